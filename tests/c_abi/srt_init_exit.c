/* A C process that starts the library's asynchronous init and then leaves
 * before any build -- what Shadow does when it calls srt_init_async at the top
 * of main and then exits on --help, --version or a config/GML error
 * (sim_config.rs:136-140 runs only after those checks).  The process must end
 * with its own exit status, never a signal, whatever phase the init thread is
 * in when exit starts.
 *
 *   srt_init_exit <delay_us> [return|exit]
 *     delay_us: time between srt_init_async and leaving main
 *     return:   return 3 from main; exit: exit(3) from a nested call
 */
#define _POSIX_C_SOURCE 199309L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "srt.h"

static void config_error(void) {
    fprintf(stderr, "config error: leaving before the routing build\n");
    exit(3);
}

int main(int argc, char **argv) {
    const long us = argc > 1 ? atol(argv[1]) : 0;
    const int use_exit = argc > 2 && strcmp(argv[2], "exit") == 0;
    srt_init_async(0);
    if (us > 0) {
        struct timespec ts = {us / 1000000, (us % 1000000) * 1000};
        nanosleep(&ts, NULL);
    }
    if (use_exit) config_error();
    return 3;
}
