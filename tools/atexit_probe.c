/* Diagnostic (not a test, not product): which exit-time destructors get
 * registered, by which shared object, while srt_init_async's thread runs.
 *
 * glibc runs atexit / __cxa_atexit entries in reverse order of registration,
 * so an entry registered by the init thread AFTER libsrt's own join handler
 * runs BEFORE that join at exit -- while the thread may still be using the
 * object it destroys.  This executable defines __cxa_atexit (shared objects
 * bind to the executable's definition first), logs every registration with
 * its time, thread and the DSO of the destructor, and forwards to glibc.
 *
 *   gcc -O1 -rdynamic -o tools/atexit_probe tools/atexit_probe.c \
 *       -Lshadow_amd -lsrt -ldl -lpthread -Wl,-rpath,$PWD/shadow_amd
 *   tools/atexit_probe [device]
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/srt.h"

typedef int (*cxa_fn)(void (*)(void *), void *, void *);
static pthread_t g_main;
static double g_t0;
static int g_logging;

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec / 1e6;
}

int __cxa_atexit(void (*f)(void *), void *arg, void *dso) {
    static cxa_fn real;
    if (!real) real = (cxa_fn)dlsym(RTLD_NEXT, "__cxa_atexit");
    if (g_logging) {
        Dl_info fi, di;
        const char *fn = dladdr((void *)f, &fi) && fi.dli_fname ? fi.dli_fname : "?";
        const char *dn = dso && dladdr(dso, &di) && di.dli_fname ? di.dli_fname : "-";
        const char *sym = dladdr((void *)f, &fi) && fi.dli_sname ? fi.dli_sname : "";
        fprintf(stderr, "[atexit] %8.2f ms %s fn=%s %s dso=%s\n", now_ms() - g_t0,
                pthread_equal(pthread_self(), g_main) ? "main  " : "thread", fn, sym, dn);
    }
    return real(f, arg, dso);
}

int main(int argc, char **argv) {
    const int dev = argc > 1 ? atoi(argv[1]) : 0;
    g_main = pthread_self();
    g_t0 = now_ms();
    g_logging = 1;
    fprintf(stderr, "[atexit] srt_init_async(%d)\n", dev);
    srt_init_async(dev);
    fprintf(stderr, "[atexit] %8.2f ms srt_init_async returned\n", now_ms() - g_t0);
    srt_err err;
    memset(&err, 0, sizeof err);
    srt_status s = srt_init(dev, &err);
    fprintf(stderr, "[atexit] %8.2f ms srt_init (wait) -> %d %s\n", now_ms() - g_t0, (int)s, err.msg);
    return s == SRT_OK ? 0 : 1;
}
