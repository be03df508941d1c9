// stream_gap.hip -- cost of a cross-stream dependency between back-to-back
// kernels on the main stream (the FW round schedule's rest(kb) -> rest(kb+1)
// hand-off, ~15 us between rest kernels in every rocprofv3 trace).
//
// M runs N busy kernels back to back; before each one, variant:
//   none      no wait
//   event     hipStreamWaitEvent on an event S recorded after a tiny kernel
//   event_nf  same, events created with hipEventDisableSystemFence
//   value     hipStreamWaitValue64 on a flag S sets with hipStreamWriteValue64
// S is always far ahead (its work is tiny), so every wait is already satisfied
// when M reaches it: the difference to "none" is the packet overhead alone.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

__global__ void busy_kernel(double *out, int iters) {
    double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
    for (int i = 0; i < iters; ++i) {
        a = a * 0.999 + b;
        b = b * 0.998 + a;
    }
    if (a == 12345.0) out[threadIdx.x] = b;  // keeps the loop
}

// busy + writes: every thread stores `per` doubles (dirty lines left in L2)
__global__ void busy_write_kernel(double *out, int iters, int per) {
    double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
    for (int i = 0; i < iters; ++i) {
        a = a * 0.999 + b;
        b = b * 0.998 + a;
    }
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x, nt = (size_t)gridDim.x * blockDim.x;
    for (int k = 0; k < per; ++k) out[t + k * nt] = a + k;
}

__global__ void tiny_kernel(double *out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] += 1.0;
}

int main(int argc, char **argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 200;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 4000;
    double *buf;
    CK(hipMalloc(&buf, 1 << 20));
    uint64_t *flag;
    CK(hipMalloc(&flag, 4096));
    CK(hipMemset(flag, 0, 4096));
    hipStream_t M, S;
    CK(hipStreamCreateWithFlags(&M, hipStreamNonBlocking));
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithPriority(&S, hipStreamNonBlocking, hi));
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    const char *names[] = {"none", "event", "event_nf", "value"};
    for (int rep = 0; rep < 2; ++rep)
        for (int v = 0; v < 4; ++v) {
            std::vector<hipEvent_t> evs(N);
            for (int i = 0; i < N; ++i)
                CK(hipEventCreateWithFlags(&evs[i], hipEventDisableTiming |
                                                       (v == 2 ? hipEventDisableSystemFence : 0u)));
            CK(hipMemset(flag, 0, 4096));
            CK(hipDeviceSynchronize());
            // S: all its hand-offs first (tiny), so every M wait is satisfied
            for (int i = 0; i < N; ++i) {
                hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, S, buf + 1024);
                if (v == 1 || v == 2) CK(hipEventRecord(evs[i], S));
                if (v == 3) CK(hipStreamWriteValue64(S, flag, (uint64_t)(i + 1), 0));
            }
            CK(hipStreamSynchronize(S));
            CK(hipEventRecord(t0, M));
            for (int i = 0; i < N; ++i) {
                if (v == 1 || v == 2) CK(hipStreamWaitEvent(M, evs[i], 0));
                if (v == 3) CK(hipStreamWaitValue64(M, flag, (uint64_t)(i + 1), hipStreamWaitValueGte, ~0ull));
                hipLaunchKernelGGL(busy_kernel, dim3(512), dim3(256), 0, M, buf, iters);
            }
            CK(hipEventRecord(t1, M));
            CK(hipEventSynchronize(t1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, t0, t1));
            std::printf("rep %d %-9s %d kernels: %.3f ms total, %.2f us per kernel\n", rep, names[v], N, ms,
                        ms * 1e3 / N);
            for (auto e : evs) CK(hipEventDestroy(e));
        }
    // concurrent variant: S's hand-off is produced while M's previous kernel runs
    // (the real schedule), event wait vs none
    for (int v = 0; v < 2; ++v) {
        std::vector<hipEvent_t> evs(N);
        for (int i = 0; i < N; ++i) CK(hipEventCreateWithFlags(&evs[i], hipEventDisableTiming));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(t0, M));
        for (int i = 0; i < N; ++i) {
            hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, S, buf + 1024);
            CK(hipEventRecord(evs[i], S));
            if (v) CK(hipStreamWaitEvent(M, evs[i], 0));
            hipLaunchKernelGGL(busy_kernel, dim3(512), dim3(256), 0, M, buf, iters);
        }
        CK(hipEventRecord(t1, M));
        CK(hipEventSynchronize(t1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, t0, t1));
        std::printf("interleaved %-6s %d kernels: %.3f ms total, %.2f us per kernel\n", v ? "event" : "none", N, ms,
                    ms * 1e3 / N);
        for (auto e : evs) CK(hipEventDestroy(e));
    }
    // write-heavy kernels (each leaves `per` x 1 MB... of stores): gap with no
    // events, with an event recorded after each kernel (system fence / none)
    const int per = argc > 3 ? std::atoi(argv[3]) : 64;
    double *big;
    CK(hipMalloc(&big, (size_t)512 * 256 * per * 8));
    const char *wn[] = {"w_none", "w_ev_sys", "w_ev_nofence", "w_ev_timing_nf"};
    for (int rep = 0; rep < 2; ++rep)
        for (int v = 0; v < 4; ++v) {
            std::vector<hipEvent_t> evs(N);
            const unsigned fl = v == 1 ? hipEventDisableTiming
                                : v == 2 ? (hipEventDisableTiming | hipEventDisableSystemFence)
                                         : hipEventDisableSystemFence;
            for (int i = 0; i < N; ++i) CK(hipEventCreateWithFlags(&evs[i], fl));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(t0, M));
            for (int i = 0; i < N; ++i) {
                hipLaunchKernelGGL(busy_write_kernel, dim3(512), dim3(256), 0, M, big, iters, per);
                if (v) CK(hipEventRecord(evs[i], M));
            }
            CK(hipEventRecord(t1, M));
            CK(hipEventSynchronize(t1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, t0, t1));
            std::printf("rep %d %-15s %d kernels x %d MB stores: %.3f ms total, %.2f us per kernel\n", rep, wn[v], N,
                        512 * 256 * per * 8 >> 20, ms, ms * 1e3 / N);
            for (auto e : evs) CK(hipEventDestroy(e));
        }
    // the FW round schedule, mimicked: M = [wait pivot(i)] [timing ev] rest(i)
    // [timing ev = rest_done(i)]; S = [wait rest_done(i-1)] cross, p1, p2row,
    // p2col [record pivot(i+1)].  Variants: sync events with / without the
    // system fence, with / without timing events on M.
    for (int rep = 0; rep < 2; ++rep)
        for (int v = 0; v < 4; ++v) {
            const bool sync_nf = v & 1, timing = !(v & 2);
            std::vector<hipEvent_t> piv(N + 1), rd(N), tb(N);
            for (int i = 0; i <= N; ++i)
                CK(hipEventCreateWithFlags(&piv[i], hipEventDisableTiming | (sync_nf ? hipEventDisableSystemFence : 0u)));
            for (int i = 0; i < N; ++i) {
                CK(hipEventCreateWithFlags(&rd[i], timing ? hipEventDisableSystemFence
                                                          : (hipEventDisableTiming | (sync_nf ? hipEventDisableSystemFence : 0u))));
                CK(hipEventCreateWithFlags(&tb[i], hipEventDisableSystemFence));
            }
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(t0, M));
            CK(hipEventRecord(piv[0], M));
            for (int i = 0; i < N; ++i) {
                if (i) CK(hipStreamWaitEvent(S, rd[i - 1], 0));
                if (i) CK(hipStreamWaitEvent(M, piv[i], 0));
                if (timing) CK(hipEventRecord(tb[i], M));
                hipLaunchKernelGGL(busy_write_kernel, dim3(512), dim3(256), 0, M, big, iters, per);
                CK(hipEventRecord(rd[i], M));
                // chain: 4 small write kernels (quarter of the chip, short)
                for (int c = 0; c < 4; ++c)
                    hipLaunchKernelGGL(busy_write_kernel, dim3(128), dim3(256), 0, S, big, iters / 8, 4);
                CK(hipEventRecord(piv[i + 1], S));
            }
            CK(hipEventRecord(t1, M));
            CK(hipEventSynchronize(t1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, t0, t1));
            std::printf("rep %d sched sync_nf=%d timing=%d: %.3f ms total, %.2f us per round\n", rep, (int)sync_nf,
                        (int)timing, ms, ms * 1e3 / N);
            for (auto e : piv) CK(hipEventDestroy(e));
            for (auto e : rd) CK(hipEventDestroy(e));
            for (auto e : tb) CK(hipEventDestroy(e));
        }
    return 0;
}
