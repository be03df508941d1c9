// Cross-stream dependency latency on one GPU (measurement tool, not shipped):
// stream M runs a spin kernel, stream S a tiny kernel that must start after
// it.  Each mode orders them differently; the kernels stamp the wall clock
// (s_memrealtime, 100 MHz) so the gap "M kernel end -> S kernel start" is
// read back without a profiler.  "satisfied": S is still busy with a longer
// spin when M finishes, so the wait is already satisfied when S reaches it
// (the symmetric sharded chain's case).
//   modes: 0 hipEventRecord / hipStreamWaitEvent
//          1 hipStreamWriteValue32 / hipStreamWaitValue32
//          2 the M kernel's last store releases a flag / hipStreamWaitValue32
//          3 no dependency (the plain kernel-to-kernel gap on S)
// build: hipcc --offload-arch=gfx950 -O2 tools/wait_probe.hip -o /tmp/wait_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }

__global__ void spin_kernel(long long ticks, unsigned long long *stamp, unsigned *flag, unsigned v) {
    const unsigned long long t0 = now();
    while ((long long)(now() - t0) < ticks) __builtin_amdgcn_s_sleep(1);
    if (threadIdx.x == 0) {
        stamp[0] = now();
        if (flag) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ void tiny_kernel(unsigned long long *stamp) {
    if (threadIdx.x == 0) stamp[0] = now();
}

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

int main() {
    int can = 0;
    CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0));
    std::printf("CanUseStreamWaitValue=%d\n", can);
    hipStream_t M, S;
    CK(hipStreamCreateWithFlags(&M, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&S, hipStreamNonBlocking));
    const int IT = 64;
    unsigned long long *st;
    unsigned *flag;
    CK(hipMalloc(&st, 4 * IT * 8));
    CK(hipMalloc(&flag, 64));
    std::vector<hipEvent_t> ev(IT), back(IT);
    for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
    for (auto &e : back) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
    for (int sat = 0; sat < 2; ++sat)
        for (int mode = 0; mode < 4; ++mode) {
            if ((mode == 1 || mode == 2) && !can) continue;
            CK(hipMemset(flag, 0, 64));
            CK(hipMemset(st, 0, 4 * IT * 8));
            CK(hipDeviceSynchronize());
            for (int i = 0; i < IT; ++i) {
                const unsigned v = (unsigned)(i + 1);
                // M: 40 us spin; S: (satisfied) 60 us spin first, then the wait and the tiny kernel
                hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, M, 4000LL, st + 4 * i, mode == 2 ? flag : nullptr,
                                   v);
                if (sat) hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, S, 6000LL, st + 4 * i + 2, nullptr, 0u);
                if (mode == 3) {
                } else if (mode == 0) {
                    CK(hipEventRecord(ev[i], M));
                    CK(hipStreamWaitEvent(S, ev[i], 0));
                } else {
                    if (mode == 1) CK(hipStreamWriteValue32(M, flag, v, 0));
                    CK(hipStreamWaitValue32(S, flag, v, hipStreamWaitValueGte, 0xffffffffu));
                }
                hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, S, st + 4 * i + 1);
                // keep M behind S so iterations do not overlap
                CK(hipEventRecord(back[i], S));
                CK(hipStreamWaitEvent(M, back[i], 0));
            }
            CK(hipDeviceSynchronize());
            std::vector<unsigned long long> h(4 * IT);
            CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
            std::vector<double> gap;
            for (int i = 4; i < IT; ++i) {
                const unsigned long long ready = sat ? std::max(h[4 * i], h[4 * i + 2]) : h[4 * i];
                gap.push_back(((long long)(h[4 * i + 1] - ready)) / 100.0);
            }
            std::sort(gap.begin(), gap.end());
            std::printf("%s mode %d: gap us  min %.2f  median %.2f  p90 %.2f\n", sat ? "satisfied" : "pending  ", mode,
                        gap.front(), gap[gap.size() / 2], gap[gap.size() * 9 / 10]);
        }
    return 0;
}
