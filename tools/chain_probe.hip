// Chain-kernel latency probe (measurement tool, not shipped): the symmetric
// sharded chain's small launches timed alone on an idle GPU and beside a
// long kernel that keeps every CU busy, next to empty / copy-only launches
// of the same grid, to split a chain launch's ~15 us into launch, memory
// latency, compute and end-of-kernel cost.  Run it under
//   rocprofv3 --kernel-trace --stats -- ./chain_probe.bin
// build (in-tree, includes the library's kernels):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I shadow_amd/csrc -I include tools/chain_probe.hip \
//         -o tools/chain_probe.bin -Lshadow_amd -lsrt -Wl,-rpath,'$ORIGIN/../shadow_amd'
#include "../shadow_amd/csrc/srt_fw.hip"

#include <cstdio>
#include <vector>

namespace srt {
namespace {

__global__ void empty_kernel(uint16_t *) {}

// one 64 x 64 quarter of tile (k, c) per workgroup: read, write back, plus
// its transposed mirror -- the p2row launch's memory traffic, no compute
__global__ __launch_bounds__(256) void copy_quarter_kernel(uint16_t *D, uint32_t Vp, uint32_t k) {
    __shared__ uint16_t T[SQ][SQ + 1];
    uint32_t c = blockIdx.x >> 2;
    if (c >= k) ++c;
    const uint32_t q = blockIdx.x & 3;
    const uint64_t i0 = (uint64_t)k * B + (q >> 1) * SQ, j0 = (uint64_t)c * B + (q & 1) * SQ;
    const int tx = threadIdx.x % 16, ty = threadIdx.x / 16;
    uint2 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = *reinterpret_cast<const uint2 *>(D + (i0 + ty * 4 + i) * Vp + j0 + tx * 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[i].x = v[i].x < 0x7fff7fffu ? v[i].x : 0x7fff7fffu;
        *reinterpret_cast<uint2 *>(D + (i0 + ty * 4 + i) * Vp + j0 + tx * 4) = v[i];
        const uint16_t *h = reinterpret_cast<const uint16_t *>(&v[i]);
        for (int e = 0; e < 4; ++e) T[tx * 4 + e][ty * 4 + i] = h[e];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = ty * 4 + i;
        uint2 w;
        w.x = (uint32_t)T[r][tx * 4] | ((uint32_t)T[r][tx * 4 + 1] << 16);
        w.y = (uint32_t)T[r][tx * 4 + 2] | ((uint32_t)T[r][tx * 4 + 3] << 16);
        *reinterpret_cast<uint2 *>(D + (j0 + r) * Vp + i0 + tx * 4) = w;
    }
}

// the busy neighbour: many short workgroups (like the rest launch's tiles),
// each spinning for `ticks` and writing to a buffer (dirty lines in every L2)
__global__ __launch_bounds__(256) void busy_kernel(uint32_t *buf, long long ticks) {
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    uint32_t x = threadIdx.x;
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        for (int r = 0; r < 64; ++r) x = x * 1664525u + 1013904223u;
        buf[i] = x;
        i = (i + 256ull * 1024) % (64ull << 20);
    }
}

}  // namespace
}  // namespace srt

using namespace srt;

int main() {
    const uint32_t Vp = 16384, nblk = Vp / B, k = 37;
    uint16_t *D;
    uint32_t *buf;
    if (hipMalloc(&D, (size_t)Vp * Vp * 2) != hipSuccess || hipMalloc(&buf, 256u << 20) != hipSuccess) return 1;
    std::vector<uint16_t> row((size_t)Vp);
    for (uint32_t i = 0; i < Vp; ++i) row[i] = (uint16_t)(1 + (i * 2654435761u >> 22) % 200);
    for (uint32_t r = 0; r < Vp; ++r) hipMemcpy(D + (size_t)r * Vp, row.data(), Vp * 2, hipMemcpyHostToDevice);
    hipStream_t M, S;
    hipStreamCreateWithFlags(&M, hipStreamNonBlocking);
    int lo, hi;
    hipDeviceGetStreamPriorityRange(&lo, &hi);
    hipStreamCreateWithPriority(&S, hipStreamNonBlocking, hi);
    const Rect row_r{make_span(k, k + 1), make_span(0, nblk, k)};
    const Rect none{make_span(0, 0), make_span(0, 0)};
    const PackSpec nopack{nullptr, 0u, 0u, 1u, 1u};
    const uint32_t nq = 4 * row_r.c.n;
    for (int busy = 0; busy < 2; ++busy) {
        if (busy) hipLaunchKernelGGL(busy_kernel, dim3(40000), dim3(256), 0, M, buf, 2000LL);  // 20 us a workgroup
        for (int rep = 0; rep < 20; ++rep) {
            hipLaunchKernelGGL(empty_kernel, dim3(nq), dim3(256), 0, S, D);
            hipLaunchKernelGGL(copy_quarter_kernel, dim3(nq), dim3(256), 0, S, D, Vp, k);
            hipLaunchKernelGGL((minplus_q16_kernel<1, 1, true>), dim3(nq), dim3(256), 0, S, D, Vp, k, row_r, none, 1u,
                               nopack);
            hipLaunchKernelGGL((fw_phase1_pk2_kernel<4, true>), dim3(1), dim3(512), 0, S, D, Vp, k);
        }
        hipDeviceSynchronize();
        std::printf("pass %d (%s) done\n", busy, busy ? "beside a busy kernel" : "idle GPU");
    }
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
