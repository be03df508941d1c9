// srt_peer.hip -- the copy kernel of the in-process communicator (srt_comm.cpp,
// srt_comm_init_local): every rank's slot gathered straight from the other
// ranks' device buffers (xGMI peer reads on a multi-GPU node; plain device
// copies when several ranks share one GPU), one launch per collective.
#include <algorithm>

#include "srt_internal.h"

namespace srt {

namespace {

// grid-stride copy of every source rank's slot [q * bytes, (q+1) * bytes) of
// src[q] into the same range of dst (skip: the calling rank's own slot), or,
// for a broadcast (only = root, not slotted), [0, bytes) of the root's buffer.
// Widest access the alignment of all pointers and the slot size allows.
template <typename T>
__global__ __launch_bounds__(256) void peer_gather_kernel(uint8_t *dst, PeerSrcs src, uint64_t bytes, int nranks,
                                                          int skip, int only, int slotted) {
    const uint64_t n = bytes / sizeof(T);
    const uint64_t total = n * (uint64_t)nranks;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const int q = (int)(e / n);
        if (q == skip || (only >= 0 && q != only)) continue;
        const uint64_t i = e % n;
        const uint64_t off = (slotted ? (uint64_t)q * bytes : 0) + i * sizeof(T);
        *reinterpret_cast<T *>(dst + off) = *reinterpret_cast<const T *>(src.p[q] + off);
    }
}

}  // namespace

// dst's slots <- src[q]'s slots (q != skip; only >= 0: that slot alone), on s
void peer_gather(uint8_t *dst, const PeerSrcs &src, uint64_t bytes, int nranks, int skip, int only, hipStream_t s) {
    const int slotted = only < 0;
    uintptr_t a = (uintptr_t)dst | (uintptr_t)bytes;
    for (int q = 0; q < nranks; ++q) a |= (uintptr_t)src.p[q];
    const uint64_t copied = bytes * (uint64_t)(only >= 0 ? 1 : nranks - 1);
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(2048, std::max<uint64_t>(1, copied / 4096));
    if (a % 16 == 0)
        hipLaunchKernelGGL(peer_gather_kernel<uint4>, dim3(blocks), dim3(256), 0, s, dst, src, bytes, nranks, skip,
                           only, slotted);
    else if (a % 4 == 0)
        hipLaunchKernelGGL(peer_gather_kernel<uint32_t>, dim3(blocks), dim3(256), 0, s, dst, src, bytes, nranks, skip,
                           only, slotted);
    else
        hipLaunchKernelGGL(peer_gather_kernel<uint8_t>, dim3(blocks), dim3(256), 0, s, dst, src, bytes, nranks, skip,
                           only, slotted);
}

}  // namespace srt
