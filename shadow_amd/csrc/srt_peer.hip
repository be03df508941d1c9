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

// Position-weighted checksum of a buffer: the sum over its u32 words w_i of
// (w_i + 1) (2 i + 1) mod 2^64 (bytes, weighted by byte position, when the
// buffer is not word-aligned).  One flipped bit changes it (the weights are
// odd), and so does a word moved to another place.
__global__ __launch_bounds__(256) void cksum_kernel(const uint8_t *__restrict__ p, uint64_t bytes, int words,
                                                    unsigned long long *out) {
    unsigned long long acc = 0;
    const uint64_t n = words ? bytes / 4 : bytes;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t w = words ? reinterpret_cast<const uint32_t *>(p)[i] : p[i];
        acc += (w + 1ull) * (2ull * i + 1ull);
    }
    if (words && blockIdx.x == 0 && threadIdx.x == 0)
        for (uint64_t b = n * 4; b < bytes; ++b) acc += ((uint64_t)p[b] + 1ull) * (2ull * (n + b) + 1ull);
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

__global__ void cksum_cmp_kernel(const unsigned long long *a, const unsigned long long *b, uint32_t *bad) {
    if (*a != *b) atomicOr(bad, 1u);
}

__global__ void flip_byte_kernel(uint8_t *p) { p[0] ^= 0x40u; }  // a value bit of the slot's last word

}  // namespace

void checksum(const void *d, uint64_t bytes, unsigned long long *out, hipStream_t s) {
    (void)hipMemsetAsync(out, 0, sizeof *out, s);
    if (!bytes) return;
    const int words = ((uintptr_t)d % 4) == 0;
    const uint64_t n = words ? bytes / 4 : bytes;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(1024, std::max<uint64_t>(1, n / 2048));
    hipLaunchKernelGGL(cksum_kernel, dim3(blocks), dim3(256), 0, s, (const uint8_t *)d, bytes, words, out);
}

void checksum_cmp(const unsigned long long *a, const unsigned long long *b, uint32_t *bad, hipStream_t s) {
    hipLaunchKernelGGL(cksum_cmp_kernel, dim3(1), dim3(1), 0, s, a, b, bad);
}

void corrupt_byte(void *d, uint64_t bytes, hipStream_t s) {
    if (bytes) hipLaunchKernelGGL(flip_byte_kernel, dim3(1), dim3(1), 0, s, (uint8_t *)d + bytes - 1);
}

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
