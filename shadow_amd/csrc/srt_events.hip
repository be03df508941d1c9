// srt_events.hip -- batched packet-event push for one round.
//
// Reference: Worker::push_packet_to_host (src/main/core/worker.rs:629-639)
// wraps every packet send_packet marked SENT in Event::new_packet
// (core/work/event.rs:20-31) -- src_host_event_id = the source host's next
// event id, Host::get_new_event_id (host/host.rs:691-695), taken in send
// order -- and pushes it on the destination host's event queue, which pops
// events by (time, then data): packet data orders by (src_host_id,
// src_host_event_id) (event.rs:85-150).
//
// Here, for the whole batch at once: (A) one lane per source host walks its
// packets in send order and hands out event ids to the sent ones; (B) the sent
// packets are sorted by (destination host, deliver time), stably from batch
// order -- which is (source host, send order), i.e. (src_host_id,
// src_host_event_id) order, since host segments are laid out by host index ==
// HostId order.  One reduction finds the sent deliver-time span; when its bits
// plus the destination bits fit 64, one rocPRIM radix sort of the combined key
// (destination << tbits | deliver - tmin) over exactly those bits does it (C5:
// 43 bits), else two stable LSD sorts (time, then destination); (C) per
// destination host the offsets of its events (its queue's pop order).
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>

#include "srt_internal.h"

namespace {

// (A) event ids; keys for (B)
__global__ __launch_bounds__(64) void event_id_kernel(const uint32_t *__restrict__ host_ptr, uint32_t n_hosts,
                                                      const uint32_t *__restrict__ flags,
                                                      uint64_t *__restrict__ base, uint64_t *__restrict__ event_id) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= n_hosts) return;
    uint64_t next = base[h];
    const uint32_t b = host_ptr[h], e = host_ptr[h + 1];
    for (uint32_t p = b; p < e; ++p) event_id[p] = flags[p] == SRT_PDS_INET_SENT ? next++ : ~0ull;
    base[h] = next;
}

// Range of the sent packets' deliver times and the destination range check:
// per-block partials {min, max, bad} -> range[0..2] by one workgroup (no
// same-address atomics from every block).
constexpr int RB = 256;
__global__ __launch_bounds__(RB) void event_range_kernel(const uint32_t *__restrict__ flags,
                                                         const uint64_t *__restrict__ deliver,
                                                         const uint32_t *__restrict__ dst, uint32_t n_dst, uint64_t n,
                                                         unsigned long long *__restrict__ part) {
    unsigned long long mn = ~0ull, mx = 0, bad = 0;
    for (uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x) {
        if (flags[p] != SRT_PDS_INET_SENT) continue;
        const unsigned long long d = deliver[p];
        mn = d < mn ? d : mn;
        mx = d > mx ? d : mx;
        bad |= dst[p] >= n_dst;
    }
    __shared__ unsigned long long r[3][RB];
    r[0][threadIdx.x] = mn;
    r[1][threadIdx.x] = mx;
    r[2][threadIdx.x] = bad;
    __syncthreads();
    for (int s = RB / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            r[0][threadIdx.x] = r[0][threadIdx.x + s] < r[0][threadIdx.x] ? r[0][threadIdx.x + s] : r[0][threadIdx.x];
            r[1][threadIdx.x] = r[1][threadIdx.x + s] > r[1][threadIdx.x] ? r[1][threadIdx.x + s] : r[1][threadIdx.x];
            r[2][threadIdx.x] |= r[2][threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part[3 * blockIdx.x] = r[0][0];
        part[3 * blockIdx.x + 1] = r[1][0];
        part[3 * blockIdx.x + 2] = r[2][0];
    }
}

__global__ __launch_bounds__(RB) void event_range_final_kernel(const unsigned long long *__restrict__ part,
                                                               uint32_t nb, unsigned long long *__restrict__ range) {
    unsigned long long mn = ~0ull, mx = 0, bad = 0;
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) {
        mn = part[3 * b] < mn ? part[3 * b] : mn;
        mx = part[3 * b + 1] > mx ? part[3 * b + 1] : mx;
        bad |= part[3 * b + 2];
    }
    __shared__ unsigned long long r[3][RB];
    r[0][threadIdx.x] = mn;
    r[1][threadIdx.x] = mx;
    r[2][threadIdx.x] = bad;
    __syncthreads();
    for (int s = RB / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            r[0][threadIdx.x] = r[0][threadIdx.x + s] < r[0][threadIdx.x] ? r[0][threadIdx.x + s] : r[0][threadIdx.x];
            r[1][threadIdx.x] = r[1][threadIdx.x + s] > r[1][threadIdx.x] ? r[1][threadIdx.x + s] : r[1][threadIdx.x];
            r[2][threadIdx.x] |= r[2][threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        range[0] = r[0][0];
        range[1] = r[1][0];
        range[2] = r[2][0];
    }
}

// one combined key per packet: (destination << tbits) | (deliver - tmin);
// unsent packets get destination n_dst (they sort last)
__global__ void event_keys_kernel(const uint32_t *__restrict__ flags, const uint64_t *__restrict__ deliver,
                                  const uint32_t *__restrict__ dst, uint32_t n_dst, uint64_t tmin, int tbits,
                                  uint64_t n, uint64_t *__restrict__ key, uint32_t *__restrict__ idx) {
    for (uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x) {
        const bool sent = flags[p] == SRT_PDS_INET_SENT;
        key[p] = sent ? ((uint64_t)dst[p] << tbits) | (deliver[p] - tmin) : (uint64_t)n_dst << tbits;
        idx[p] = (uint32_t)p;
    }
}

// (C) for the combined-key path: dst_ptr[d] = first sorted key >= d << tbits
__global__ void event_dst_ptr64_kernel(const uint64_t *__restrict__ key, uint64_t n, uint32_t n_dst, int tbits,
                                       uint32_t *__restrict__ dst_ptr) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d > n_dst) return;
    const uint64_t kd = (uint64_t)d << tbits;
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (key[mid] < kd) lo = mid + 1;
        else hi = mid;
    }
    dst_ptr[d] = (uint32_t)lo;
}

// general path (time span + destination bits > 64): time keys first
__global__ void event_time_keys_kernel(const uint32_t *__restrict__ flags, const uint64_t *__restrict__ deliver,
                                       uint64_t n, uint64_t *__restrict__ ktime, uint32_t *__restrict__ idx) {
    for (uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x) {
        ktime[p] = flags[p] == SRT_PDS_INET_SENT ? deliver[p] : ~0ull;
        idx[p] = (uint32_t)p;
    }
}

// destination key in time order; unsent packets sort last (key n_dst)
__global__ void event_dst_keys_kernel(const uint32_t *__restrict__ idx, const uint32_t *__restrict__ flags,
                                      const uint32_t *__restrict__ dst, uint32_t n_dst, uint64_t n,
                                      uint32_t *__restrict__ kdst) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t p = idx[i];
        uint32_t k = n_dst;
        if (flags[p] == SRT_PDS_INET_SENT) k = dst[p];  // range-checked by event_range_kernel
        kdst[i] = k;
    }
}

// (C) dst_ptr[d] = first position of destination d in the sorted keys
__global__ void event_dst_ptr_kernel(const uint32_t *__restrict__ kdst, uint64_t n, uint32_t n_dst,
                                     uint32_t *__restrict__ dst_ptr) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d > n_dst) return;
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (kdst[mid] < d) lo = mid + 1;
        else hi = mid;
    }
    dst_ptr[d] = (uint32_t)lo;
}

void set_err(srt_err *err, srt_status code, const char *msg) {
    if (!err) return;
    err->code = code;
    std::snprintf(err->msg, sizeof err->msg, "%s", msg);
}

int bit_width64(uint64_t x) {
    int b = 0;
    while (x) {
        ++b;
        x >>= 1;
    }
    return b;
}

int bit_width(uint32_t x) {
    int b = 0;
    while (x) {
        ++b;
        x >>= 1;
    }
    return b;
}

}  // namespace

namespace srt {
// srt_init: loads this unit's code object (srt::preload_kernels)
hipError_t preload_events() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&event_id_kernel));
}
}  // namespace srt

extern "C" srt_status srt_packet_events(srt_plan *plan, const uint32_t *d_host_pkt_ptr, uint32_t n_hosts,
                                        uint64_t n_pkts, const uint32_t *d_flags, const uint64_t *d_deliver,
                                        const uint32_t *d_dst_host, uint32_t n_dst_hosts, uint64_t *d_event_base,
                                        uint64_t *d_event_id, uint32_t *d_order, uint32_t *d_dst_ptr,
                                        srt_err *err) {
    if (err) std::memset(err, 0, sizeof *err);
    if (!plan || !d_host_pkt_ptr || !d_dst_ptr || (n_hosts && !d_event_base) ||
        (n_pkts && (!d_flags || !d_deliver || !d_dst_host || !d_event_id || !d_order))) {
        set_err(err, SRT_ERR_INVALID, "null argument");
        return SRT_ERR_INVALID;
    }
    if (n_pkts >= 0xffffffffull || n_dst_hosts >= 0xffffffffu) {
        set_err(err, SRT_ERR_INVALID, "more than 2^32-2 packets or destination hosts in one batch");
        return SRT_ERR_INVALID;
    }
    if (hipSetDevice(plan->device) != hipSuccess) return SRT_ERR_HIP;
    hipStream_t s = plan->stream;
    const uint32_t n = (uint32_t)n_pkts;
    if (n_hosts)
        hipLaunchKernelGGL(event_id_kernel, dim3((n_hosts + 63) / 64), dim3(64), 0, s, d_host_pkt_ptr, n_hosts, d_flags,
                           d_event_base, d_event_id);
    if (!n) {
        hipLaunchKernelGGL(event_dst_ptr_kernel, dim3(n_dst_hosts / 256 + 1), dim3(256), 0, s,
                           (const uint32_t *)nullptr, 0ull, n_dst_hosts, d_dst_ptr);
        return hipGetLastError() == hipSuccess ? SRT_OK : SRT_ERR_HIP;
    }
    const int dbits = std::max(bit_width(n_dst_hosts), 1);  // keys 0..n_dst_hosts
    // scratch: key[2n] u64, idx[2n] u32, kdst[2n] u32, range partials, rocPRIM temp
    const uint32_t rblocks = std::min<uint32_t>((n + RB - 1) / RB, 1024);
    size_t t1 = 0, t2 = 0;
    rocprim::radix_sort_pairs((void *)nullptr, t1, (uint64_t *)nullptr, (uint64_t *)nullptr, (uint32_t *)nullptr,
                              (uint32_t *)nullptr, n, 0, 64, s);
    rocprim::radix_sort_pairs((void *)nullptr, t2, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                              (uint32_t *)nullptr, n, 0, (unsigned)dbits, s);
    const size_t temp = std::max(t1, t2);
    const size_t need = 16ull * n + 16ull * n + 8ull * (3 * rblocks + 4) + 512 + temp;
    if (need > plan->ev_scratch_cap) {
        if (plan->d_ev_scratch) (void)hipFree(plan->d_ev_scratch);
        plan->d_ev_scratch = nullptr;
        plan->ev_scratch_cap = 0;
        if (hipMalloc(&plan->d_ev_scratch, need) != hipSuccess) {
            set_err(err, SRT_ERR_OOM, "hipMalloc(event scratch) failed");
            return SRT_ERR_OOM;
        }
        plan->ev_scratch_cap = need;
    }
    char *sp = (char *)plan->d_ev_scratch;
    uint64_t *key = (uint64_t *)sp, *key_s = key + n;
    uint32_t *idx = (uint32_t *)(key_s + n), *idx1 = idx + n;
    uint32_t *kdst = idx1 + n, *kdst_s = kdst + n;
    unsigned long long *part = (unsigned long long *)(kdst_s + n), *range = part + 3 * rblocks;
    // rocPRIM partitions its temporary storage assuming an aligned base
    void *tmp = (void *)(((uintptr_t)(range + 4) + 255) & ~(uintptr_t)255);
    // sent range + destination check (the one host round trip of the call)
    hipLaunchKernelGGL(event_range_kernel, dim3(rblocks), dim3(RB), 0, s, d_flags, d_deliver, d_dst_host, n_dst_hosts,
                       (uint64_t)n, part);
    hipLaunchKernelGGL(event_range_final_kernel, dim3(1), dim3(RB), 0, s, part, rblocks, range);
    unsigned long long h_range[3] = {0, 0, 0};
    if (hipMemcpyAsync(h_range, range, sizeof h_range, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        set_err(err, SRT_ERR_HIP, "packet events: stream failed");
        return SRT_ERR_HIP;
    }
    if (h_range[2]) {
        set_err(err, SRT_ERR_INVALID, "destination host index out of range");
        return SRT_ERR_INVALID;
    }
    const uint32_t blocks = std::min<uint32_t>((n + 255) / 256, 4096);
    const uint64_t tmin = h_range[0] == ~0ull ? 0 : h_range[0];
    const int tbits = h_range[0] == ~0ull ? 0 : bit_width64(h_range[1] - h_range[0]);
    size_t ts = temp;
    if (tbits + dbits <= 64) {
        size_t tc = 0;  // this sort's own size (bit count dependent): never more than allotted
        rocprim::radix_sort_pairs((void *)nullptr, tc, (uint64_t *)nullptr, (uint64_t *)nullptr, (uint32_t *)nullptr,
                                  (uint32_t *)nullptr, n, 0, (unsigned)(tbits + dbits), s);
        if (tc > temp) {
            set_err(err, SRT_ERR_HIP, "radix sort temporary storage larger than sized");
            return SRT_ERR_HIP;
        }
        // one sort of (destination, deliver - tmin) keys, stable from batch order
        hipLaunchKernelGGL(event_keys_kernel, dim3(blocks), dim3(256), 0, s, d_flags, d_deliver, d_dst_host,
                           n_dst_hosts, tmin, tbits, (uint64_t)n, key, idx);
        if (rocprim::radix_sort_pairs(tmp, ts, key, key_s, idx, d_order, n, 0, (unsigned)(tbits + dbits), s) !=
            hipSuccess) {
            set_err(err, SRT_ERR_HIP, "radix sort (destination, deliver time) failed");
            return SRT_ERR_HIP;
        }
        hipLaunchKernelGGL(event_dst_ptr64_kernel, dim3(n_dst_hosts / 256 + 1), dim3(256), 0, s, key_s, (uint64_t)n,
                           n_dst_hosts, tbits, d_dst_ptr);
    } else {
        // general: stable sort by deliver time, then stable sort by destination
        hipLaunchKernelGGL(event_time_keys_kernel, dim3(blocks), dim3(256), 0, s, d_flags, d_deliver, (uint64_t)n,
                           key, idx);
        if (rocprim::radix_sort_pairs(tmp, ts, key, key_s, idx, idx1, n, 0, 64, s) != hipSuccess) {
            set_err(err, SRT_ERR_HIP, "radix sort (deliver time) failed");
            return SRT_ERR_HIP;
        }
        hipLaunchKernelGGL(event_dst_keys_kernel, dim3(blocks), dim3(256), 0, s, idx1, d_flags, d_dst_host,
                           n_dst_hosts, (uint64_t)n, kdst);
        ts = temp;
        if (rocprim::radix_sort_pairs(tmp, ts, kdst, kdst_s, idx1, d_order, n, 0, (unsigned)dbits, s) != hipSuccess) {
            set_err(err, SRT_ERR_HIP, "radix sort (destination host) failed");
            return SRT_ERR_HIP;
        }
        hipLaunchKernelGGL(event_dst_ptr_kernel, dim3(n_dst_hosts / 256 + 1), dim3(256), 0, s, kdst_s, (uint64_t)n,
                           n_dst_hosts, d_dst_ptr);
    }
    return hipGetLastError() == hipSuccess ? SRT_OK : SRT_ERR_HIP;
}
