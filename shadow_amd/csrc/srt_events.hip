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
// HostId order.  One rocPRIM radix sort of the combined key (destination <<
// tbits | deliver - tmin) with tmin reduced on the device and a 48-bit key
// (C5: 14 destination + 34 time bits, a 17 s span) does it, so the call never
// waits for the device; a batch whose deliver times span 2^tbits ns or more
// is flagged and srt_packet_events_status redoes it exactly (two stable
// sorts: time, then destination); (C) per destination host the offsets of its
// events (its queue's pop order).
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>

#include "srt_internal.h"

namespace {

// (A) event ids: one wave per source host; its packets in send order, 64 at
// a time, the sent ones numbered by a ballot prefix count.  The same pass
// takes the earliest deliver time of the sent packets (block-reduced, one
// atomic per workgroup into *tmin, which the previous call's last kernel left
// at ~0).
__global__ __launch_bounds__(256) void event_id_kernel(const uint32_t *__restrict__ host_ptr, uint32_t n_hosts,
                                                       const uint32_t *__restrict__ flags,
                                                       const uint64_t *__restrict__ deliver,
                                                       uint64_t *__restrict__ base, uint64_t *__restrict__ event_id,
                                                       unsigned long long *__restrict__ tmin) {
    __shared__ unsigned long long wmin[4];
    const uint32_t h = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned long long mn = ~0ull;
    if (h < n_hosts) {
        uint64_t next = base[h];
        const uint32_t b = host_ptr[h], e = host_ptr[h + 1];
        for (uint32_t p0 = b; p0 < e; p0 += 64) {
            const uint32_t p = p0 + lane;
            const bool sent = p < e && flags[p] == SRT_PDS_INET_SENT;
            const uint64_t m = __ballot(sent);
            if (p < e) event_id[p] = sent ? next + (uint64_t)__popcll(m & ((1ull << lane) - 1ull)) : ~0ull;
            if (sent) {
                const unsigned long long d = deliver[p];
                mn = d < mn ? d : mn;
            }
            next += (uint64_t)__popcll(m);
        }
        if (lane == 0) base[h] = next;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(mn, off);
        mn = o < mn ? o : mn;
    }
    if (lane == 0) wmin[wv] = mn;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int q = 1; q < 4; ++q) mn = wmin[q] < mn ? wmin[q] : mn;
        if (mn != ~0ull) atomicMin(tmin, mn);
    }
}

// one combined key per packet: (destination << tbits) | (deliver - tmin),
// tmin from the device (range[0]: no host round trip), tbits = 64 - the
// destination bits; unsent packets get destination n_dst (they sort last).
// A sent packet past the key (span >= 2^tbits ns) or with a destination out
// of range raises *bad (bit 1 / bit 0; srt_packet_events_status reports it).
__global__ void event_keys_kernel(const uint32_t *__restrict__ flags, const uint64_t *__restrict__ deliver,
                                  const uint32_t *__restrict__ dst, uint32_t n_dst,
                                  const unsigned long long *__restrict__ range, int tbits, uint64_t n,
                                  uint64_t *__restrict__ key, uint32_t *__restrict__ idx, uint32_t *__restrict__ bad) {
    const uint64_t tmin = range[0] == ~0ull ? 0 : range[0];
    const uint64_t tmask = tbits >= 64 ? ~0ull : (1ull << tbits) - 1;
    uint32_t b = 0;
    for (uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t k = (uint64_t)n_dst << tbits;
        if (flags[p] == SRT_PDS_INET_SENT) {
            const uint32_t d = dst[p];
            const uint64_t t = deliver[p] - tmin;
            if (d >= n_dst) b |= 1u;
            else if (t > tmask) b |= 2u;
            else k = ((uint64_t)d << tbits) | t;
        }
        key[p] = k;
        idx[p] = (uint32_t)p;
    }
    if (b) atomicOr(bad, b);
}

// (C) for the combined-key path: dst_ptr[d] = first sorted key >= d << tbits
__global__ void event_dst_ptr64_kernel(const uint64_t *__restrict__ key, uint64_t n, uint32_t n_dst, int tbits,
                                       uint32_t *__restrict__ dst_ptr, unsigned long long *__restrict__ tmin) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d == 0) *tmin = ~0ull;  // for the next call (its keys were built from it already)
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

// exact fallback (srt_packet_events_status, when a batch's deliver-time span
// overflowed the combined key): stable sort by time, then by destination
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
        if (flags[p] == SRT_PDS_INET_SENT && dst[p] < n_dst) k = dst[p];
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
    if (!plan->d_ev_bad) {  // status flags [0], then the earliest deliver time [1..2] (u64)
        if (hipMalloc(&plan->d_ev_bad, 16) != hipSuccess) {
            set_err(err, SRT_ERR_OOM, "hipMalloc(event status) failed");
            return SRT_ERR_OOM;
        }
        (void)hipMemsetAsync(plan->d_ev_bad, 0, 4, s);
        (void)hipMemsetAsync(plan->d_ev_bad + 2, 0xff, 8, s);
    }
    unsigned long long *tmin = reinterpret_cast<unsigned long long *>(plan->d_ev_bad + 2);
    if (n_hosts)
        hipLaunchKernelGGL(event_id_kernel, dim3((n_hosts + 3) / 4), dim3(256), 0, s, d_host_pkt_ptr, n_hosts, d_flags,
                           d_deliver, d_event_base, d_event_id, tmin);
    if (!n) {
        (void)hipMemsetAsync(tmin, 0xff, 8, s);
        (void)hipMemsetAsync(d_dst_ptr, 0, ((size_t)n_dst_hosts + 1) * 4, s);
        return hipGetLastError() == hipSuccess ? SRT_OK : SRT_ERR_HIP;
    }
    // (B) one sort of (destination, deliver - tmin) keys, stable from batch
    // order, tmin reduced on the device: the call needs nothing from the
    // device on the host (no round trip).  The key is 48 bits (6 radix
    // passes) while the destinations leave the time field >= 30 bits (~1 s
    // of deliver-time span; C5: 34 bits, 17 s), else 64; a batch spanning
    // more is flagged and srt_packet_events_status redoes it exactly.
    const int dbits = std::max(bit_width(n_dst_hosts), 1);  // keys 0..n_dst_hosts
    const int kbits = dbits <= 18 ? 48 : 64;
    const int tbits = kbits - dbits;
    size_t temp = 0;
    rocprim::radix_sort_pairs((void *)nullptr, temp, (uint64_t *)nullptr, (uint64_t *)nullptr, (uint32_t *)nullptr,
                              (uint32_t *)nullptr, n, 0, (unsigned)kbits, s);
    // scratch: key[2n] u64, idx[n] u32, rocPRIM temp
    const size_t need = 16ull * n + 4ull * n + 512 + temp;
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
    uint32_t *idx = (uint32_t *)(key_s + n);
    // rocPRIM partitions its temporary storage assuming an aligned base
    void *tmp = (void *)(((uintptr_t)(idx + n) + 255) & ~(uintptr_t)255);
    const uint32_t blocks = std::min<uint32_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(event_keys_kernel, dim3(blocks), dim3(256), 0, s, d_flags, d_deliver, d_dst_host, n_dst_hosts,
                       (const unsigned long long *)tmin, tbits, (uint64_t)n, key, idx, plan->d_ev_bad);
    size_t ts = temp;
    if (rocprim::radix_sort_pairs(tmp, ts, key, key_s, idx, d_order, n, 0, (unsigned)kbits, s) != hipSuccess) {
        set_err(err, SRT_ERR_HIP, "radix sort (destination, deliver time) failed");
        return SRT_ERR_HIP;
    }
    hipLaunchKernelGGL(event_dst_ptr64_kernel, dim3(n_dst_hosts / 256 + 1), dim3(256), 0, s, key_s, (uint64_t)n,
                       n_dst_hosts, tbits, d_dst_ptr, tmin);
    // the call, for srt_packet_events_status's exact fallback
    plan->ev_last = srt_plan::EvCall{d_flags, d_deliver, d_dst_host, n_dst_hosts, d_order, d_dst_ptr, n};
    return hipGetLastError() == hipSuccess ? SRT_OK : SRT_ERR_HIP;
}

extern "C" srt_status srt_packet_events_status(srt_plan *plan, srt_err *err) {
    if (err) std::memset(err, 0, sizeof *err);
    if (!plan) {
        set_err(err, SRT_ERR_INVALID, "null plan");
        return SRT_ERR_INVALID;
    }
    if (!plan->d_ev_bad) return SRT_OK;
    if (hipSetDevice(plan->device) != hipSuccess) return SRT_ERR_HIP;
    uint32_t bad = 0;
    if (hipMemcpyAsync(&bad, plan->d_ev_bad, 4, hipMemcpyDeviceToHost, plan->stream) != hipSuccess ||
        hipStreamSynchronize(plan->stream) != hipSuccess) {
        set_err(err, SRT_ERR_HIP, "packet events: stream failed");
        return SRT_ERR_HIP;
    }
    if (bad) {
        (void)hipMemsetAsync(plan->d_ev_bad, 0, 4, plan->stream);
        if (bad & 1u) {
            set_err(err, SRT_ERR_INVALID, "destination host index out of range");
            return SRT_ERR_INVALID;
        }
        // the last batch's deliver times spanned more than the key's time
        // field: redo its sort exactly -- by time (64 bits), then stably by
        // destination -- on the same (still valid) arrays
        const srt_plan::EvCall &c = plan->ev_last;
        const uint32_t n = c.n;
        hipStream_t s = plan->stream;
        const int dbits = std::max(bit_width(c.n_dst), 1);
        size_t t1 = 0, t2 = 0;
        rocprim::radix_sort_pairs((void *)nullptr, t1, (uint64_t *)nullptr, (uint64_t *)nullptr, (uint32_t *)nullptr,
                                  (uint32_t *)nullptr, n, 0, 64, s);
        rocprim::radix_sort_pairs((void *)nullptr, t2, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                  (uint32_t *)nullptr, n, 0, (unsigned)dbits, s);
        const size_t temp = std::max(t1, t2), need = 16ull * n + 16ull * n + 512 + temp;
        void *buf = nullptr;
        if (hipMalloc(&buf, need) != hipSuccess) {
            set_err(err, SRT_ERR_OOM, "hipMalloc(event fallback) failed");
            return SRT_ERR_OOM;
        }
        uint64_t *ktime = (uint64_t *)buf, *ktime_s = ktime + n;
        uint32_t *idx = (uint32_t *)(ktime_s + n), *idx1 = idx + n, *kdst = idx1 + n, *kdst_s = kdst + n;
        void *tmp = (void *)(((uintptr_t)(kdst_s + n) + 255) & ~(uintptr_t)255);
        const uint32_t blocks = std::min<uint32_t>((n + 255) / 256, 4096);
        size_t ts = temp;
        hipLaunchKernelGGL(event_time_keys_kernel, dim3(blocks), dim3(256), 0, s, c.flags, c.deliver, (uint64_t)n,
                           ktime, idx);
        hipError_t e = rocprim::radix_sort_pairs(tmp, ts, ktime, ktime_s, idx, idx1, n, 0, 64, s);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(event_dst_keys_kernel, dim3(blocks), dim3(256), 0, s, idx1, c.flags, c.dst, c.n_dst,
                               (uint64_t)n, kdst);
            ts = temp;
            e = rocprim::radix_sort_pairs(tmp, ts, kdst, kdst_s, idx1, c.order, n, 0, (unsigned)dbits, s);
        }
        if (e == hipSuccess) {
            hipLaunchKernelGGL(event_dst_ptr_kernel, dim3(c.n_dst / 256 + 1), dim3(256), 0, s, kdst_s, (uint64_t)n,
                               c.n_dst, c.dst_ptr);
            e = hipStreamSynchronize(s);
        }
        (void)hipFree(buf);
        if (e != hipSuccess) {
            set_err(err, SRT_ERR_HIP, "packet events: exact fallback failed");
            return SRT_ERR_HIP;
        }
        return SRT_OK;
    }
    return SRT_OK;
}
