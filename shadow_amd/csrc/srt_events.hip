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
// Here, for the whole batch at once, asynchronously (the call never waits for
// the device): (A) one wave per source host walks its packets in send order,
// hands out event ids to the sent ones and counts them per destination; an
// exclusive scan of the counts gives each destination's group offsets; (B)
// every sent packet is scattered into its destination's group (any order
// within the group), then one workgroup per destination sorts its group in
// LDS by (deliver time, batch index) -- batch order is (source host, send
// order), i.e. (src_host_id, src_host_event_id) order, since host segments are
// laid out by host index == HostId order -- a rank sort: each element's place
// is the number of smaller keys.  No key-width limit on the deliver times.  A
// group larger than EV_CAP events, or a sent packet whose destination is out
// of range, is flagged: srt_packet_events_status reports the latter and redoes
// a batch with a big group exactly (two stable radix sorts: time, then
// destination).
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>

#include "srt_internal.h"

namespace {

constexpr uint32_t EV_CAP = 1024;  // events a destination group may hold for the LDS sort

// (A) event ids: one wave per source host; its packets in send order, 64 at
// a time, the sent ones numbered by a ballot prefix count and counted per
// destination (cnt, zeroed by the call); an out-of-range destination raises
// bit 0 of *bad.
__global__ __launch_bounds__(256) void event_id_kernel(const uint32_t *__restrict__ host_ptr, uint32_t n_hosts,
                                                       const uint32_t *__restrict__ flags,
                                                       const uint32_t *__restrict__ dst, uint32_t n_dst,
                                                       uint64_t *__restrict__ base, uint64_t *__restrict__ event_id,
                                                       uint32_t *__restrict__ cnt, uint32_t *__restrict__ bad) {
    const uint32_t h = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
    if (h >= n_hosts) return;
    uint64_t next = base[h];
    const uint32_t b = host_ptr[h], e = host_ptr[h + 1];
    bool oob = false;
    for (uint32_t p0 = b; p0 < e; p0 += 64) {
        const uint32_t p = p0 + lane;
        const bool sent = p < e && flags[p] == SRT_PDS_INET_SENT;
        const uint64_t m = __ballot(sent);
        if (p < e) event_id[p] = sent ? next + (uint64_t)__popcll(m & ((1ull << lane) - 1ull)) : ~0ull;
        if (sent) {
            const uint32_t d = dst[p];
            if (d >= n_dst) oob = true;
            else if (cnt) atomicAdd(&cnt[d], 1u);
        }
        next += (uint64_t)__popcll(m);
    }
    if (lane == 0) base[h] = next;
    if (__ballot(oob) && lane == 0) atomicOr(bad, 1u);
}

// one workgroup: dst_ptr = exclusive scan of cnt (dst_ptr[n_dst] = the sent
// total), cur = dst_ptr (the scatter's cursors)
__global__ __launch_bounds__(1024) void event_scan_kernel(const uint32_t *__restrict__ cnt, uint32_t n_dst,
                                                          uint32_t *__restrict__ dst_ptr, uint32_t *__restrict__ cur) {
    __shared__ uint32_t wsum[16];
    const uint32_t t = threadIdx.x, per = (n_dst + 1023) / 1024;
    const uint32_t b = min(n_dst, t * per), e = min(n_dst, b + per);
    uint32_t sum = 0;
#pragma unroll 8
    for (uint32_t i = b; i < e; ++i) sum += cnt[i];
    const int lane = t & 63, w = t >> 6;
    uint32_t x = sum;  // inclusive scan over the block
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t before = 0;
    for (int q = 0; q < w; ++q) before += wsum[q];
    uint32_t run = before + x - sum;  // exclusive prefix of this thread's chunk
    for (uint32_t i = b; i < e; ++i) {
        dst_ptr[i] = run;
        cur[i] = run;
        run += cnt[i];
    }
    if (t == 1023) dst_ptr[n_dst] = before + x;
}

// Counting without global atomics (n_dst <= EV_LDS_DST, the usual case): the
// packets in chunks of EV_CHUNK, one workgroup each.  (1) every chunk counts
// its sent packets per destination in LDS and writes the row hist[chunk][d];
// (2) per destination a running sum down the chunks turns the rows into the
// chunk's offset inside the destination's group (and the group sizes into
// cnt); (3) event_scan_kernel; (4) every chunk scatters its packets from
// cursors dst_ptr[d] + hist[chunk][d] in LDS.  (Device-scope atomics on 10k
// counters from 1M packets cost ~45 us a pass on C5.)
constexpr uint32_t EV_CHUNK = 4096, EV_LDS_DST = 15872;  // LDS: n_dst cursors + n_dst / 64 block prefixes

__global__ __launch_bounds__(1024) void event_chunk_count_kernel(const uint32_t *__restrict__ flags,
                                                                 const uint32_t *__restrict__ dst, uint32_t n_dst,
                                                                 uint32_t n, uint32_t *__restrict__ hist) {
    extern __shared__ uint32_t h[];
    for (uint32_t d = threadIdx.x; d < n_dst; d += blockDim.x) h[d] = 0;
    __syncthreads();
    const uint32_t p0 = blockIdx.x * EV_CHUNK, p1 = min(n, p0 + EV_CHUNK);
    for (uint32_t p = p0 + threadIdx.x; p < p1; p += blockDim.x)
        if (flags[p] == SRT_PDS_INET_SENT) {
            const uint32_t d = dst[p];
            if (d < n_dst) atomicAdd(&h[d], 1u);
        }
    __syncthreads();
    uint32_t *row = hist + (uint64_t)blockIdx.x * n_dst;
    for (uint32_t d = threadIdx.x; d < n_dst; d += blockDim.x) row[d] = h[d];
}

// four lanes per destination, each over a quarter of the chunks (16 loads in
// flight), joined by shuffles (one lane a destination: 61 us on C5)
// Also the destinations' group offsets, in two levels without a separate
// scan launch: loc[d] = offset of d among the 64 destinations of its
// workgroup, part[w] = the workgroup's total (event_chunk_scatter_kernel adds
// the prefix of part).  Thread 0 resets the big-group list for this call.
__global__ __launch_bounds__(256) void event_col_scan_kernel(uint32_t *__restrict__ hist, uint32_t chunks,
                                                             uint32_t n_dst, uint32_t *__restrict__ loc,
                                                             uint32_t *__restrict__ part, uint32_t *__restrict__ big) {
    __shared__ uint32_t tot[64];
    if (blockIdx.x == 0 && threadIdx.x == 0) big[0] = 0;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, d = t >> 2, q = t & 3;
    const bool live = d < n_dst;
    const uint32_t per = (chunks + 3) / 4, c0 = min(chunks, q * per), c1 = min(chunks, c0 + per);
    uint32_t v[16], mine = 0;
    for (uint32_t c = c0; live && c < c1; c += 16) {
#pragma unroll
        for (int k = 0; k < 16; ++k) mine += c + k < c1 ? hist[(uint64_t)(c + k) * n_dst + d] : 0u;
    }
    // exclusive prefix over the 4 lanes of d
    uint32_t x = mine;
    for (int off = 1; off < 4; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 4);
        if (q >= (uint32_t)off) x += y;
    }
    uint32_t run = x - mine;
    const uint32_t total = __shfl(x, 3, 4);
    for (uint32_t c = c0; live && c < c1; c += 16) {
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = c + k < c1 ? hist[(uint64_t)(c + k) * n_dst + d] : 0u;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (c + k < c1) {
                hist[(uint64_t)(c + k) * n_dst + d] = run;
                run += v[k];
            }
    }
    // exclusive scan of the 64 totals of this workgroup (wave 0)
    if (q == 0) tot[threadIdx.x >> 2] = live ? total : 0u;
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t own = tot[threadIdx.x];
        uint32_t y = own;
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t z = __shfl_up(y, off);
            if ((int)threadIdx.x >= off) y += z;
        }
        const uint32_t dd = blockIdx.x * 64 + threadIdx.x;
        if (dd < n_dst) loc[dd] = y - own;
        if (threadIdx.x == 63) part[blockIdx.x] = y;
    }
}

// group offsets: dst_ptr[d] = prefix of part over the 64-destination blocks
// below d + loc[d] (workgroup 0 writes dst_ptr, every workgroup derives its
// cursors from the same values)
__global__ __launch_bounds__(1024) void event_chunk_scatter_kernel(const uint32_t *__restrict__ flags,
                                                                   const uint32_t *__restrict__ dst, uint32_t n_dst,
                                                                   uint32_t n, const uint32_t *__restrict__ hist,
                                                                   const uint32_t *__restrict__ loc,
                                                                   const uint32_t *__restrict__ part,
                                                                   uint32_t *__restrict__ dst_ptr,
                                                                   uint32_t *__restrict__ order) {
    extern __shared__ uint32_t c[];  // n_dst cursors, then the block prefixes
    const uint32_t nparts = (n_dst + 63) / 64;
    uint32_t *pbase = c + n_dst;
    // exclusive scan of part (nparts <= 250) by wave 0, 64 at a time
    if (threadIdx.x < 64) {
        uint32_t carry = 0;
        for (uint32_t b0 = 0; b0 < nparts; b0 += 64) {
            const uint32_t i = b0 + threadIdx.x;
            const uint32_t own = i < nparts ? part[i] : 0u;
            uint32_t y = own;
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t z = __shfl_up(y, off);
                if ((int)threadIdx.x >= off) y += z;
            }
            if (i < nparts) pbase[i] = carry + y - own;
            carry += __shfl(y, 63);
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) dst_ptr[n_dst] = carry;
    }
    __syncthreads();
    const uint32_t *row = hist + (uint64_t)blockIdx.x * n_dst;
    for (uint32_t d = threadIdx.x; d < n_dst; d += blockDim.x) {
        const uint32_t g = pbase[d >> 6] + loc[d];
        if (blockIdx.x == 0) dst_ptr[d] = g;
        c[d] = g + row[d];
    }
    __syncthreads();
    const uint32_t p0 = blockIdx.x * EV_CHUNK, p1 = min(n, p0 + EV_CHUNK);
    for (uint32_t p = p0 + threadIdx.x; p < p1; p += blockDim.x)
        if (flags[p] == SRT_PDS_INET_SENT) {
            const uint32_t d = dst[p];
            if (d < n_dst) order[atomicAdd(&c[d], 1u)] = p;
        }
}

// (B) every sent packet into its destination's group, in any order (the
// global-atomic form, for more than EV_LDS_DST destinations)
__global__ void event_scatter_kernel(const uint32_t *__restrict__ flags, const uint32_t *__restrict__ dst,
                                     uint32_t n_dst, uint32_t n, uint32_t *__restrict__ cur,
                                     uint32_t *__restrict__ order) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
        if (flags[p] != SRT_PDS_INET_SENT) continue;
        const uint32_t d = dst[p];
        if (d < n_dst) order[atomicAdd(&cur[d], 1u)] = p;
    }
}

// (B) one workgroup per destination: its group sorted by (deliver time, batch
// index) in LDS, in place.  Keys are distinct (the index breaks every tie), so
// an element's rank among them is its place.  CAP events fit the kernel's LDS:
// the common form (CAP = EV_SMALL, 3 KB, many workgroups a CU) appends a
// bigger group to a list (big[0] = count) for the EV_CAP form, which walks the
// list; a group over EV_CAP raises bit 2 of *bad (srt_packet_events_status
// redoes the batch exactly).
constexpr uint32_t EV_SMALL = 256;

template <uint32_t CAP>
__device__ __forceinline__ void group_rank_sort(uint32_t b, uint32_t m, const uint64_t *__restrict__ deliver,
                                                uint32_t *__restrict__ order, uint64_t *key, uint32_t *idx) {
    for (uint32_t i = threadIdx.x; i < m; i += 64) {
        const uint32_t p = order[b + i];
        idx[i] = p;
        key[i] = deliver[p];
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < m; i += 64) {
        const uint64_t ki = key[i];
        const uint32_t pi = idx[i];
        uint32_t r = 0;
        for (uint32_t j = 0; j < m; ++j) {
            const uint64_t kj = key[j];
            r += (kj < ki) | ((kj == ki) & (idx[j] < pi));
        }
        order[b + r] = pi;
    }
}

// one single-wave workgroup per destination (four destinations per 256-lane
// workgroup measured slower: 24.4 against 21.0 us on C5)
__global__ __launch_bounds__(64) void event_group_sort_kernel(const uint32_t *__restrict__ dst_ptr,
                                                              const uint64_t *__restrict__ deliver,
                                                              uint32_t *__restrict__ order, uint32_t *__restrict__ big) {
    __shared__ uint64_t key[EV_SMALL];
    __shared__ uint32_t idx[EV_SMALL];
    const uint32_t d = blockIdx.x, b = dst_ptr[d], m = dst_ptr[d + 1] - b;
    if (m <= 1) return;
    if (m > EV_SMALL) {
        if (threadIdx.x == 0) big[1 + atomicAdd(&big[0], 1u)] = d;
        return;
    }
    group_rank_sort<EV_SMALL>(b, m, deliver, order, key, idx);
}

__global__ __launch_bounds__(64) void event_big_group_sort_kernel(const uint32_t *__restrict__ dst_ptr,
                                                                  const uint64_t *__restrict__ deliver,
                                                                  uint32_t *__restrict__ order,
                                                                  const uint32_t *__restrict__ big,
                                                                  uint32_t *__restrict__ bad) {
    __shared__ uint64_t key[EV_CAP];
    __shared__ uint32_t idx[EV_CAP];
    const uint32_t nb = big[0];
    for (uint32_t k = blockIdx.x; k < nb; k += gridDim.x) {
        const uint32_t d = big[1 + k], b = dst_ptr[d], m = dst_ptr[d + 1] - b;
        if (m > EV_CAP) {
            if (threadIdx.x == 0) atomicOr(bad, 4u);
            continue;
        }
        group_rank_sort<EV_CAP>(b, m, deliver, order, key, idx);
        __syncthreads();  // LDS reused by the next group
    }
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

namespace {
// start of a batch: an unchecked big-group flag of the previous batch (bit 2)
// moves to bit 3 ("an earlier batch is wrong and can no longer be redone")
__global__ void event_carry_kernel(uint32_t *bad) {
    const uint32_t b = *bad;
    if (b & 4u) *bad = (b & ~4u) | 8u;
}
}  // namespace

extern "C" srt_status srt_packet_events(srt_plan *plan, const uint32_t *d_host_pkt_ptr, uint32_t n_hosts,
                                        uint64_t n_pkts, const uint32_t *d_flags, const uint64_t *d_deliver,
                                        const uint32_t *d_dst_host, uint32_t n_dst_hosts, uint64_t *d_event_base,
                                        uint64_t *d_event_id, uint32_t *d_order, uint32_t *d_dst_ptr,
                                        srt_err *err) {
    srt::init_wait();  // a pending srt_init_async finishes first
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
    if (!plan->d_ev_bad) {  // status flags (bit 0 destination out of range, bit 2 a group over EV_CAP)
        if (hipMalloc(&plan->d_ev_bad, 16) != hipSuccess) {
            set_err(err, SRT_ERR_OOM, "hipMalloc(event status) failed");
            return SRT_ERR_OOM;
        }
        (void)hipMemsetAsync(plan->d_ev_bad, 0, 4, s);
    } else {
        // a big group of an earlier, unchecked batch cannot be redone any more
        // (only the last call's arrays are kept): bit 2 becomes bit 3, which
        // srt_packet_events_status reports as an error
        hipLaunchKernelGGL(event_carry_kernel, dim3(1), dim3(1), 0, s, plan->d_ev_bad);
    }
    // scratch: per destination a count and a scatter cursor; for the chunked
    // count the per-chunk rows
    const uint32_t chunks = (n + EV_CHUNK - 1) / EV_CHUNK;
    const bool chunked = n && n_dst_hosts && n_dst_hosts <= EV_LDS_DST && (uint64_t)chunks * n_dst_hosts <= (64u << 20);
    const size_t need = 12ull * ((size_t)n_dst_hosts + 1) + (chunked ? 4ull * chunks * n_dst_hosts : 0);
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
    // cnt, cur, the big-group list (count + ids), the chunk rows
    uint32_t *cnt = (uint32_t *)plan->d_ev_scratch, *cur = cnt + n_dst_hosts + 1, *big = cur + n_dst_hosts + 1;
    uint32_t *hist = big + n_dst_hosts + 1;
    if (!chunked) {
        (void)hipMemsetAsync(cnt, 0, 4ull * (n_dst_hosts + 1), s);
        (void)hipMemsetAsync(big, 0, 4, s);
    }
    if (n_hosts)
        hipLaunchKernelGGL(event_id_kernel, dim3((n_hosts + 3) / 4), dim3(256), 0, s, d_host_pkt_ptr, n_hosts, d_flags,
                           d_dst_host, n_dst_hosts, d_event_base, d_event_id, chunked ? nullptr : cnt,
                           plan->d_ev_bad);
    const size_t lds = 4ull * n_dst_hosts;
    if (chunked) {
        hipLaunchKernelGGL(event_chunk_count_kernel, dim3(chunks), dim3(1024), lds, s, d_flags, d_dst_host, n_dst_hosts,
                           n, hist);
        // loc = cnt, part = cur (both n_dst + 1 long)
        hipLaunchKernelGGL(event_col_scan_kernel, dim3((n_dst_hosts + 63) / 64), dim3(256), 0, s, hist, chunks,
                           n_dst_hosts, cnt, cur, big);
    } else {
        hipLaunchKernelGGL(event_scan_kernel, dim3(1), dim3(1024), 0, s, (const uint32_t *)cnt, n_dst_hosts,
                           d_dst_ptr, cur);
    }
    if (n) {
        const uint32_t blocks = std::min<uint32_t>((n + 255) / 256, 4096);
        if (chunked)
            hipLaunchKernelGGL(event_chunk_scatter_kernel, dim3(chunks), dim3(1024),
                               lds + 4ull * ((n_dst_hosts + 63) / 64), s, d_flags, d_dst_host, n_dst_hosts, n,
                               (const uint32_t *)hist, (const uint32_t *)cnt, (const uint32_t *)cur, d_dst_ptr,
                               d_order);
        else
            hipLaunchKernelGGL(event_scatter_kernel, dim3(blocks), dim3(256), 0, s, d_flags, d_dst_host, n_dst_hosts, n,
                               cur, d_order);
        if (n_dst_hosts) {
            hipLaunchKernelGGL(event_group_sort_kernel, dim3(n_dst_hosts), dim3(64), 0, s, (const uint32_t *)d_dst_ptr,
                               d_deliver, d_order, big);
            hipLaunchKernelGGL(event_big_group_sort_kernel, dim3(std::min<uint32_t>(n_dst_hosts, 512)), dim3(64), 0, s,
                               (const uint32_t *)d_dst_ptr, d_deliver, d_order, (const uint32_t *)big, plan->d_ev_bad);
        }
    }
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
        if (bad & 8u) {
            set_err(err, SRT_ERR_INVALID,
                    "packet events: an earlier batch had a destination group over 1024 events and was not checked "
                    "(call srt_packet_events_status after every batch that may hold one)");
            return SRT_ERR_INVALID;
        }
        // a destination group of the last batch was too big for the LDS
        // sort: redo the batch's sort exactly -- by time (64 bits), then
        // stably by destination -- on the same (still valid) arrays
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
