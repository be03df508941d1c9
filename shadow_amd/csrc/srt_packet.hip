// srt_packet.hip -- batched Worker::send_packet decision for one round.
//
// Reference: src/main/core/worker.rs:326-410 (+ WorkerShared::latency /
// reliability :539-553, RoutingInfo::increment_packet_count mod.rs:449-456,
// Worker::update_lowest_used_latency :291-300, update_next_event_time :314-322).
// Per packet, in the source host's send order:
//   completed  = t >= sim_end            -> nothing, and NO RNG draw (:336-339)
//   chance     = host_rng.gen::<f64>()   = (next_u64 >> 11) * 2^-53 (rand 0.8.5)
//   reliability= (1.0f32 - loss) as f64  (f32 subtraction, then widened)
//   drop iff !(t < bootstrap_end) && chance >= reliability && payload > 0
//   else: delay = latency; counter++; SENT; deliver = max(t + delay, round_end)
//
// Two kernels: (A) one lane per host walks its packets and advances its
// xoshiro256++ state -- the only sequential part, ~20 integer ops per draw;
// (B) one lane per packet does the table gather and the decision, HBM-bound.
#include <cstdlib>
#include <cstring>

#include "srt_internal.h"

namespace {

__device__ __forceinline__ uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

// rand_xoshiro 0.6.0 Xoshiro256PlusPlus::next_u64
__device__ __forceinline__ uint64_t xoshiro_next(uint64_t &s0, uint64_t &s1, uint64_t &s2,
                                                 uint64_t &s3) {
    const uint64_t r = rotl(s0 + s3, 23) + s0;
    const uint64_t t = s1 << 17;
    s2 ^= s0;
    s3 ^= s1;
    s1 ^= s2;
    s0 ^= s3;
    s2 ^= t;
    s3 = rotl(s3, 45);
    return r;
}

// One lane per host; the walk is a dependent chain per lane, so the grid is
// spread thin (DT threads per block: 10k hosts -> 157 CUs at DT = 64, not 40)
// and the send times are fetched PF at a time (independent loads in flight)
// so the walk is not one memory latency per packet.
template <int DT, int PF>
__global__ __launch_bounds__(DT) void draw_kernel(const srt_pkt *__restrict__ pkts,
                                                  const uint32_t *__restrict__ host_ptr, uint32_t n_hosts,
                                                  uint64_t *__restrict__ rng, uint64_t sim_end,
                                                  uint64_t *__restrict__ draws) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= n_hosts) return;
    uint64_t s0 = rng[4 * (uint64_t)h], s1 = rng[4 * (uint64_t)h + 1];
    uint64_t s2 = rng[4 * (uint64_t)h + 2], s3 = rng[4 * (uint64_t)h + 3];
    const uint32_t b = host_ptr[h], e = host_ptr[h + 1];
    for (uint32_t p0 = b; p0 < e; p0 += PF) {
        uint64_t tt[PF];
#pragma unroll
        for (int q = 0; q < PF; ++q) tt[q] = p0 + q < e ? pkts[p0 + q].t_ns : 0;
#pragma unroll
        for (int q = 0; q < PF; ++q) {
            if (p0 + q >= e || tt[q] >= sim_end) continue;  // completed: no draw
            draws[p0 + q] = xoshiro_next(s0, s1, s2, s3);
        }
    }
    rng[4 * (uint64_t)h] = s0;
    rng[4 * (uint64_t)h + 1] = s1;
    rng[4 * (uint64_t)h + 2] = s2;
    rng[4 * (uint64_t)h + 3] = s3;
}

constexpr int DECIDE_THREADS = 256;

__global__ __launch_bounds__(DECIDE_THREADS) void decide_kernel(const srt_pkt *__restrict__ pkts, uint64_t n_pkts,
                              const uint64_t *__restrict__ draws,
                              const uint64_t *__restrict__ lat, const float *__restrict__ loss,
                              uint32_t n, srt_round r, uint32_t *__restrict__ flags,
                              uint64_t *__restrict__ deliver, unsigned long long *counters,
                              unsigned long long *__restrict__ partial) {
    unsigned long long min_lat = ~0ull, min_deliver = ~0ull;
    for (uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; p < n_pkts;
         p += (uint64_t)gridDim.x * blockDim.x) {
        const srt_pkt k = pkts[p];
        uint32_t f = SRT_PDS_NONE;
        uint64_t d = 0;
        if (k.t_ns < r.sim_end_ns) {
            const uint64_t o = (uint64_t)k.src_row * n + k.dst_row;
            const float rel32 = 1.0f - loss[o];
            const double reliability = (double)rel32;
            const double chance = (double)(draws[p] >> 11) * 0x1.0p-53;
            const bool bootstrapping = k.t_ns < r.bootstrap_end_ns;
            if (!bootstrapping && chance >= reliability && k.payload_size > 0) {
                f = SRT_PDS_INET_DROPPED;
            } else {
                const uint64_t delay = lat[o];
                f = SRT_PDS_INET_SENT;
                d = k.t_ns + delay;
                if (d < r.round_end_ns) d = r.round_end_ns;
                if (counters) atomicAdd(&counters[o], 1ull);
                min_lat = delay < min_lat ? delay : min_lat;
                min_deliver = d < min_deliver ? d : min_deliver;
            }
        }
        flags[p] = f;
        deliver[p] = d;
    }
    // wave, then block reduction: one pair of atomics per block (same-address
    // atomics from every wave serialise at the memory-side atomic unit)
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long a = __shfl_xor(min_lat, off), b = __shfl_xor(min_deliver, off);
        min_lat = a < min_lat ? a : min_lat;
        min_deliver = b < min_deliver ? b : min_deliver;
    }
    __shared__ unsigned long long red[2][DECIDE_THREADS / 64];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][w] = min_lat;
        red[1][w] = min_deliver;
    }
    __syncthreads();
    if (threadIdx.x == 0 && partial) {
        for (int k = 1; k < DECIDE_THREADS / 64; ++k) {
            min_lat = red[0][k] < min_lat ? red[0][k] : min_lat;
            min_deliver = red[1][k] < min_deliver ? red[1][k] : min_deliver;
        }
        partial[2 * blockIdx.x] = min_lat;
        partial[2 * blockIdx.x + 1] = min_deliver;
    }
}

// Block partials -> the caller's stats (min-combined).  Same-address atomics
// from every block of decide_kernel serialise at the memory-side atomic unit
// (2048 blocks x 2 = ~60 us measured, more than the whole decision pass), so
// they are combined here by one workgroup: two atomics per round.
__global__ __launch_bounds__(1024) void stats_kernel(const unsigned long long *__restrict__ partial, uint32_t nblocks,
                                                     unsigned long long *stats) {
    unsigned long long a = ~0ull, b = ~0ull;
    for (uint32_t i = threadIdx.x; i < nblocks; i += blockDim.x) {
        a = partial[2 * i] < a ? partial[2 * i] : a;
        b = partial[2 * i + 1] < b ? partial[2 * i + 1] : b;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long x = __shfl_xor(a, off), y = __shfl_xor(b, off);
        a = x < a ? x : a;
        b = y < b ? y : b;
    }
    __shared__ unsigned long long red[2][16];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][w] = a;
        red[1][w] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < (int)(blockDim.x >> 6); ++k) {
            a = red[0][k] < a ? red[0][k] : a;
            b = red[1][k] < b ? red[1][k] : b;
        }
        if (a != ~0ull) atomicMin(&stats[0], a);
        if (b != ~0ull) atomicMin(&stats[1], b);
    }
}

}  // namespace

namespace srt {
// srt_init: loads this unit's code object (srt::preload_kernels)
hipError_t preload_packet() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&decide_kernel));
}
}  // namespace srt

extern "C" srt_status srt_packet_batch(srt_plan *plan, const srt_pkt *d_pkts,
                                       const uint32_t *d_host_pkt_ptr, uint32_t n_hosts,
                                       uint64_t n_pkts, uint64_t *d_rng, const srt_round *round,
                                       uint32_t *d_flags, uint64_t *d_deliver,
                                       uint64_t *d_counters, uint64_t *d_stats, srt_err *err) {
    srt::init_wait();  // a pending srt_init_async finishes first
    if (err) std::memset(err, 0, sizeof *err);
    if (!plan || !round || (n_pkts && (!d_pkts || !d_flags || !d_deliver)) || !d_host_pkt_ptr ||
        (n_hosts && !d_rng)) {
        if (err) {
            err->code = SRT_ERR_INVALID;
            std::snprintf(err->msg, sizeof err->msg, "null argument");
        }
        return SRT_ERR_INVALID;
    }
    if (!plan->ran) {
        if (err) {
            err->code = SRT_ERR_INVALID;
            std::snprintf(err->msg, sizeof err->msg, "routing table not built (run the plan first)");
        }
        return SRT_ERR_INVALID;
    }
    if (hipSetDevice(plan->device) != hipSuccess) return SRT_ERR_HIP;
    // scratch: one draw per packet, then {min latency, min deliver} per decide block
    constexpr uint64_t MAX_DECIDE_BLOCKS = 2048;  // grid-stride: 8 blocks per CU
    const uint64_t need = n_pkts + 2 * MAX_DECIDE_BLOCKS;
    if (need > plan->draws_cap) {
        if (plan->d_draws) (void)hipFree(plan->d_draws);
        plan->d_draws = nullptr;
        plan->draws_cap = 0;
        if (hipMalloc(&plan->d_draws, need * sizeof(uint64_t)) != hipSuccess) {
            if (err) {
                err->code = SRT_ERR_OOM;
                std::snprintf(err->msg, sizeof err->msg, "hipMalloc(draws) failed");
            }
            return SRT_ERR_OOM;
        }
        plan->draws_cap = need;
    }
    unsigned long long *partial = (unsigned long long *)(plan->d_draws + n_pkts);
    hipStream_t s = plan->stream;
    if (n_hosts) {
        // 64 threads x 16 packets in flight a host (C5: 103 us/round vs 137
        // at 256 threads; 32 in flight no faster)
        hipLaunchKernelGGL((draw_kernel<64, 16>), dim3((n_hosts + 63) / 64), dim3(64), 0, s, d_pkts,
                           d_host_pkt_ptr, n_hosts, d_rng, round->sim_end_ns, plan->d_draws);
    }
    if (n_pkts) {
        uint64_t blocks = (n_pkts + DECIDE_THREADS - 1) / DECIDE_THREADS;
        if (blocks > MAX_DECIDE_BLOCKS) blocks = MAX_DECIDE_BLOCKS;
        hipLaunchKernelGGL(decide_kernel, dim3((uint32_t)blocks), dim3(DECIDE_THREADS), 0, s, d_pkts, n_pkts,
                           plan->d_draws, plan->d_out_lat, plan->d_out_loss, plan->n, *round,
                           d_flags, d_deliver, (unsigned long long *)d_counters, d_stats ? partial : nullptr);
        if (d_stats)
            hipLaunchKernelGGL(stats_kernel, dim3(1), dim3(1024), 0, s, partial, (uint32_t)blocks,
                               (unsigned long long *)d_stats);
    }
    if (hipGetLastError() != hipSuccess) {
        if (err) {
            err->code = SRT_ERR_HIP;
            std::snprintf(err->msg, sizeof err->msg, "packet kernel launch failed");
        }
        return SRT_ERR_HIP;
    }
    return SRT_OK;
}
