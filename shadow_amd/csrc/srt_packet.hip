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
// One kernel a round (round_kernel): a workgroup takes HB consecutive source
// hosts.  One lane per host walks its packets in send order and advances its
// xoshiro256++ state -- the only sequential part, a dependent chain of ~20
// integer ops a draw -- leaving the draws in LDS, while every lane loads its
// packets (the record, then one 16-B gather of the packed {latency, loss}
// table record, packed once per build); then every lane decides its packets:
// the drop rule, the deliver-time clamp, the per-path counter, block minima.
// The draws never travel through HBM (a block whose packets overflow its LDS
// keeps them in a global scratch instead).
//
// The packet's table row and column come either from srt_pkt (resolved by the
// caller) or, in srt_packet_batch_ip, from its IPv4 addresses through the
// frozen IpAssignment (srt_ip.cpp): the reference's per-packet
// ip_assignment.get_node + routing_info.path lookups (worker.rs:539-553).
#include <cstdlib>
#include <cstring>

#include "srt_internal.h"

namespace {

__host__ __device__ __forceinline__ uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

// rand_xoshiro 0.6.0 Xoshiro256PlusPlus::next_u64
__host__ __device__ __forceinline__ uint64_t xoshiro_next(uint64_t &s0, uint64_t &s1, uint64_t &s2, uint64_t &s3) {
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

constexpr int RT = 256;          // threads a round workgroup
#ifndef SRT_PKT_HB
#define SRT_PKT_HB 16
#endif
constexpr int HB = SRT_PKT_HB;   // source hosts a workgroup (C5: 625 workgroups, ~1,600 packets each)
constexpr uint32_t DCAP = 3072;  // draws a workgroup keeps in LDS (24 KB)
constexpr int KP = 8;            // packets a lane holds across the host walks (RT * KP = 2,048 a workgroup)
constexpr int PF = 16;           // send times in flight a host walk (the exact walk)

// the packet's (row, column) of the table: resolved by the caller, or from its
// addresses (network byte order); -1 when an address has no row
template <bool IP>
__device__ __forceinline__ void pkt_rows(const srt_pkt &k, const srt::IpTable &ipt, int32_t &i, int32_t &j) {
    if (IP) {
        i = srt::ip_lookup(ipt, __builtin_bswap32(k.src_row));
        j = srt::ip_lookup(ipt, __builtin_bswap32(k.dst_row));
    } else {
        i = (int32_t)k.src_row;
        j = (int32_t)k.dst_row;
    }
}

// a packet's inputs once its record and table entry are loaded
struct PktIn {
    uint64_t t, delay;
    uint64_t o;          // table index (~0: completed or unresolved)
    uint32_t payload;
    float ls;
    bool live, unresolved;
};

template <bool IP, bool TAB16>
__device__ __forceinline__ PktIn load_pkt(const srt_pkt *__restrict__ pkts, uint32_t p, const srt_round &r,
                                          const uint4 *__restrict__ tab, const uint64_t *__restrict__ lat,
                                          const float *__restrict__ loss, uint32_t n, const srt::IpTable &ipt) {
    const srt_pkt k = pkts[p];
    PktIn x{k.t_ns, 0, ~0ull, k.payload_size, 0.0f, false, false};
    if (k.t_ns < r.sim_end_ns) {
        int32_t i, j;
        pkt_rows<IP>(k, ipt, i, j);
        if (i < 0 || j < 0) {
            x.unresolved = true;  // the reference's reliability(..).unwrap() panics (worker.rs:359)
        } else {
            x.live = true;
            x.o = (uint64_t)(uint32_t)i * n + (uint32_t)j;
            if (TAB16) {
                const uint4 rec = tab[x.o];
                x.delay = (uint64_t)rec.x | (uint64_t)rec.y << 32;
                x.ls = __uint_as_float(rec.z);
            } else {
                x.delay = lat[x.o];
                x.ls = loss[x.o];
            }
        }
    }
    return x;
}

// The round of HB source hosts.  The walks are dependent chains (one draw a
// packet, host.rs:233 stream order) and the loads are independent, so they
// overlap: every lane issues the loads of its packets (record, then the 16-B
// table record) while one lane per host runs its chain speculatively -- a draw
// for every packet, which is exact unless a packet is completed (t >= sim_end:
// no draw, worker.rs:336-339).  The block then knows which hosts had one;
// those (rare: the last round of a simulation) redo their walk exactly from
// the saved state.  Then every lane decides its packets from the draws in LDS.
template <bool IP, bool TAB16>
__global__ __launch_bounds__(RT) void round_kernel(const srt_pkt *__restrict__ pkts,
                                                   const uint32_t *__restrict__ host_ptr, uint32_t n_hosts,
                                                   uint64_t *__restrict__ rng, srt_round r,
                                                   const uint4 *__restrict__ tab, const uint64_t *__restrict__ lat,
                                                   const float *__restrict__ loss, uint32_t n, srt::IpTable ipt,
                                                   uint32_t *__restrict__ flags, uint64_t *__restrict__ deliver,
                                                   unsigned long long *counters,
                                                   unsigned long long *__restrict__ partial,
                                                   uint64_t *__restrict__ gdraws, uint32_t *__restrict__ bad) {
    __shared__ uint64_t sdraw[DCAP];
    __shared__ uint32_t sptr[HB + 1];
    __shared__ uint32_t scomp;  // bit i: host i of the block has a completed packet
    __shared__ unsigned long long red[2][RT / 64];
    const uint32_t t = threadIdx.x;
    const uint32_t h0 = blockIdx.x * HB;
    const uint32_t nh = min((uint32_t)HB, n_hosts - h0);
    if (t <= nh) sptr[t] = host_ptr[h0 + t];
    if (t == 0) scomp = 0;
    __syncthreads();
    const uint32_t pb = sptr[0], pe = sptr[nh];
    const bool in_lds = pe - pb <= DCAP;
    auto put = [&](uint32_t p, uint64_t d) {
        if (in_lds) sdraw[p - pb] = d;
        else gdraws[p] = d;
    };
    // (1) the lane's packets: loads issued first (they do not depend on the draws)
    PktIn mine[KP];
#pragma unroll
    for (int q = 0; q < KP; ++q) {
        const uint32_t p = pb + t + q * RT;
        if (p < pe) mine[q] = load_pkt<IP, TAB16>(pkts, p, r, tab, lat, loss, n, ipt);
    }
    // (2) one lane a host, all in wave 0: the speculative walk (no send-time
    // loads).  A chain instruction costs its wave a full issue slot however
    // few lanes are active, so the walkers share one wave: the other three
    // waves' SIMDs stay free for other workgroups' walks and loads (walkers
    // spread one or two a wave measured 54-72 us a C5 round, VALU issue-bound)
    const uint32_t wi = t;
    const bool walker = t < nh;
    uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    if (walker) {
        const uint64_t h = h0 + wi;
        a0 = s0 = rng[4 * h];
        a1 = s1 = rng[4 * h + 1];
        a2 = s2 = rng[4 * h + 2];
        a3 = s3 = rng[4 * h + 3];
        for (uint32_t p = sptr[wi], e = sptr[wi + 1]; p < e; ++p) put(p, xoshiro_next(s0, s1, s2, s3));
    }
    // hosts with a completed packet (their walks skip its draw)
#pragma unroll
    for (int q = 0; q < KP; ++q) {
        const uint32_t p = pb + t + q * RT;
        if (p < pe && mine[q].t >= r.sim_end_ns) {
            uint32_t i = 0;
            while (i + 1 < nh && sptr[i + 1] <= p) ++i;
            atomicOr(&scomp, 1u << i);
        }
    }
    for (uint32_t p = pb + t + KP * RT; p < pe; p += RT)  // past KP a lane: the send time only
        if (pkts[p].t_ns >= r.sim_end_ns) {
            uint32_t i = 0;
            while (i + 1 < nh && sptr[i + 1] <= p) ++i;
            atomicOr(&scomp, 1u << i);
        }
    __syncthreads();
    if (walker) {
        if ((scomp >> wi) & 1u) {  // the exact walk, from the saved state
            s0 = a0;
            s1 = a1;
            s2 = a2;
            s3 = a3;
            const uint32_t b = sptr[wi], e = sptr[wi + 1];
            for (uint32_t p0 = b; p0 < e; p0 += PF) {
                uint64_t tt[PF];
#pragma unroll
                for (int q = 0; q < PF; ++q) tt[q] = p0 + q < e ? pkts[p0 + q].t_ns : ~0ull;
#pragma unroll
                for (int q = 0; q < PF; ++q) {
                    if (p0 + q >= e || tt[q] >= r.sim_end_ns) continue;  // completed: no draw
                    put(p0 + q, xoshiro_next(s0, s1, s2, s3));
                }
            }
        }
        const uint64_t h = h0 + wi;
        rng[4 * h] = s0;
        rng[4 * h + 1] = s1;
        rng[4 * h + 2] = s2;
        rng[4 * h + 3] = s3;
    }
    __syncthreads();
    // (3) the decisions
    unsigned long long min_lat = ~0ull, min_deliver = ~0ull;
    bool unresolved = false;
    auto decide = [&](uint32_t p, const PktIn &x) {
        uint32_t f = SRT_PDS_NONE;
        uint64_t d = 0;
        unresolved |= x.unresolved;
        if (x.live) {
            const float rel32 = 1.0f - x.ls;
            const double reliability = (double)rel32;
            const uint64_t draw = in_lds ? sdraw[p - pb] : gdraws[p];
            const double chance = (double)(draw >> 11) * 0x1.0p-53;
            const bool bootstrapping = x.t < r.bootstrap_end_ns;
            if (!bootstrapping && chance >= reliability && x.payload > 0) {
                f = SRT_PDS_INET_DROPPED;
            } else {
                f = SRT_PDS_INET_SENT;
                d = x.t + x.delay;
                if (d < r.round_end_ns) d = r.round_end_ns;
                if (counters) atomicAdd(&counters[x.o], 1ull);
                min_lat = x.delay < min_lat ? x.delay : min_lat;
                min_deliver = d < min_deliver ? d : min_deliver;
            }
        }
        flags[p] = f;
        deliver[p] = d;
    };
#pragma unroll
    for (int q = 0; q < KP; ++q) {
        const uint32_t p = pb + t + q * RT;
        if (p < pe) decide(p, mine[q]);
    }
    for (uint32_t p = pb + t + KP * RT; p < pe; p += RT) decide(p, load_pkt<IP, TAB16>(pkts, p, r, tab, lat, loss, n, ipt));
    if (IP && __any(unresolved) && (t & 63) == 0) atomicOr(bad, 1u);
    // wave, then block reduction: one pair of partials per block (same-address
    // atomics from every wave serialise at the memory-side atomic unit)
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long a = __shfl_xor(min_lat, off), b = __shfl_xor(min_deliver, off);
        min_lat = a < min_lat ? a : min_lat;
        min_deliver = b < min_deliver ? b : min_deliver;
    }
    const int w = t >> 6;
    if ((t & 63) == 0) {
        red[0][w] = min_lat;
        red[1][w] = min_deliver;
    }
    __syncthreads();
    if (t == 0 && partial) {
        for (int q = 1; q < RT / 64; ++q) {
            min_lat = red[0][q] < min_lat ? red[0][q] : min_lat;
            min_deliver = red[1][q] < min_deliver ? red[1][q] : min_deliver;
        }
        partial[2 * blockIdx.x] = min_lat;
        partial[2 * blockIdx.x + 1] = min_deliver;
    }
}

// the built table as 16-B records {latency lo, latency hi, loss bits, 0}: one
// gather a packet instead of two (the table is static through a simulation)
__global__ __launch_bounds__(256) void pack_tab16_kernel(const uint64_t *__restrict__ lat,
                                                         const float *__restrict__ loss, uint64_t count,
                                                         uint4 *__restrict__ out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t l = lat[i];
        out[i] = make_uint4((uint32_t)l, (uint32_t)(l >> 32), __float_as_uint(loss[i]), 0u);
    }
}

// Block partials -> the caller's stats (min-combined).  Same-address atomics
// from every block serialise at the memory-side atomic unit, so they are
// combined here by one workgroup: two atomics per round.
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

void perr(srt_err *err, int code, const char *msg) {
    if (!err) return;
    err->code = code;
    std::snprintf(err->msg, sizeof err->msg, "%s", msg);
}

// tables up to this size are packed into 16-B records for the round's gathers
constexpr uint64_t TAB16_MAX_BYTES = 1ull << 30;

srt_status packet_round(srt_plan *plan, const srt_pkt *d_pkts, const uint32_t *d_host_pkt_ptr, uint32_t n_hosts,
                        uint64_t n_pkts, uint64_t *d_rng, const srt_round *round, uint32_t *d_flags,
                        uint64_t *d_deliver, uint64_t *d_counters, uint64_t *d_stats, const srt::IpTable *ipt,
                        srt_err *err) {
    srt::init_wait();  // a pending srt_init_async finishes first
    if (err) std::memset(err, 0, sizeof *err);
    if (!plan || !round || (n_pkts && (!d_pkts || !d_flags || !d_deliver)) || !d_host_pkt_ptr ||
        (n_hosts && !d_rng)) {
        perr(err, SRT_ERR_INVALID, "null argument");
        return SRT_ERR_INVALID;
    }
    if (!plan->ran) {
        perr(err, SRT_ERR_INVALID, "routing table not built (run the plan first)");
        return SRT_ERR_INVALID;
    }
    if (plan->row_shard || plan->row0 != 0 || plan->row1 != plan->n) {
        perr(err, SRT_ERR_INVALID, "the packet stage needs the whole table on the plan's device");
        return SRT_ERR_INVALID;
    }
    if (hipSetDevice(plan->device) != hipSuccess) return SRT_ERR_HIP;
    hipStream_t s = plan->stream;
    const uint32_t blocks = (n_hosts + HB - 1) / HB;
    // scratch: the draws of blocks whose packets overflow their LDS, then
    // {min latency, min deliver} per block
    const uint64_t need = n_pkts + 2 * (uint64_t)std::max<uint32_t>(blocks, 1);
    if (need > plan->draws_cap) {
        if (plan->d_draws) (void)hipFree(plan->d_draws);
        plan->d_draws = nullptr;
        plan->draws_cap = 0;
        if (hipMalloc(&plan->d_draws, need * sizeof(uint64_t)) != hipSuccess) {
            perr(err, SRT_ERR_OOM, "hipMalloc(draws) failed");
            return SRT_ERR_OOM;
        }
        plan->draws_cap = need;
    }
    const uint64_t nn = (uint64_t)plan->n * plan->n;
    // knob SRT_PKT_TAB16=0: the two-gather form tables over 1 GiB use (tests)
    static const bool tab16_off = [] {
        const char *e = std::getenv("SRT_PKT_TAB16");
        return e && std::atoi(e) == 0;
    }();
    const bool tab16 = nn * 16 <= TAB16_MAX_BYTES && nn > 0 && !tab16_off;
    if (tab16 && plan->pkt_tab_run != plan->run_no) {
        if (!plan->d_pkt_tab && hipMalloc(&plan->d_pkt_tab, nn * 16) != hipSuccess) {
            plan->d_pkt_tab = nullptr;
            perr(err, SRT_ERR_OOM, "hipMalloc(packed table) failed");
            return SRT_ERR_OOM;
        }
        hipLaunchKernelGGL(pack_tab16_kernel, dim3((uint32_t)std::min<uint64_t>((nn + 255) / 256, 8192)), dim3(256),
                           0, s, plan->d_out_lat, plan->d_out_loss, nn, plan->d_pkt_tab);
        plan->pkt_tab_run = plan->run_no;
    }
    if (ipt && !plan->d_pkt_bad) {
        if (hipMalloc(&plan->d_pkt_bad, 4) != hipSuccess) {
            plan->d_pkt_bad = nullptr;
            perr(err, SRT_ERR_OOM, "hipMalloc(status) failed");
            return SRT_ERR_OOM;
        }
        (void)hipMemsetAsync(plan->d_pkt_bad, 0, 4, s);
    }
    unsigned long long *partial = (unsigned long long *)(plan->d_draws + n_pkts);
    const srt::IpTable none{};
    if (blocks) {
        auto *k = ipt ? (tab16 ? round_kernel<true, true> : round_kernel<true, false>)
                      : (tab16 ? round_kernel<false, true> : round_kernel<false, false>);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(RT), 0, s, d_pkts, d_host_pkt_ptr, n_hosts, d_rng, *round,
                           plan->d_pkt_tab, plan->d_out_lat, plan->d_out_loss, plan->n, ipt ? *ipt : none, d_flags,
                           d_deliver, (unsigned long long *)d_counters, d_stats ? partial : nullptr, plan->d_draws,
                           plan->d_pkt_bad);
        if (d_stats)
            hipLaunchKernelGGL(stats_kernel, dim3(1), dim3(1024), 0, s, partial, blocks,
                               (unsigned long long *)d_stats);
    }
    if (hipGetLastError() != hipSuccess) {
        perr(err, SRT_ERR_HIP, "packet kernel launch failed");
        return SRT_ERR_HIP;
    }
    return SRT_OK;
}

}  // namespace

namespace srt {
// srt_init: loads this unit's code object (srt::preload_kernels)
hipError_t preload_packet() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&round_kernel<false, true>));
}
}  // namespace srt

extern "C" srt_status srt_packet_batch(srt_plan *plan, const srt_pkt *d_pkts, const uint32_t *d_host_pkt_ptr,
                                       uint32_t n_hosts, uint64_t n_pkts, uint64_t *d_rng, const srt_round *round,
                                       uint32_t *d_flags, uint64_t *d_deliver, uint64_t *d_counters,
                                       uint64_t *d_stats, srt_err *err) {
    return packet_round(plan, d_pkts, d_host_pkt_ptr, n_hosts, n_pkts, d_rng, round, d_flags, d_deliver, d_counters,
                        d_stats, nullptr, err);
}

extern "C" srt_status srt_packet_batch_ip(srt_plan *plan, srt_ip_resolver *res, const srt_pkt_ip *d_pkts,
                                          const uint32_t *d_host_pkt_ptr, uint32_t n_hosts, uint64_t n_pkts,
                                          uint64_t *d_rng, const srt_round *round, uint32_t *d_flags,
                                          uint64_t *d_deliver, uint64_t *d_counters, uint64_t *d_stats,
                                          srt_err *err) {
    if (err) std::memset(err, 0, sizeof *err);
    if (!plan || !res) {
        perr(err, SRT_ERR_INVALID, "null argument");
        return SRT_ERR_INVALID;
    }
    static_assert(sizeof(srt_pkt_ip) == sizeof(srt_pkt), "srt_pkt_ip mirrors srt_pkt's layout");
    srt::IpTable t{};
    if (srt_status st = srt::ip_table_device(res, plan->device, &t, err); st != SRT_OK) return st;
    return packet_round(plan, reinterpret_cast<const srt_pkt *>(d_pkts), d_host_pkt_ptr, n_hosts, n_pkts, d_rng,
                        round, d_flags, d_deliver, d_counters, d_stats, &t, err);
}

extern "C" srt_status srt_packet_status(srt_plan *plan, srt_err *err) {
    if (err) std::memset(err, 0, sizeof *err);
    if (!plan) return SRT_ERR_INVALID;
    if (hipSetDevice(plan->device) != hipSuccess || hipStreamSynchronize(plan->stream) != hipSuccess) {
        perr(err, SRT_ERR_HIP, "hipStreamSynchronize failed");
        return SRT_ERR_HIP;
    }
    if (!plan->d_pkt_bad) return SRT_OK;
    uint32_t bad = 0;
    if (hipMemcpy(&bad, plan->d_pkt_bad, 4, hipMemcpyDeviceToHost) != hipSuccess) return SRT_ERR_HIP;
    if (bad) {
        (void)hipMemset(plan->d_pkt_bad, 0, 4);
        // WorkerShared::reliability(src, dst).unwrap() (worker.rs:359-361)
        perr(err, SRT_ERR_INVALID, "a packet's source or destination address has no node in the routing table");
        return SRT_ERR_INVALID;
    }
    return SRT_OK;
}

// ------------------------------------------------------------------ host RNG
// The per-host stream lives in Shadow's Host (host.rs:122, 233); these are the
// library's host-side copies of its three steps, so a caller can seed, advance
// and check the 4 x u64 states it hands to srt_packet_batch.
extern "C" void srt_xoshiro_seed_from_u64(uint64_t seed, uint64_t state[4]) {
    // rand_core 0.6 SeedableRng::seed_from_u64 for Xoshiro256PlusPlus
    // (rand_xoshiro 0.6.0): SplitMix64 outputs as the four state words
    uint64_t x = seed;
    for (int i = 0; i < 4; ++i) {
        x += 0x9E3779B97F4A7C15ull;
        uint64_t z = x;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        state[i] = z ^ (z >> 31);
    }
}

extern "C" void srt_xoshiro_next_u64(uint64_t state[4], uint64_t count, uint64_t *out) {
    uint64_t s0 = state[0], s1 = state[1], s2 = state[2], s3 = state[3];
    for (uint64_t i = 0; i < count; ++i) {
        const uint64_t v = xoshiro_next(s0, s1, s2, s3);
        if (out) out[i] = v;
    }
    state[0] = s0;
    state[1] = s1;
    state[2] = s2;
    state[3] = s3;
}

namespace {
// std::hash::DefaultHasher (SipHash-1-3, keys 0, 0; Rust 1.76) of a &str:
// the bytes, then 0xFF (str's Hash impl)
uint64_t siphash13_str(const char *s, size_t len) {
    uint64_t v0 = 0x736F6D6570736575ull, v1 = 0x646F72616E646F6Dull, v2 = 0x6C7967656E657261ull,
             v3 = 0x7465646279746573ull;
    auto round = [&] {
        v0 += v1; v1 = rotl(v1, 13); v1 ^= v0; v0 = rotl(v0, 32);
        v2 += v3; v3 = rotl(v3, 16); v3 ^= v2;
        v0 += v3; v3 = rotl(v3, 21); v3 ^= v0;
        v2 += v1; v1 = rotl(v1, 17); v1 ^= v2; v2 = rotl(v2, 32);
    };
    const size_t n = len + 1;
    auto byte = [&](size_t i) -> uint64_t { return i < len ? (uint8_t)s[i] : 0xffu; };
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w = 0;
        for (int k = 0; k < 8; ++k) w |= byte(i + k) << (8 * k);
        v3 ^= w;
        round();
        v0 ^= w;
    }
    uint64_t b = (uint64_t)(n & 0xff) << 56;
    for (size_t k = 0; i + k < n; ++k) b |= byte(i + k) << (8 * k);
    v3 ^= b;
    round();
    v0 ^= b;
    v2 ^= 0xff;
    round();
    round();
    round();
    return v0 ^ v1 ^ v2 ^ v3;
}
}  // namespace

extern "C" uint64_t srt_host_node_seed(uint32_t general_seed, const char *hostname, size_t len) {
    // sim_config.rs:47-53: randomness_for_seed_calc = the first u64 of
    // Xoshiro256PlusPlus::seed_from_u64(general.seed); :222-227, :244: the
    // host's seed = that ^ DefaultHasher(hostname)
    uint64_t st[4], r = 0;
    srt_xoshiro_seed_from_u64(general_seed, st);
    srt_xoshiro_next_u64(st, 1, &r);
    return r ^ siphash13_str(hostname ? hostname : "", hostname ? len : 0);
}
