// srt_fw.hip -- blocked min-plus Floyd-Warshall over packed path keys, gfx950.
//
// Replaces NetworkGraph::compute_shortest_paths (src/main/network/graph/mod.rs:183-228):
// instead of one petgraph Dijkstra per in-use source on a rayon pool, the whole
// graph is closed in HBM with a three-phase blocked Floyd-Warshall, B = 128:
//   round kb:  phase 1: close the B x B pivot block P in LDS (one workgroup);
//              phase 2: pivot block-row    R <- P* (x) R,
//                       pivot block-column Q <- Q (x) P*      (min-plus products:
//                       with the closed P* the in-block sequential sweep of FW
//                       collapses to one product);
//              phase 3: every other block C <- min(C, Q(i) (x) R(j)) -- the N^3
//                       hot loop, a min-plus "GEMM" with K = B.
// Phases 2 and 3 run the same tile kernel (minplus_tile_kernel).
//
// Path keys (see KeyParams, srt_internal.h) are path LATENCIES in units of g,
// exact integers carried either as f64 (< 2^53, the fast path: v_add_f64 +
// v_min_f64 = 2 VALU ops per relaxation) or as u64 (< 2^62: v_lshl_add_u64 +
// v_cmp_lt_u64 + 2 v_cndmask = 4 ops).  Both give bit-identical latencies; the
// host picks f64 whenever its bound proof fits in 53 bits.  packet_loss is not
// carried through the closure: the exact-loss pass (srt_loss.hip) folds it
// over the tight shortest-path DAG afterwards, bit for bit as the reference.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "srt_internal.h"

namespace srt {

namespace {

constexpr int B = FW_B;  // 128: pivot block / tile edge
constexpr int KC = 16;   // k-chunk staged in LDS per pipeline step of the tile kernel
constexpr int NT3 = 256; // tile kernel: 4 waves; 66 KB LDS -> 2 workgroups per CU
constexpr int TR = 8;    // rows per thread   (128 / 16 row-threads)
constexpr int TC = 8;    // cols per thread   (128 / 16 col-threads)

template <typename K>
struct KeyOps;

template <>
struct KeyOps<uint64_t> {
    static __device__ __forceinline__ uint64_t inf() { return KEY_INF; }
    static __device__ __forceinline__ uint64_t zero() { return 0ull; }
    static __device__ __forceinline__ uint64_t kmin(uint64_t a, uint64_t b) { return a < b ? a : b; }
    static __device__ __forceinline__ uint64_t from_int(uint64_t v) { return v; }
    static __device__ __forceinline__ bool is_inf(uint64_t k) { return k >= KEY_INF; }
    static __device__ __forceinline__ uint64_t to_int(uint64_t k) { return k; }
};

// u32 latency keys (2 lmax < KEY32_INF, host-proved): INF + INF < 2^32, so a
// candidate never wraps and min keeps every value <= KEY32_INF
template <>
struct KeyOps<uint32_t> {
    static __device__ __forceinline__ uint32_t inf() { return KEY32_INF; }
    static __device__ __forceinline__ uint32_t zero() { return 0u; }
    static __device__ __forceinline__ uint32_t kmin(uint32_t a, uint32_t b) { return a < b ? a : b; }
    static __device__ __forceinline__ uint32_t from_int(uint64_t v) { return (uint32_t)v; }
    static __device__ __forceinline__ bool is_inf(uint32_t k) { return k >= KEY32_INF; }
    static __device__ __forceinline__ uint64_t to_int(uint32_t k) { return k; }
};

// u16 latency keys (2 lmax < KEY16_INF, host-proved -- a complete graph's
// shortest paths never exceed its longest edge): INF + INF < 2^16, like u32
template <>
struct KeyOps<uint16_t> {
    static __device__ __forceinline__ uint16_t inf() { return KEY16_INF; }
    static __device__ __forceinline__ uint16_t zero() { return 0; }
    static __device__ __forceinline__ uint16_t kmin(uint32_t a, uint32_t b) { return (uint16_t)(a < b ? a : b); }
    static __device__ __forceinline__ uint16_t from_int(uint64_t v) { return (uint16_t)v; }
    static __device__ __forceinline__ bool is_inf(uint16_t k) { return k >= KEY16_INF; }
    static __device__ __forceinline__ uint64_t to_int(uint16_t k) { return k; }
};

template <>
struct KeyOps<double> {
    static __device__ __forceinline__ double inf() { return __builtin_huge_val(); }
    static __device__ __forceinline__ double zero() { return 0.0; }
    // Keys are never NaN, so v_min_f64 needs no IEEE-mode input quieting; with
    // __builtin_fmin hipcc emits a v_max_f64 x,x,x canonicalisation per operand
    // on loop-carried values (+50% VALU in the hot loop), hence the asm.
    static __device__ __forceinline__ double kmin(double a, double b) {
        double r;
        asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
        return r;
    }
    static __device__ __forceinline__ double from_int(uint64_t v) { return (double)v; }
    static __device__ __forceinline__ bool is_inf(double k) { return !(k < 9007199254740992.0); }
    static __device__ __forceinline__ uint64_t to_int(double k) { return (uint64_t)k; }
};

// One row of the register tile: acc[j] = min(acc[j], a + b[j]), j < 8.
// f64: the 8 adds are issued before the 8 mins (dependency distance 8) -- left
// to itself hipcc reuses one temporary and pairs every add with its min.
template <typename K>
__device__ __forceinline__ void relax_row8(K (&acc)[8], K a, const K (&b)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = KeyOps<K>::kmin(acc[j], a + b[j]);
}

template <>
__device__ __forceinline__ void relax_row8<uint16_t>(uint16_t (&acc)[8], uint16_t a, const uint16_t (&b)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t t = (uint32_t)a + b[j];  // < 2^16: both operands <= KEY16_INF
        acc[j] = (uint16_t)(acc[j] < t ? acc[j] : t);
    }
}

template <>
__device__ __forceinline__ void relax_row8<double>(double (&acc)[8], double a, const double (&b)[8]) {
    double t0, t1, t2, t3, t4, t5, t6, t7;
    asm("v_add_f64 %0, %16, %17\n\t"
        "v_add_f64 %1, %16, %18\n\t"
        "v_add_f64 %2, %16, %19\n\t"
        "v_add_f64 %3, %16, %20\n\t"
        "v_add_f64 %4, %16, %21\n\t"
        "v_add_f64 %5, %16, %22\n\t"
        "v_add_f64 %6, %16, %23\n\t"
        "v_add_f64 %7, %16, %24\n\t"
        "v_min_f64 %8, %8, %0\n\t"
        "v_min_f64 %9, %9, %1\n\t"
        "v_min_f64 %10, %10, %2\n\t"
        "v_min_f64 %11, %11, %3\n\t"
        "v_min_f64 %12, %12, %4\n\t"
        "v_min_f64 %13, %13, %5\n\t"
        "v_min_f64 %14, %14, %6\n\t"
        "v_min_f64 %15, %15, %7"
        : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "=&v"(t4), "=&v"(t5), "=&v"(t6), "=&v"(t7),
          "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]),
          "+v"(acc[6]), "+v"(acc[7])
        : "v"(a), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]),
          "v"(b[7]));
}

// ------------------------------------------------------------------ init
// rows [r0, r1) of D: 0 on the diagonal, +inf elsewhere
constexpr uint16_t F16_INF_BITS = 0x6400;  // 1024.0: f16 plans' INF (below)

template <typename K>
__global__ void fill_kernel(K *__restrict__ D, uint32_t Vp, uint32_t r0, uint32_t r1, bool f16) {
    const uint64_t first = (uint64_t)r0 * Vp, total = (uint64_t)(r1 - r0) * Vp;
    const K inf = f16 ? (K)F16_INF_BITS : KeyOps<K>::inf();  // f16: 2-byte keys only
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t r = (uint32_t)((first + e) / Vp), c = (uint32_t)((first + e) % Vp);
        D[first + e] = (r == c) ? KeyOps<K>::zero() : inf;
    }
}

// f16-key plans (srt_plan::fw_f16): the closure runs on f16 integer keys
// (exact below 2048, INF = 1024 = 0x6400) and every other stage -- init, the
// loss pass, the exchanges, fetch -- sees the u16 integer keys
// (KEY16_INF = unreachable).  One pass each way over D (2 x 2 B per pair,
// ~0.1 ms at 16k).  Values >= 1024 saturate to INF: exact, since the host
// proved every finite distance < 1024 (every stored key is then min(real
// walk, INF), as for u16 / u32 keys).
__global__ void keys_to_f16_kernel(uint16_t *__restrict__ D, uint64_t n8) {
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < n8; e += (uint64_t)gridDim.x * blockDim.x) {
        uint4 v = reinterpret_cast<uint4 *>(D)[e];
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t o = 0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t k = (w[q] >> (16 * h)) & 0xffffu;
                const uint16_t f = k >= 1024u ? F16_INF_BITS : __builtin_bit_cast(uint16_t, (_Float16)(float)k);
                o |= (uint32_t)f << (16 * h);
            }
            w[q] = o;
        }
        reinterpret_cast<uint4 *>(D)[e] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}
__global__ void keys_from_f16_kernel(uint16_t *__restrict__ D, uint64_t n8) {
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < n8; e += (uint64_t)gridDim.x * blockDim.x) {
        uint4 v = reinterpret_cast<uint4 *>(D)[e];
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t o = 0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint16_t f = (uint16_t)((w[q] >> (16 * h)) & 0xffffu);
                const uint32_t k =
                    f >= F16_INF_BITS ? (uint32_t)KEY16_INF : (uint32_t)(float)__builtin_bit_cast(_Float16, f);
                o |= k << (16 * h);
            }
            w[q] = o;
        }
        reinterpret_cast<uint4 *>(D)[e] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

// key of an edge: its latency in units of g (g divides every edge latency;
// below 2^53 the f64 quotient of two exact integers is exact, and cheaper
// than the u64 division)
__device__ __forceinline__ uint64_t edge_key(uint64_t lat, const KeyParams &kp) {
    if (lat < (1ull << 53)) return (uint64_t)((double)lat / (double)kp.g);
    return lat / kp.g;
}

// D[u][v] = min over parallel edges u->v (one wave per graph row).  The
// diagonal keeps 0: a self-loop never shortens a path, and the table's
// diagonal is the raw self-loop written by the loss pass (mod.rs:210-217).
// UNIQUE (host-checked: no parallel edges) stores the key instead of the
// memory-side atomic min (16k complete graph: 2.5 ms -> one plain store pass).
// f16 (2-byte keys of an f16 plan): the keys stored as f16 integer bits
// straight away (the conversion pass before the closure is skipped)
template <typename K, bool UNIQUE>
__global__ void scatter_edges_kernel(K *__restrict__ D, uint32_t Vp,
                                     const uint64_t *__restrict__ row_ptr,
                                     const uint32_t *__restrict__ col,
                                     const uint64_t *__restrict__ lat, uint32_t u0, uint32_t u1, KeyParams kp,
                                     bool f16) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t u = u0 + wave; u < u1; u += nwaves) {
        const uint64_t b = row_ptr[u], e = row_ptr[u + 1];
        for (uint64_t k = b + lane; k < e; k += 64) {
            const uint32_t v = col[k];
            if (v == u) continue;
            // integer key order == f64 order for exact integers: atomicMin on the
            // u64 value works for both representations (f64 bits of non-negative
            // doubles order like the doubles)
            // an edge longer than the proved bound (possible under the
            // eccentricity proof) is never on a shortest path: stored as INF
            uint64_t key = edge_key(lat[k], kp);
            if constexpr (std::is_same<K, double>::value) {
                if (key >= (1ull << 53)) key = 0x7ff0000000000000ull;  // marker, mapped to +inf below
            } else {
                const uint64_t inf = KeyOps<K>::to_int(KeyOps<K>::inf());
                key = key < inf ? key : inf;
            }
            if constexpr (sizeof(K) == 2) {
                if (f16)  // non-negative f16 bit patterns order like the values: the min below still holds
                    key = key >= 1024u ? F16_INF_BITS : __builtin_bit_cast(uint16_t, (_Float16)(float)key);
                K *dst = &D[(uint64_t)u * Vp + v];
                if constexpr (UNIQUE) {
                    *dst = (K)key;
                } else {
                    // 16-bit atomic min: CAS on the aligned 32-bit word
                    unsigned int *w = (unsigned int *)((uintptr_t)dst & ~(uintptr_t)3);
                    const unsigned sh = ((uintptr_t)dst & 2) ? 16u : 0u;
                    unsigned int old = *w, assumed;
                    do {
                        assumed = old;
                        if (((assumed >> sh) & 0xffffu) <= key) break;
                        old = atomicCAS(w, assumed, (assumed & ~(0xffffu << sh)) | ((unsigned)key << sh));
                    } while (old != assumed);
                }
            } else if constexpr (sizeof(K) == 4) {
                if constexpr (UNIQUE)
                    D[(uint64_t)u * Vp + v] = (K)key;
                else
                    atomicMin((unsigned int *)&D[(uint64_t)u * Vp + v], (unsigned int)key);
            } else {
                uint64_t bits;
                if constexpr (std::is_same<K, double>::value) {
                    const double d = key == 0x7ff0000000000000ull ? KeyOps<double>::inf() : (double)key;
                    bits = __builtin_bit_cast(uint64_t, d);
                } else {
                    bits = key;
                }
                if constexpr (UNIQUE)
                    reinterpret_cast<uint64_t *>(D)[(uint64_t)u * Vp + v] = bits;
                else
                    atomicMin((unsigned long long *)&D[(uint64_t)u * Vp + v], (unsigned long long)bits);
            }
        }
    }
}

// ------------------------------------------------------------- phase 1
// Close the 128x128 pivot block.  Same footprint as the tile kernel (256
// threads, 8x8 keys per thread in registers) so that, under look-ahead, it can
// take the slot of any retiring phase-3 workgroup.  Thread (tx, ty) holds rows
// ty*8+i and cols tx*8+j.  Step k needs row k and column k; their owners
// publish them (after their own step k-1 update) into double-buffered LDS
// vectors: one barrier per step.  The k loop is unrolled by 8 so the owned
// element index (k & 7) is static (a runtime index would send p to scratch).
// P1R = rows per thread (8: 256 threads, one wave per SIMD; 4: 512 threads,
// two waves per SIMD so one wave's LDS/barrier wait hides behind the other's
// VALU work -- the kernel is latency bound, 128 dependent steps).
template <typename K, int P1R>
__global__ __launch_bounds__(16 * (B / P1R)) void fw_phase1_kernel(K *__restrict__ D, uint32_t Vp, uint32_t kb) {
    __shared__ K rowbuf[2][B];
    __shared__ K colbuf[2][B];
    __builtin_amdgcn_s_setprio(3);  // critical path of the look-ahead chain
    const int tid = threadIdx.x, tx = tid % 16, ty = tid / 16;
    const uint64_t k0 = (uint64_t)kb * B;
    K p[P1R][TC];
#pragma unroll
    for (int i = 0; i < P1R; ++i) {
        const K *src = D + (k0 + ty * P1R + i) * Vp + k0 + tx * TC;
#pragma unroll
        for (int j = 0; j < TC; ++j) p[i][j] = src[j];
    }
    // step k = 8g + e: row k lives in thread-row k / P1R at element k % P1R,
    // column k in thread-column g at element e -- both static once e is
    auto publish = [&](int g, int e, int buf) {
        const int k = 8 * g + e;
        if (ty == k / P1R) {
#pragma unroll
            for (int j = 0; j < TC; ++j) rowbuf[buf][tx * TC + j] = p[e % P1R][j];
        }
        if (tx == g) {
#pragma unroll
            for (int i = 0; i < P1R; ++i) colbuf[buf][ty * P1R + i] = p[i][e];
        }
    };
    publish(0, 0, 0);
    __syncthreads();
#pragma unroll 1
    for (int g = 0; g < B / 8; ++g) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int cur = e & 1;  // k = 8g + e, parity of k == parity of e
            K a[P1R], b[TC];
#pragma unroll
            for (int i = 0; i < P1R; ++i) a[i] = colbuf[cur][ty * P1R + i];
#pragma unroll
            for (int j = 0; j < TC; ++j) b[j] = rowbuf[cur][tx * TC + j];
#pragma unroll
            for (int i = 0; i < P1R; ++i) relax_row8<K>(p[i], a[i], b);
            // publish step k+1 = 8g + e + 1
            if (e < 7) publish(g, e + 1, cur ^ 1);
            else if (g + 1 < B / 8) publish(g + 1, 0, cur ^ 1);
            __syncthreads();
        }
    }
#pragma unroll
    for (int i = 0; i < P1R; ++i) {
        K *dst = D + (k0 + ty * P1R + i) * Vp + k0 + tx * TC;
#pragma unroll
        for (int j = 0; j < TC; ++j) dst[j] = p[i][j];
    }
}

// Phase 1 for u16 keys: the layout of fw_phase1_kernel<uint16_t, P1R> with each
// thread's 8 columns as 4 packed pairs, relaxed by v_pk_add_u16 +
// v_pk_min_u16 (a broadcast to both halves): a third of the scalar u16
// version's VALU (add, min, and the u16 widening) per step.  Sums stay below
// 2^16 (both operands <= KEY16_INF), so the packed add never wraps.
typedef unsigned short us2 __attribute__((ext_vector_type(2)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
// a2 + b of packed keys: u16 integers, or f16 integers (F16; exact below 2048)
template <bool F16>
__device__ __forceinline__ us2 add_keys2(us2 a, us2 b) {
    if constexpr (F16) return __builtin_bit_cast(us2, __builtin_bit_cast(h2, a) + __builtin_bit_cast(h2, b));
    else return a + b;
}
// F16: f16 integer keys (the sum in f16; the min on the bits, which order
// like the values for non-negative f16)
template <int P1R, bool F16 = false>
__global__ __launch_bounds__(16 * (B / P1R)) void fw_phase1_u16pk_kernel(uint16_t *__restrict__ D, uint32_t Vp,
                                                                        uint32_t kb) {
    __shared__ us2 rowbuf[2][B / 2];
    __shared__ uint16_t colbuf[2][B];
    __builtin_amdgcn_s_setprio(3);  // critical path of the look-ahead chain
    const int tid = threadIdx.x, tx = tid % 16, ty = tid / 16;
    const uint64_t k0 = (uint64_t)kb * B;
    us2 p[P1R][4];
#pragma unroll
    for (int i = 0; i < P1R; ++i) {
        const uint4 v = *reinterpret_cast<const uint4 *>(D + (k0 + ty * P1R + i) * Vp + k0 + tx * 8);
        p[i][0] = __builtin_bit_cast(us2, v.x);
        p[i][1] = __builtin_bit_cast(us2, v.y);
        p[i][2] = __builtin_bit_cast(us2, v.z);
        p[i][3] = __builtin_bit_cast(us2, v.w);
    }
    // step k = 8g + e: row k in thread-row k / P1R at element k % P1R, column
    // k in thread-column g at element e (pair e / 2, half e % 2)
    auto publish = [&](int g, int e, int buf) {
        const int k = 8 * g + e;
        if (ty == k / P1R) {
#pragma unroll
            for (int q = 0; q < 4; ++q) rowbuf[buf][tx * 4 + q] = p[k % P1R][q];
        }
        if (tx == g) {
#pragma unroll
            for (int i = 0; i < P1R; ++i) colbuf[buf][ty * P1R + i] = p[i][e / 2][e % 2];
        }
    };
    publish(0, 0, 0);
    __syncthreads();
#pragma unroll 1
    for (int g = 0; g < B / 8; ++g) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int cur = e & 1;
            us2 b[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) b[q] = rowbuf[cur][tx * 4 + q];
#pragma unroll
            for (int i = 0; i < P1R; ++i) {
                const uint16_t a = colbuf[cur][ty * P1R + i];
                const us2 a2 = {a, a};
#pragma unroll
                for (int q = 0; q < 4; ++q) p[i][q] = __builtin_elementwise_min(p[i][q], add_keys2<F16>(a2, b[q]));
            }
            if (e < 7) publish(g, e + 1, cur ^ 1);
            else if (g + 1 < B / 8) publish(g + 1, 0, cur ^ 1);
            __syncthreads();
        }
    }
#pragma unroll
    for (int i = 0; i < P1R; ++i) {
        uint4 v;
        v.x = __builtin_bit_cast(uint32_t, p[i][0]);
        v.y = __builtin_bit_cast(uint32_t, p[i][1]);
        v.z = __builtin_bit_cast(uint32_t, p[i][2]);
        v.w = __builtin_bit_cast(uint32_t, p[i][3]);
        *reinterpret_cast<uint4 *>(D + (k0 + ty * P1R + i) * Vp + k0 + tx * 8) = v;
    }
}

// ------------------------------------------------------ phases 2 and 3
// Every min-plus update of a round is C(bi,bj) <- min(C, A(bi,kb) (x) Bm(kb,bj)):
//   phase 2 row:  bi = kb  (A = P*, Bm aliases C);
//   phase 2 col:  bj = kb  (Bm = P*, A aliases C);
//   phase 3:      bi, bj != kb.
// A launch covers up to two rectangles of tiles, each rows x cols where a
// Span is [lo, hi) minus one skipped range of block indices [x0, x1).  Aliased operands
// are fully staged in LDS before C is written and each tile has exactly one
// owner workgroup, so phase-2 tiles are safe to update in place.  TAG only
// gives each use its own kernel symbol (rocprof attribution).
struct Span {
    uint32_t lo, hi, x0, x1, n;  // skipped [x0, x1) inside [lo, hi); none: x0 = NONE
};
struct Rect {
    Span r, c;
};
constexpr uint32_t NONE = 0xffffffffu;

__host__ __device__ inline uint32_t span_at(const Span &s, uint32_t i) {
    uint32_t v = s.lo + i;
    if (v >= s.x0) v += s.x1 - s.x0;
    return v;
}

// [lo, hi) minus [x0, x1) (clipped; empty or NONE: nothing skipped)
inline Span make_range(uint32_t lo, uint32_t hi, uint32_t x0, uint32_t x1) {
    if (x0 == NONE || x1 <= lo || x0 >= hi || x1 <= x0) return Span{lo, hi, NONE, NONE, hi - lo};
    x0 = std::max(x0, lo);
    x1 = std::min(x1, hi);
    return Span{lo, hi, x0, x1, (hi - lo) - (x1 - x0)};
}

// [lo, hi) minus block a and (optionally) its neighbour b = a + 1
inline Span make_span(uint32_t lo, uint32_t hi, uint32_t a = NONE, uint32_t b = NONE) {
    if (a == NONE) return make_range(lo, hi, NONE, NONE);
    if (b != NONE && b != a + 1) std::abort();  // every schedule skips adjacent blocks
    return make_range(lo, hi, a, b == NONE ? a + 1 : b + 1);
}

template <typename K, int TAG>
__global__ __launch_bounds__(NT3, 2) void minplus_tile_kernel(K *__restrict__ D, uint32_t Vp,
                                                           uint32_t kb, Rect r1, Rect r2) {
    __shared__ K As[2][B][KC + 1];  // As[buf][row][k]  (double-buffered)
    __shared__ K Bs[2][KC][B];      // Bs[buf][k][col]
    const uint32_t n1 = r1.r.n * r1.c.n;
    uint32_t t = blockIdx.x, bi, bj;
    if (t < n1) {
        if (gridDim.x == n1 && n1 >= 64) {
            // XCD-aware bijective remap: blocks b and b+8 share an XCD (round-robin
            // dispatch); each XCD gets a contiguous run of row-major tiles, so the
            // A-panel rows and many B-panel columns stay in its 4 MB L2.
            const uint32_t q = n1 / 8, rr = n1 % 8, xcd = t % 8;
            t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + t / 8;
        }
        bi = span_at(r1.r, t / r1.c.n);
        bj = span_at(r1.c, t % r1.c.n);
    } else {
        t -= n1;
        bi = span_at(r2.r, t / r2.c.n);
        bj = span_at(r2.c, t % r2.c.n);
    }
    const uint64_t i0 = (uint64_t)bi * B, j0 = (uint64_t)bj * B, k0 = (uint64_t)kb * B;
    const int tid = threadIdx.x;
    const int tx = tid % 16, ty = tid / 16;  // 16 column-threads x 16 row-threads

    // C sub-tile: rows ty*8 .. ty*8+7 (A reads: 4 distinct rows per wave, broadcast),
    // cols tx + 16 j (B reads and C stores: 16 consecutive keys per wave row)
    K acc[TR][TC];
#pragma unroll
    for (int i = 0; i < TR; ++i) {
        const K *src = D + (i0 + ty * TR + i) * Vp + j0 + tx;
#pragma unroll
        for (int j = 0; j < TC; ++j) acc[i][j] = src[16 * j];
    }
    // Two LDS buffers, one barrier per chunk.  With PREFETCH the next chunk is
    // fetched into registers while the current one is consumed (needs 32 more
    // VGPRs); without it the next chunk is staged into the other buffer before
    // the current one is consumed and the 2 workgroups per CU overlap each
    // other's staging.  Geometry (256 thr): A chunk 128 x KC, B chunk KC x 128.
    constexpr int NA = B * KC / NT3, NB = KC * B / NT3;
    constexpr bool PREFETCH = false;
    K ra[NA], rb[NB];
    auto fetch = [&](int kc) {
#pragma unroll
        for (int m2 = 0; m2 < NA; ++m2) {
            const int e = tid + NT3 * m2, r = e / KC, c = e % KC;
            ra[m2] = D[(i0 + r) * Vp + k0 + kc + c];
        }
#pragma unroll
        for (int m2 = 0; m2 < NB; ++m2) {
            const int e = tid + NT3 * m2, r = e / B, c = e % B;
            rb[m2] = D[(k0 + kc + r) * Vp + j0 + c];
        }
    };
    auto stash = [&](int buf) {
#pragma unroll
        for (int m2 = 0; m2 < NA; ++m2) {
            const int e = tid + NT3 * m2, r = e / KC, c = e % KC;
            As[buf][r][c] = ra[m2];
        }
#pragma unroll
        for (int m2 = 0; m2 < NB; ++m2) {
            const int e = tid + NT3 * m2, r = e / B, c = e % B;
            Bs[buf][r][c] = rb[m2];
        }
    };
    fetch(0);
    stash(0);
    __syncthreads();
    constexpr int NCH = B / KC;
#pragma unroll 1
    for (int ch = 0; ch < NCH; ++ch) {
        const int cur = ch & 1;
        if (PREFETCH && ch + 1 < NCH) fetch((ch + 1) * KC);
        if (!PREFETCH && ch + 1 < NCH) {  // the other buffer's readers all passed the last barrier
            fetch((ch + 1) * KC);
            stash(cur ^ 1);
        }
#pragma unroll 2
        for (int k = 0; k < KC; ++k) {
            K a[TR], b[TC];
#pragma unroll
            for (int i = 0; i < TR; ++i) a[i] = As[cur][ty * TR + i][k];
#pragma unroll
            for (int j = 0; j < TC; ++j) b[j] = Bs[cur][k][tx + 16 * j];
#pragma unroll
            for (int i = 0; i < TR; ++i) relax_row8<K>(acc[i], a[i], b);
        }
        if (PREFETCH && ch + 1 < NCH) stash(cur ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < TR; ++i) {
        K *dst = D + (i0 + ty * TR + i) * Vp + j0 + tx;
#pragma unroll
        for (int j = 0; j < TC; ++j) dst[16 * j] = acc[i][j];
    }
}

// Same tile and per-thread 8x8 register block as minplus_tile_kernel, but the
// K-chunks are staged with LDS-DMA (global_load_lds_dwordx4: no VGPR round
// trip, so the loads of chunk c+1 are issued before chunk c is consumed and
// stay in flight under its 16 k-steps; -32 VGPRs of staging registers).
// One __shared__ array holds both double-buffered images (a second __shared__
// object can make hipcc drain vmcnt before every ds_read):
//   A image [buf][16 pieces][8 rows][16 k] + 16 B pad per piece: one 1-KiB
//     lane-linear wave-instruction per piece; the pad puts the two pieces a
//     half-wave reads (rows ty*8.., ty even / odd) on different banks;
//   B image [buf][16 k][128 cols], one 1-KiB wave-instruction per k row.
constexpr int APIECE = 8 * KC + 2;          // elements per padded A piece (1040 B)
constexpr int AIMG = (B / 8) * APIECE;      // 2080
constexpr int BIMG = KC * B;                // 2048
constexpr int GBUF = AIMG + BIMG;           // elements per buffer

typedef double f64x2 __attribute__((ext_vector_type(2)));

// Operands of one k-step: a[i] for the thread's 8 rows (as 4 pairs) and b[j]
// for its 8 columns.
struct StepOps {
    f64x2 a[4];
    double b[8];
};

// LDS reads of step k into o, by inline asm so hipcc neither merges steps nor
// inserts waits: the caller waits with an explicit lgkmcnt.  abase = byte
// address of the thread's A piece, bbase = of its first B column.
template <int k>
__device__ __forceinline__ void lds_step(StepOps &o, uint32_t abase, uint32_t bbase) {
    asm volatile("ds_read2_b64 %0, %1 offset0:%2 offset1:%3" : "=v"(o.a[0]) : "v"(abase), "i"(k), "i"(16 + k));
    asm volatile("ds_read2_b64 %0, %1 offset0:%2 offset1:%3" : "=v"(o.a[1]) : "v"(abase), "i"(32 + k), "i"(48 + k));
    asm volatile("ds_read2_b64 %0, %1 offset0:%2 offset1:%3" : "=v"(o.a[2]) : "v"(abase), "i"(64 + k), "i"(80 + k));
    asm volatile("ds_read2_b64 %0, %1 offset0:%2 offset1:%3" : "=v"(o.a[3]) : "v"(abase), "i"(96 + k), "i"(112 + k));
#pragma unroll
    for (int j = 0; j < 8; ++j)
        asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(o.b[j]) : "v"(bbase), "i"(k * B * 8 + j * 128));
}

// acc[j] = min(acc[j], a + b[j]), j < 8, as one volatile asm block so it stays
// in program order with the explicit waits.
__device__ __forceinline__ void relax_row8_v(double (&acc)[8], double a, const double (&b)[8]) {
    double t0, t1, t2, t3, t4, t5, t6, t7;
    asm volatile(
        "v_add_f64 %0, %16, %17\n\t"
        "v_add_f64 %1, %16, %18\n\t"
        "v_add_f64 %2, %16, %19\n\t"
        "v_add_f64 %3, %16, %20\n\t"
        "v_add_f64 %4, %16, %21\n\t"
        "v_add_f64 %5, %16, %22\n\t"
        "v_add_f64 %6, %16, %23\n\t"
        "v_add_f64 %7, %16, %24\n\t"
        "v_min_f64 %8, %8, %0\n\t"
        "v_min_f64 %9, %9, %1\n\t"
        "v_min_f64 %10, %10, %2\n\t"
        "v_min_f64 %11, %11, %3\n\t"
        "v_min_f64 %12, %12, %4\n\t"
        "v_min_f64 %13, %13, %5\n\t"
        "v_min_f64 %14, %14, %6\n\t"
        "v_min_f64 %15, %15, %7"
        : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "=&v"(t4), "=&v"(t5), "=&v"(t6), "=&v"(t7),
          "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]),
          "+v"(acc[7])
        : "v"(a), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]));
}

// Steps k .. KC-1 of a chunk: wait for step k's operands (issued during step
// k-1), issue step k+1's reads into the other operand set, then 128 VALU ops.
template <int k>
__device__ __forceinline__ void chunk_steps(double (&acc)[TR][TC], StepOps (&o)[2], uint32_t abase,
                                            uint32_t bbase) {
    if constexpr (k < KC) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (k + 1 < KC) lds_step<k + 1>(o[(k + 1) & 1], abase, bbase);
        const StepOps &c = o[k & 1];
#pragma unroll
        for (int i = 0; i < TR; ++i) relax_row8_v(acc[i], (i & 1) ? c.a[i >> 1].y : c.a[i >> 1].x, c.b);
        chunk_steps<k + 1>(acc, o, abase, bbase);
    }
}

template <typename K, int TAG>
__global__ __launch_bounds__(NT3, 2) void minplus_glds_kernel(K *__restrict__ D, uint32_t Vp, uint32_t kb,
                                                           Rect r1, Rect r2, uint32_t ng) {
    static_assert(sizeof(K) == 8, "8-byte keys");
    __shared__ K lds[2 * GBUF];
    // the look-ahead chain (phase 2 row/col, cross) shares SIMDs with the
    // rest(kb) waves it overlaps: give it issue priority so the next round's
    // pivot work, not the bulk update, sets the pace at high rank counts
    if constexpr (TAG != 0) __builtin_amdgcn_s_setprio(2);
    const uint32_t n1 = r1.r.n * r1.c.n;
    uint32_t t = blockIdx.x, bi, bj;
    const uint32_t ngr = ng & 0xffffu;
    if (t < n1) {
        if (gridDim.x == n1 && n1 >= 64) {  // XCD-aware bijective remap (see minplus_tile_kernel)
            const uint32_t q = n1 / 8, rr = n1 % 8, xcd = t % 8;
            t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + t / 8;
        }
        const uint32_t nc = r1.c.n, full = (r1.r.n / 8) * 8 * nc;
        if ((ng & 0x10000u) && t < full) {
            // banded order (grouped launches): an XCD's ~64 resident tiles
            // cover 8 rows x 8 columns, so one round's 16 A/B panels (2 MB)
            // stay in its L2 instead of 65
            const uint32_t w = t % (8 * nc);
            bi = span_at(r1.r, (t / (8 * nc)) * 8 + w % 8);
            bj = span_at(r1.c, w / 8);
        } else {
            bi = span_at(r1.r, t / nc);
            bj = span_at(r1.c, t % nc);
        }
    } else {
        t -= n1;
        bi = span_at(r2.r, t / r2.c.n);
        bj = span_at(r2.c, t % r2.c.n);
    }
    // grouped rounds kb .. kb+ng-1 (ng > 1, see fw_rounds_group_t): chunks
    // [r NCH, (r+1) NCH) are round kb+r's update.  A tile whose highest
    // row/column index inside the group is q had rounds <= q done by the chain
    // (phase 2 of q, the in-group cross before it) and runs rounds q+1 ..; a
    // tile in row/column kb+ng-1 is all chain work and exits.
    constexpr int NCH = B / KC;
    int ch0 = 0;
    const uint32_t ng_ = ngr;
    const int ch1 = (int)ng_ * NCH;
    if (ng_ > 1) {
        const uint32_t qi = bi - kb < ng_ ? bi - kb : 0u, qj = bj - kb < ng_ ? bj - kb : 0u;
        const bool in = bi - kb < ng_ || bj - kb < ng_;
        const uint32_t q = std::max(qi, qj);
        if (in && q == ng_ - 1) return;  // workgroup-uniform, before any barrier
        ch0 = in ? (int)(q + 1) * NCH : 0;
    }
    const uint64_t i0 = (uint64_t)bi * B, j0 = (uint64_t)bj * B;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tx = tid % 16, ty = tid / 16;

    K acc[TR][TC];
#pragma unroll
    for (int i = 0; i < TR; ++i) {
        const K *src = D + (i0 + ty * TR + i) * Vp + j0 + tx;
#pragma unroll
        for (int j = 0; j < TC; ++j) acc[i][j] = src[16 * j];
    }
    // 32 wave-instructions of 1 KiB per chunk, 8 per wave: 4 A pieces (8 rows
    // each) and 4 B rows
    auto stage = [&](int ch, int buf) {
        const uint64_t kk = (uint64_t)(kb + ch / NCH) * B + (ch % NCH) * KC;  // first k row of the chunk
        K *img = lds + buf * GBUF;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int piece = wave * 4 + q;  // rows piece*8 .. +7
            const K *g = D + (i0 + piece * 8 + lane / 8) * Vp + kk + (lane % 8) * 2;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                             (__attribute__((address_space(3))) void *)(img + piece * APIECE), 16,
                                             0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int kr = wave * 4 + q;  // B row
            const K *g = D + (kk + kr) * Vp + j0 + lane * 2;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                             (__attribute__((address_space(3))) void *)(img + AIMG + kr * B), 16,
                                             0, 0);
        }
    };
    stage(ch0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll 1
    for (int ch = ch0; ch < ch1; ++ch) {
        const int cur = (ch - ch0) & 1;
        if (ch + 1 < ch1) stage(ch + 1, cur ^ 1);  // the other buffer's readers passed the last barrier
        const K *As = lds + cur * GBUF + ty * APIECE;     // the thread's A piece
        const K *Bs = lds + cur * GBUF + AIMG + tx;       // the thread's first B column
        if constexpr (std::is_same<K, double>::value) {
            const uint32_t abase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) K *)As;
            const uint32_t bbase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) K *)Bs;
            StepOps o[2];
            lds_step<0>(o[0], abase, bbase);
            chunk_steps<0>(acc, o, abase, bbase);
        } else {
#pragma unroll 2
            for (int k = 0; k < KC; ++k) {
                K a[TR], b[TC];
#pragma unroll
                for (int i = 0; i < TR; ++i) a[i] = As[i * KC + k];
#pragma unroll
                for (int j = 0; j < TC; ++j) b[j] = Bs[k * B + 16 * j];
#pragma unroll
                for (int i = 0; i < TR; ++i) relax_row8<K>(acc[i], a[i], b);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < TR; ++i) {
        K *dst = D + (i0 + ty * TR + i) * Vp + j0 + tx;
#pragma unroll
        for (int j = 0; j < TC; ++j) dst[16 * j] = acc[i][j];
    }
}

// ------------------------------------------------------------ u32 keys
// The same 128 x 128 tile per 256-thread workgroup, for 4-byte latency keys
// (the host proves 2 lmax < KEY32_INF).  Two k-steps are relaxed together,
//     acc = min3(acc, a_k + b_k, a_{k+1} + b_{k+1})
// = 2 v_add_u32 (issued at twice the rate of other VALU ops) + 1 v_min3_u32
// per 2 relaxations, against v_add_f64 + v_min_f64 per relaxation for f64
// keys (profiles/r01_valu_bench.txt: 61 / 35 / 36.5 / 36.4 Tlane-ops/s).
// Thread (tx, ty) holds rows ty + 16 i (i < 8) and columns tx*4 + c and
// 64 + tx*4 + c (c < 4): C loads/stores are 16-B per lane, 256 B contiguous
// per 16 lanes.  K-chunks of KC32 = 16 are staged by LDS-DMA (16 wave-
// instructions of 1 KiB, 4 per wave, lane-linear):
//   A image: 8 pieces of [16 rows][16 k] + 16 B pad -- a thread's row i sits
//     in piece i at row ty, so the two rows a half-wave reads with one
//     ds_read_b64 (ty and ty+1) are 16 dwords apart: distinct banks;
//   B image: [16 k][128 cols] (2 k-rows per piece); a thread reads its 4+4
//     columns of a k-row with 2 ds_read_b128, 256 contiguous bytes per 16
//     lanes: conflict-free.
constexpr int KC32 = 16;
constexpr int NCH32 = B / KC32;
constexpr int APIECE32 = 16 * KC32 + 4;       // u32 per padded A piece (1040 B)
constexpr int AIMG32 = (B / 16) * APIECE32;   // 2080
constexpr int BIMG32 = KC32 * B;              // 2048
constexpr int GBUF32 = AIMG32 + BIMG32;       // u32 per buffer

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct StepOps32 {
    u32x2 a[8];  // a[i] = (A[row i][k], A[row i][k+1])
    u32x4 b[4];  // b[0] / b[1]: k-row k, columns lo / hi; b[2] / b[3]: k-row k+1
};

// LDS reads of step-pair s (k = 2s, 2s+1) into o; abase = byte address of the
// thread's row in piece 0, bbase = of its first column in k-row 0.
template <int s>
__device__ __forceinline__ void lds_step32(StepOps32 &o, uint32_t abase, uint32_t bbase) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
        asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(o.a[i]) : "v"(abase), "i"(i * APIECE32 * 4 + 8 * s));
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(o.b[0]) : "v"(bbase), "i"((2 * s) * B * 4));
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(o.b[1]) : "v"(bbase), "i"((2 * s) * B * 4 + 256));
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(o.b[2]) : "v"(bbase), "i"((2 * s + 1) * B * 4));
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(o.b[3]) : "v"(bbase), "i"((2 * s + 1) * B * 4 + 256));
}

// acc[c] = min3(acc[c], a0 + b0[c], a1 + b1[c]), c < 4: two rounds of 4 adds
// + 2 min3 through 4 temporaries (one volatile block so it stays in order
// with the explicit waits; 4 temporaries instead of 8 keep the kernel under
// 168 VGPRs, the 3-workgroups-per-CU budget)
__device__ __forceinline__ void relax_quad32(uint32_t &c0, uint32_t &c1, uint32_t &c2, uint32_t &c3, uint32_t a0,
                                             uint32_t a1, u32x4 b0, u32x4 b1) {
    uint32_t t0, t1, t2, t3;
    asm volatile(
        "v_add_u32 %0, %8, %10\n\t"
        "v_add_u32 %1, %9, %14\n\t"
        "v_add_u32 %2, %8, %11\n\t"
        "v_add_u32 %3, %9, %15\n\t"
        "v_min3_u32 %4, %4, %0, %1\n\t"
        "v_min3_u32 %5, %5, %2, %3\n\t"
        "v_add_u32 %0, %8, %12\n\t"
        "v_add_u32 %1, %9, %16\n\t"
        "v_add_u32 %2, %8, %13\n\t"
        "v_add_u32 %3, %9, %17\n\t"
        "v_min3_u32 %6, %6, %0, %1\n\t"
        "v_min3_u32 %7, %7, %2, %3"
        : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3)
        : "v"(a0), "v"(a1), "v"(b0.x), "v"(b0.y), "v"(b0.z), "v"(b0.w), "v"(b1.x), "v"(b1.y), "v"(b1.z),
          "v"(b1.w));
}

template <int s>
__device__ __forceinline__ void chunk_steps32(uint32_t (&acc)[8][8], StepOps32 (&o)[2], uint32_t abase,
                                              uint32_t bbase) {
    if constexpr (s < KC32 / 2) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (s + 1 < KC32 / 2) lds_step32<s + 1>(o[(s + 1) & 1], abase, bbase);
        const StepOps32 &c = o[s & 1];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            relax_quad32(acc[i][0], acc[i][1], acc[i][2], acc[i][3], c.a[i].x, c.a[i].y, c.b[0], c.b[2]);
            relax_quad32(acc[i][4], acc[i][5], acc[i][6], acc[i][7], c.a[i].x, c.a[i].y, c.b[1], c.b[3]);
        }
        chunk_steps32<s + 1>(acc, o, abase, bbase);
    }
}

// tile (bi, bj) of workgroup t in the launch's rectangles (XCD-aware remap,
// banded order for grouped launches: see minplus_glds_kernel)
__device__ __forceinline__ void tile_of(uint32_t t, const Rect &r1, const Rect &r2, uint32_t ng, uint32_t &bi,
                                        uint32_t &bj) {
    const uint32_t n1 = r1.r.n * r1.c.n;
    if (t < n1) {
        if (gridDim.x == n1 && n1 >= 64 && !(ng & (1u << 26))) {  // bit 26: no remap (rest launches)
            const uint32_t q = n1 / 8, rr = n1 % 8, xcd = t % 8;
            t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + t / 8;
        }
        const uint32_t nc = r1.c.n, full = (r1.r.n / 8) * 8 * nc;
        if ((ng & 0x10000u) && t < full) {
            const uint32_t w = t % (8 * nc);
            bi = span_at(r1.r, (t / (8 * nc)) * 8 + w % 8);
            bj = span_at(r1.c, w / 8);
        } else {
            bi = span_at(r1.r, t / nc);
            bj = span_at(r1.c, t % nc);
        }
    } else {
        t -= n1;
        bi = span_at(r2.r, t / r2.c.n);
        bj = span_at(r2.c, t % r2.c.n);
    }
}

template <int TAG>
__global__ __launch_bounds__(NT3, 2) void minplus_u32_kernel(uint32_t *__restrict__ D, uint32_t Vp, uint32_t kb,
                                                               Rect r1, Rect r2, uint32_t ng) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[2 * GBUF32];
    if constexpr (TAG != 0) __builtin_amdgcn_s_setprio(2);  // look-ahead chain: issue priority
    uint32_t bi, bj;
    tile_of(blockIdx.x, r1, r2, ng, bi, bj);
    // grouped rounds (see minplus_glds_kernel)
    const uint32_t ng_ = ng & 0xffffu;
    int ch0 = 0;
    const int ch1 = (int)ng_ * NCH32;
    if (ng_ > 1) {
        const uint32_t qi = bi - kb < ng_ ? bi - kb : 0u, qj = bj - kb < ng_ ? bj - kb : 0u;
        const bool in = bi - kb < ng_ || bj - kb < ng_;
        const uint32_t q = std::max(qi, qj);
        if (in && q == ng_ - 1) return;  // workgroup-uniform, before any barrier
        ch0 = in ? (int)(q + 1) * NCH32 : 0;
    }
    const uint64_t i0 = (uint64_t)bi * B, j0 = (uint64_t)bj * B;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tx = tid % 16, ty = tid / 16;

    uint32_t acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t *src = D + (i0 + ty + 16 * i) * Vp + j0 + tx * 4;
        const u32x4 lo = *reinterpret_cast<const u32x4 *>(src), hi = *reinterpret_cast<const u32x4 *>(src + 64);
        acc[i][0] = lo.x;
        acc[i][1] = lo.y;
        acc[i][2] = lo.z;
        acc[i][3] = lo.w;
        acc[i][4] = hi.x;
        acc[i][5] = hi.y;
        acc[i][6] = hi.z;
        acc[i][7] = hi.w;
    }
    auto stage = [&](int ch, int buf) {
        const uint64_t kk = (uint64_t)(kb + ch / NCH32) * B + (ch % NCH32) * KC32;  // first k of the chunk
        uint32_t *img = lds + buf * GBUF32;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int piece = wave * 2 + q;  // A rows piece*16 .. +15
            const uint32_t *g = D + (i0 + piece * 16 + lane / 4) * Vp + kk + (lane % 4) * 4;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                             (__attribute__((address_space(3))) void *)(img + piece * APIECE32), 16,
                                             0, 0);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int piece = wave * 2 + q;  // B k-rows 2 piece, 2 piece + 1
            const uint32_t *g = D + (kk + piece * 2 + lane / 32) * Vp + j0 + (lane % 32) * 4;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                             (__attribute__((address_space(3))) void *)(img + AIMG32 + piece * 256),
                                             16, 0, 0);
        }
    };
    stage(ch0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll 1
    for (int ch = ch0; ch < ch1; ++ch) {
        const int cur = (ch - ch0) & 1;
        if (ch + 1 < ch1 ) stage(ch + 1, cur ^ 1);  // the other buffer's readers passed the last barrier
        const uint32_t *As = lds + cur * GBUF32 + ty * KC32;      // row ty of piece 0
        const uint32_t *Bs = lds + cur * GBUF32 + AIMG32 + tx * 4;  // columns tx*4 of k-row 0
        const uint32_t abase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t *)As;
        const uint32_t bbase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t *)Bs;
        StepOps32 o[2];
        lds_step32<0>(o[0], abase, bbase);
        chunk_steps32<0>(acc, o, abase, bbase);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t *dst = D + (i0 + ty + 16 * i) * Vp + j0 + tx * 4;
        u32x4 lo, hi;
        lo.x = acc[i][0];
        lo.y = acc[i][1];
        lo.z = acc[i][2];
        lo.w = acc[i][3];
        hi.x = acc[i][4];
        hi.y = acc[i][5];
        hi.z = acc[i][6];
        hi.w = acc[i][7];
        *reinterpret_cast<u32x4 *>(dst) = lo;
        *reinterpret_cast<u32x4 *>(dst + 64) = hi;
    }
}

// ------------------------------------------------------------ u16 keys
// Packed 16-bit latency keys (the host proves 2 lmax < KEY16_INF): a VGPR
// holds the keys of two adjacent columns and
//     acc = v_pk_min_u16(acc, v_pk_add_u16(a_k, b_pair))
// relaxes both with 2 instructions (A's key is broadcast to both halves by
// op_sel) -- 1 VALU slot per relaxation, where u32 keys measure 1.4
// (tools/valu_bench.hip: the u16 mix 37.6 / 34.5, the u32 mix 28.1 / 23.9
// Trelax/s at 8 / 2 waves per SIMD), and half the LDS and HBM bytes.
// Same 128 x 128 tile per 256-thread workgroup; thread (tx, ty) holds rows
// ty + 16 i (i < 8) and the 8 columns tx*8 .. tx*8+7 as 4 pairs: C loads and
// stores are 16 B per lane, 256 contiguous bytes per 16 lanes.  K-chunks of
// KC16 = 32 keys staged by LDS-DMA (16 wave-instructions of 1 KiB per chunk):
//   A image: 8 pieces of [16 rows][32 k] + 16 B pad -- byte for byte the u32
//     kernel's layout (64-B rows), so a thread reads k .. k+3 of its row i
//     with one ds_read_b64;
//   B image: [32 k][128 cols], 4 k-rows per 1-KiB piece; a thread reads its 8
//     columns of a k-row with one ds_read_b128 (16 lanes: 256 contiguous B).
constexpr int KC16 = 32;
constexpr int NCH16 = B / KC16;
constexpr int APIECE16 = 16 * KC16 + 8;      // u16 per padded A piece (1040 B)
constexpr int AIMG16 = (B / 16) * APIECE16;  // 4160
constexpr int BIMG16 = KC16 * B;             // 4096
constexpr int GBUF16 = AIMG16 + BIMG16;      // u16 per buffer (16.5 KB)

struct StepOps16 {
    u32x2 a[8];  // a[i] = A[row i][k .. k+3] (2 keys per dword)
    u32x4 b[4];  // b[m] = B[k+m][the thread's 8 columns] (4 pairs)
};

// LDS reads of step-quad s (k = 4s .. 4s+3) into o; abase = byte address of
// the thread's row in piece 0, bbase = of its first column in k-row 0.
template <int s>
__device__ __forceinline__ void lds_step16(StepOps16 &o, uint32_t abase, uint32_t bbase) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
        asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(o.a[i]) : "v"(abase), "i"(i * APIECE16 * 2 + 8 * s));
#pragma unroll
    for (int m = 0; m < 4; ++m)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(o.b[m]) : "v"(bbase), "i"((4 * s + m) * B * 2));
}

// acc[p] = pk_min(acc[p], a.H + b[p]) for the 4 column pairs p, where a.H =
// the low (H = 0) or high (H = 1) key of a, broadcast to both halves
template <int H>
__device__ __forceinline__ void relax_pairs16(uint32_t (&acc)[4], uint32_t a, u32x4 b) {
    uint32_t t0, t1, t2, t3;
    if constexpr (H == 0)
        asm volatile(
            "v_pk_add_u16 %0, %8, %9 op_sel_hi:[0,1]\n\t"
            "v_pk_add_u16 %1, %8, %10 op_sel_hi:[0,1]\n\t"
            "v_pk_add_u16 %2, %8, %11 op_sel_hi:[0,1]\n\t"
            "v_pk_add_u16 %3, %8, %12 op_sel_hi:[0,1]\n\t"
            "v_pk_min_u16 %4, %4, %0\n\t"
            "v_pk_min_u16 %5, %5, %1\n\t"
            "v_pk_min_u16 %6, %6, %2\n\t"
            "v_pk_min_u16 %7, %7, %3"
            : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])
            : "v"(a), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w));
    else
        asm volatile(
            "v_pk_add_u16 %0, %8, %9 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_add_u16 %1, %8, %10 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_add_u16 %2, %8, %11 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_add_u16 %3, %8, %12 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_min_u16 %4, %4, %0\n\t"
            "v_pk_min_u16 %5, %5, %1\n\t"
            "v_pk_min_u16 %6, %6, %2\n\t"
            "v_pk_min_u16 %7, %7, %3"
            : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])
            : "v"(a), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w));
}

// f16 keys (F16 below; the host proves every finite distance < F16_INF =
// 1024 units, so a candidate -- two stored keys, each <= 1024 -- is an
// integer <= 2048, exact in f16, and non-negative f16 bits order like the
// integers): two k-steps at once,
//     acc = v_pk_minimum3_f16(acc, a_k + b_k, a_{k+1} + b_{k+1})
// for a column pair: 2 v_pk_add_f16 (A's key of step k / k+1 broadcast by
// op_sel from the packed pair a) + 1 v_pk_minimum3_f16 per 4 relaxations --
// 0.75 VALU slot per relaxation against the u16 form's 1.0
// (tools/valu_bench.hip on the box: the f16 mix 50.7 / 47.1 Trelax/s at 8 / 2
// waves per SIMD, the u16 mix 37.7 / 34.7).  Saturation at INF is exact for
// the same reason as in u16/u32 (choose_key_params): every stored key is
// min(real walk, INF).
__device__ __forceinline__ void relax_pairs_f16(uint32_t (&acc)[4], uint32_t a, u32x4 b0, u32x4 b1) {
    uint32_t t0, t1, t2, t3, t4, t5, t6, t7;
    asm volatile(
        "v_pk_add_f16 %0, %12, %13 op_sel_hi:[0,1]\n\t"
        "v_pk_add_f16 %1, %12, %17 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
        "v_pk_add_f16 %2, %12, %14 op_sel_hi:[0,1]\n\t"
        "v_pk_add_f16 %3, %12, %18 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
        "v_pk_add_f16 %4, %12, %15 op_sel_hi:[0,1]\n\t"
        "v_pk_add_f16 %5, %12, %19 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
        "v_pk_add_f16 %6, %12, %16 op_sel_hi:[0,1]\n\t"
        "v_pk_add_f16 %7, %12, %20 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
        "v_pk_minimum3_f16 %8, %8, %0, %1\n\t"
        "v_pk_minimum3_f16 %9, %9, %2, %3\n\t"
        "v_pk_minimum3_f16 %10, %10, %4, %5\n\t"
        "v_pk_minimum3_f16 %11, %11, %6, %7"
        : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "=&v"(t4), "=&v"(t5), "=&v"(t6), "=&v"(t7), "+v"(acc[0]),
          "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])
        : "v"(a), "v"(b0.x), "v"(b0.y), "v"(b0.z), "v"(b0.w), "v"(b1.x), "v"(b1.y), "v"(b1.z), "v"(b1.w));
}

// Phase 1 for u16 / f16 keys, two FW steps per barrier.  Steps k and k+1
// (k even) both follow from row/column k and row/column k+1 as they stood
// before step k: with a = D[i][k], b = D[k][j], c = D[i][k+1], d = D[k+1][j],
//     c' = min(c, a + D[k][k+1]),   d' = min(d, D[k+1][k] + b)
// are the step-k values of column / row k+1, and two sequential steps give
//     D[i][j] <- min(D[i][j], a + b, c' + d')
// (for i = k+1 or j = k+1 the third term never wins: D'[k+1][k+1] >= 0).
// So the owners publish rows k, k+1 and columns k, k+1 together, each thread
// forms d' for its 4 column pairs and c' for its rows, and one barrier covers
// two steps: 64 instead of 128 on the look-ahead chain.  F16: the three-way
// min is one v_pk_minimum3_f16 per pair (relax_pairs_f16); u16: two
// v_pk_min_u16.  Same layout as fw_phase1_u16pk_kernel (P1R even).
// The body reads the pivot block from src (row stride ss) and writes the
// closure to dst (row stride ds): D's diagonal block, or (unpack_p1_kernel)
// the block as the row all-gather delivered it.
template <int P1R, bool F16>
__device__ __forceinline__ void phase1_pk2_body(const uint16_t *__restrict__ src, uint64_t ss,
                                                uint16_t *__restrict__ dst, uint64_t ds) {
    static_assert(P1R % 2 == 0, "rows k and k+1 must share a thread-row");
    __shared__ us2 rowbuf[2][2][B / 2];  // [buffer][row k, row k+1][column pair]
    // [buffer][row]: (D[row][k], D[row][k+1]) -- the owner's register pair as is
    __shared__ __attribute__((aligned(16))) uint32_t colbuf2[2][B];
    __builtin_amdgcn_s_setprio(3);        // critical path of the look-ahead chain
    const int tid = threadIdx.x, tx = tid % 16, ty = tid / 16;
    us2 p[P1R][4];
#pragma unroll
    for (int i = 0; i < P1R; ++i) {
        const uint4 v = *reinterpret_cast<const uint4 *>(src + (ty * P1R + i) * ss + tx * 8);
        p[i][0] = __builtin_bit_cast(us2, v.x);
        p[i][1] = __builtin_bit_cast(us2, v.y);
        p[i][2] = __builtin_bit_cast(us2, v.z);
        p[i][3] = __builtin_bit_cast(us2, v.w);
    }
    // double step k = 8g + 2e (e < 4): rows k, k+1 in thread-row k / P1R at
    // elements k % P1R and +1; columns k, k+1 in thread-column g, pair e
    auto publish = [&](int g, int e, int buf) {
        const int k = 8 * g + 2 * e;
        if (ty == k / P1R) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                rowbuf[buf][0][tx * 4 + q] = p[k % P1R][q];
                rowbuf[buf][1][tx * 4 + q] = p[k % P1R + 1][q];
            }
        }
        if (tx == g) {
#pragma unroll
            for (int i = 0; i < P1R; ++i) colbuf2[buf][ty * P1R + i] = __builtin_bit_cast(uint32_t, p[i][e]);
        }
    };
    publish(0, 0, 0);
    __syncthreads();
#pragma unroll 1
    for (int g = 0; g < B / 8; ++g) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int cur = e & 1;
            const int k = 8 * g + 2 * e;
            us2 b0[4], d1[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                b0[q] = rowbuf[cur][0][tx * 4 + q];
                d1[q] = rowbuf[cur][1][tx * 4 + q];
            }
            const uint16_t s01 = rowbuf[cur][0][k / 2][1];  // D[k][k+1]
            const uint16_t s10 = rowbuf[cur][1][k / 2][0];  // D[k+1][k]
            const us2 s10p = {s10, s10};
#pragma unroll
            for (int q = 0; q < 4; ++q) d1[q] = __builtin_elementwise_min(d1[q], add_keys2<F16>(s10p, b0[q]));
            uint32_t cp[P1R];  // (a, c) = (D[i][k], D[i][k+1]) per row
#pragma unroll
            for (int i = 0; i < P1R; i += 2) {
                const uint2 v = *reinterpret_cast<const uint2 *>(&colbuf2[cur][ty * P1R + i]);
                cp[i] = v.x;
                cp[i + 1] = v.y;
            }
            // f16: (a, c') = min((a, c), (a + 2048, a + D[k][k+1])) in two packed
            // ops (a + 2048 <= 3072 is exact and > a)
            const uint32_t kk = 0x6800u | ((uint32_t)s01 << 16);
#pragma unroll
            for (int i = 0; i < P1R; ++i) {
                us2 acp;
                if constexpr (F16) {
                    uint32_t t, r;
                    asm volatile(
                        "v_pk_add_f16 %0, %2, %3 op_sel_hi:[0,1]\n\t"
                        "v_pk_min_u16 %1, %2, %0"
                        : "=&v"(t), "=v"(r)
                        : "v"(cp[i]), "v"(kk));
                    acp = __builtin_bit_cast(us2, r);
                } else {
                    const us2 ac = __builtin_bit_cast(us2, cp[i]);
                    const uint16_t a = ac[0], c = ac[1];
                    // (a, c') with c' = min(c, a + D[k][k+1])
                    const uint16_t sum = (uint16_t)(a + s01);
                    acp = us2{a, c < sum ? c : sum};
                }
                if constexpr (F16) {
                    uint32_t acc[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) acc[q] = __builtin_bit_cast(uint32_t, p[i][q]);
                    u32x4 B0, B1;
                    B0.x = __builtin_bit_cast(uint32_t, b0[0]);
                    B0.y = __builtin_bit_cast(uint32_t, b0[1]);
                    B0.z = __builtin_bit_cast(uint32_t, b0[2]);
                    B0.w = __builtin_bit_cast(uint32_t, b0[3]);
                    B1.x = __builtin_bit_cast(uint32_t, d1[0]);
                    B1.y = __builtin_bit_cast(uint32_t, d1[1]);
                    B1.z = __builtin_bit_cast(uint32_t, d1[2]);
                    B1.w = __builtin_bit_cast(uint32_t, d1[3]);
                    relax_pairs_f16(acc, __builtin_bit_cast(uint32_t, acp), B0, B1);
#pragma unroll
                    for (int q = 0; q < 4; ++q) p[i][q] = __builtin_bit_cast(us2, acc[q]);
                } else {
                    const us2 a2 = {acp[0], acp[0]}, c2 = {acp[1], acp[1]};
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        p[i][q] = __builtin_elementwise_min(__builtin_elementwise_min(p[i][q], a2 + b0[q]),
                                                            c2 + d1[q]);
                }
            }
            if (e < 3) publish(g, e + 1, cur ^ 1);
            else if (g + 1 < B / 8) publish(g + 1, 0, cur ^ 1);
            __syncthreads();
        }
    }
#pragma unroll
    for (int i = 0; i < P1R; ++i) {
        uint4 v;
        v.x = __builtin_bit_cast(uint32_t, p[i][0]);
        v.y = __builtin_bit_cast(uint32_t, p[i][1]);
        v.z = __builtin_bit_cast(uint32_t, p[i][2]);
        v.w = __builtin_bit_cast(uint32_t, p[i][3]);
        *reinterpret_cast<uint4 *>(dst + (ty * P1R + i) * ds + tx * 8) = v;
    }
}

template <int P1R, bool F16 = false>
__global__ __launch_bounds__(16 * (B / P1R)) void fw_phase1_pk2_kernel(uint16_t *__restrict__ D, uint32_t Vp,
                                                                      uint32_t kb) {
    uint16_t *blk = D + (uint64_t)kb * B * Vp + (uint64_t)kb * B;
    phase1_pk2_body<P1R, F16>(blk, Vp, blk, Vp);
}

// The symmetric sharded chain after the row all-gather, one launch: rows
// [p0, p0 + np) (one round, or a group's) arrive; block 0 closes pivot block
// (p0, p0) straight from its slot (emu: from D) into D when p1 is set; block
// 1 + (r - p0) * nblk + c copies tile (r, c) from rank (r + c) mod N's slot
// (np * S tiles a rank: index (r - p0) * S + c / N) into rows (row r at
// rows + (r - p0) * B * Vp: D's block-rows, or the emulation's scratch),
// except the pivot block p1 closes.
template <int P1R, bool F16>
__global__ __launch_bounds__(16 * (B / P1R)) void unpack_p1_kernel(uint16_t *__restrict__ D, uint32_t Vp, uint32_t p0,
                                                                  uint32_t np, uint32_t N, uint32_t S,
                                                                  const uint16_t *__restrict__ slots,
                                                                  uint16_t *__restrict__ rows, bool emu, bool p1) {
    const uint64_t diag = (uint64_t)p0 * B * Vp + (uint64_t)p0 * B;
    if (blockIdx.x == 0) {
        if (!p1) return;
        const uint16_t *src = emu ? D + diag : slots + ((uint64_t)((2 * p0) % N) * np * S + p0 / N) * B * B;
        phase1_pk2_body<P1R, F16>(src, emu ? Vp : B, D + diag, Vp);
        return;
    }
    const uint32_t nblk = Vp / B, t = blockIdx.x - 1, r = p0 + t / nblk, c = t % nblk;
    if (p1 && r == p0 && c == p0 && !emu) return;
    const uint16_t *src = slots + ((uint64_t)((r + c) % N) * np * S + (uint64_t)(r - p0) * S + c / N) * B * B;
    uint16_t *dst = rows + (uint64_t)(r - p0) * B * Vp + (uint64_t)c * B;
    for (uint32_t e = threadIdx.x; e < B * B / 8; e += blockDim.x) {
        const uint32_t rr = e / (B / 8), cc = (e % (B / 8)) * 8;
        *reinterpret_cast<u32x4 *>(dst + (uint64_t)rr * Vp + cc) =
            *reinterpret_cast<const u32x4 *>(src + rr * B + cc);
    }
}

template <int s, bool F16>
__device__ __forceinline__ void chunk_steps16(uint32_t (&acc)[8][4], StepOps16 (&o)[2], uint32_t abase,
                                              uint32_t bbase) {
    if constexpr (s < KC16 / 4) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (s + 1 < KC16 / 4) lds_step16<s + 1>(o[(s + 1) & 1], abase, bbase);
        const StepOps16 &c = o[s & 1];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (F16) {
                relax_pairs_f16(acc[i], c.a[i].x, c.b[0], c.b[1]);
                relax_pairs_f16(acc[i], c.a[i].y, c.b[2], c.b[3]);
            } else {
                relax_pairs16<0>(acc[i], c.a[i].x, c.b[0]);
                relax_pairs16<1>(acc[i], c.a[i].x, c.b[1]);
                relax_pairs16<0>(acc[i], c.a[i].y, c.b[2]);
                relax_pairs16<1>(acc[i], c.a[i].y, c.b[3]);
            }
        }
        chunk_steps16<s + 1, F16>(acc, o, abase, bbase);
    }
}

// Symmetric closures (undirected graphs: D == D^T at every round, see
// fw_sym_check): a rest launch over a square span runs only the tiles with
// span position pi <= pj and writes each off-diagonal result twice, as
// (bi, bj) and transposed as (bj, bi) -- half the relaxations.  Grid order:
// bands of up to h rows, band b = rows hb .. hb+h-1 x columns hb .. m-1, a
// column of h tiles after another (the banded order of tile_of); the band's
// h(h-1)/2 below-diagonal slots exit at once.  h = 1 (plain row-major
// triangle, no exits) without the XCD remap of tile_of is the default: C3
// rest per build, same box, with the remap, h = 32 / 16 / 8 / 4 / 2 / 1:
// 74.9 / 66.4 / 63.5 / 62.9 / 62.4 / 62.2 ms; without it h = 4 / 2 / 1:
// 62.2 / 61.1 / 60.9 ms (band heights and the XCD remap, since removed; taller bands'
// L2 reuse does not pay -- the launch is VALU-bound, not fetch-bound -- and
// the remap puts a band's short in-group tiles all on one XCD, which then
// idles in the launch's tail; a group-last order measured 62.1).  The
// mirrored tile (bj, bi)
// is never an operand the launch's grouping rule does not already allow to
// be read mid-update (its row or column is in the group exactly when
// (bi, bj)'s is), and the excluded next-group rows/cols are symmetric.
// Band height h = band_h(ng) = 1 << bits 17-19 of ng (plan field fw_band_h, a power of 2)
__host__ __device__ inline uint32_t sym_grid(uint32_t m, uint32_t h = 8) {
    uint32_t n = 0;
    for (uint32_t b0 = 0; b0 < m; b0 += h) n += std::min(h, m - b0) * (m - b0);
    return n;
}
__host__ __device__ inline uint32_t band_bits(uint32_t h) {
    uint32_t c = 0;
    while ((2u << c) <= h && c < 7) ++c;
    return c << 17;
}
__device__ __forceinline__ uint32_t band_h(uint32_t ng) { return 1u << ((ng >> 17) & 7u); }
__device__ __forceinline__ bool tile_of_sym(uint32_t t, const Span &s, uint32_t h, bool xcd_map, uint32_t &bi,
                                            uint32_t &bj) {
    const uint32_t n1 = gridDim.x;
    if (n1 >= 64 && xcd_map) {  // XCD-aware bijective remap, as tile_of
        const uint32_t q = n1 / 8, rr = n1 % 8, xcd = t % 8;
        t = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + t / 8;
    }
    const uint32_t m = s.n;
    uint32_t b0 = 0, base = 0, pi = 0, pj = 0;
    for (; b0 < m; b0 += h) {
        const uint32_t rows = min(h, m - b0), cnt = rows * (m - b0);
        if (t < base + cnt) {
            const uint32_t w = t - base;
            pi = b0 + w % rows;
            pj = b0 + w / rows;
            break;
        }
        base += cnt;
    }
    if (pi > pj) return false;
    bi = span_at(s, pi);
    bj = span_at(s, pj);
    return true;
}

// SYM: 0 = the rect(s) as given; 1 = the triangle of the square span r1.r
// (rest launches); 2 = the rect(s) as given, each off-diagonal result also
// stored transposed (the symmetric chain: p2row also writes p2col's tiles,
// one cross rect also writes the other); 3 = a tile list (symmetric sharded
// schedule), mirrored like 1 and 2.
// F16: the keys are f16 integers (see relax_pairs_f16), else u16 integers.
template <int TAG, int SYM = 0, bool F16 = false>
__global__ __launch_bounds__(NT3, 2) void minplus_u16_kernel(uint16_t *__restrict__ D, uint32_t Vp, uint32_t kb,
                                                             Rect r1, Rect r2, uint32_t ng) {
    __shared__ __attribute__((aligned(16))) uint16_t lds[2 * GBUF16];
    if constexpr (TAG != 0) __builtin_amdgcn_s_setprio(2);  // look-ahead chain: issue priority
    uint32_t bi, bj;
    if constexpr (SYM == 1) {
        if (!tile_of_sym(blockIdx.x, r1.r, band_h(ng), (ng & (1u << 24)) != 0, bi, bj))
            return;  // workgroup-uniform, before any barrier
    } else if constexpr (SYM == 3) {
        // tile list (symmetric sharded schedule): the list's device address in
        // r2.r.lo / r2.r.hi, entries (i << 16) | j; tiles in a row or column of
        // [r1.r.x0, r1.r.x1) (this group's pivots and the look-ahead group's)
        // are skipped; results are also stored mirrored (below)
        const uint32_t *tl = reinterpret_cast<const uint32_t *>(((uint64_t)r2.r.hi << 32) | r2.r.lo);
        const uint32_t e = tl[blockIdx.x];
        bi = e >> 16;
        bj = e & 0xffffu;
        if (bi - r1.r.x0 < r1.r.x1 - r1.r.x0 || bj - r1.r.x0 < r1.r.x1 - r1.r.x0) return;
    } else {
        tile_of(blockIdx.x, r1, r2, ng, bi, bj);
    }
    // grouped rounds (see minplus_glds_kernel)
    const uint32_t ng_ = ng & 0xffffu;
    int ch0 = 0;
    const int ch1 = (int)ng_ * NCH16;
    if (ng_ > 1) {
        const uint32_t qi = bi - kb < ng_ ? bi - kb : 0u, qj = bj - kb < ng_ ? bj - kb : 0u;
        const bool in = bi - kb < ng_ || bj - kb < ng_;
        const uint32_t q = std::max(qi, qj);
        if (in && q == ng_ - 1) return;  // workgroup-uniform, before any barrier
        ch0 = in ? (int)(q + 1) * NCH16 : 0;
    }
    const uint64_t i0 = (uint64_t)bi * B, j0 = (uint64_t)bj * B;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tx = tid % 16, ty = tid / 16;

    uint32_t acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const u32x4 v = *reinterpret_cast<const u32x4 *>(D + (i0 + ty + 16 * i) * Vp + j0 + tx * 8);
        acc[i][0] = v.x;
        acc[i][1] = v.y;
        acc[i][2] = v.z;
        acc[i][3] = v.w;
    }
    auto stage = [&](int ch, int buf) {
        const uint64_t kk = (uint64_t)(kb + ch / NCH16) * B + (ch % NCH16) * KC16;  // first k of the chunk
        uint16_t *img = lds + buf * GBUF16;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int piece = wave * 2 + q;  // A rows piece*16 .. +15, 64 B each
            const uint16_t *g = D + (i0 + piece * 16 + lane / 4) * Vp + kk + (lane % 4) * 8;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                             (__attribute__((address_space(3))) void *)(img + piece * APIECE16), 16,
                                             0, 0);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int piece = wave * 2 + q;  // B k-rows 4 piece .. 4 piece + 3, 256 B each
            const uint16_t *g = D + (kk + piece * 4 + lane / 16) * Vp + j0 + (lane % 16) * 8;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                             (__attribute__((address_space(3))) void *)(img + AIMG16 + piece * 512),
                                             16, 0, 0);
        }
    };
    stage(ch0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll 1
    for (int ch = ch0; ch < ch1; ++ch) {
        const int cur = (ch - ch0) & 1;
        if (ch + 1 < ch1 ) stage(ch + 1, cur ^ 1);  // the other buffer's readers passed the last barrier
        const uint16_t *As = lds + cur * GBUF16 + ty * KC16;      // row ty of piece 0
        const uint16_t *Bs = lds + cur * GBUF16 + AIMG16 + tx * 8;  // columns tx*8 of k-row 0
        const uint32_t abase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint16_t *)As;
        const uint32_t bbase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint16_t *)Bs;
        StepOps16 o[2];
        lds_step16<0>(o[0], abase, bbase);
        chunk_steps16<0, F16>(acc, o, abase, bbase);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        u32x4 v;
        v.x = acc[i][0];
        v.y = acc[i][1];
        v.z = acc[i][2];
        v.w = acc[i][3];
        *reinterpret_cast<u32x4 *>(D + (i0 + ty + 16 * i) * Vp + j0 + tx * 8) = v;
    }
    if constexpr (SYM != 0) {
        if (bi != bj) {
            // the mirror tile: transpose through LDS ([128][129] u16 = the two
            // stage buffers, idle since the last chunk's barrier; row stride 129
            // spreads a wave's 16 column groups over 16 banks)
            constexpr int LT = B + 1;
            static_assert(B * LT <= 2 * GBUF16, "transpose image fits the stage buffers");
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const int r = ty + 16 * i, c = tx * 8 + 2 * p;
                    lds[c * LT + r] = (uint16_t)(acc[i][p] & 0xffffu);
                    lds[(c + 1) * LT + r] = (uint16_t)(acc[i][p] >> 16);
                }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int c = ty + 16 * i;  // row of the mirror tile
                const uint16_t *src = lds + c * LT + tx * 8;
                u32x4 v;
                v.x = (uint32_t)src[0] | ((uint32_t)src[1] << 16);
                v.y = (uint32_t)src[2] | ((uint32_t)src[3] << 16);
                v.z = (uint32_t)src[4] | ((uint32_t)src[5] << 16);
                v.w = (uint32_t)src[6] | ((uint32_t)src[7] << 16);
                *reinterpret_cast<u32x4 *>(D + (j0 + c) * Vp + i0 + tx * 8) = v;
            }
        }
    }
}

// D == D^T?  One 64 x 64 tile pair per workgroup, through LDS; any mismatch
// clears *sym (set to 1 beforehand).  Only blocks on or above the diagonal.
template <typename K>
__global__ __launch_bounds__(256) void sym_check_kernel(const K *__restrict__ D, uint32_t Vp, uint32_t nb,
                                                        uint32_t *sym) {
    __shared__ K t[64][65];
    const uint32_t bi = blockIdx.y, bj = blockIdx.x;
    if (bi > bj) return;
    const int tid = threadIdx.x;
    const uint64_t i0 = (uint64_t)bi * 64, j0 = (uint64_t)bj * 64;
    for (int e = tid; e < 64 * 64; e += 256) t[e / 64][e % 64] = D[(j0 + e / 64) * Vp + i0 + e % 64];
    __syncthreads();
    bool ok = true;
    for (int e = tid; e < 64 * 64; e += 256) ok &= D[(i0 + e / 64) * Vp + j0 + e % 64] == t[e % 64][e / 64];
    if (!ok) *sym = 0;  // every writer stores 0
}

// ---------------------------------------------------- symmetric sharded schedule
// u16 128 x 128 tile moves through LDS (256 threads, one tile per workgroup):
// dst <- src, or src^T.  Row strides in keys.
__device__ __forceinline__ void move_tile16(const uint16_t *__restrict__ src, uint64_t ss, uint16_t *__restrict__ dst,
                                            uint64_t ds, bool transpose, uint16_t (*t)[B + 1]) {
    const int tid = threadIdx.x;
    if (!transpose) {
        for (int e = tid; e < B * B / 8; e += 256) {  // 8 keys (16 B) per thread-step
            const int r = e / (B / 8), c = (e % (B / 8)) * 8;
            *reinterpret_cast<u32x4 *>(dst + r * ds + c) = *reinterpret_cast<const u32x4 *>(src + r * ss + c);
        }
        return;
    }
    for (int e = tid; e < B * B; e += 256) t[e / B][e % B] = src[(e / B) * ss + e % B];
    __syncthreads();
    for (int e = tid; e < B * B; e += 256) dst[(e / B) * ds + e % B] = t[e % B][e / B];
}

// Own tiles of row/column k (list entries (i << 16) | j with i == k or j == k)
// into this rank's all-gather slot, as row-k tiles: tile (k, c) at slot index
// c / N (its owner is (k + c) mod N, so the indices are distinct).  The list
// kernels store every own tile's mirror too, so (k, c) is current in row
// orientation whichever of (k, c) / (c, k) the rank owns: a plain copy.
__global__ __launch_bounds__(256) void pack_row16_kernel(const uint16_t *__restrict__ D, uint32_t Vp,
                                                         const uint32_t *__restrict__ tl, uint32_t k, uint32_t N,
                                                         uint16_t *__restrict__ slot) {
    __shared__ uint16_t t[B][B + 1];
    const uint32_t e = tl[blockIdx.x], i = e >> 16, j = e & 0xffffu;
    const uint32_t c = i == k ? j : i;
    move_tile16(D + (uint64_t)k * B * Vp + (uint64_t)c * B, Vp, slot + (uint64_t)(c / N) * B * B, B, false, t);
}

// Row k assembled from every rank's slot (S tiles each): tile (k, c) from
// rank (k + c) mod N, index c / N.
__global__ __launch_bounds__(256) void unpack_row16_kernel(uint16_t *__restrict__ row, uint32_t Vp, uint32_t k,
                                                           uint32_t N, uint32_t S, const uint16_t *__restrict__ slots) {
    __shared__ uint16_t t[B][B + 1];
    const uint32_t c = blockIdx.x;  // row = block-row k of D (B x Vp keys)
    const uint16_t *src = slots + ((uint64_t)((k + c) % N) * S + c / N) * B * B;
    move_tile16(src, B, row + (uint64_t)c * B, Vp, false, t);
}

// Every tile of a list into consecutive slots (the final exchange)
__global__ __launch_bounds__(256) void pack_list16_kernel(const uint16_t *__restrict__ D, uint32_t Vp,
                                                          const uint32_t *__restrict__ tl, uint16_t *__restrict__ buf) {
    __shared__ uint16_t t[B][B + 1];
    const uint32_t e = tl[blockIdx.x], i = e >> 16, j = e & 0xffffu;
    move_tile16(D + (uint64_t)i * B * Vp + (uint64_t)j * B, Vp, buf + (uint64_t)blockIdx.x * B * B, B, false, t);
}

// Rank blockIdx.y's tiles (its list: lists + y * tmax, cnt[y] entries) from
// its buffer into D, each off-diagonal one also transposed into its mirror
__global__ __launch_bounds__(256) void unpack_list16_kernel(uint16_t *__restrict__ D, uint32_t Vp,
                                                            const uint32_t *__restrict__ lists,
                                                            const uint32_t *__restrict__ cnt, uint32_t tmax,
                                                            const uint16_t *__restrict__ bufs, uint32_t emu) {
    __shared__ uint16_t t[B][B + 1];
    const uint32_t r = emu ? 0u : blockIdx.y, x = blockIdx.x;  // emulation: rank 0's tiles, N times
    if (x >= cnt[r]) return;
    const uint32_t e = lists[(uint64_t)r * tmax + x], i = e >> 16, j = e & 0xffffu;
    const uint16_t *src = bufs + ((uint64_t)r * tmax + x) * B * B;
    move_tile16(src, B, D + (uint64_t)i * B * Vp + (uint64_t)j * B, Vp, false, t);
    if (i != j) {
        __syncthreads();
        move_tile16(src, B, D + (uint64_t)j * B * Vp + (uint64_t)i * B, Vp, true, t);
    }
}

// Latency-oriented variant for the look-ahead chain of the sharded schedule
// (phase 2 row/col and cross): each 128x128 tile is split into four 64x64
// quadrants, one 256-thread workgroup each (4x4 keys per thread), so a chain
// launch finishes in about a quarter of a full tile's time when it is on the
// critical path (8 ranks: the per-rank rest(kb) is only ~4 tile-waves).  In
// phase 2 a quadrant reads the whole aliased pivot block-row/column while
// sibling quadrants update it: P* (x) R_mixed == P* (x) R_old because P* is
// closed (P* (x) P* == P*) and min-plus is monotone, and 8-byte stores are
// atomic, so the result is the same bits as the unsplit update.
constexpr int SQ = 64;
template <typename K, int TAG>
__global__ __launch_bounds__(256) void minplus_small_kernel(K *__restrict__ D, uint32_t Vp, uint32_t kb, Rect r1,
                                                          Rect r2) {
    __shared__ K As[2][SQ][KC + 1];
    __shared__ K Bs[2][KC][SQ];
    __builtin_amdgcn_s_setprio(2);
    const uint32_t n1 = r1.r.n * r1.c.n;
    uint32_t t = blockIdx.x >> 2, bi, bj;
    const uint32_t q = blockIdx.x & 3;
    if (t < n1) {
        bi = span_at(r1.r, t / r1.c.n);
        bj = span_at(r1.c, t % r1.c.n);
    } else {
        t -= n1;
        bi = span_at(r2.r, t / r2.c.n);
        bj = span_at(r2.c, t % r2.c.n);
    }
    const uint64_t i0 = (uint64_t)bi * B + (q >> 1) * SQ, j0 = (uint64_t)bj * B + (q & 1) * SQ;
    const uint64_t k0 = (uint64_t)kb * B;
    const int tid = threadIdx.x, tx = tid % 16, ty = tid / 16;
    K acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = D[(i0 + ty * 4 + i) * Vp + j0 + tx + 16 * j];
    K ra[4], rb[4];
    auto fetch = [&](int kc) {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int e = tid + 256 * m;
            ra[m] = D[(i0 + e / KC) * Vp + k0 + kc + e % KC];
            rb[m] = D[(k0 + kc + e / SQ) * Vp + j0 + e % SQ];
        }
    };
    auto stash = [&](int buf) {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int e = tid + 256 * m;
            As[buf][e / KC][e % KC] = ra[m];
            Bs[buf][e / SQ][e % SQ] = rb[m];
        }
    };
    fetch(0);
    stash(0);
    __syncthreads();
    constexpr int NCH = B / KC;
#pragma unroll 1
    for (int ch = 0; ch < NCH; ++ch) {
        const int cur = ch & 1;
        if (ch + 1 < NCH) fetch((ch + 1) * KC);
#pragma unroll 4
        for (int k = 0; k < KC; ++k) {
            K a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = As[cur][ty * 4 + i][k];
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = Bs[cur][k][tx + 16 * j];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = KeyOps<K>::kmin(acc[i][j], a[i] + b[j]);
        }
        if (ch + 1 < NCH) stash(cur ^ 1);  // the other buffer's readers passed the last barrier
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) D[(i0 + ty * 4 + i) * Vp + j0 + tx + 16 * j] = acc[i][j];
}

// Quarter-tile chain kernel for u16 keys with packed relaxations: a 64 x 64
// quarter of a 128 x 128 tile per 256-thread workgroup (4 per tile), thread
// (tx, ty) holding rows ty*4 .. +3 and columns tx*4 .. +3 as 2 packed pairs
// (v_pk_add_u16 + v_pk_min_u16: 8 + 8 VALU per k against the scalar quarter
// kernel's ~48).  K chunks of 32 staged through LDS, double-buffered.  Every
// off-diagonal result is also stored transposed into its mirror (symmetric D).
// MODE 2: tiles from a list (entries (i << 16) | j, address in r2.r.lo/hi,
// rows or columns r1.r.x0 / r1.r.x1 skipped), mirrored; MODE 1: the rect r1,
// mirrored; MODE 0: the rects r1 then r2, not mirrored (the look-ahead chain
// of one GPU at chain-bound sizes and of the row-sharded schedule).  F16: f16
// integer keys (see relax_pairs_f16).  nr rounds (k from kb * B to (kb + nr)
// * B: a grouped cross).  pk.slot (MODE 2, the symmetric sharded cross):
// every result tile in a row or column r of [pk.p0, pk.p0 + pk.np) also goes,
// in row-r orientation, to this rank's all-gather slot -- tile (r, c) at slot
// index (r - p0) * S + c / N (the pack of fw_rounds_sym_sharded, fused).
struct PackSpec {
    uint16_t *slot;
    uint32_t p0, np, N, S;
};
template <int TAG, int MODE, bool F16>
__global__ __launch_bounds__(256) void minplus_q16_kernel(uint16_t *__restrict__ D, uint32_t Vp, uint32_t kb, Rect r1,
                                                          Rect r2, uint32_t nr, PackSpec pk) {
    uint16_t *__restrict__ slot = pk.slot;
    const uint32_t N = pk.N;
    auto in_pack = [&](uint32_t b) { return b - pk.p0 < pk.np; };
    auto slot_tile = [&](uint32_t r, uint32_t c) {
        return slot + ((uint64_t)(r - pk.p0) * pk.S + c / N) * B * B;
    };
    constexpr int QK = 32;
    __shared__ __attribute__((aligned(16))) uint32_t At2[2][QK / 2][SQ + 4];  // [k pair][row]: (A[row][2kp], A[row][2kp+1])
    __shared__ __attribute__((aligned(16))) us2 Bs[2][QK][SQ / 2];           // [k][column pair]
    __shared__ uint16_t T[SQ][SQ + 1];
    __builtin_amdgcn_s_setprio(2);
    uint32_t t = blockIdx.x >> 2, bi, bj;
    const uint32_t q = blockIdx.x & 3;
    if constexpr (MODE == 2) {
        const uint32_t *tl = reinterpret_cast<const uint32_t *>(((uint64_t)r2.r.hi << 32) | r2.r.lo);
        const uint32_t e = tl[t];
        bi = e >> 16;
        bj = e & 0xffffu;
        if (bi - r1.r.x0 < r1.r.x1 - r1.r.x0 || bj - r1.r.x0 < r1.r.x1 - r1.r.x0) {  // skipped range [x0, x1)
            // a skipped tile of a packed row / column is current already: into the slot as it is
            if (slot && (in_pack(bi) || in_pack(bj))) {
                const uint64_t si0 = (uint64_t)bi * B + (q >> 1) * SQ, sj0 = (uint64_t)bj * B + (q & 1) * SQ;
                const int tx = threadIdx.x % 16, ty = threadIdx.x / 16;
                if (in_pack(bi)) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        *reinterpret_cast<uint2 *>(slot_tile(bi, bj) + ((q >> 1) * SQ + ty * 4 + i) * B +
                                                   (q & 1) * SQ + tx * 4) =
                            *reinterpret_cast<const uint2 *>(D + (si0 + ty * 4 + i) * Vp + sj0 + tx * 4);
                }
                if (in_pack(bj) && bi != bj) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int c = 0; c < 4; ++c)
                            T[tx * 4 + c][ty * 4 + i] = D[(si0 + ty * 4 + i) * Vp + sj0 + tx * 4 + c];
                    __syncthreads();
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int r = ty * 4 + i;
                        uint2 v;
                        v.x = (uint32_t)T[r][tx * 4] | ((uint32_t)T[r][tx * 4 + 1] << 16);
                        v.y = (uint32_t)T[r][tx * 4 + 2] | ((uint32_t)T[r][tx * 4 + 3] << 16);
                        *reinterpret_cast<uint2 *>(slot_tile(bj, bi) + ((q & 1) * SQ + r) * B + (q >> 1) * SQ +
                                                   tx * 4) = v;
                    }
                }
            }
            return;
        }
    } else {
        const uint32_t n1 = r1.r.n * r1.c.n;
        if (MODE == 1 || t < n1) {
            bi = span_at(r1.r, t / r1.c.n);
            bj = span_at(r1.c, t % r1.c.n);
        } else {
            t -= n1;
            bi = span_at(r2.r, t / r2.c.n);
            bj = span_at(r2.c, t % r2.c.n);
        }
    }
    const uint64_t i0 = (uint64_t)bi * B + (q >> 1) * SQ, j0 = (uint64_t)bj * B + (q & 1) * SQ;
    const uint64_t k0 = (uint64_t)kb * B;
    const int tid = threadIdx.x, tx = tid % 16, ty = tid / 16;
    const int NCH = (int)nr * (B / 32);  // K chunks of 32 over the nr rounds
    us2 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint2 v = *reinterpret_cast<const uint2 *>(D + (i0 + ty * 4 + i) * Vp + j0 + tx * 4);
        acc[i][0] = __builtin_bit_cast(us2, v.x);
        acc[i][1] = __builtin_bit_cast(us2, v.y);
    }
    // a chunk: A = 64 rows x 32 k (8 keys a thread), B = 32 k x 64 columns (8
    // keys).  Chunks are fetched PF ahead into a register ring, so a launch
    // of one round (4 chunks) waits on global memory once, not per chunk:
    // these launches are latency-bound chain steps
    constexpr int PF = 4;
    uint4 ra[PF], rb[PF];
    auto fetch = [&](int slot, int kc) {
        ra[slot] = *reinterpret_cast<const uint4 *>(D + (i0 + tid / 4) * Vp + k0 + kc + (tid % 4) * 8);
        rb[slot] = *reinterpret_cast<const uint4 *>(D + (k0 + kc + tid / 8) * Vp + j0 + (tid % 8) * 8);
    };
    auto stash = [&](int slot, int buf) {
        // the thread's 8 keys of row tid / 4 = 4 k pairs, at k pairs (tid % 4) * 4 ..
        const uint32_t *r = reinterpret_cast<const uint32_t *>(&ra[slot]);
#pragma unroll
        for (int x = 0; x < 4; ++x) At2[buf][(tid % 4) * 4 + x][tid / 4] = r[x];
        us2 *b = &Bs[buf][tid / 8][(tid % 8) * 4];
        b[0] = __builtin_bit_cast(us2, rb[slot].x);
        b[1] = __builtin_bit_cast(us2, rb[slot].y);
        b[2] = __builtin_bit_cast(us2, rb[slot].z);
        b[3] = __builtin_bit_cast(us2, rb[slot].w);
    };
#pragma unroll
    for (int c = 0; c < PF; ++c) fetch(c, c * QK);  // NCH is a multiple of 4 = PF
    stash(0, 0);
    __syncthreads();
    uint32_t ac[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        ac[i][0] = __builtin_bit_cast(uint32_t, acc[i][0]);
        ac[i][1] = __builtin_bit_cast(uint32_t, acc[i][1]);
    }
#pragma unroll 1
    for (int c0 = 0; c0 < NCH; c0 += PF) {
#pragma unroll
        for (int j = 0; j < PF; ++j) {
            const int ch = c0 + j, cur = j & 1;
            // two k a step: per row and column pair, acc <- min(acc, a_k + b_k,
            // a_k+1 + b_k+1) -- f16: 2 v_pk_add_f16 + 1 v_pk_minimum3_f16 (A's
            // pair broadcast by op_sel, as relax_pairs_f16); u16: 2 adds + 2 mins
#pragma unroll 4
            for (int kp = 0; kp < QK / 2; ++kp) {
                const uint4 a4 = *reinterpret_cast<const uint4 *>(&At2[cur][kp][ty * 4]);
                const uint2 b0 = *reinterpret_cast<const uint2 *>(&Bs[cur][2 * kp][tx * 2]);
                const uint2 b1 = *reinterpret_cast<const uint2 *>(&Bs[cur][2 * kp + 1][tx * 2]);
                const uint32_t av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    uint32_t t0, t1, t2, t3;
                    if constexpr (F16)
                        asm volatile(
                            "v_pk_add_f16 %0, %6, %7 op_sel_hi:[0,1]\n\t"
                            "v_pk_add_f16 %1, %6, %9 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
                            "v_pk_add_f16 %2, %6, %8 op_sel_hi:[0,1]\n\t"
                            "v_pk_add_f16 %3, %6, %10 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
                            "v_pk_minimum3_f16 %4, %4, %0, %1\n\t"
                            "v_pk_minimum3_f16 %5, %5, %2, %3"
                            : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "+v"(ac[i][0]), "+v"(ac[i][1])
                            : "v"(av[i]), "v"(b0.x), "v"(b0.y), "v"(b1.x), "v"(b1.y));
                    else
                        asm volatile(
                            "v_pk_add_u16 %0, %6, %7 op_sel_hi:[0,1]\n\t"
                            "v_pk_add_u16 %1, %6, %9 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
                            "v_pk_add_u16 %2, %6, %8 op_sel_hi:[0,1]\n\t"
                            "v_pk_add_u16 %3, %6, %10 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
                            "v_pk_min_u16 %4, %4, %0\n\t"
                            "v_pk_min_u16 %5, %5, %2\n\t"
                            "v_pk_min_u16 %4, %4, %1\n\t"
                            "v_pk_min_u16 %5, %5, %3"
                            : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "+v"(ac[i][0]), "+v"(ac[i][1])
                            : "v"(av[i]), "v"(b0.x), "v"(b0.y), "v"(b1.x), "v"(b1.y));
                }
            }
            if (ch + 1 < NCH) {
                stash((j + 1) % PF, cur ^ 1);  // the other buffer's readers passed the last barrier
                if (ch + 1 + PF - 1 < NCH) fetch(j, (ch + PF) * QK);  // slot j is free again
            }
            __syncthreads();
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        acc[i][0] = __builtin_bit_cast(us2, ac[i][0]);
        acc[i][1] = __builtin_bit_cast(us2, ac[i][1]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint2 v;
        v.x = __builtin_bit_cast(uint32_t, acc[i][0]);
        v.y = __builtin_bit_cast(uint32_t, acc[i][1]);
        *reinterpret_cast<uint2 *>(D + (i0 + ty * 4 + i) * Vp + j0 + tx * 4) = v;
        // the slot takes the quarter as computed when it is a packed row's
        if (MODE == 2 && slot && in_pack(bi))
            *reinterpret_cast<uint2 *>(slot_tile(bi, bj) + ((q >> 1) * SQ + ty * 4 + i) * B + (q & 1) * SQ +
                                       tx * 4) = v;
    }
    if (MODE != 0 && bi != bj) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int c = 0; c < 4; ++c) T[tx * 4 + c][ty * 4 + i] = acc[i][c / 2][c % 2];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = ty * 4 + i;  // row of the mirror quarter
            uint2 v;
            v.x = (uint32_t)T[r][tx * 4] | ((uint32_t)T[r][tx * 4 + 1] << 16);
            v.y = (uint32_t)T[r][tx * 4 + 2] | ((uint32_t)T[r][tx * 4 + 3] << 16);
            *reinterpret_cast<uint2 *>(D + (j0 + r) * Vp + i0 + tx * 4) = v;
            // ... or transposed, when it is a packed column's (tile (bi, r) = mirror (r, bi))
            if (MODE == 2 && slot && in_pack(bj))
                *reinterpret_cast<uint2 *>(slot_tile(bj, bi) + ((q & 1) * SQ + r) * B + (q >> 1) * SQ + tx * 4) =
                    v;
        }
    }
}

__global__ void pack_kernel(const uint64_t *__restrict__ lat, const float *__restrict__ loss,
                            srt_path *__restrict__ out, uint64_t total) {
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        srt_path p;
        p.latency_ns = lat[e];
        p.packet_loss = loss[e];
        p._pad = 0;
        out[e] = p;
    }
}

// 8-byte download form of a table entry: latency in units of g (u32, the
// unreachable ~0 as 0xFFFFFFFF) + the f32 loss bits; the host expands it into
// srt_path.  Needs every finite latency / g < 2^32 - 1 (KeyParams::lat32;
// the diagonal's self-loop latency is an edge latency, so a multiple of g).
__global__ void pack8_kernel(const uint64_t *__restrict__ lat, const float *__restrict__ loss, uint2 *__restrict__ out,
                             uint64_t total, uint64_t g) {
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t l = lat[e];
        out[e] = make_uint2(l == ~0ull ? 0xffffffffu : (uint32_t)(l / g), __float_as_uint(loss[e]));
    }
}

// 6-byte download form for u16-key plans (every finite latency / g < 0x4000):
// the piece's latencies as u16 (unreachable 0xFFFF), then its f32 losses at
// byte offset loss_off
__global__ void pack6_kernel(const uint64_t *__restrict__ lat, const float *__restrict__ loss, uint8_t *__restrict__ out,
                             uint64_t total, uint64_t g, uint64_t loss_off) {
    uint16_t *l16 = reinterpret_cast<uint16_t *>(out);
    float *lf = reinterpret_cast<float *>(out + loss_off);
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t l = lat[e];
        l16[e] = l == ~0ull ? (uint16_t)0xffffu : (uint16_t)(l / g);
        lf[e] = loss[e];
    }
}

// 5-byte download records (closures whose every finite latency is <= 510
// units): the low 8 bits of the units in one array, then (16-byte aligned)
// the loss bits with the units' 9th bit in the sign bit (a table loss is
// never negative: folds give +0, and the diagonal, whose self-loop may be
// -0.0, is rewritten on the host).  511 = unreachable.
__global__ void pack5_kernel(const uint64_t *__restrict__ lat, const float *__restrict__ loss, uint8_t *__restrict__ out,
                             uint64_t total, uint64_t g, uint64_t loss_off) {
    uint32_t *lw = reinterpret_cast<uint32_t *>(out + loss_off);
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t l = lat[e];
        const uint64_t u = l == ~0ull ? 511u : l / g;
        const uint32_t u9 = u < 511u ? (uint32_t)u : 511u;
        out[e] = (uint8_t)u9;
        lw[e] = (__float_as_uint(loss[e]) & 0x7fffffffu) | ((u9 >> 8) << 31);
    }
}

__global__ void widen_u32_kernel(uint64_t *__restrict__ dst, const uint32_t *__restrict__ src, uint64_t count) {
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < count; e += (uint64_t)gridDim.x * blockDim.x)
        dst[e] = src[e];
}

// ShadowEdge::try_from's loss range (mod.rs:72-111) on the device, over the
// losses as the end-to-end build uploads them: the first entry (k0 + index)
// outside [0, 1] (or NaN; -0.0 is valid) atomic-min'ed into *first
__global__ void loss_check_kernel(const uint32_t *__restrict__ bits, uint64_t count, uint64_t k0,
                                  unsigned long long *first) {
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < count; e += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t q = bits[e];
        if (q > 0x3f800000u && q != 0x80000000u) atomicMin(first, (unsigned long long)(k0 + e));
    }
}

__global__ void iota_rows_kernel(uint32_t *__restrict__ dst, uint64_t count, uint32_t V) {
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < count; e += (uint64_t)gridDim.x * blockDim.x)
        dst[e] = (uint32_t)(e % V);
}

template <typename K>
void fw_init_t(srt_plan *p) {
    K *D = reinterpret_cast<K *>(p->d_D);
    // sharded: only the local block-rows -- every other row this rank ever
    // reads arrives whole first (pivot-row broadcasts, the final all-gather)
    // (the symmetric sharded schedule needs every row: fw_sym_check runs on
    // the first build's full init, and symmetric plans keep it)
    const bool local = p->comm && !(sizeof(K) == 2 && (p->fw_sym || !p->fw_sym_known));
    const uint32_t r0 = local ? p->rb0 * B : 0, r1 = local ? p->rb1 * B : p->Vp;
    const uint32_t u0 = std::min(r0, p->V), u1 = std::min(r1, p->V);
    // f16 plans initialised in full: D in f16 keys from the start (the
    // closure's keys_to_f16 pass is skipped: C3 -0.19 ms)
    const bool f16 = sizeof(K) == 2 && p->fw_f16 && !local;
    p->d_f16 = f16;
    hipLaunchKernelGGL(fill_kernel<K>, dim3(4096), dim3(256), 0, p->stream, D, p->Vp, r0, r1, f16);
    if (p->fw_unique_edges)
        hipLaunchKernelGGL((scatter_edges_kernel<K, true>), dim3(2048), dim3(256), 0, p->stream, D, p->Vp,
                           p->d_row_ptr, p->d_col, p->d_lat, u0, u1, p->kp, f16);
    else
        hipLaunchKernelGGL((scatter_edges_kernel<K, false>), dim3(2048), dim3(256), 0, p->stream, D, p->Vp,
                           p->d_row_ptr, p->d_col, p->d_lat, u0, u1, p->kp, f16);
}

// Measurement only (N-rank emulation): stands in for the pivot-row broadcast
// on the chain stream -- one wave waits `ticks` of the constant wall clock.
__global__ void delay_kernel(long long ticks) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

// the u16 kernels of a plan's key arithmetic (f16: fw_f16 plans)
template <int TAG, int SYM>
auto u16k(bool f16) {
    return f16 ? &minplus_u16_kernel<TAG, SYM, true> : &minplus_u16_kernel<TAG, SYM, false>;
}
template <int TAG, int MODE>
auto q16k(bool f16) {
    return f16 ? &minplus_q16_kernel<TAG, MODE, true> : &minplus_q16_kernel<TAG, MODE, false>;
}
template <int P1R>
auto p1k(bool f16) {
    return f16 ? &fw_phase1_u16pk_kernel<P1R, true> : &fw_phase1_u16pk_kernel<P1R, false>;
}
template <int P1R>
auto p1k2(bool f16) {
    return f16 ? &fw_phase1_pk2_kernel<P1R, true> : &fw_phase1_pk2_kernel<P1R, false>;
}

// two: u16 / f16 keys, two FW steps per barrier (fw_phase1_pk2_kernel)
template <typename K>
void launch_p1(int rows, hipStream_t s, K *D, uint32_t Vp, uint32_t kb, bool f16 = false, int mode = 0) {
    if constexpr (sizeof(K) == 2) {
        uint16_t *D16 = reinterpret_cast<uint16_t *>(D);
        if (mode == 1) {
            if (rows == 2)
                hipLaunchKernelGGL(p1k2<2>(f16), dim3(1), dim3(16 * (B / 2)), 0, s, D16, Vp, kb);
            else if (rows == 4)
                hipLaunchKernelGGL(p1k2<4>(f16), dim3(1), dim3(16 * (B / 4)), 0, s, D16, Vp, kb);
            else
                hipLaunchKernelGGL(p1k2<8>(f16), dim3(1), dim3(16 * (B / 8)), 0, s, D16, Vp, kb);
            return;
        }
        if (rows == 2)
            hipLaunchKernelGGL(p1k<2>(f16), dim3(1), dim3(16 * (B / 2)), 0, s, D16, Vp, kb);
        else if (rows == 4)
            hipLaunchKernelGGL(p1k<4>(f16), dim3(1), dim3(16 * (B / 4)), 0, s, D16, Vp, kb);
        else
            hipLaunchKernelGGL(p1k<8>(f16), dim3(1), dim3(16 * (B / 8)), 0, s, D16, Vp, kb);
        return;
    }
    if (rows == 2)
        hipLaunchKernelGGL((fw_phase1_kernel<K, 2>), dim3(1), dim3(16 * (B / 2)), 0, s, D, Vp, kb);
    else if (rows == 4)
        hipLaunchKernelGGL((fw_phase1_kernel<K, 4>), dim3(1), dim3(16 * (B / 4)), 0, s, D, Vp, kb);
    else
        hipLaunchKernelGGL((fw_phase1_kernel<K, 8>), dim3(1), dim3(16 * (B / 8)), 0, s, D, Vp, kb);
}

template <typename K, int TAG>
void launch_tiles(srt_plan *p, hipStream_t s, uint32_t kb, const Rect &r1, const Rect &r2) {
    const uint32_t n = r1.r.n * r1.c.n + r2.r.n * r2.c.n;
    if (!n) return;
    if (TAG != 0 && p->fw_small_chain) {  // look-ahead chain: quarter tiles, lower latency
        if constexpr (sizeof(K) == 2)
            hipLaunchKernelGGL((q16k<TAG, 0>(p->fw_f16)), dim3(4 * n), dim3(256), 0, s,
                               reinterpret_cast<uint16_t *>(p->d_D), p->Vp, kb, r1, r2, 1u,
                               PackSpec{nullptr, 0u, 0u, 1u, 1u});
        else
            hipLaunchKernelGGL((minplus_small_kernel<K, TAG>), dim3(4 * n), dim3(256), 0, s,
                               reinterpret_cast<K *>(p->d_D), p->Vp, kb, r1, r2);
    } else if (p->fw_glds) {
        if constexpr (sizeof(K) == 2)
            hipLaunchKernelGGL((u16k<TAG, 0>(p->fw_f16)), dim3(n), dim3(NT3), 0, s,
                               reinterpret_cast<uint16_t *>(p->d_D), p->Vp, kb, r1, r2, 1u);
        else if constexpr (sizeof(K) == 4)
            hipLaunchKernelGGL((minplus_u32_kernel<TAG>), dim3(n), dim3(NT3), 0, s,
                               reinterpret_cast<uint32_t *>(p->d_D), p->Vp, kb, r1, r2, 1u);
        else
            hipLaunchKernelGGL((minplus_glds_kernel<K, TAG>), dim3(n), dim3(NT3), 0, s,
                               reinterpret_cast<K *>(p->d_D), p->Vp, kb, r1, r2, 1u);
    }
    else
        hipLaunchKernelGGL((minplus_tile_kernel<K, TAG>), dim3(n), dim3(NT3), 0, s,
                           reinterpret_cast<K *>(p->d_D), p->Vp, kb, r1, r2);
}

// A single round's rest over a square span, as its triangle (u16 keys)
template <typename K>
void launch_rest_sym(srt_plan *p, hipStream_t s, uint32_t kb, const Rect &r1) {
    if constexpr (sizeof(K) == 2)
        hipLaunchKernelGGL((u16k<0, 1>(p->fw_f16)), dim3(sym_grid(r1.r.n, p->fw_band_h)), dim3(NT3), 0, s,
                           reinterpret_cast<uint16_t *>(p->d_D), p->Vp, kb, r1,
                           Rect{make_span(0, 0), make_span(0, 0)},
                           1u | band_bits(p->fw_band_h) | (p->fw_xcd ? 1u << 24 : 0u));
}

// One rect of chain tiles that also stores each off-diagonal result
// transposed (symmetric D, u16 keys): the mirror of a phase-2 row tile is the
// phase-2 column tile, so p2col needs no launch; in a cross rect the
// corner's tiles appear with their mirrors, both writing the same bits.
template <typename K, int TAG>
void launch_mirror(srt_plan *p, hipStream_t s, uint32_t kb, const Rect &r1) {
    const uint32_t n = r1.r.n * r1.c.n;
    if (!n) return;
    if constexpr (sizeof(K) == 2)
        hipLaunchKernelGGL((u16k<TAG, 2>(p->fw_f16)), dim3(n), dim3(NT3), 0, s,
                           reinterpret_cast<uint16_t *>(p->d_D), p->Vp, kb, r1,
                           Rect{make_span(0, 0), make_span(0, 0)}, 1u);
}

// Round schedule with one block of look-ahead, per rank (block-rows [rb0,rb1)):
//   main stream M:  (wait pivot kb) rest(kb) | (wait pivot kb+1) rest(kb+1) | ...
//   side stream S:  (after rest(kb-1))  cross(kb), p1(kb+1), p2row(kb+1) on
//                   the owner of kb+1, the pivot-row broadcast of kb+1
//                   (multi-GPU), then p2col(kb+1) for the local rows
// cross(kb) = the round-kb phase-3 tiles that round kb+1's pivot work needs
// (column kb+1 of the local rows; row kb+1 on its owner), rest(kb) = all other
// phase-3 tiles.  The two sets are disjoint and both read only pivot kb's row
// and column, so the whole S chain of pivot kb+1 overlaps rest(kb): M runs
// phase-3 kernels back to back and the round period is max(rest, chain).
// (Measured before, with cross(kb) on M: 10 us gaps either side of it and a
// half-empty GPU during it, 3.4% of the 16k build on one GPU.)  Single GPU =
// one rank, no broadcast.
template <typename K>
srt_status fw_rounds_group_t(srt_plan *p, int p1r, uint32_t g);

template <typename K>
srt_status fw_rounds_group_sharded_t(srt_plan *p, int p1r, uint32_t g, uint32_t rb0, uint32_t rb1, bool emu,
                                     long long emu_bcast_ticks, srt_err *err);

// Symmetric D on N ranks (u16 keys): the triangle's tiles (i, j), i <= j,
// are dealt to ranks by (i + j) mod N -- every block-row then has
// ceil(nblk / N) or fewer tiles on each rank, and every rank ~1/N of the
// triangle.  Each rank keeps a full D; its own tiles are current, the rest
// only where a round needs them.  Per round kb (k1 = kb + 1):
//   M: rest(kb) over the own list, minus rows/cols kb and k1 (operands: row kb
//      and its mirror, column kb, both complete on every rank);
//   S: cross(kb) = own tiles in row/col k1, round kb; pack them into this
//      rank's slot as row-k1 tiles; C: all-gather the slots (ceil(nblk/N)
//      tiles a rank); S: unpack row k1 from all slots, p1(k1) and p2row(k1)
//      with its mirror (column k1) -- the same bits on every rank.
// After the last round the own tiles are all-gathered and written with their
// mirrors, so every rank holds the whole closure (the sharded loss tail then
// reads its own rows).  Half the relaxations of the row-sharded schedule,
// one all-gather of ceil(nblk/N) tiles a round instead of a broadcast of
// nblk.  The prologue needs no exchange: every rank starts from the same
// full initial D.
// Groups of g rounds (fw_rounds_sym_grouped; g = 1: fw_rounds_sym_sharded):
// tl_cross_off[a] .. [a + 1] = the own tiles with a row or column in group a,
// d_rowslots = N slots of g * ceil(nblk / N) tiles.
srt_status sym_sharded_setup(srt_plan *p, uint32_t N, uint32_t r, uint32_t g, srt_err *err) {
    if (p->d_tl_all && p->sym_g == g) return SRT_OK;
    if (p->d_tl_all) {  // another group size: rebuild
        hipFree(p->d_tl_all);
        hipFree(p->d_tl_cnt);
        hipFree(p->d_tl_cross);
        hipFree(p->d_rowslots);
        hipFree(p->d_fbuf);
        p->d_tl_all = p->d_tl_cnt = p->d_tl_cross = nullptr;
        p->d_rowslots = p->d_fbuf = nullptr;
    }
    p->sym_g = g;
    const uint32_t nblk = p->Vp / B, ngrp = (nblk + g - 1) / g;
    std::vector<std::vector<uint32_t>> lists(N);
    for (uint32_t i = 0; i < nblk; ++i)
        for (uint32_t j = i; j < nblk; ++j) lists[(i + j) % N].push_back((i << 16) | j);
    uint32_t tmax = 0;
    for (auto &l : lists) tmax = std::max<uint32_t>(tmax, (uint32_t)l.size());
    std::vector<uint32_t> all((size_t)N * tmax, 0), cnt(N);
    for (uint32_t q = 0; q < N; ++q) {
        cnt[q] = (uint32_t)lists[q].size();
        std::copy(lists[q].begin(), lists[q].end(), all.begin() + (size_t)q * tmax);
    }
    std::vector<uint32_t> cross;
    p->tl_cross_off.assign(ngrp + 1, 0);
    for (uint32_t a = 0; a < ngrp; ++a) {
        p->tl_cross_off[a] = (uint32_t)cross.size();
        for (uint32_t e : lists[r])
            if ((e >> 16) / g == a || (e & 0xffffu) / g == a) cross.push_back(e);
    }
    p->tl_cross_off[ngrp] = (uint32_t)cross.size();
    p->tl_max = tmax;
    p->tl_own = cnt[r];
    const uint32_t S = (nblk + N - 1) / N;
    hipError_t e = hipMalloc(&p->d_tl_all, all.size() * 4);
    if (e == hipSuccess) e = hipMalloc(&p->d_tl_cnt, N * 4);
    if (e == hipSuccess) e = hipMalloc(&p->d_tl_cross, std::max<size_t>(cross.size(), 1) * 4);
    if (e == hipSuccess) e = hipMalloc(&p->d_rowslots, (size_t)N * g * S * B * B * 2);
    // the final exchange; also the emulation's scratch rows (g block-rows)
    if (e == hipSuccess) e = hipMalloc(&p->d_fbuf, std::max<size_t>((size_t)N * tmax, (size_t)g * nblk) * B * B * 2);
    if (e == hipSuccess) e = hipMemcpy(p->d_tl_all, all.data(), all.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_tl_cnt, cnt.data(), N * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess && !cross.empty())
        e = hipMemcpy(p->d_tl_cross, cross.data(), cross.size() * 4, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (err) {
            err->code = SRT_ERR_HIP;
            std::snprintf(err->msg, sizeof err->msg, "symmetric sharded setup: %s", hipGetErrorString(e));
        }
        return SRT_ERR_HIP;
    }
    return SRT_OK;
}

// the fused row unpack + (two-step) phase 1 kernel at p1r rows a thread
struct UnpackP1 {
    void (*fn)(uint16_t *, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, const uint16_t *, uint16_t *, bool, bool);
    uint32_t threads;
};
UnpackP1 unpack_p1_for(int p1r, bool f16) {
    if (p1r == 2) return {f16 ? &unpack_p1_kernel<2, true> : &unpack_p1_kernel<2, false>, 16u * (B / 2)};
    if (p1r == 4) return {f16 ? &unpack_p1_kernel<4, true> : &unpack_p1_kernel<4, false>, 16u * (B / 4)};
    return {f16 ? &unpack_p1_kernel<8, true> : &unpack_p1_kernel<8, false>, 16u * (B / 8)};
}

// a list launch of the SYM == 3 rest kernel: n entries at tl, ng rounds from
// kb, skipping tiles in a row or column of [a, b)
void launch_list16(hipStream_t s, uint16_t *D, uint32_t Vp, uint32_t kb, const uint32_t *tl, uint32_t n, uint32_t a,
                   uint32_t b, bool f16, uint32_t ng = 1) {
    if (!n) return;
    Span skip{0, 0, a, b, 0};
    const uint64_t addr = reinterpret_cast<uint64_t>(tl);
    Span ptr{(uint32_t)addr, (uint32_t)(addr >> 32), NONE, NONE, 0};
    hipLaunchKernelGGL((u16k<0, 3>(f16)), dim3(n), dim3(NT3), 0, s, D, Vp, kb, Rect{skip, skip},
                       Rect{ptr, ptr}, ng);
}

// Emulation (measurement only, SRT_FW_EMULATE_RANKS=N, one GPU, D already
// closed): rank 0's schedule, each all-gather a wait of SRT_FW_EMU_AG_US +
// received bytes / SRT_FW_EMU_AG_GBPS (as the loss tail's); the row unpack
// goes to scratch (the other ranks' slots hold no real rows) and the final
// unpack writes rank 0's tiles N times (every rank's volume), so D stays the
// closure for the loss tail that follows.
// the all-gather of the symmetric sharded schedules: RCCL in place, or the
// emulation's stand-in wait (latency + bytes / bandwidth, see below)
struct SymGather {
    srt_plan *p;
    srt_err *err;
    bool emu;
    uint32_t N;
    long long ag_lat = 0;
    double ag_per_byte = 0.0;
    SymGather(srt_plan *p_, uint32_t N_, srt_err *e) : p(p_), err(e), emu(p_->comm == nullptr), N(N_) {
        if (!emu) return;
        int khz = 100000;
        (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, p->device);
        const double lat_us = std::getenv("SRT_FW_EMU_AG_US") ? std::atof(std::getenv("SRT_FW_EMU_AG_US")) : 25.0;
        const double gbps = std::getenv("SRT_FW_EMU_AG_GBPS") ? std::atof(std::getenv("SRT_FW_EMU_AG_GBPS")) : 300.0;
        ag_lat = (long long)(lat_us * khz / 1000.0);
        ag_per_byte = (double)(N - 1) / (gbps * 1e3) * khz / 1000.0;  // ticks per byte a rank sends
    }
    srt_status operator()(void *buf, size_t bytes_per_rank, hipStream_t s) const {
        if (!emu) return comm_allgather_inplace(p->comm, buf, bytes_per_rank, s, err);
        hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, s, ag_lat + (long long)(bytes_per_rank * ag_per_byte));
        return SRT_OK;
    }
};

// the final exchange of the symmetric sharded schedules: every rank's tiles,
// written with their mirrors (after M's last rest)
srt_status sym_final_exchange(srt_plan *p, uint32_t N, uint32_t r, const SymGather &gather) {
    uint16_t *D = reinterpret_cast<uint16_t *>(p->d_D);
    hipStream_t M = p->stream, C = p->comm_stream;
    const uint32_t *own = p->d_tl_all + (size_t)r * p->tl_max;
    if (p->tl_own)
        hipLaunchKernelGGL(pack_list16_kernel, dim3(p->tl_own), dim3(256), 0, M, D, p->Vp, own,
                           p->d_fbuf + (size_t)r * p->tl_max * B * B);
    hipEventRecord(p->ev_row, M);
    hipStreamWaitEvent(C, p->ev_row, 0);
    if (srt_status st = gather(p->d_fbuf, (size_t)p->tl_max * B * B * 2, C); st != SRT_OK) return st;
    hipEventRecord(p->ev_bcast, C);
    hipStreamWaitEvent(M, p->ev_bcast, 0);
    hipLaunchKernelGGL(unpack_list16_kernel, dim3(p->tl_max, N), dim3(256), 0, M, D, p->Vp,
                       (const uint32_t *)p->d_tl_all, (const uint32_t *)p->d_tl_cnt, p->tl_max,
                       (const uint16_t *)p->d_fbuf, gather.emu ? 1u : 0u);
    return SRT_OK;
}

srt_status fw_rounds_sym_grouped(srt_plan *p, int p1r, uint32_t g, srt_err *err);

srt_status fw_rounds_sym_sharded(srt_plan *p, int p1r, srt_err *err) {
    const bool emu = p->comm == nullptr;
    const uint32_t N = emu ? p->emulate_ranks : (uint32_t)p->comm->nranks, r = emu ? 0u : (uint32_t)p->comm->rank;
    const uint32_t nblk = p->Vp / B;
    {
        uint32_t g = p->fw_sym_group;
        if (const char *e = std::getenv("SRT_FW_SYM_GROUP")) g = (uint32_t)std::max(1, std::atoi(e));
        g = std::min<uint32_t>(g, std::max<uint32_t>(1, nblk / 2));
        if (g > 1 && (p1r == 2 || p1r == 4 || p1r == 8)) return fw_rounds_sym_grouped(p, p1r, g, err);
    }
    if (srt_status st = sym_sharded_setup(p, N, r, 1u, err); st != SRT_OK) return st;
    uint16_t *D = reinterpret_cast<uint16_t *>(p->d_D);
    const uint32_t S_t = (nblk + N - 1) / N;
    const SymGather gather(p, N, err);
    hipStream_t M = p->stream, S = p->side_stream;
    const uint32_t *own = p->d_tl_all + (size_t)r * p->tl_max;
    uint16_t *myslot = p->d_rowslots + (size_t)r * S_t * B * B;
    p->p3_launches = 0;
    p->p3_work = 0.0;
    p->p3_tiles = 0;
    while (p->ev.size() < 2 * (size_t)nblk + 2) {
        hipEvent_t e;
        hipEventCreateWithFlags(&e, (unsigned)hipEventDisableSystemFence);
        p->ev.push_back(e);
    }
    srt_status st = SRT_OK;
    // the chain as packed quarter tiles (minplus_q16_kernel) when a rank's
    // rest is short (< 4096 own tiles: from 4 ranks on at 16k) -- it is then
    // the round's critical path; knob SRT_FW_SYM_SMALL=0/1 for A/B
    bool small = p->tl_own < 4096;
    if (const char *e = std::getenv("SRT_FW_SYM_SMALL")) small = std::atoi(e) != 0;
    // the quarter-tile cross also packs row k1 into the slot ...
    const bool fuse_pack = true;
    // ... and the unpack of row k1 runs beside p1(k1) in one launch (two-step
    // phase 1)
    const bool fuse_p1 = p->fw_p1 >= 1;
    auto p2row_mirror = [&](hipStream_t s, uint32_t k) {
        const Rect row{make_span(k, k + 1), make_span(0, nblk, k)};
        if (small)
            hipLaunchKernelGGL((q16k<1, 1>(p->fw_f16)), dim3(4 * row.c.n), dim3(256), 0, s, D, p->Vp, k, row,
                               Rect{make_span(0, 0), make_span(0, 0)}, 1u, PackSpec{nullptr, 0u, 0u, 1u, 1u});
        else
            launch_mirror<uint16_t, 1>(p, s, k, row);
    };
    // prologue: pivot 0 on every rank (the same full initial D)
    launch_p1<uint16_t>(p1r, M, D, p->Vp, 0u, p->fw_f16, p->fw_p1);
    p2row_mirror(M, 0);
    hipEventRecord(p->ev_cross, M);
    hipEvent_t rest_done = p->ev_cross;
    for (uint32_t kb = 0; kb < nblk; ++kb) {
        const bool nxt = kb + 1 < nblk;
        const uint32_t k1 = kb + 1;
        if (nxt) hipStreamWaitEvent(S, rest_done, 0);
        if (kb) hipStreamWaitEvent(M, p->ev_pivot, 0);
        hipEventRecord(p->ev[2 * p->p3_launches], M);
        launch_list16(M, D, p->Vp, kb, own, p->tl_own, kb, nxt ? k1 + 1 : k1, p->fw_f16);
        rest_done = p->ev[2 * p->p3_launches + 1];
        hipEventRecord(rest_done, M);
        p->p3_launches++;
        p->p3_work += (double)p->tl_own * B * B * B;  // minus the few skipped row/col tiles
        p->p3_tiles += p->tl_own;
        if (!nxt) break;
        const uint32_t *cl = p->d_tl_cross + p->tl_cross_off[k1];
        const uint32_t cn = p->tl_cross_off[k1 + 1] - p->tl_cross_off[k1];
        if (small && cn) {
            Span skip{0, 0, kb, kb + 1, 0};
            const uint64_t addr = reinterpret_cast<uint64_t>(cl);
            Span ptr{(uint32_t)addr, (uint32_t)(addr >> 32), NONE, NONE, 0};
            // cross(kb) and the pack of row k1 into this rank's slot, one launch
            hipLaunchKernelGGL((q16k<4, 2>(p->fw_f16)), dim3(4 * cn), dim3(256), 0, S, D, p->Vp, kb,
                               Rect{skip, skip}, Rect{ptr, ptr}, 1u,
                               PackSpec{fuse_pack ? myslot : (uint16_t *)nullptr, k1, 1u, N, S_t});
            if (!fuse_pack)
                hipLaunchKernelGGL(pack_row16_kernel, dim3(cn), dim3(256), 0, S, D, p->Vp, cl, k1, N, myslot);
        } else {
            launch_list16(S, D, p->Vp, kb, cl, cn, kb, kb + 1, p->fw_f16);
            if (cn) hipLaunchKernelGGL(pack_row16_kernel, dim3(cn), dim3(256), 0, S, D, p->Vp, cl, k1, N, myslot);
        }
        // the row all-gather on S itself: nothing else waits on S meanwhile,
        // and two cross-stream event hops (~13 us each) fewer per round
        if ((st = gather(p->d_rowslots, (size_t)S_t * B * B * 2, S)) != SRT_OK) return st;
        // emulation: the other slots hold no real rows, so the unpack (same
        // volume) goes to scratch and the closed D stays as it is
        uint16_t *rowdst = emu ? p->d_fbuf : D + (uint64_t)k1 * B * p->Vp;
        if (fuse_p1 && (p1r == 2 || p1r == 4 || p1r == 8)) {
            // unpack of row k1 and p1(k1) from its slot, one launch
            const UnpackP1 u = unpack_p1_for(p1r, p->fw_f16);
            hipLaunchKernelGGL(u.fn, dim3(nblk + 1), dim3(u.threads), 0, S, D, p->Vp, k1, 1u, N, S_t,
                               (const uint16_t *)p->d_rowslots, rowdst, emu, true);
        } else {
            hipLaunchKernelGGL(unpack_row16_kernel, dim3(nblk), dim3(256), 0, S, rowdst, p->Vp, k1, N, S_t,
                               (const uint16_t *)p->d_rowslots);
            launch_p1<uint16_t>(p1r, S, D, p->Vp, k1, p->fw_f16, p->fw_p1);
        }
        p2row_mirror(S, k1);
        hipEventRecord(p->ev_pivot, S);
    }
    return sym_final_exchange(p, N, r, gather);
}

// The symmetric sharded schedule in groups of g rounds: one row all-gather
// per group instead of per round.  Group a = blocks [a g, a g + g) (the last
// one shorter); A = group a, Bn = group a + 1.  Invariant at group a: the
// panel of A (its block-rows and, mirrored, block-columns) is closed through
// A's last round on every rank; own tiles elsewhere are current through the
// rounds before A.  Per group:
//   M: rest(A) = own tiles outside the rows / columns of A and Bn, the |A|
//      rounds of A in one pass (they read only A's closed panel);
//   S: cross(A) = own tiles in a row or column of Bn (outside A's), the |A|
//      rounds of A, each result of rows Bn also packed into this rank's slot
//      (g ceil(nblk / N) tiles); the all-gather; the unpack of rows Bn and
//      p1(Bn.lo) in one launch; then Bn's panel closed round by round on every
//      rank: p1(q), p2row(q) with its mirror, and round q on the other rows
//      of Bn (mirrored).
// rest(A) and the chain of Bn touch disjoint tiles, as in the one-round
// schedule; S waits for rest(A - 1) (the rows of Bn took A - 1's rounds there)
// and M for Bn's panel.  Relaxations as the one-round schedule, g times fewer
// all-gathers, p1 / p2row / cross launches, and stream hops.
srt_status fw_rounds_sym_grouped(srt_plan *p, int p1r, uint32_t g, srt_err *err) {
    const bool emu = p->comm == nullptr;
    const uint32_t N = emu ? p->emulate_ranks : (uint32_t)p->comm->nranks, r = emu ? 0u : (uint32_t)p->comm->rank;
    if (srt_status st = sym_sharded_setup(p, N, r, g, err); st != SRT_OK) return st;
    uint16_t *D = reinterpret_cast<uint16_t *>(p->d_D);
    const uint32_t nblk = p->Vp / B, ngrp = (nblk + g - 1) / g;
    const uint32_t S_t = (nblk + N - 1) / N;
    const SymGather gather(p, N, err);
    hipStream_t M = p->stream, S = p->side_stream;
    const uint32_t *own = p->d_tl_all + (size_t)r * p->tl_max;
    p->p3_launches = 0;
    p->p3_work = 0.0;
    p->p3_tiles = 0;
    while (p->ev.size() < 2 * (size_t)ngrp + 2) {
        hipEvent_t e;
        hipEventCreateWithFlags(&e, (unsigned)hipEventDisableSystemFence);
        p->ev.push_back(e);
    }
    const bool f16 = p->fw_f16;
    const Rect none{make_span(0, 0), make_span(0, 0)};
    const PackSpec nopack{nullptr, 0u, 0u, 1u, 1u};
    auto lo = [&](uint32_t a) { return a * g; };
    auto hi = [&](uint32_t a) { return std::min(nblk, a * g + g); };
    // Bn's panel after rows Bn arrived: round q on row q (mirrored), then on
    // the other rows of Bn (mirrored; column q is p2row's mirror, row q and
    // column q are the operands); p1(q) before each but the first when first
    // is set (the unpack closed it)
    auto close_panel = [&](hipStream_t s, uint32_t a, bool first_done) {
        const uint32_t b0 = lo(a), b1 = hi(a);
        for (uint32_t q = b0; q < b1; ++q) {
            if (q > b0 || !first_done) launch_p1<uint16_t>(p1r, s, D, p->Vp, q, f16, p->fw_p1);
            const Rect row{make_span(q, q + 1), make_span(0, nblk, q)};
            hipLaunchKernelGGL((q16k<1, 1>(f16)), dim3(4 * row.c.n), dim3(256), 0, s, D, p->Vp, q, row, none, 1u,
                               nopack);
            if (b1 - b0 > 1) {
                const Rect pan{make_span(b0, b1, q), make_span(0, nblk, q)};
                hipLaunchKernelGGL((q16k<1, 1>(f16)), dim3(4 * pan.r.n * pan.c.n), dim3(256), 0, s, D, p->Vp, q,
                                   pan, none, 1u, nopack);
            }
        }
    };
    // prologue: group 0's panel on every rank (the same full initial D)
    close_panel(M, 0, false);
    hipEventRecord(p->ev_cross, M);
    hipEvent_t rest_done = p->ev_cross;
    srt_status st = SRT_OK;
    for (uint32_t a = 0; a < ngrp; ++a) {
        const bool nxt = a + 1 < ngrp;
        const uint32_t A0 = lo(a), A1 = hi(a), na = A1 - A0;
        if (nxt) hipStreamWaitEvent(S, rest_done, 0);
        if (a) hipStreamWaitEvent(M, p->ev_pivot, 0);
        hipEventRecord(p->ev[2 * p->p3_launches], M);
        launch_list16(M, D, p->Vp, A0, own, p->tl_own, A0, nxt ? hi(a + 1) : A1, f16, na);
        rest_done = p->ev[2 * p->p3_launches + 1];
        hipEventRecord(rest_done, M);
        p->p3_launches++;
        p->p3_work += (double)p->tl_own * B * B * B * na;  // minus the skipped row/col tiles
        p->p3_tiles += p->tl_own;
        if (!nxt) break;
        const uint32_t B0 = lo(a + 1), nb = hi(a + 1) - B0;
        const uint32_t *cl = p->d_tl_cross + p->tl_cross_off[a + 1];
        const uint32_t cn = p->tl_cross_off[a + 2] - p->tl_cross_off[a + 1];
        uint16_t *myslot = p->d_rowslots + (size_t)r * nb * S_t * B * B;
        if (cn) {
            Span skip{0, 0, A0, A1, 0};
            const uint64_t addr = reinterpret_cast<uint64_t>(cl);
            Span ptr{(uint32_t)addr, (uint32_t)(addr >> 32), NONE, NONE, 0};
            // cross(A) and the pack of rows Bn into this rank's slot, one launch
            hipLaunchKernelGGL((q16k<4, 2>(f16)), dim3(4 * cn), dim3(256), 0, S, D, p->Vp, A0, Rect{skip, skip},
                               Rect{ptr, ptr}, na, PackSpec{myslot, B0, nb, N, S_t});
        }
        if ((st = gather(p->d_rowslots, (size_t)nb * S_t * B * B * 2, S)) != SRT_OK) return st;
        // emulation: the other slots hold no real rows, so the unpack (same
        // volume) goes to scratch and the closed D stays as it is
        uint16_t *rowdst = emu ? p->d_fbuf : D + (uint64_t)B0 * B * p->Vp;
        const bool p1 = p->fw_p1 >= 1;  // the fused p1 is the two-step body
        const UnpackP1 u = unpack_p1_for(p1r, f16);
        hipLaunchKernelGGL(u.fn, dim3(1 + nb * nblk), dim3(u.threads), 0, S, D, p->Vp, B0, nb, N, S_t,
                           (const uint16_t *)p->d_rowslots, rowdst, emu, p1);
        close_panel(S, a + 1, p1);
        hipEventRecord(p->ev_pivot, S);
    }
    return sym_final_exchange(p, N, r, gather);
}

template <typename K>
srt_status fw_rounds_t(srt_plan *p, srt_err *err) {
    K *D = reinterpret_cast<K *>(p->d_D);
    const uint32_t nblk = p->Vp / B;
    // measurement-only emulation of one rank of an N-rank run on one GPU
    // (SRT_FW_EMULATE_RANKS): local rows = 1/N of the block-rows, and this
    // rank plays the owner of every pivot (p1 + p2row each round: the longest
    // per-round chain any rank has), no collectives -- the table is not valid
    // (after the first run, which closes D for real: see srt_plan_run_async)
    const uint32_t emu = (!p->comm && p->emulate_ranks > 1 && p->emu_closed) ? p->emulate_ranks : 0;
    const uint32_t rb0 = p->rb0, rb1 = emu ? std::max<uint32_t>(1, nblk / emu) : p->rb1;
    const bool sharded = p->comm != nullptr;  // a 1-rank comm runs the same schedule (tested)
    // quarter-tile chain kernels whenever a round's rest() is short (sharded
    // ranks; one GPU below ~8 tile-waves of rest, e.g. 4k nodes: 8.4 -> 7.0 ms),
    // where the chain, not rest, would set the round period; knobs force it
    // on / off for A/B timing
    const uint64_t rest_tiles = (uint64_t)(rb1 - rb0) * nblk;
    p->fw_small_chain = std::getenv("SRT_FW_SMALL_CHAIN") != nullptr ||
                        ((sharded || emu || rest_tiles < 8ull * 512) && !std::getenv("SRT_FW_NO_SMALL_CHAIN"));
    const uint32_t per_rank = sharded ? nblk / p->comm->nranks : nblk;
    const size_t pivot_bytes = (size_t)B * p->Vp * sizeof(K);
    hipStream_t M = p->stream, S = p->side_stream, C = p->comm_stream;
    auto own = [&](uint32_t b) { return emu ? true : (b >= rb0 && b < rb1); };
    const Rect none{make_span(0, 0), make_span(0, 0)};
    p->p3_launches = 0;
    p->p3_work = 0.0;
    // phase-3 launches bracketed by timing events (kernel_stats), every round
    const uint32_t ev_every = 1;
    const size_t need = 2 * (size_t)nblk + 2;
    while (p->ev.size() < need) {
        hipEvent_t e;
        // timing-only events: no system-scope fence
        hipEventCreateWithFlags(&e, (unsigned)hipEventDisableSystemFence);
        p->ev.push_back(e);
    }
    // phase-1 rows per thread (knob SRT_FW_P1_ROWS in {2,4,8}, measurement only)
    // (u16 keys: the packed kernel at 4 rows a thread, 512 threads -- emulated
    // 8 ranks 29.4 -> 28.3 ms, where phase 1 is on the round's critical path;
    // one GPU unchanged)
    int p1r = sizeof(K) == 2 ? 4 : 8;
    if (const char *e = std::getenv("SRT_FW_P1_ROWS")) p1r = std::atoi(e);
    // emulation only: SRT_FW_EMU_BCAST_US stands in for the pivot-row broadcast latency
    long long emu_bcast_ticks = 0;
    if (const char *e = std::getenv("SRT_FW_EMU_BCAST_US"); e && emu) {
        int khz = 100000;
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, p->device);
        emu_bcast_ticks = (long long)(std::atof(e) * khz / 1000.0);
    }
    // one GPU, rest-bound (no quarter-tile chain): rounds in groups of g = 4
    // from 96 blocks (12k nodes) on, 2 below or when the block count is not a
    // multiple of 4 (measured, same box: 8k 39.0 / 37.2 / 37.6 ms for g = 1 /
    // 2 / 4; 12k 122.8 / 118.2 / 117.2; 16k 285.4 / 274.9 / 270.7; knob
    // SRT_FW_GROUP=1/2/4 for A/B timing, SRT_FW_PAIR forces grouping at
    // chain-bound sizes too: parity tests)
    uint32_t grp = (nblk % 4 == 0 && nblk >= 96) ? 4 : 2;
    if (nblk < 96 && std::getenv("SRT_FW_PAIR") && nblk % 4 == 0 && nblk >= 8) grp = 4;
    if (const char *e = std::getenv("SRT_FW_GROUP")) grp = (uint32_t)std::atoi(e);
    if (std::getenv("SRT_FW_NO_PAIR")) grp = 1;
    if (!sharded && !emu && p->fw_glds && (!p->fw_small_chain || std::getenv("SRT_FW_PAIR")) && grp > 1 &&
        grp <= 8 && nblk % grp == 0 && nblk >= 2 * grp)
        return fw_rounds_group_t<K>(p, p1r, grp);
    // symmetric D on several ranks: the triangle dealt by (i + j) mod N
    if constexpr (sizeof(K) == 2)
        if ((sharded || emu) && p->fw_sym && p->fw_glds) {
            p->fw_full_d = true;  // the final tile exchange leaves the whole closure on every rank
            return fw_rounds_sym_sharded(p, p1r, err);
        }
    // sharded: groups of 2 when a rank holds >= 32 block-rows (rest-bound)
    // that split into whole groups (one owner per group) and there are >= 2
    // groups.  Emulated C3 (16k, u16 keys), g = 1 / 2 / 4: 2 ranks 82.7 / 80.6
    // / 82.6 ms, 4 ranks 47.8 / 45.7 / 50.2, 8 ranks 33.4 / 35.8 / 39.8 -- at 16
    // block-rows a rank the chain (X(b) + g x (p1, p2row, p2col, cross))
    // outlasts F(a) (knob SRT_FW_SHARD_GROUP=0 / 2 / 4 for A/B timing)
    {
        const uint32_t per_local = emu ? std::max<uint32_t>(1, nblk / emu) : per_rank;
        uint32_t sg = per_local >= 32 ? 2 : 0;
        if (const char *e = std::getenv("SRT_FW_SHARD_GROUP")) sg = (uint32_t)std::atoi(e);
        if ((sharded || emu) && p->fw_glds && sg > 1 && sg <= 8 && per_local % sg == 0 && nblk % sg == 0 &&
            nblk >= 2 * sg)
            return fw_rounds_group_sharded_t<K>(p, p1r, sg, rb0, rb1, emu != 0, emu_bcast_ticks, err);
    }
    p->p3_tiles = 0;
    srt_status st = SRT_OK;
    // prologue: pivot 0
    if (own(0)) {
        launch_p1<K>(p1r, M, D, p->Vp, 0u, p->fw_f16, p->fw_p1);
        launch_tiles<K, 1>(p, M, 0, Rect{make_span(0, 1), make_span(0, nblk, 0)}, none);
    }
    if (sharded && (st = comm_bcast(p->comm, D, pivot_bytes, 0, M, err)) != SRT_OK) return st;
    launch_tiles<K, 2>(p, M, 0, Rect{make_span(rb0, rb1, 0), make_span(0, 1)}, none);

    // S may start round 0's cross tiles once the prologue is done; C's
    // broadcasts follow the prologue's
    hipEventRecord(p->ev_cross, M);
    hipStreamWaitEvent(C, p->ev_cross, 0);
    hipEvent_t rest_done = p->ev_cross;  // the latest point S's next cross tiles wait for
    for (uint32_t kb = 0; kb < nblk; ++kb) {
        const bool nxt = kb + 1 < nblk;
        const uint32_t k1 = kb + 1;
        // host order matters: ev_cross / ev_pivot are re-recorded every round,
        // and a wait binds to the record enqueued before it
        if (nxt) hipStreamWaitEvent(S, rest_done, 0);  // rest(kb-1) (or the prologue) done
        if (kb) hipStreamWaitEvent(M, p->ev_pivot, 0);  // pivot kb ready (round 0: stream order)
        // rest(kb): local rows and all columns, minus kb and (look-ahead) k1
        Rect rest{make_span(rb0, rb1, kb, nxt ? k1 : NONE), make_span(0, nblk, kb, nxt ? k1 : NONE)};
        const uint32_t nt = rest.r.n * rest.c.n;
        // symmetric D on one GPU: the rest runs its triangle (see minplus_u16_kernel)
        const bool tri = p->fw_sym && sizeof(K) == 2 && !sharded && !emu && p->fw_glds;
        if (nt && kb % ev_every == 0) {
            hipEventRecord(p->ev[2 * p->p3_launches], M);
            if (tri) launch_rest_sym<K>(p, M, kb, rest);
            else launch_tiles<K, 0>(p, M, kb, rest, none);
            // the timing event after rest(kb) doubles as S's hand-off (one
            // event packet fewer per round on the main stream)
            rest_done = p->ev[2 * p->p3_launches + 1];
            hipEventRecord(rest_done, M);
            p->p3_launches++;
            const double run = tri ? (double)rest.r.n * (rest.r.n + 1) / 2 : (double)nt;  // tiles run
            p->p3_work += run * B * B * B;
            p->p3_tiles += (uint64_t)run;
        } else {
            if (nt && tri) launch_rest_sym<K>(p, M, kb, rest);
            else if (nt) launch_tiles<K, 0>(p, M, kb, rest, none);
            if (nxt) {
                hipEventRecord(p->ev_cross, M);
                rest_done = p->ev_cross;
            }
        }
        if (nxt) {
            // for round k1's cross tiles on S: rest_done (waited at the top of
            // the next iteration)
            // cross(kb) on S, concurrent with rest(kb) (disjoint tiles; both
            // read only the pivot-kb row and column): column k1 of the local
            // rows (+ row k1 on its owner)
            Rect col{make_span(rb0, rb1, kb, k1), make_span(k1, k1 + 1)};
            Rect row = own(k1) ? Rect{make_span(k1, k1 + 1), make_span(0, nblk, kb)} : none;
            launch_tiles<K, 4>(p, S, kb, col, row);
            if (own(k1)) {
                launch_p1<K>(p1r, S, D, p->Vp, k1, p->fw_f16, p->fw_p1);
                launch_tiles<K, 1>(p, S, k1, Rect{make_span(k1, k1 + 1), make_span(0, nblk, k1)}, none);
            }
            // pivot-row broadcast on the comm stream C: the owner's chain goes
            // on without it (it holds row k1; its next cross/p1/p2row are
            // local), so the transfer overlaps the owner's next pivot and only
            // the other ranks' p2col(k1) -> rest(k1) wait for it.  Reading
            // row k1 while the owner's later rounds lower it is harmless: every
            // key is a real path's key, so receivers only see valid upper
            // bounds at least as tight as round k1's (the FW invariant holds).
            if (sharded || emu_bcast_ticks) {
                if (own(k1)) {
                    hipEventRecord(p->ev_row, S);
                    hipStreamWaitEvent(C, p->ev_row, 0);
                }
                if (sharded &&
                    (st = comm_bcast(p->comm, D + (uint64_t)k1 * B * p->Vp, pivot_bytes, (int)(k1 / per_rank), C,
                                     err)) != SRT_OK)
                    return st;
                if (emu_bcast_ticks) hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, C, emu_bcast_ticks);
                if (!own(k1)) {
                    hipEventRecord(p->ev_bcast, C);
                    hipStreamWaitEvent(S, p->ev_bcast, 0);
                }
            }
            // p2col(k1): column k1 of the local rows through P*(k1); rest(kb)
            // never touches column k1, so this also overlaps rest(kb)
            launch_tiles<K, 2>(p, S, k1, Rect{make_span(rb0, rb1, k1), make_span(k1, k1 + 1)}, none);
            hipEventRecord(p->ev_pivot, S);
        }
    }
    // collectives on one communicator stay ordered: the loss pass's
    // exchanges (srt_loss.hip) follow the last broadcast.  The closure rows
    // stay sharded: the loss pass of a rank only reads its own rows, and
    // fw_gather_keys is its fallback.
    hipEventRecord(p->ev_bcast, C);
    hipStreamWaitEvent(M, p->ev_bcast, 0);
    return SRT_OK;
}

// One GPU, rest-bound sizes: rounds are fused in groups of g (2 or 4) rounds
// a .. a+g-1 (a a multiple of g), so each rest tile is loaded and stored once
// per g rounds (the per-tile prologue/epilogue both workgroups of a CU wait out
// together is ~9% of a single-round launch) and there are 1/g as many rest
// launches, launch gaps and launch tails.
//   chain (pivots of the group) = for r = a .. a+g-1: p1(r), p2row(r),
//       p2col(r), then round r on rows/cols r+1 .. a+g-1 (in-group cross)
//   F(a) on M = rounds a .. a+g-1 on every tile outside rows/cols of the next
//       group (a tile whose highest in-group row/column is q runs rounds > q)
//   X(a+g) on S = the same rounds on rows/cols a+g .. a+2g-1 (overlaps F(a)),
//       then the chain of the next group.
// Operands of round r > a are final chain output; round r's column D(i, r)
// may be lowered by a later round of the same launch while other tiles read
// it -- a tighter key of a real path, so the FW invariant holds and the
// closure is the same bits (the argument of the look-ahead chain and the
// broadcast).  Tiles that two rectangles of one launch both cover (the g x g
// corners) are updated twice with the same inputs: min is idempotent.
template <typename K>
void launch_group(srt_plan *p, hipStream_t s, uint32_t a, uint32_t g, const Rect &r1, const Rect &r2, bool chain) {
    const uint32_t n = r1.r.n * r1.c.n + r2.r.n * r2.c.n;
    if (!n) return;
    K *D = reinterpret_cast<K *>(p->d_D);
    // bit 16: banded tile order (plan knob SRT_FW_BAND=0 turns it off for A/B timing)
    // bit 24: XCD remap of the triangle order (measured no faster; plan field fw_xcd off)
    const uint32_t arg = g | (p->fw_band ? 0x10000u : 0u) | band_bits(p->fw_band_h) |
                         (p->fw_xcd ? 1u << 24 : 0u) |
                         (chain ? 0u : 1u << 26);
    if constexpr (sizeof(K) == 2) {
        if (chain && p->fw_sym)  // r1 only; its transposes are r2 (fw_rounds_group_t)
            hipLaunchKernelGGL((u16k<5, 2>(p->fw_f16)), dim3(r1.r.n * r1.c.n), dim3(NT3), 0, s, D, p->Vp, a, r1,
                               Rect{make_span(0, 0), make_span(0, 0)}, arg);
        else if (chain)
            hipLaunchKernelGGL((u16k<5, 0>(p->fw_f16)), dim3(n), dim3(NT3), 0, s, D, p->Vp, a, r1, r2, arg);
        else if (p->fw_sym)  // square span, r2 empty (fw_rounds_group_t)
            hipLaunchKernelGGL((u16k<0, 1>(p->fw_f16)), dim3(sym_grid(r1.r.n, p->fw_band_h)), dim3(NT3), 0, s, D,
                               p->Vp, a, r1, r2, arg);
        else
            hipLaunchKernelGGL((u16k<0, 0>(p->fw_f16)), dim3(n), dim3(NT3), 0, s, D, p->Vp, a, r1, r2, arg);
    } else if constexpr (sizeof(K) == 4) {
        if (chain)
            hipLaunchKernelGGL((minplus_u32_kernel<5>), dim3(n), dim3(NT3), 0, s, D, p->Vp, a, r1, r2, arg);
        else
            hipLaunchKernelGGL((minplus_u32_kernel<0>), dim3(n), dim3(NT3), 0, s, D, p->Vp, a, r1, r2, arg);
    } else {
        if (chain)
            hipLaunchKernelGGL((minplus_glds_kernel<K, 5>), dim3(n), dim3(NT3), 0, s, D, p->Vp, a, r1, r2, arg);
        else
            hipLaunchKernelGGL((minplus_glds_kernel<K, 0>), dim3(n), dim3(NT3), 0, s, D, p->Vp, a, r1, r2, arg);
    }
}

void group_work_sym(const Span &r, uint32_t a, uint32_t g, double &work, double &tiles);

template <typename K>
srt_status fw_rounds_group_t(srt_plan *p, int p1r, uint32_t g) {
    K *D = reinterpret_cast<K *>(p->d_D);
    const uint32_t nblk = p->Vp / B;
    hipStream_t M = p->stream, S = p->side_stream;
    const Rect none{make_span(0, 0), make_span(0, 0)};
    // the pivots of group a on stream s (rows/cols a .. a+g-1 already hold rounds < a)
    // symmetric D (u16 keys, see fw_sym_check): p2row also stores p2col's
    // tiles transposed, and the cross runs one rect and stores the other
    const bool symc = p->fw_sym && sizeof(K) == 2 && !p->fw_small_chain;
    auto pivots = [&](hipStream_t s, uint32_t a) {
        for (uint32_t r = a; r < a + g; ++r) {
            launch_p1<K>(p1r, s, D, p->Vp, r, p->fw_f16, p->fw_p1);
            if (symc) {
                launch_mirror<K, 1>(p, s, r, Rect{make_span(r, r + 1), make_span(0, nblk, r)});
                if (r + 1 < a + g)
                    launch_mirror<K, 4>(p, s, r, Rect{make_span(0, nblk, r), make_range(r + 1, a + g, NONE, NONE)});
                continue;
            }
            launch_tiles<K, 1>(p, s, r, Rect{make_span(r, r + 1), make_span(0, nblk, r)}, none);
            launch_tiles<K, 2>(p, s, r, Rect{make_span(0, nblk, r), make_span(r, r + 1)}, none);
            if (r + 1 < a + g)  // round r on rows/cols r+1 .. a+g-1 (the corner twice: idempotent)
                launch_tiles<K, 4>(p, s, r, Rect{make_span(0, nblk, r), make_range(r + 1, a + g, NONE, NONE)},
                                   Rect{make_range(r + 1, a + g, NONE, NONE), make_span(0, nblk, r)});
        }
    };
    p->p3_launches = 0;
    p->p3_work = 0.0;
    p->p3_tiles = 0;
    const size_t need = 2 * (nblk / g) + 2;
    while (p->ev.size() < need) {
        hipEvent_t e;
        hipEventCreateWithFlags(&e, (unsigned)hipEventDisableSystemFence);
        p->ev.push_back(e);
    }
    pivots(M, 0);
    hipEventRecord(p->ev_cross, M);
    hipEvent_t rest_done = p->ev_cross;
    for (uint32_t a = 0; a < nblk; a += g) {
        const bool nxt = a + g < nblk;
        const uint32_t c0 = nxt ? a + g : NONE, c1 = a + 2 * g;
        if (nxt) hipStreamWaitEvent(S, rest_done, 0);  // F(a-g) (or the prologue) done
        if (a) hipStreamWaitEvent(M, p->ev_pivot, 0);  // the group's pivots ready
        const Rect all{make_range(0, nblk, c0, c1), make_range(0, nblk, c0, c1)};
        hipEventRecord(p->ev[2 * p->p3_launches], M);
        launch_group<K>(p, M, a, g, all, none, false);
        rest_done = p->ev[2 * p->p3_launches + 1];
        hipEventRecord(rest_done, M);
        p->p3_launches++;
        // tiles (i, j) of the launch: with t = number of in-group indices
        // above max(i,j)'s group position, rounds = g for out-of-group tiles
        const double m = all.r.n, o = m - g;  // o: rows outside the group
        double work = o * o * g, tiles = o * o;
        for (uint32_t q = 0; q + 1 < g; ++q) {
            // tiles whose highest in-group index is q: (q+1)^2 - q^2 inside, 2 * o * 1 mixed
            const double cnt = (2.0 * q + 1) + 2.0 * o;
            work += cnt * (g - 1 - q);
            tiles += cnt;
        }
        if (p->fw_sym && sizeof(K) == 2) {
            // the triangle actually run: pi <= pj (a tile computed once, stored twice)
            work = tiles = 0.0;
            group_work_sym(all.r, a, g, work, tiles);
        }
        p->p3_work += work * B * B * B;
        p->p3_tiles += (uint64_t)tiles;
        if (nxt) {
            // X(a+g): rows/cols a+g .. a+2g-1 through the group's rounds
            const Span nx = make_range(a + g, a + 2 * g, NONE, NONE);
            launch_group<K>(p, S, a, g, Rect{make_span(0, nblk), nx}, Rect{nx, make_span(0, nblk)}, true);
            pivots(S, a + g);
            hipEventRecord(p->ev_pivot, S);
        }
    }
    return SRT_OK;
}

// group_work over the symmetric launch's tiles pi <= pj of the square span r
void group_work_sym(const Span &r, uint32_t a, uint32_t g, double &work, double &tiles) {
    for (uint32_t i = 0; i < r.n; ++i) {
        const uint32_t bi = span_at(r, i);
        for (uint32_t j = i; j < r.n; ++j) {
            const uint32_t bj = span_at(r, j);
            const bool ii = bi - a < g, jj = bj - a < g;
            uint32_t rounds = g;
            if (ii || jj) rounds = g - 1 - std::max(ii ? bi - a : 0u, jj ? bj - a : 0u);
            if (rounds) {
                work += rounds;
                tiles += 1;
            }
        }
    }
}

// Tiles and relaxations of a grouped launch over rows x cols for the group
// a .. a+g-1: a tile whose highest in-group row/column position is q runs
// rounds q+1 .. (g - 1 - q of them), others all g.
void group_work(const Span &r, const Span &c, uint32_t a, uint32_t g, double &work, double &tiles) {
    for (uint32_t i = 0; i < r.n; ++i) {
        const uint32_t bi = span_at(r, i);
        for (uint32_t j = 0; j < c.n; ++j) {
            const uint32_t bj = span_at(c, j);
            const bool ii = bi - a < g, jj = bj - a < g;
            uint32_t rounds = g;
            if (ii || jj) rounds = g - 1 - std::max(ii ? bi - a : 0u, jj ? bj - a : 0u);
            if (rounds) {
                work += rounds;
                tiles += 1;
            }
        }
    }
}

// Sharded build (or its one-GPU emulation), rounds in groups of g; g divides
// every rank's block-row count, so the pivot rows of a group have one owner.
// Per group a (b = a + g the next, G(x) = block-rows/cols x .. x+g-1):
//   M: F(a) = rounds G(a) on the local rows x all columns, minus columns G(b)
//      and (on b's owner) rows G(b) -- the grouped rule of fw_rounds_group_t
//      for tiles in G(a)
//   S: X(b) = rounds G(a) on the local rows x columns G(b), and on b's owner
//      rows G(b) x all columns; then chain(b): per r in G(b), on the owner
//      p1(r), p2row(r), then the broadcast of block-row r on C (pipelined:
//      row r is final for the chain once p2row(r) ran), p2col(r) on the local
//      rows, round r on rows r+1.. of G(b) x all columns and on the local rows
//      x columns r+1.. of G(b); on the other ranks, per r: row r received,
//      p2col(r), round r on the local rows x columns r+1.. of G(b).
// One broadcast per pivot block-row as before, 1/g as many rest launches,
// each tile loaded and stored once per g rounds.  Operands read while a
// concurrent launch lowers them are real paths' keys at least as tight as
// the round's (the FW invariant of the look-ahead chain), so the closure is
// the same bits.  Emulation (measurement only): this rank owns every group
// and also waits out each row's modelled broadcast (SRT_FW_EMU_BCAST_US) as a
// receiver would -- the longest chain any rank has.
template <typename K>
srt_status fw_rounds_group_sharded_t(srt_plan *p, int p1r, uint32_t g, uint32_t rb0, uint32_t rb1, bool emu,
                                     long long emu_bcast_ticks, srt_err *err) {
    K *D = reinterpret_cast<K *>(p->d_D);
    const uint32_t nblk = p->Vp / B;
    const bool sharded = p->comm != nullptr;
    const uint32_t per_rank = sharded ? nblk / p->comm->nranks : nblk;
    const size_t pivot_bytes = (size_t)B * p->Vp * sizeof(K);
    hipStream_t M = p->stream, S = p->side_stream, C = p->comm_stream;
    const Rect none{make_span(0, 0), make_span(0, 0)};
    auto own = [&](uint32_t blk) { return emu || (blk >= rb0 && blk < rb1); };
    p->p3_launches = 0;
    p->p3_work = 0.0;
    p->p3_tiles = 0;
    const size_t need = 2 * (nblk / g) + 2;
    while (p->ev.size() < need) {
        hipEvent_t e;
        hipEventCreateWithFlags(&e, (unsigned)hipEventDisableSystemFence);
        p->ev.push_back(e);
    }
    auto chain = [&](hipStream_t s, uint32_t a) -> srt_status {
        const bool o = own(a);
        for (uint32_t r = a; r < a + g; ++r) {
            if (o) {
                launch_p1<K>(p1r, s, D, p->Vp, r, p->fw_f16, p->fw_p1);
                launch_tiles<K, 1>(p, s, r, Rect{make_span(r, r + 1), make_span(0, nblk, r)}, none);
            }
            if (sharded || emu_bcast_ticks) {
                if (o) {
                    hipEventRecord(p->ev_row, s);
                    hipStreamWaitEvent(C, p->ev_row, 0);
                }
                if (sharded) {
                    const srt_status st =
                        comm_bcast(p->comm, D + (uint64_t)r * B * p->Vp, pivot_bytes, (int)(r / per_rank), C, err);
                    if (st != SRT_OK) return st;
                }
                if (emu_bcast_ticks) hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, C, emu_bcast_ticks);
                if (!o || emu_bcast_ticks) {
                    hipEventRecord(p->ev_bcast, C);
                    hipStreamWaitEvent(s, p->ev_bcast, 0);
                }
            }
            launch_tiles<K, 2>(p, s, r, Rect{make_span(rb0, rb1, r), make_span(r, r + 1)}, none);
            if (r + 1 < a + g)
                launch_tiles<K, 4>(p, s, r, Rect{make_span(rb0, rb1, r), make_range(r + 1, a + g, NONE, NONE)},
                                   o ? Rect{make_range(r + 1, a + g, NONE, NONE), make_span(0, nblk, r)} : none);
        }
        return SRT_OK;
    };
    // S starts after fw_init on M; chain(0)
    hipEventRecord(p->ev_cross, M);
    hipStreamWaitEvent(S, p->ev_cross, 0);
    srt_status st = chain(S, 0);
    if (st != SRT_OK) return st;
    hipEventRecord(p->ev_pivot, S);
    hipEvent_t rest_done = p->ev_cross;
    for (uint32_t a = 0; a < nblk; a += g) {
        const bool nxt = a + g < nblk;
        const uint32_t b = a + g, c0 = nxt ? b : NONE, c1 = b + g;
        if (nxt) hipStreamWaitEvent(S, rest_done, 0);  // F(a-g) done
        hipStreamWaitEvent(M, p->ev_pivot, 0);         // chain(a) done
        // rows of the next group this rank's S stream runs (X(b) rows): G(b)
        // on its owner; in the emulation a local group stands in for it, so
        // the emulated rank carries exactly an owner's load
        const uint32_t lg = emu ? rb0 + ((b / g) % ((rb1 - rb0) / g)) * g : b;
        const bool xr = nxt && own(b);
        const Rect f{make_range(rb0, rb1, xr ? lg : NONE, lg + g), make_range(0, nblk, c0, c1)};
        hipEventRecord(p->ev[2 * p->p3_launches], M);
        launch_group<K>(p, M, a, g, f, none, false);
        rest_done = p->ev[2 * p->p3_launches + 1];
        hipEventRecord(rest_done, M);
        p->p3_launches++;
        double work = 0.0, tiles = 0.0;
        group_work(f.r, f.c, a, g, work, tiles);
        p->p3_work += work * B * B * B;
        p->p3_tiles += (uint64_t)tiles;
        if (nxt) {
            const Span nx = make_range(b, b + g, NONE, NONE);
            launch_group<K>(p, S, a, g, Rect{make_span(rb0, rb1), nx},
                            xr ? Rect{make_range(lg, lg + g, NONE, NONE), make_range(0, nblk, b, b + g)} : none, true);
            if ((st = chain(S, b)) != SRT_OK) return st;
            hipEventRecord(p->ev_pivot, S);
        }
    }
    hipEventRecord(p->ev_bcast, C);
    hipStreamWaitEvent(M, p->ev_bcast, 0);
    return SRT_OK;
}

// ------------------------------------------------ key-width proof (eccentricity)
// Bellman-Ford sweeps from one source s over the CSR, both directions at
// once: dout[v] = d(s, v) by pushes along u -> v (atomic min), din[u] =
// d(u, s) by the row's own pull over its out-edges (min over k of lat[k] +
// din[col[k]]; only u's wave writes din[u]).  Values only decrease and every
// value is a real walk's latency, so racing readers stay correct; the sweeps
// repeat until one changes nothing.  Sums saturate instead of wrapping.
__global__ __launch_bounds__(256) void ecc_sweep_kernel(const uint64_t *__restrict__ row_ptr,
                                                        const uint32_t *__restrict__ col,
                                                        const uint64_t *__restrict__ lat, uint32_t V,
                                                        unsigned long long *dout, unsigned long long *din,
                                                        uint32_t *changed) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    bool ch = false;
    for (uint32_t u = wave; u < V; u += nwaves) {
        const uint64_t du = __atomic_load_n(&dout[u], __ATOMIC_RELAXED);
        uint64_t best = ~0ull;
        for (uint64_t k = row_ptr[u] + lane; k < row_ptr[u + 1]; k += 64) {
            const uint32_t v = col[k];
            const uint64_t w = lat[k];
            if (du != ~0ull && du + w >= du) {
                const uint64_t nd = du + w;
                if (nd < __atomic_load_n(&dout[v], __ATOMIC_RELAXED)) {
                    atomicMin(&dout[v], (unsigned long long)nd);
                    ch = true;
                }
            }
            const uint64_t dv = __atomic_load_n(&din[v], __ATOMIC_RELAXED);
            if (dv != ~0ull && dv + w >= dv && dv + w < best) best = dv + w;
        }
        for (int off = 32; off > 0; off >>= 1) {
            const uint64_t o = __shfl_xor(best, off);
            best = o < best ? o : best;
        }
        if (lane == 0 && best < __atomic_load_n(&din[u], __ATOMIC_RELAXED)) {
            __atomic_store_n(&din[u], (unsigned long long)best, __ATOMIC_RELAXED);
            ch = true;
        }
    }
    if (__builtin_amdgcn_ballot_w64(ch) && lane == 0) *changed = 1;  // every writer stores 1
}

// out[0] = max dout, out[1] = max din (~0 if any node is unreached)
__global__ __launch_bounds__(256) void ecc_max_kernel(const unsigned long long *__restrict__ dout,
                                                      const unsigned long long *__restrict__ din, uint32_t V,
                                                      unsigned long long *out) {
    uint64_t a = 0, b = 0;
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < V; v += gridDim.x * blockDim.x) {
        a = dout[v] > a ? dout[v] : a;
        b = din[v] > b ? din[v] : b;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t x = __shfl_xor(a, off), y = __shfl_xor(b, off);
        a = x > a ? x : a;
        b = y > b ? y : b;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&out[0], (unsigned long long)a);
        atomicMax(&out[1], (unsigned long long)b);
    }
}

}  // namespace

// Once per plan, after the first init (one GPU, u16 keys, knob SRT_FW_SYM=0
// off): is the initial D symmetric?  FW keeps a symmetric D symmetric, so
// every later round may then run the triangle (minplus_u16_kernel<0, true>).
srt_status fw_sym_check(srt_plan *p, srt_err *err) {
    p->fw_sym_known = true;
    p->fw_sym = false;
    if (p->key_type != KEY_U16) return SRT_OK;
    if (const char *e = std::getenv("SRT_FW_SYM"); e && std::atoi(e) == 0) return SRT_OK;
    const uint32_t nb = p->Vp / 64;
    uint32_t one = 1, h = 0;
    hipError_t e = hipMemcpyAsync(p->d_flag32, &one, 4, hipMemcpyHostToDevice, p->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(sym_check_kernel<uint16_t>, dim3(nb, nb), dim3(256), 0, p->stream,
                           reinterpret_cast<const uint16_t *>(p->d_D), p->Vp, nb, p->d_flag32);
        e = hipMemcpyAsync(&h, p->d_flag32, 4, hipMemcpyDeviceToHost, p->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
    if (e != hipSuccess) {
        if (err) {
            err->code = SRT_ERR_HIP;
            std::snprintf(err->msg, sizeof err->msg, "symmetry check: %s", hipGetErrorString(e));
        }
        return SRT_ERR_HIP;
    }
    p->fw_sym = h != 0;
    if (p->fw_sym) p->desc += " sym=triangle";
    return SRT_OK;
}

// Key-width proof from the graph's real diameter: for a node
// s that reaches every node and is reached by every node, any pair has
// d(u, v) <= d(u, s) + d(s, v) <= max_u d(u, s) + max_v d(s, v).  Runs the
// sweeps above from s = 0 on the uploaded CSR (p->stream, synchronous);
// *bound_ns = ~0 when s misses a node either way or the sweeps do not settle
// within max_sweeps (the caller keeps its (V - 1) * max edge bound).
srt_status fw_ecc_bound(srt_plan *p, uint32_t max_sweeps, uint64_t *bound_ns, uint32_t *sweeps, srt_err *err) {
    *bound_ns = ~0ull;
    *sweeps = 0;
    const uint32_t V = p->V;
    if (!V) return SRT_OK;
    unsigned long long *buf = nullptr;  // dout[V], din[V], out[2], flag
    hipError_t e = hipMalloc(&buf, ((size_t)2 * V + 3) * 8);
    unsigned long long *dout = buf, *din = buf + V, *out = buf + 2 * (size_t)V;
    uint32_t *flag = reinterpret_cast<uint32_t *>(buf + 2 * (size_t)V + 2);
    const unsigned long long zero = 0;
    if (e == hipSuccess) e = hipMemsetAsync(buf, 0xff, (size_t)2 * V * 8, p->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dout, &zero, 8, hipMemcpyHostToDevice, p->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(din, &zero, 8, hipMemcpyHostToDevice, p->stream);
    if (e == hipSuccess) e = hipMemsetAsync(out, 0, 16, p->stream);
    const uint32_t blocks = std::min<uint32_t>(4096, (V + 3) / 4);
    bool settled = false;
    for (uint32_t it = 0; e == hipSuccess && it < max_sweeps; ++it) {
        uint32_t h = 0;
        e = hipMemsetAsync(flag, 0, 4, p->stream);
        if (e != hipSuccess) break;
        cspan_begin(p);
        hipLaunchKernelGGL(ecc_sweep_kernel, dim3(blocks), dim3(256), 0, p->stream, p->d_row_ptr, p->d_col, p->d_lat,
                           V, dout, din, flag);
        cspan_end(p);
        e = hipMemcpyAsync(&h, flag, 4, hipMemcpyDeviceToHost, p->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
        *sweeps = it + 1;
        if (e == hipSuccess && !h) {
            settled = true;
            break;
        }
    }
    unsigned long long m[2] = {~0ull, ~0ull};
    if (e == hipSuccess && settled) {
        cspan_begin(p);
        hipLaunchKernelGGL(ecc_max_kernel, dim3(std::min<uint32_t>(1024, (V + 255) / 256)), dim3(256), 0, p->stream,
                           dout, din, V, out);
        cspan_end(p);
        e = hipMemcpyAsync(m, out, 16, hipMemcpyDeviceToHost, p->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
    }
    hipFree(buf);
    if (e != hipSuccess) {
        if (err) {
            err->code = SRT_ERR_HIP;
            std::snprintf(err->msg, sizeof err->msg, "eccentricity sweeps: %s", hipGetErrorString(e));
        }
        return SRT_ERR_HIP;
    }
    if (settled && m[0] != ~0ull && m[1] != ~0ull && m[0] + m[1] >= m[0]) *bound_ns = m[0] + m[1];
    return SRT_OK;
}

void fw_init(srt_plan *p) {
    if (p->key_type == KEY_U16) fw_init_t<uint16_t>(p);
    else if (p->key_type == KEY_U32) fw_init_t<uint32_t>(p);
    else if (p->key_type == KEY_F64) fw_init_t<double>(p);
    else fw_init_t<uint64_t>(p);
}

srt_status fw_gather_keys(srt_plan *p, srt_err *err) {
    const uint32_t per_rank = (p->Vp / FW_B) / p->comm->nranks;
    return comm_allgather_inplace(p->comm, p->d_D, (size_t)per_rank * FW_B * p->Vp * key_bytes(p->key_type),
                                  p->stream, err);
}

srt_status fw_rounds(srt_plan *p, srt_err *err) {
    p->fw_full_d = false;
    if (p->key_type == KEY_U16) {
        // f16 plans: D to f16 keys and back around the closure, on the main
        // stream (every schedule's last kernel runs there, or joins it)
        const uint64_t n8 = (uint64_t)p->Vp * p->Vp / 8;
        uint16_t *D = reinterpret_cast<uint16_t *>(p->d_D);
        if (p->fw_f16 && !p->d_f16) hipLaunchKernelGGL(keys_to_f16_kernel, dim3(4096), dim3(256), 0, p->stream, D, n8);
        const srt_status st = fw_rounds_t<uint16_t>(p, err);
        if (p->fw_f16) hipLaunchKernelGGL(keys_from_f16_kernel, dim3(4096), dim3(256), 0, p->stream, D, n8);
        p->d_f16 = false;
        return st;
    }
    if (p->key_type == KEY_U32) return fw_rounds_t<uint32_t>(p, err);
    return p->key_type == KEY_F64 ? fw_rounds_t<double>(p, err) : fw_rounds_t<uint64_t>(p, err);
}

void pack_paths8(srt_plan *p, uint64_t first, uint64_t count, void *dst, hipStream_t s) {
    hipLaunchKernelGGL(pack8_kernel, dim3(4096), dim3(256), 0, s, p->d_out_lat + first, p->d_out_loss + first,
                       reinterpret_cast<uint2 *>(dst), count, p->kp.g);
}

void widen_u32(uint64_t *dst, const uint32_t *src, uint64_t count, hipStream_t s) {
    hipLaunchKernelGGL(widen_u32_kernel, dim3(2048), dim3(256), 0, s, dst, src, count);
}

void loss_check(const float *d_loss, uint64_t count, uint64_t k0, unsigned long long *d_first, hipStream_t s) {
    if (count)
        hipLaunchKernelGGL(loss_check_kernel, dim3(2048), dim3(256), 0, s, reinterpret_cast<const uint32_t *>(d_loss),
                           count, k0, d_first);
}

void iota_rows(uint32_t *dst, uint64_t count, uint32_t V, hipStream_t s) {
    hipLaunchKernelGGL(iota_rows_kernel, dim3(2048), dim3(256), 0, s, dst, count, V);
}

void pack_paths6(srt_plan *p, uint64_t first, uint64_t count, void *dst, uint64_t loss_off, hipStream_t s) {
    hipLaunchKernelGGL(pack6_kernel, dim3(4096), dim3(256), 0, s, p->d_out_lat + first, p->d_out_loss + first,
                       reinterpret_cast<uint8_t *>(dst), count, p->kp.g, loss_off);
}

void pack_paths5(srt_plan *p, uint64_t first, uint64_t count, void *dst, uint64_t loss_off, hipStream_t s) {
    hipLaunchKernelGGL(pack5_kernel, dim3(4096), dim3(256), 0, s, p->d_out_lat + first, p->d_out_loss + first,
                       reinterpret_cast<uint8_t *>(dst), count, p->kp.g, loss_off);
}

void pack_paths(srt_plan *p, uint64_t first, uint64_t count, srt_path *dst, hipStream_t s) {
    hipLaunchKernelGGL(pack_kernel, dim3(4096), dim3(256), 0, s, p->d_out_lat + first, p->d_out_loss + first, dst,
                       count);
}

// srt_init: loads this unit's code object (srt::preload_kernels)
hipError_t preload_fw() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&fill_kernel<uint16_t>));
}

hipError_t preload_loss();
hipError_t preload_sssp();
hipError_t preload_packet();
hipError_t preload_direct();
hipError_t preload_events();
hipError_t preload_kernels() {
    hipError_t e = preload_fw();
    if (e == hipSuccess) e = preload_loss();
    if (e == hipSuccess) e = preload_sssp();
    if (e == hipSuccess) e = preload_packet();
    if (e == hipSuccess) e = preload_direct();
    if (e == hipSuccess) e = preload_events();
    return e;
}

}  // namespace srt
