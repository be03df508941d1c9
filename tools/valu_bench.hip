// valu_bench.hip -- measured VALU issue rates on gfx950 for the instructions a
// min-plus relaxation can be built from (to pick the path-key representation
// and to state the roofline peak from measurement, not from a datasheet).
//
//   hipcc -O3 --offload-arch=gfx950 tools/valu_bench.hip -o tools/valu_bench && ./tools/valu_bench
//
// Each kernel runs 8 independent chains of one instruction kind in inline asm,
// ITER iterations, on a full grid (2048 x 256 threads); reported as wave64
// instructions per CU per cycle-equivalent and as lane-ops/s.
#include <hip/hip_runtime.h>

#include <cstdio>

#define ITER 4096


#define V32(i) unsigned a##i = seed + i + threadIdx.x;
#define DECL32 V32(0) V32(1) V32(2) V32(3) V32(4) V32(5) V32(6) V32(7) unsigned b = seed * 3u;
#define SINK32 unsigned sink = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7

#define ASM8(op)                                                        \
    asm volatile(op " %0, %0, %1" : "+v"(a0) : "v"(b));                \
    asm volatile(op " %0, %0, %1" : "+v"(a1) : "v"(b));                \
    asm volatile(op " %0, %0, %1" : "+v"(a2) : "v"(b));                \
    asm volatile(op " %0, %0, %1" : "+v"(a3) : "v"(b));                \
    asm volatile(op " %0, %0, %1" : "+v"(a4) : "v"(b));                \
    asm volatile(op " %0, %0, %1" : "+v"(a5) : "v"(b));                \
    asm volatile(op " %0, %0, %1" : "+v"(a6) : "v"(b));                \
    asm volatile(op " %0, %0, %1" : "+v"(a7) : "v"(b));


// plain 32-bit ops
#define K32(kname, op)                                                           \
    __global__ __launch_bounds__(256) void kname(unsigned *out, unsigned seed) { \
        DECL32;                                                                  \
        for (int it = 0; it < ITER; ++it) { ASM8(op) }                           \
        SINK32;                                                                  \
        if (seed == 12345u) out[threadIdx.x] = sink;                             \
    }
K32(k_add_u32, "v_add_u32")
K32(k_min_u32, "v_min_u32")
K32(k_pk_add_u16, "v_pk_add_u16")
K32(k_pk_min_u16, "v_pk_min_u16")

#define ASM8_3(op)                                                              \
    asm volatile(op " %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(a7));           \
    asm volatile(op " %0, %0, %1, %2" : "+v"(a1) : "v"(b), "v"(a0));           \
    asm volatile(op " %0, %0, %1, %2" : "+v"(a2) : "v"(b), "v"(a1));           \
    asm volatile(op " %0, %0, %1, %2" : "+v"(a3) : "v"(b), "v"(a2));           \
    asm volatile(op " %0, %0, %1, %2" : "+v"(a4) : "v"(b), "v"(a3));           \
    asm volatile(op " %0, %0, %1, %2" : "+v"(a5) : "v"(b), "v"(a4));           \
    asm volatile(op " %0, %0, %1, %2" : "+v"(a6) : "v"(b), "v"(a5));           \
    asm volatile(op " %0, %0, %1, %2" : "+v"(a7) : "v"(b), "v"(a6));
#define K32_3(kname, op)                                                         \
    __global__ __launch_bounds__(256) void kname(unsigned *out, unsigned seed) { \
        DECL32;                                                                  \
        for (int it = 0; it < ITER; ++it) { ASM8_3(op) }                         \
        SINK32;                                                                  \
        if (seed == 12345u) out[threadIdx.x] = sink;                             \
    }
K32_3(k_min3_u32, "v_min3_u32")

// 64-bit ops
#define V64(i) unsigned long long a##i = (unsigned long long)(seed + i + threadIdx.x) << 20;
#define DECL64 V64(0) V64(1) V64(2) V64(3) V64(4) V64(5) V64(6) V64(7) unsigned long long b = seed * 3ull;
#define SINK64 unsigned sink = (unsigned)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7)
#define ASM8_64(op)                                                             \
    asm volatile(op : "+v"(a0) : "v"(b));                                       \
    asm volatile(op : "+v"(a1) : "v"(b));                                       \
    asm volatile(op : "+v"(a2) : "v"(b));                                       \
    asm volatile(op : "+v"(a3) : "v"(b));                                       \
    asm volatile(op : "+v"(a4) : "v"(b));                                       \
    asm volatile(op : "+v"(a5) : "v"(b));                                       \
    asm volatile(op : "+v"(a6) : "v"(b));                                       \
    asm volatile(op : "+v"(a7) : "v"(b));
#define K64(kname, op)                                                           \
    __global__ __launch_bounds__(256) void kname(unsigned *out, unsigned seed) { \
        DECL64;                                                                  \
        for (int it = 0; it < ITER; ++it) { ASM8_64(op) }                        \
        SINK64;                                                                  \
        if (seed == 12345u) out[threadIdx.x] = sink;                             \
    }
K64(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 0, %1")
K64(k_add_f64, "v_add_f64 %0, %0, %1")
K64(k_min_f64, "v_min_f64 %0, %0, %1")

// the full packed-key relaxation as the compiler emits it: c = min(c, a + b)
__global__ __launch_bounds__(256) void k_relax_u64(unsigned *out, unsigned seed) {
    DECL64;
    unsigned long long c0 = ~0ull >> 2, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0, c7 = c0;
    for (int it = 0; it < ITER; ++it) {
#define R(i) { unsigned long long t = a##i + b; c##i = t < c##i ? t : c##i; asm volatile("" : "+v"(a##i), "+v"(c##i)); }
        R(0) R(1) R(2) R(3) R(4) R(5) R(6) R(7)
#undef R
    }
    unsigned sink = (unsigned)(c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7);
    if (seed == 12345u) out[threadIdx.x] = sink;
}

__global__ __launch_bounds__(256) void k_relax_u32sat(unsigned *out, unsigned seed) {
    DECL32;
    unsigned c0 = ~0u, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0, c7 = c0;
    for (int it = 0; it < ITER; ++it) {
#define R(i) { unsigned t = __builtin_elementwise_add_sat(a##i, b); c##i = t < c##i ? t : c##i; asm volatile("" : "+v"(a##i), "+v"(c##i)); }
        R(0) R(1) R(2) R(3) R(4) R(5) R(6) R(7)
#undef R
    }
    unsigned sink = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
    if (seed == 12345u) out[threadIdx.x] = sink;
}

// the u32 rest kernel's instruction mix (relax_quad32: 4 v_add_u32 + 2
// v_min3_u32 per 4 relaxations), 64 accumulators per lane like the kernel
__global__ __launch_bounds__(256) void k_mix_u32(unsigned *out, unsigned seed) {
    unsigned acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = ~0u >> 1;
    unsigned a0 = seed + threadIdx.x, a1 = a0 * 3u, b0 = seed * 5u, b1 = b0 + 1, b2 = b0 + 2, b3 = b0 + 3,
             b4 = b0 + 4, b5 = b0 + 5, b6 = b0 + 6, b7 = b0 + 7;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            unsigned t0, t1, t2, t3;
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
                : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "+v"(acc[4 * q]), "+v"(acc[4 * q + 1]),
                  "+v"(acc[4 * q + 2]), "+v"(acc[4 * q + 3])
                : "v"(a0), "v"(a1), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7));
        }
    }
    unsigned sink = 0;
    for (int i = 0; i < 16; ++i) sink ^= acc[i];
    if (seed == 12345u) out[threadIdx.x] = sink;
}

// packed u16 keys: acc pair (c, c+1) = pk_min(acc, sat(a_k + b_pair)), the A
// value broadcast to both halves with op_sel; 2 relaxations per instruction pair
__global__ __launch_bounds__(256) void k_mix_u16(unsigned *out, unsigned seed) {
    unsigned acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = 0x7fff7fffu;
    unsigned a0 = seed + threadIdx.x, b0 = seed * 5u, b1 = b0 + 1, b2 = b0 + 2, b3 = b0 + 3;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            unsigned t0, t1, t2, t3;
            asm volatile(
                "v_pk_add_u16 %0, %8, %9 op_sel_hi:[0,1] clamp\n\t"
                "v_pk_add_u16 %1, %8, %10 op_sel_hi:[0,1] clamp\n\t"
                "v_pk_add_u16 %2, %8, %11 op_sel:[1,0] op_sel_hi:[1,1] clamp\n\t"
                "v_pk_add_u16 %3, %8, %12 op_sel:[1,0] op_sel_hi:[1,1] clamp\n\t"
                "v_pk_min_u16 %4, %4, %0\n\t"
                "v_pk_min_u16 %5, %5, %1\n\t"
                "v_pk_min_u16 %6, %6, %2\n\t"
                "v_pk_min_u16 %7, %7, %3"
                : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "+v"(acc[4 * q]), "+v"(acc[4 * q + 1]),
                  "+v"(acc[4 * q + 2]), "+v"(acc[4 * q + 3])
                : "v"(a0), "v"(b0), "v"(b1), "v"(b2), "v"(b3));
        }
    }
    unsigned sink = 0;
    for (int i = 0; i < 16; ++i) sink ^= acc[i];
    if (seed == 12345u) out[threadIdx.x] = sink;
}

// f16 integer keys (exact below 2048): per row and k-pair, two packed adds
// (A[r][k] / A[r][k+1] broadcast by op_sel) and one v_pk_minimum3_f16 fold
// four candidates into a column pair: 3 instructions per 4 relaxations
K32(k_pk_add_f16, "v_pk_add_f16")
K32(k_pk_min_f16, "v_pk_min_f16")
K32_3(k_pk_minimum3_f16, "v_pk_minimum3_f16")
K32_3(k_minimum3_f32, "v_minimum3_f32")
K32_3(k_min3_f32, "v_min3_f32")
K64(k_pk_add_f32, "v_pk_add_f32 %0, %0, %1")
__global__ __launch_bounds__(256) void k_mix_f16(unsigned *out, unsigned seed) {
    unsigned acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = 0x64006400u;  // (1024, 1024)
    unsigned a0 = 0x3c003c00u + (threadIdx.x & 7), b0 = 0x40004000u + seed, b1 = b0 + 1, b2 = b0 + 2,
             b3 = b0 + 3, b4 = b0 + 4, b5 = b0 + 5, b6 = b0 + 6, b7 = b0 + 7;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            unsigned t0, t1, t2, t3;
            asm volatile(
                "v_pk_add_f16 %0, %8, %9 op_sel_hi:[0,1]\n\t"
                "v_pk_add_f16 %1, %8, %10 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
                "v_pk_add_f16 %2, %8, %11 op_sel_hi:[0,1]\n\t"
                "v_pk_add_f16 %3, %8, %12 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
                "v_pk_minimum3_f16 %4, %4, %0, %1\n\t"
                "v_pk_minimum3_f16 %5, %5, %2, %3\n\t"
                "v_pk_add_f16 %0, %8, %13 op_sel_hi:[0,1]\n\t"
                "v_pk_add_f16 %1, %8, %14 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
                "v_pk_add_f16 %2, %8, %15 op_sel_hi:[0,1]\n\t"
                "v_pk_add_f16 %3, %8, %16 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
                "v_pk_minimum3_f16 %6, %6, %0, %1\n\t"
                "v_pk_minimum3_f16 %7, %7, %2, %3"
                : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "+v"(acc[4 * q]), "+v"(acc[4 * q + 1]),
                  "+v"(acc[4 * q + 2]), "+v"(acc[4 * q + 3])
                : "v"(a0), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7));
        }
    }
    unsigned sink = 0;
    for (int i = 0; i < 16; ++i) sink ^= acc[i];
    if (seed == 12345u) out[threadIdx.x] = sink;
}

// f32 integer keys (exact below 2^24): v_pk_add_f32 forms two candidates (A
// broadcast), v_min3_f32 folds two into one accumulator: 2 instructions per 2
// relaxations if the packed add issues at full rate
__global__ __launch_bounds__(256) void k_mix_f32(unsigned *out, unsigned seed) {
    float acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = 1e9f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 a0 = {1.0f + (threadIdx.x & 7), 2.0f}, b0 = {(float)seed, 3.0f}, b1 = b0 + 1.0f, b2 = b0 + 2.0f,
       b3 = b0 + 3.0f;
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            f2 t0, t1, t2, t3;
            asm volatile(
                "v_pk_add_f32 %0, %4, %5 op_sel_hi:[0,1]\n\t"
                "v_pk_add_f32 %1, %4, %6 op_sel:[1,0] op_sel_hi:[1,1]\n\t"
                "v_pk_add_f32 %2, %4, %7 op_sel_hi:[0,1]\n\t"
                "v_pk_add_f32 %3, %4, %8 op_sel:[1,0] op_sel_hi:[1,1]"
                : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3)
                : "v"(a0), "v"(b0), "v"(b1), "v"(b2), "v"(b3));
            asm volatile(
                "v_min3_f32 %0, %0, %4, %5\n\t"
                "v_min3_f32 %1, %1, %6, %7\n\t"
                "v_min3_f32 %2, %2, %8, %9\n\t"
                "v_min3_f32 %3, %3, %10, %11"
                : "+v"(acc[4 * q]), "+v"(acc[4 * q + 1]), "+v"(acc[4 * q + 2]), "+v"(acc[4 * q + 3])
                : "v"(t0.x), "v"(t1.x), "v"(t0.y), "v"(t1.y), "v"(t2.x), "v"(t3.x), "v"(t2.y), "v"(t3.y));
        }
    }
    float sink = 0;
    for (int i = 0; i < 16; ++i) sink += acc[i];
    if (seed == 12345u) out[threadIdx.x] = __float_as_uint(sink);
}

typedef void (*kfn)(unsigned *, unsigned);

static void run(const char *name, kfn k, int instr_per_iter, unsigned *d, int grid = 2048) {
    const int block = 256;
    hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, d, 1u);  // warm
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, d, 1u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double lane_ops = (double)reps * grid * block * ITER * instr_per_iter;
    const double rate = lane_ops / (ms * 1e-3);
    printf("%-16s %8.3f ms  %7.2f Tlane-ops/s  (%.3f of 78.6)\n", name, ms / reps, rate / 1e12,
           rate / 78.6e12);
}

int main() {
    unsigned *d;
    hipMalloc(&d, 4096);
    run("v_add_u32", k_add_u32, 8, d);
    run("v_min_u32", k_min_u32, 8, d);
    run("v_min3_u32", k_min3_u32, 8, d);
    run("v_pk_add_u16", k_pk_add_u16, 8, d);
    run("v_pk_min_u16", k_pk_min_u16, 8, d);
    run("v_lshl_add_u64", k_lshl_add_u64, 8, d);
    run("v_add_f64", k_add_f64, 8, d);
    run("v_min_f64", k_min_f64, 8, d);
    run("relax_u64(x1)", k_relax_u64, 8, d);  // reported per relaxation
    run("relax_u32sat(x1)", k_relax_u32sat, 8, d);
    // per relaxation (16 per asm block x 4 blocks per iteration = 32 relax... see k_mix_u32)
    run("mix_u32 8w/SIMD", k_mix_u32, 32, d);
    run("mix_u32 2w/SIMD", k_mix_u32, 32, d, 512);
    run("mix_u32 1w/SIMD", k_mix_u32, 32, d, 256);
    run("v_add_u32 2w/SIMD", k_add_u32, 8, d, 512);
    // 4 blocks x 8 instructions = 32 instructions = 32 relaxations (2 per packed pair of ops)
    run("mix_u16 8w/SIMD", k_mix_u16, 32, d);
    run("mix_u16 2w/SIMD", k_mix_u16, 32, d, 512);
    run("v_min3 2w/SIMD", k_min3_u32, 8, d, 512);
    run("v_pk_add_f16", k_pk_add_f16, 8, d);
    run("v_pk_min_f16", k_pk_min_f16, 8, d);
    run("v_pk_minimum3_f16", k_pk_minimum3_f16, 8, d);
    run("v_minimum3_f32", k_minimum3_f32, 8, d);
    run("v_min3_f32", k_min3_f32, 8, d);
    run("v_pk_add_f32", k_pk_add_f32, 8, d);
    // per relaxation: 4 blocks x 16 relaxations (12 instructions) per iteration
    run("mix_f16 8w/SIMD", k_mix_f16, 64, d);
    run("mix_f16 2w/SIMD", k_mix_f16, 64, d, 512);
    // per relaxation: 4 blocks x 8 relaxations (8 instructions) per iteration
    run("mix_f32 8w/SIMD", k_mix_f32, 32, d);
    run("mix_f32 2w/SIMD", k_mix_f32, 32, d, 512);
    hipFree(d);
    return 0;
}
