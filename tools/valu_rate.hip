// valu_rate.hip -- measurement tool (not part of the library): issue rate of
// the VALU instructions a min-plus relaxation can be built from, on gfx950.
// Every kernel runs ITERS x 16 independent instances of one instruction per
// wave (16 accumulators, no dependency between them), 2 workgroups of 256
// threads per CU; the time per instruction per SIMD is printed relative to
// v_fma_f32 and v_add_f64.
//   hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip && ./valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITERS = 4096;

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

__global__ __launch_bounds__(256) void k_add_f64(double *out, double s) {
    double a[16];
#define I(i) a[i] = s + i;
    REP16(I)
#undef I
    for (int it = 0; it < ITERS; ++it) {
#define I(i) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[i]) : "v"(s));
        REP16(I)
#undef I
    }
    double r = 0;
#define I(i) r += a[i];
    REP16(I)
#undef I
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_min_f64(double *out, double s) {
    double a[16];
#define I(i) a[i] = s + i;
    REP16(I)
#undef I
    for (int it = 0; it < ITERS; ++it) {
#define I(i) asm volatile("v_min_f64 %0, %0, %1" : "+v"(a[i]) : "v"(s));
        REP16(I)
#undef I
    }
    double r = 0;
#define I(i) r += a[i];
    REP16(I)
#undef I
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int OP>
__global__ __launch_bounds__(256) void k_u32(double *out, unsigned s) {
    unsigned a[16];
#define I(i) a[i] = s + i;
    REP16(I)
#undef I
    for (int it = 0; it < ITERS; ++it) {
        if constexpr (OP == 0) {
#define I(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(s));
            REP16(I)
#undef I
        } else if constexpr (OP == 1) {
#define I(i) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[i]) : "v"(s));
            REP16(I)
#undef I
        } else if constexpr (OP == 2) {
#define I(i) asm volatile("v_min3_u32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(s));
            REP16(I)
#undef I
        } else if constexpr (OP == 3) {
#define I(i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(s));
            REP16(I)
#undef I
        } else if constexpr (OP == 4) {
#define I(i) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(s));
            REP16(I)
#undef I
        } else if constexpr (OP == 5) {
#define I(i) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(a[i]) : "v"(s));
            REP16(I)
#undef I
        } else if constexpr (OP == 6) {
#define I(i) asm volatile("v_min3_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(s));
            REP16(I)
#undef I
        }
    }
    unsigned r = 0;
#define I(i) r += a[i];
    REP16(I)
#undef I
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_u64(double *out, unsigned long long s) {
    unsigned long long a[16];
#define I(i) a[i] = s + i;
    REP16(I)
#undef I
    for (int it = 0; it < ITERS; ++it) {
#define I(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[i]) : "v"(s));
        REP16(I)
#undef I
    }
    unsigned long long r = 0;
#define I(i) r += a[i];
    REP16(I)
#undef I
    out[blockIdx.x * blockDim.x + threadIdx.x] = (double)r;
}

__global__ __launch_bounds__(256) void k_pk_add_f32(double *out, double s) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 a[16];
    f2 v = {(float)s, (float)s};
#define I(i) a[i] = v + (float)i;
    REP16(I)
#undef I
    for (int it = 0; it < ITERS; ++it) {
#define I(i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(v));
        REP16(I)
#undef I
    }
    float r = 0;
#define I(i) r += a[i].x + a[i].y;
    REP16(I)
#undef I
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <typename F>
float time_it(F launch) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const int blocks = 2 * cus, threads = 256;
    double *out;
    hipMalloc(&out, sizeof(double) * blocks * threads);
    const double instr_per_simd = (double)ITERS * 16 * 2;  // 2 waves per SIMD, 16 per iteration
    struct Row {
        const char *name;
        float ms;
    } rows[] = {
        {"v_fma_f32", time_it([&] { hipLaunchKernelGGL(k_u32<3>, blocks, threads, 0, 0, out, 0x3f800000u); })},
        {"v_add_f64", time_it([&] { hipLaunchKernelGGL(k_add_f64, blocks, threads, 0, 0, out, 1.0); })},
        {"v_min_f64", time_it([&] { hipLaunchKernelGGL(k_min_f64, blocks, threads, 0, 0, out, 1.0); })},
        {"v_add_u32", time_it([&] { hipLaunchKernelGGL(k_u32<0>, blocks, threads, 0, 0, out, 1u); })},
        {"v_min_u32", time_it([&] { hipLaunchKernelGGL(k_u32<1>, blocks, threads, 0, 0, out, 1u); })},
        {"v_min3_u32", time_it([&] { hipLaunchKernelGGL(k_u32<2>, blocks, threads, 0, 0, out, 1u); })},
        {"v_add3_u32", time_it([&] { hipLaunchKernelGGL(k_u32<4>, blocks, threads, 0, 0, out, 1u); })},
        {"v_pk_min_u16", time_it([&] { hipLaunchKernelGGL(k_u32<5>, blocks, threads, 0, 0, out, 1u); })},
        {"v_min3_f32", time_it([&] { hipLaunchKernelGGL(k_u32<6>, blocks, threads, 0, 0, out, 0x3f800000u); })},
        {"v_lshl_add_u64", time_it([&] { hipLaunchKernelGGL(k_u64, blocks, threads, 0, 0, out, 1ull); })},
        {"v_pk_add_f32", time_it([&] { hipLaunchKernelGGL(k_pk_add_f32, blocks, threads, 0, 0, out, 1.0); })},
    };
    const double f64ms = rows[1].ms;
    std::printf("{\"cus\": %d, \"rows\": [\n", cus);
    for (size_t i = 0; i < sizeof rows / sizeof rows[0]; ++i)
        std::printf("  {\"instr\": \"%s\", \"ms\": %.4f, \"ns_per_instr_per_simd\": %.4f, \"rel_to_add_f64\": %.3f}%s\n",
                    rows[i].name, rows[i].ms, rows[i].ms * 1e6 / instr_per_simd, rows[i].ms / f64ms,
                    i + 1 < sizeof rows / sizeof rows[0] ? "," : "");
    std::printf("]}\n");
    hipFree(out);
    return 0;
}
