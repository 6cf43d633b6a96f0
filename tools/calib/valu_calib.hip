// Calibration of the SQ instruction counters and of the VALU issue rate on gfx950.
// (1) SQ_INSTS_VALU / SQ_WAVES against a known count per wave: compiler-scheduled FMA chains
//     (fma32: the compiler packs pairs into v_pk_fma_f32; fma64: v_fma_f64).
// (2) Issue rate: inline-asm blocks of 8 independent v_fma_f32 / v_fma_f64 / v_add_f64 /
//     v_pk_fma_f32 per iteration, 8 waves per SIMD -- wave-instructions per second per type.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 4096;

__global__ void __launch_bounds__(256) fma32(float *out, float a, float b) {
    float x = float(threadIdx.x), y = x + 1.f, z = x + 2.f, w = x + 3.f;
#pragma unroll 64
    for (int i = 0; i < N; ++i) {
        x = fmaf(x, a, b);
        y = fmaf(y, a, b);
        z = fmaf(z, a, b);
        w = fmaf(w, a, b);
    }
    out[blockIdx.x * 256 + threadIdx.x] = x + y + z + w;
}

__global__ void __launch_bounds__(256) fma64(double *out, double a, double b) {
    double x = double(threadIdx.x), y = x + 1.0, z = x + 2.0, w = x + 3.0;
#pragma unroll 64
    for (int i = 0; i < N; ++i) {
        x = fma(x, a, b);
        y = fma(y, a, b);
        z = fma(z, a, b);
        w = fma(w, a, b);
    }
    out[blockIdx.x * 256 + threadIdx.x] = x + y + z + w;
}

constexpr int M = 1024;   // iterations of 8 independent instructions

#define ASM8_F32(OP)                                                                       \
    asm volatile(OP " %0, %8, %9, %0\n\t" OP " %1, %8, %9, %1\n\t" OP " %2, %8, %9, %2\n\t" \
                 OP " %3, %8, %9, %3\n\t" OP " %4, %8, %9, %4\n\t" OP " %5, %8, %9, %5\n\t" \
                 OP " %6, %8, %9, %6\n\t" OP " %7, %8, %9, %7"                             \
                 : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) \
                 : "v"(a), "v"(b))

__global__ void __launch_bounds__(256) issue_f32(float *out, float a, float b) {
    float r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5,
          r6 = r0 + 6, r7 = r0 + 7;
    for (int i = 0; i < M; ++i) ASM8_F32("v_fma_f32");
    out[blockIdx.x * 256 + threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
}

__global__ void __launch_bounds__(256) issue_f64(double *out, double a, double b) {
    double r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5,
           r6 = r0 + 6, r7 = r0 + 7;
    for (int i = 0; i < M; ++i) ASM8_F32("v_fma_f64");
    out[blockIdx.x * 256 + threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
}

__global__ void __launch_bounds__(256) issue_add64(double *out, double a, double b) {
    double r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5,
           r6 = r0 + 6, r7 = r0 + 7;
    for (int i = 0; i < M; ++i)
        asm volatile("v_add_f64 %0, %8, %0\n\tv_add_f64 %1, %8, %1\n\tv_add_f64 %2, %8, %2\n\t"
                     "v_add_f64 %3, %8, %3\n\tv_add_f64 %4, %8, %4\n\tv_add_f64 %5, %8, %5\n\t"
                     "v_add_f64 %6, %8, %6\n\tv_add_f64 %7, %8, %7"
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6),
                       "+v"(r7)
                     : "v"(a));
    (void)b;
    out[blockIdx.x * 256 + threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
}

// (3) f64 MFMA throughput (could the normals' f64 cumulant sums run as
//     v_mfma_f64_16x16x4f64 tiles?): 8 independent accumulators per wave, 8 waves per SIMD.
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) mfma64(double *out, double a, double b) {
    d4 c0 = {a, b, a, b}, c1 = c0, c2 = c0, c3 = c0, c4 = c0, c5 = c0, c6 = c0, c7 = c0;
    const double x = a + threadIdx.x * 1e-9, y = b - threadIdx.x * 1e-9;
    for (int i = 0; i < M; ++i) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c3, 0, 0, 0);
        c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c4, 0, 0, 0);
        c5 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c5, 0, 0, 0);
        c6 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c6, 0, 0, 0);
        c7 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c7, 0, 0, 0);
    }
    const d4 s = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
    out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y + s.z + s.w;
}

template <typename K, typename T>
float timed(K k, T *o, T a, T b, int blocks) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    k<<<blocks, 256>>>(o, a, b);   // warm
    (void)hipEventRecord(e0);
    k<<<blocks, 256>>>(o, a, b);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    const int blocks = 2048;   // 8192 waves: 8 per SIMD on 256 CUs
    float *o32;
    double *o64;
    if (hipMalloc(&o32, blocks * 256 * 4) != hipSuccess || hipMalloc(&o64, blocks * 256 * 8) != hipSuccess) return 1;
    const double waves = blocks * 4.0;
    float ms = timed(fma32, o32, 0.999f, 0.001f, blocks);
    printf("fma32 (compiler, v_pk_fma_f32): %.3f ms, %.1f G wave-instr/s\n", ms, waves * (N * 2.0) / ms / 1e6);
    ms = timed(fma64, o64, 0.999, 0.001, blocks);
    printf("fma64 (compiler, v_fma_f64): %.3f ms, %.1f G wave-instr/s\n", ms, waves * (N * 4.0) / ms / 1e6);
    ms = timed(issue_f32, o32, 0.999f, 0.001f, blocks);
    printf("issue v_fma_f32 x8: %.3f ms, %.1f G wave-instr/s\n", ms, waves * (M * 8.0) / ms / 1e6);
    ms = timed(issue_f64, o64, 0.999, 0.001, blocks);
    printf("issue v_fma_f64 x8: %.3f ms, %.1f G wave-instr/s\n", ms, waves * (M * 8.0) / ms / 1e6);
    ms = timed(issue_add64, o64, 0.999, 0.001, blocks);
    printf("issue v_add_f64 x8: %.3f ms, %.1f G wave-instr/s\n", ms, waves * (M * 8.0) / ms / 1e6);
    ms = timed(mfma64, o64, 0.999, 0.001, blocks);
    {
        const double inst = waves * (M * 8.0);
        printf("mfma v_mfma_f64_16x16x4f64 x8: %.3f ms, %.2f G wave-instr/s, %.1f TFLOP/s "
               "(2048 FLOP each), %.1f cycles/SIMD each at 2.4 GHz\n", ms, inst / ms / 1e6,
               inst * 2048.0 / ms / 1e9, 1024.0 * 2.4e9 / (inst / (ms * 1e-3)));
    }
    printf("(peak assumed by bench.py: 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles = 1228.8 G/s)\n");
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
