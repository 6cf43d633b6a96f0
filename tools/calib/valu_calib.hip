// Calibration of the SQ instruction counters on gfx950: kernels with a known number of VALU
// instructions per wave (f32 FMA chains, f64 FMA chains), run under rocprofv3 --pmc SQ_WAVES
// SQ_INSTS_VALU ... The ratio SQ_INSTS_VALU / SQ_WAVES against the disassembly's count per wave
// tells how the counter counts a wave64 instruction (bench.py's roofline_normals divides by it).
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 4096;

__global__ void __launch_bounds__(256) fma32(float *out, float a, float b) {
    float x = float(threadIdx.x), y = x + 1.f, z = x + 2.f, w = x + 3.f;
#pragma unroll 64
    for (int i = 0; i < N; ++i) {   // 4 independent chains: 4 v_fma_f32 per iteration
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

int main() {
    const int blocks = 1024;
    float *o32;
    double *o64;
    if (hipMalloc(&o32, blocks * 256 * 4) != hipSuccess || hipMalloc(&o64, blocks * 256 * 8) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        fma32<<<blocks, 256>>>(o32, 0.999f, 0.001f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms32;
        hipEventElapsedTime(&ms32, e0, e1);
        hipEventRecord(e0);
        fma64<<<blocks, 256>>>(o64, 0.999, 0.001);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms64;
        hipEventElapsedTime(&ms64, e0, e1);
        const double insts = double(blocks) * 4 * 4.0 * N;   // wave-instructions of the chains
        printf("rep %d: f32 %.3f ms (%.1f G wave-FMA/s), f64 %.3f ms (%.1f G wave-FMA/s); waves %d, "
               "chain FMAs per wave %d\n", rep, ms32, insts / ms32 / 1e6, ms64, insts / ms64 / 1e6,
               blocks * 4, 4 * N);
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
