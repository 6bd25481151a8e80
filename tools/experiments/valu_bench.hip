// VALU throughput microbenchmark: scalar v_fma_f32 (SGPR coefficient) vs
// packed v_pk_fma_f32 on gfx950, many waves per SIMD, independent chains.
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_bench.hip -o build/valu_bench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void fma_scalar(float *out, float c0, float c1, int iters) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = fmaf(c0, a[i], c1);
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void fma_packed(float *out, float c0, float c1, int iters) {
    f2 a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = f2{threadIdx.x * 0.001f + i, threadIdx.x * 0.002f + i};
    const f2 cc0 = {c0, c0}, cc1 = {c1, c1};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = __builtin_elementwise_fma(cc0, a[i], cc1);
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) s += a[i].x + a[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    const int blocks = 256 * 8, threads = 256, iters = 4096;
    float *out;
    hipMalloc(&out, sizeof(float) * blocks * threads);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 3; ++rep) {
        for (int k = 0; k < 2; ++k) {
            if (k == 0) hipLaunchKernelGGL(fma_scalar, dim3(blocks), dim3(threads), 0, 0, out, 0.999f, 0.001f, iters);
            else hipLaunchKernelGGL(fma_packed, dim3(blocks), dim3(threads), 0, 0, out, 0.999f, 0.001f, iters);
            hipDeviceSynchronize();
            hipEventRecord(a);
            if (k == 0) hipLaunchKernelGGL(fma_scalar, dim3(blocks), dim3(threads), 0, 0, out, 0.999f, 0.001f, iters);
            else hipLaunchKernelGGL(fma_packed, dim3(blocks), dim3(threads), 0, 0, out, 0.999f, 0.001f, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double flops = 2.0 * 8 * iters * (double)blocks * threads;
            const double wave_instr = (k == 0 ? 8.0 : 4.0) * iters * (double)blocks * threads / 64.0;
            const double cycles_per_simd = ms * 1e-3 * 2.4e9;
            std::printf("{\"kernel\": \"%s\", \"ms\": %.3f, \"TFLOPs\": %.1f, \"cyc_per_wave_instr_at_2.4GHz\": %.2f}\n",
                        k == 0 ? "v_fma_f32" : "v_pk_fma_f32", ms, flops / ms / 1e9, cycles_per_simd / (wave_instr / 1024));
        }
    }
    return 0;
}
