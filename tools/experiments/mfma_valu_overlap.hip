// Does an int8 MFMA stream overlap with VALU work on gfx950? (lab3 question,
// profiles/lab3_classify.md). Three kernels with the same loop trip count:
//   mfma  : 4 independent v_mfma_i32_32x32x32_i8 chains per iteration
//   valu  : 32 independent fp32 FMAs per iteration (the ranking-style stream)
//   both  : the two bodies interleaved in one wave (independent data)
// 2 waves per SIMD; time with hipEvents; prints one JSON line.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_valu_overlap.hip -o bin/mfma_valu_overlap
#include <hip/hip_runtime.h>

#include <cstdio>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

template <bool MF, bool VA>
__global__ __launch_bounds__(256) void body(int iters, int *out, float *fout) {
    const int t = threadIdx.x;
    v4i a = {t, t + 1, t + 2, t + 3}, b = {t * 3, t ^ 5, t + 7, t - 1};
    v16i c0 = {}, c1 = {}, c2 = {}, c3 = {};
    float f[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) f[i] = (float)(t + i);
    const float m = 1.0000001f, d = 0.5f;
    for (int it = 0; it < iters; ++it) {
        if constexpr (MF) {
            c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, b, c3, 0, 0, 0);
        }
        if constexpr (VA) {
#pragma unroll
            for (int i = 0; i < 32; ++i) f[i] = __builtin_fmaf(f[i], m, d);
        }
    }
    int s = 0;
    if constexpr (MF) {
#pragma unroll
        for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
    }
    float fs = 0.0f;
#pragma unroll
    for (int i = 0; i < 32; ++i) fs += f[i];
    out[blockIdx.x * 256 + t] = s;
    fout[blockIdx.x * 256 + t] = fs;
}

template <bool MF, bool VA>
float run(int iters, int blocks, int *o, float *fo) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL((body<MF, VA>), dim3(blocks), dim3(256), 0, 0, iters, o, fo);  // warm-up
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL((body<MF, VA>), dim3(blocks), dim3(256), 0, 0, iters, o, fo);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    const int blocks = 256 * 2;  // 2 waves per SIMD on 256 CUs (4 waves per block)
    const int iters = 20000;
    int *o;
    float *fo;
    CHECK(hipMalloc(&o, blocks * 256 * sizeof(int)));
    CHECK(hipMalloc(&fo, blocks * 256 * sizeof(float)));
    const float tm = run<true, false>(iters, blocks, o, fo);
    const float tv = run<false, true>(iters, blocks, o, fo);
    const float tb = run<true, true>(iters, blocks, o, fo);
    CHECK(hipGetLastError());
    const double waves = blocks * 4.0;
    const double mfma_ops = waves * iters * 4 * 32.0 * 32 * 32 * 2;  // int ops
    const double valu_ops = waves * 64 * iters * 32 * 2.0;           // fp32 flops
    printf("{\"mfma_ms\": %.3f, \"valu_ms\": %.3f, \"both_ms\": %.3f, \"overlap\": %.3f, "
           "\"i8_tops\": %.1f, \"valu_tflops\": %.1f}\n",
           tm, tv, tb, (tm + tv - tb) / (tm < tv ? tm : tv), mfma_ops / tm / 1e9, valu_ops / tv / 1e9);
    return 0;
}
