// Operand / result layout of v_mfma_i32_4x4x4_16b_i8 on gfx950 (probe for the
// small-class-count lab3 ranking, classify.hip). Prints one JSON line:
//   a_src[l][r]: which lane's A operand (byte 0) reaches lane l, result reg r
//   b_src[l][r]: which lane's B operand (byte 0) reaches lane l, result reg r
//   kpair_ok: byte k of A multiplies byte k of B (k = 0..3)
// Build: hipcc --offload-arch=gfx950 -O2 tools/experiments/mfma4_layout.hip -o bin/mfma4_layout
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(int mode, int *out) {
    const int l = threadIdx.x;
    int a = 0, b = 0;
    if (mode == 0) { a = l + 1; b = 1; }          // D = A row value: identifies the A lane
    else if (mode == 1) { a = 1; b = l + 1; }     // identifies the B lane
    else {                                        // k pairing: A byte k = 1 << k, B byte k = k + 1
        a = 0x08040201; b = 0x04030201;
    }
    i32x4 acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_i32_4x4x4i8(a, b, acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[l * 4 + r] = acc[r];
}

// back-to-back issue cost: 4 independent accumulator chains, 1024 rounds
__global__ void rate(int a0, long long *cyc, int *sink) {
    i32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    const int a = a0 + threadIdx.x;
    const long long t0 = clock64();
    for (int i = 0; i < 1024; ++i) {
        c0 = __builtin_amdgcn_mfma_i32_4x4x4i8(a, a, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_4x4x4i8(a, a + 1, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_4x4x4i8(a, a + 2, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_4x4x4i8(a, a + 3, c3, 0, 0, 0);
    }
    const long long t1 = clock64();
    if (threadIdx.x == 0) *cyc = t1 - t0;
    sink[threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}

int main() {
    int *d;
    int h[3][256];
    if (hipMalloc(&d, 256 * sizeof(int)) != hipSuccess) return 1;
    for (int m = 0; m < 3; ++m) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, m, d);
        if (hipMemcpy(h[m], d, 256 * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    }
    printf("{\"a_src\": [");
    for (int l = 0; l < 64; ++l) {
        printf("%s[", l ? "," : "");
        for (int r = 0; r < 4; ++r) printf("%s%d", r ? "," : "", h[0][l * 4 + r] - 1);
        printf("]");
    }
    printf("], \"b_src\": [");
    for (int l = 0; l < 64; ++l) {
        printf("%s[", l ? "," : "");
        for (int r = 0; r < 4; ++r) printf("%s%d", r ? "," : "", h[1][l * 4 + r] - 1);
        printf("]");
    }
    // sum_k (1 << k) (k + 1) = 1 + 4 + 12 + 32 = 49 when byte k meets byte k
    long long *cyc;
    if (hipMalloc(&cyc, sizeof(long long)) != hipSuccess) return 1;
    hipLaunchKernelGGL(rate, dim3(1), dim3(64), 0, 0, 3, cyc, d);
    long long hc = 0;
    if (hipMemcpy(&hc, cyc, sizeof(hc), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("], \"kpair\": %d, \"kpair_ok\": %s, \"cycles_per_mfma\": %.2f}\n", h[2][0],
           h[2][0] == 49 ? "true" : "false", (double)hc / 4096.0);
    (void)hipFree(cyc);
    (void)hipFree(d);
    return 0;
}
