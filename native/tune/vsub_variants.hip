// Tuning variants of lab1's vector subtraction (tools/experiments/vsub_sweep.py):
// V 16-B vectors per thread, contiguous, optionally non-temporal loads. Built
// into libmpx_tune.so only; the production kernel is in
// native/src/kernels/vsub.hip.
#include <algorithm>

#include "../src/kernels/internal.hpp"

namespace mpx {
namespace {

typedef double d2_t __attribute__((ext_vector_type(2)));
typedef float f4_t __attribute__((ext_vector_type(4)));
template <typename T> struct Vec16;
template <> struct Vec16<double> { using type = d2_t; static constexpr int n = 2; };
template <> struct Vec16<float> { using type = f4_t; static constexpr int n = 4; };

template <typename V> __device__ __forceinline__ V vsub(V a, V b) { return a - b; }

// Tuning variants (mpx_vsub_variant): V 16-B vectors per thread, contiguous
// (thread t owns vectors V*t .. V*t+V-1), optionally non-temporal loads.
template <typename T, int V, bool NTLD>
__global__ void vsub_var_kernel(const T *__restrict__ a, const T *__restrict__ b, T *__restrict__ c, int64_t n) {
    using W = typename Vec16<T>::type;
    constexpr int kV = Vec16<T>::n;
    const int64_t nvec = n / kV;
    const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * V;
    const W *__restrict__ av = reinterpret_cast<const W *>(a);
    const W *__restrict__ bv = reinterpret_cast<const W *>(b);
    W *__restrict__ cv = reinterpret_cast<W *>(c);
    W x[V], y[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int64_t i = min(i0 + v, nvec - 1);
        if constexpr (NTLD) {
            x[v] = __builtin_nontemporal_load(&av[i]);
            y[v] = __builtin_nontemporal_load(&bv[i]);
        } else {
            x[v] = av[i];
            y[v] = bv[i];
        }
    }
#pragma unroll
    for (int v = 0; v < V; ++v)
        if (i0 + v < nvec) __builtin_nontemporal_store(vsub(x[v], y[v]), &cv[i0 + v]);
    if (i0 == 0)
        for (int64_t t = nvec * kV; t < n; ++t) c[t] = a[t] - b[t];
}

template <typename T>
int launch_vsub_variant(const T *a, const T *b, T *c, int64_t n, int kind, int block, void *stream) {
    MPX_CHECK_ARG(n > 0 && a && b && c && aligned16(a) && aligned16(b) && aligned16(c), "bad arguments");
    if (block <= 0) block = 1024;
    const int v = (kind & 1) ? 2 : 1;
    const int64_t nvec = n / Vec16<T>::n;
    const int64_t threads = (nvec + v - 1) / v;
    const unsigned grid = (unsigned)std::max<int64_t>(1, (threads + block - 1) / block);
    hipStream_t s = as_stream(stream);
    switch (kind) {
        case 0: hipLaunchKernelGGL((vsub_var_kernel<T, 1, false>), dim3(grid), dim3(block), 0, s, a, b, c, n); break;
        case 1: hipLaunchKernelGGL((vsub_var_kernel<T, 2, false>), dim3(grid), dim3(block), 0, s, a, b, c, n); break;
        case 2: hipLaunchKernelGGL((vsub_var_kernel<T, 1, true>), dim3(grid), dim3(block), 0, s, a, b, c, n); break;
        case 3: hipLaunchKernelGGL((vsub_var_kernel<T, 2, true>), dim3(grid), dim3(block), 0, s, a, b, c, n); break;
        default: set_error("unknown vsub variant %d", kind); return MPX_ERR_ARG;
    }
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}

}  // namespace
}  // namespace mpx

extern "C" int mpx_vsub_variant(const void *a, const void *b, void *c, int64_t n, int fp64, int kind, int block,
                                void *stream) {
    if (fp64)
        return mpx::launch_vsub_variant<double>(static_cast<const double *>(a), static_cast<const double *>(b),
                                                static_cast<double *>(c), n, kind, block, stream);
    return mpx::launch_vsub_variant<float>(static_cast<const float *>(a), static_cast<const float *>(b),
                                           static_cast<float *>(c), n, kind, block, stream);
}

