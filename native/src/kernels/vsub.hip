// lab1: element-wise vector subtraction c = a - b (fp64 and fp32).
//
// Reference: lab1/src/main.cu:22-29 (one scalar element per thread per
// grid-stride step). MI355X design: pure HBM streaming (AI = 1/24 flop/B), so
// every lane moves 16 B per access (double2 / float4), keeps four independent
// 16-B loads per operand in flight per grid-stride step, and both reads and
// writes are non-temporal: nothing is re-read by this kernel, so none of it
// should displace L2/MALL lines (tools/vsub_sweep.py: non-temporal loads take
// 2^26 fp32 from 131.7 to 122.4 us, 6.12 -> 6.58 TB/s).
// Launch geometry is honoured exactly when the caller passes one (the harness
// sweeps [grid, block] pairs); 0/0 picks one vector per thread (see below).
#include <algorithm>

#include "internal.hpp"

namespace mpx {
namespace {

// clang ext_vector types: element-wise '-' and accepted by __builtin_nontemporal_store
typedef double d2_t __attribute__((ext_vector_type(2)));
typedef float f4_t __attribute__((ext_vector_type(4)));
template <typename T> struct Vec16;
template <> struct Vec16<double> { using type = d2_t; static constexpr int n = 2; };
template <> struct Vec16<float> { using type = f4_t; static constexpr int n = 4; };

template <typename V> __device__ __forceinline__ V vsub(V a, V b) { return a - b; }

// kUnroll independent 16-B vectors per operand in flight per thread and
// grid-stride step: 4 for launches that fill the GPU, 8 for "thin" harness
// geometries ([1, 32], [4, 64] ...: a few waves streaming a whole vector are
// latency-bound, and only loads in flight per lane help them)
// LB: workgroup-size bound; the 16-deep thin form is compiled for <= 256
// threads, which lifts the 128-VGPR cap of a 1024-thread bound (no spills)
template <typename T, int kUnroll, int LB = 1024>
__global__ __launch_bounds__(LB) void vsub_vec_kernel(const T *__restrict__ a, const T *__restrict__ b, T *__restrict__ c,
                                                      int64_t n) {
    using V = typename Vec16<T>::type;
    constexpr int kV = Vec16<T>::n;
    const int64_t nvec = n / kV;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const V *__restrict__ av = reinterpret_cast<const V *>(a);
    const V *__restrict__ bv = reinterpret_cast<const V *>(b);
    V *__restrict__ cv = reinterpret_cast<V *>(c);
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // main body: kUnroll independent vectors per thread in flight
    for (; i + (kUnroll - 1) * stride < nvec; i += kUnroll * stride) {
        V x[kUnroll], y[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            x[u] = __builtin_nontemporal_load(&av[i + u * stride]);
            y[u] = __builtin_nontemporal_load(&bv[i + u * stride]);
        }
        // every load issued before the first use: left alone the scheduler
        // interleaves load pairs with the (possibly aliasing, to its mind)
        // stores and waits for each pair
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) __builtin_nontemporal_store(vsub(x[u], y[u]), &cv[i + u * stride]);
    }
    for (; i < nvec; i += stride)
        __builtin_nontemporal_store(vsub(__builtin_nontemporal_load(&av[i]), __builtin_nontemporal_load(&bv[i])), &cv[i]);
    // scalar tail (n not a multiple of the vector width)
    for (int64_t t = nvec * kV + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += stride)
        c[t] = a[t] - b[t];
}

template <typename T>
__global__ void vsub_scalar_kernel(const T *__restrict__ a, const T *__restrict__ b, T *__restrict__ c,
                                   int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) c[i] = a[i] - b[i];
}

template <typename T>
int launch_vsub(const T *a, const T *b, T *c, int64_t n, int grid, int block, void *stream) {
    MPX_CHECK_ARG(n >= 0, "n must be >= 0");
    MPX_CHECK_ARG(grid >= 0 && block >= 0 && block <= 1024, "grid/block out of range");
    if (n == 0) return MPX_OK;
    MPX_CHECK_ARG(a && b && c, "null pointer");
    const bool vec = aligned16(a) && aligned16(b) && aligned16(c);
    if (grid == 0) {
        // one 16-B vector per thread in 1024-thread blocks: measured on MI355X
        // at 2^26 fp32 / 2^25 fp64 (tools/vsub_sweep.py, profiles/lab1_vsub.md)
        // 5.95 / 6.06 TB/s, = torch's own elementwise kernel, against 4.3-5.8
        // TB/s for persistent grid-stride geometries (2048x256 .. 256x256):
        // with one access per wave in flight per address range, the DRAM
        // pages are consumed in order instead of by 4 strided streams per wave
        if (block == 0) block = 1024;
        const int64_t per_block = (int64_t)block * (vec ? Vec16<T>::n : 1);
        int64_t g = (n + per_block - 1) / per_block;
        const int64_t cap = (int64_t)1 << 30;
        grid = (int)(g < 1 ? 1 : (g > cap ? cap : g));
    }
    if (block == 0) block = 256;
    // empty workgroups of an oversized caller grid dropped (useful_grid): the
    // vector kernel's thread t handles vector t and tail element t; the scalar
    // kernel element t
    {
        const int64_t items = vec ? std::max<int64_t>(n / Vec16<T>::n, Vec16<T>::n) : n;
        grid = (int)useful_grid(grid, items, block);
    }
    const bool thin = (int64_t)grid * block < 16384;
    // very thin ([1, 32] .. [4, 64]: at most one wave per CU): 16 vectors in
    // flight per operand — each lane walks thousands of vectors, so the
    // round trips, not the issue, bound it
    // (measured on MI355X, n = 10^6 fp64: [1, 32] 1383 -> 915 us, [4, 64] 151
    // -> 113 us vs 8 deep; 32 deep is slower again, 1380 us: 64 loads exceed
    // the 63 a wave's vmcnt can track, so the loop waits every trip)
    const bool very_thin = (int64_t)grid * block <= 2048 && block <= 256;
    if (vec && very_thin)
        hipLaunchKernelGGL((vsub_vec_kernel<T, 16, 256>), dim3(grid), dim3(block), 0, as_stream(stream), a, b, c, n);
    else if (vec && thin)
        hipLaunchKernelGGL((vsub_vec_kernel<T, 8>), dim3(grid), dim3(block), 0, as_stream(stream), a, b, c, n);
    else if (vec)
        hipLaunchKernelGGL((vsub_vec_kernel<T, 4>), dim3(grid), dim3(block), 0, as_stream(stream), a, b, c, n);
    else
        hipLaunchKernelGGL(vsub_scalar_kernel<T>, dim3(grid), dim3(block), 0, as_stream(stream), a, b, c, n);
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}

}  // namespace
MPX_MODULE_ANCHOR(vsub)

}  // namespace mpx

extern "C" int mpx_vsub_f64(const double *a, const double *b, double *c, int64_t n, int grid, int block,
                            void *stream) {
    return mpx::launch_vsub<double>(a, b, c, n, grid, block, stream);
}

// tuning entry (tools/vsub_sweep.py): kind bit 0 = two vectors per thread, bit 1 = non-temporal loads
extern "C" int mpx_vsub_f32(const float *a, const float *b, float *c, int64_t n, int grid, int block,
                            void *stream) {
    return mpx::launch_vsub<float>(a, b, c, n, grid, block, stream);
}
