// 2-D Jacobi sweep for the distributed stencil tier (the MPI north star of
// BASELINE.json, re-expressed over RCCL): slab rows with one halo row above
// and below, Dirichlet columns 0 and cols-1, fused L-infinity residual.
//
// MI355X design: HBM-bound 5-point stencil. Each lane owns a 16-B column
// vector (double2 / float4) and slides down kRows rows keeping the up/centre
// rows in registers, so each input row is fetched from HBM once per sweep; the
// left/right neighbours at the vector edges come from the L1 (the adjacent
// lanes just loaded them). The residual is reduced wave -> lane 0 -> one
// device-scope atomic max per wave on the bit pattern (non-negative IEEE
// values order like unsigned integers), so no second kernel is needed.
#include "internal.hpp"

namespace mpx {
namespace {

template <typename T> struct JVec;
template <> struct JVec<double> {
    using type = double2;
    using bits = unsigned long long;
    static constexpr int n = 2;
};
template <> struct JVec<float> {
    using type = float4;
    using bits = unsigned int;
    static constexpr int n = 4;
};

constexpr int kRows = 16;  // rows swept per lane (vertical register reuse)

template <typename T>
__device__ __forceinline__ T lane_of(const typename JVec<T>::type &v, int i) {
    if constexpr (JVec<T>::n == 2) return i == 0 ? v.x : v.y;
    else return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void jacobi_kernel(const T *__restrict__ u, T *__restrict__ un, int cols,
                                                     int pitch, int r0, int r1, T *__restrict__ resid) {
    using V = typename JVec<T>::type;
    constexpr int NV = VEC ? JVec<T>::n : 1;
    const int j0 = NV * (blockIdx.x * blockDim.x + threadIdx.x);
    const int i0 = r0 + blockIdx.y * kRows;
    const int i1 = min(i0 + kRows, r1);
    T rmax = (T)0;
    if (j0 < cols && i0 < i1) {
        T up[NV], cen[NV], dn[NV];
        auto load_row = [&](int i, T (&dst)[NV]) {
            const T *row = u + (int64_t)i * pitch;
            if constexpr (VEC) {
                if (j0 + NV <= cols) {
                    const V q = *reinterpret_cast<const V *>(row + j0);
#pragma unroll
                    for (int k = 0; k < NV; ++k) dst[k] = lane_of<T>(q, k);
                    return;
                }
            }
#pragma unroll
            for (int k = 0; k < NV; ++k) dst[k] = (j0 + k < cols) ? row[j0 + k] : (T)0;
        };
        load_row(i0 - 1, up);
        load_row(i0, cen);
        for (int i = i0; i < i1; ++i) {
            load_row(i + 1, dn);
            const T *crow = u + (int64_t)i * pitch;
            const T left = j0 > 0 ? crow[j0 - 1] : (T)0;
            const T right = (j0 + NV < cols) ? crow[j0 + NV] : (T)0;
            T res[NV];
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                const int j = j0 + k;
                const T l = k == 0 ? left : cen[k - 1];
                const T r = k == NV - 1 ? right : cen[k + 1];
                const T s = ((up[k] + dn[k]) + (l + r)) * (T)0.25;
                const bool interior = j > 0 && j < cols - 1;
                res[k] = interior ? s : cen[k];
                if (interior && j < cols) {
                    const T d = s > cen[k] ? s - cen[k] : cen[k] - s;
                    rmax = d > rmax ? d : rmax;
                }
            }
            T *orow = un + (int64_t)i * pitch;
            bool stored = false;
            if constexpr (VEC) {
                if (j0 + NV <= cols) {
                    if constexpr (JVec<T>::n == 2)
                        *reinterpret_cast<double2 *>(orow + j0) = make_double2(res[0], res[1]);
                    else
                        *reinterpret_cast<float4 *>(orow + j0) = make_float4(res[0], res[1], res[2], res[3]);
                    stored = true;
                }
            }
            if (!stored) {
#pragma unroll
                for (int k = 0; k < NV; ++k)
                    if (j0 + k < cols) orow[j0 + k] = res[k];
            }
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                up[k] = cen[k];
                cen[k] = dn[k];
            }
        }
    }
    if (resid) {
        using B = typename JVec<T>::bits;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            const T o = __shfl_xor(rmax, m);
            rmax = o > rmax ? o : rmax;
        }
        if ((threadIdx.x & 63) == 0 && rmax > (T)0) atomicMax(reinterpret_cast<B *>(resid), __builtin_bit_cast(B, rmax));
    }
}

template <typename T>
int launch_jacobi(const T *u, T *un, int cols, int pitch, int r0, int r1, T *resid, void *stream) {
    MPX_CHECK_ARG(u && un, "null pointer");
    MPX_CHECK_ARG(cols >= 1 && pitch >= cols && r0 >= 1 && r1 >= r0, "bad slab geometry");
    if (r1 == r0) return MPX_OK;
    constexpr int NV = JVec<T>::n;
    const bool vec = (pitch % NV == 0) && aligned16(u) && aligned16(un);
    const int lanes = vec ? (cols + NV - 1) / NV : cols;
    const dim3 blk(256);
    const dim3 grd((lanes + 255) / 256, (r1 - r0 + kRows - 1) / kRows);
    if (vec)
        hipLaunchKernelGGL((jacobi_kernel<T, true>), grd, blk, 0, as_stream(stream), u, un, cols, pitch, r0, r1, resid);
    else
        hipLaunchKernelGGL((jacobi_kernel<T, false>), grd, blk, 0, as_stream(stream), u, un, cols, pitch, r0, r1,
                           resid);
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}

}  // namespace
}  // namespace mpx

extern "C" int mpx_jacobi_f64(const double *u, double *un, int cols, int pitch, int r0, int r1, double *resid,
                              void *stream) {
    return mpx::launch_jacobi<double>(u, un, cols, pitch, r0, r1, resid, stream);
}

extern "C" int mpx_jacobi_f32(const float *u, float *un, int cols, int pitch, int r0, int r1, float *resid,
                              void *stream) {
    return mpx::launch_jacobi<float>(u, un, cols, pitch, r0, r1, resid, stream);
}
