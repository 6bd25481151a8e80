// lab2: Roberts cross and its KxK generalisation (gradient-magnitude / linear
// convolution on fp32 luminance of RGBA8 images).
//
// Reference behaviour: lab2/src/main.cu:15-52 — per pixel, four tex2D fetches
// (clamp addressing), luminance recomputed for each of them, Gx = Y11 - Y00,
// Gy = Y10 - Y01, G = sqrtf(Gx^2 + Gy^2) clamped and truncated, alpha of p00
// preserved. The reference reads through a texture cache; CDNA has no reason
// to: this file stages each tile's luminance ONCE per input pixel in LDS
// (160 KiB per CU), moves 16 B per lane from HBM, and writes 8-16 B per lane.
//
// Numerics are defined by native/src/cpu/cpu_kernels.c and reproduced bit for
// bit: luminance and the gradient magnitude without FMA contraction (this TU
// is compiled with -ffp-contract=off), correctly rounded sqrtf (hipcc default),
// taps accumulated with one explicit fmaf each in (dy, dx) row-major order.
#include <algorithm>

#include "edge_kernels.hpp"

namespace mpx {
using edge::Taps;
namespace {

// ---------------------------------------------------------------------------
// Generic direct kernel: any K <= MPX_MAX_K and any anchor, one output pixel
// per thread straight from global memory. Used for (K, anchor) pairs without a
// tiled instantiation and as the naive baseline in profiles.
// ---------------------------------------------------------------------------
template <int MODE>
__global__ void conv_direct_kernel(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, int w,
                                   int pitch, int oy0, int oy1, int y_lo, int y_hi, int k, int anchor,
                                   Taps taps) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = oy0 + blockIdx.y * blockDim.y + threadIdx.y;
    if (x >= w || y >= oy1) return;
    float ax = 0.0f, ay = 0.0f;
    for (int dy = 0; dy < k; ++dy) {
        const uint32_t *row = in + (int64_t)mpx_clampi(y + dy - anchor, y_lo, y_hi) * pitch;
        for (int dx = 0; dx < k; ++dx) {
            const float l = mpx_luma(row[mpx_clampi(x + dx - anchor, 0, w - 1)]);
            ax = fmaf(taps.wx[dy * k + dx], l, ax);
            if (MODE == MPX_CONV_MAG2) ay = fmaf(taps.wy[dy * k + dx], l, ay);
        }
    }
    out[(int64_t)y * pitch + x] = edge::gray_px<MODE, false>(ax, ay, mpx_px_a(in[(int64_t)y * pitch + x]));
}

// ---------------------------------------------------------------------------
// Roberts with the caller's launch geometry (harness contract). Block (bx, by)
// threads, each thread VEC horizontally adjacent pixels of one row, so a tile
// is (VEC*bx) x by pixels; grid (gx, gy) grid-strides over tiles. Luminance of
// the tile plus its 1-pixel right/bottom halo is staged in LDS once.
// ---------------------------------------------------------------------------
template <int VEC>
__global__ void roberts_geom_kernel(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, int w,
                                    int h) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int bx = blockDim.x, by = blockDim.y;
    const int tx = threadIdx.x, ty = threadIdx.y;
    const int TW = VEC * bx, TH = by;
    const int LW = TW + 4;  // 16-B aligned rows; column TW holds the right halo
    const int tiles_x = (w + TW - 1) / TW, tiles_y = (h + TH - 1) / TH;
    for (int tyt = blockIdx.y; tyt < tiles_y; tyt += gridDim.y) {
        for (int txt = blockIdx.x; txt < tiles_x; txt += gridDim.x) {
            const int x0 = txt * TW, y0 = tyt * TH;
            const int xs = x0 + VEC * tx;
            const int yrow = min(y0 + ty, h - 1);
            uint32_t own[VEC];
            // own pixels (clamped copies beyond the right/bottom edge)
            if constexpr (VEC == 4) {
                const uint4 q = *reinterpret_cast<const uint4 *>(in + (int64_t)yrow * w + min(xs, w - 4));
                const bool right = xs >= w;
                own[0] = right ? q.w : q.x;
                own[1] = right ? q.w : q.y;
                own[2] = right ? q.w : q.z;
                own[3] = q.w;
                *reinterpret_cast<float4 *>(&lds[ty * LW + VEC * tx]) =
                    make_float4(mpx_luma(own[0]), mpx_luma(own[1]), mpx_luma(own[2]), mpx_luma(own[3]));
            } else {
                own[0] = in[(int64_t)yrow * w + min(xs, w - 1)];
                lds[ty * LW + tx] = mpx_luma(own[0]);
            }
            const int ybot = min(y0 + TH, h - 1);
            if (ty == 0) {  // bottom halo row
                if constexpr (VEC == 4) {
                    const uint4 q = *reinterpret_cast<const uint4 *>(in + (int64_t)ybot * w + min(xs, w - 4));
                    const bool right = xs >= w;
                    *reinterpret_cast<float4 *>(&lds[TH * LW + VEC * tx]) =
                        make_float4(mpx_luma(right ? q.w : q.x), mpx_luma(right ? q.w : q.y),
                                    mpx_luma(right ? q.w : q.z), mpx_luma(q.w));
                } else {
                    lds[TH * LW + tx] = mpx_luma(in[(int64_t)ybot * w + min(xs, w - 1)]);
                }
            }
            if (tx == 0) {  // right halo column
                const int xr = min(x0 + TW, w - 1);
                lds[ty * LW + TW] = mpx_luma(in[(int64_t)yrow * w + xr]);
                if (ty == 0) lds[TH * LW + TW] = mpx_luma(in[(int64_t)ybot * w + xr]);
            }
            __syncthreads();
            const int y = y0 + ty;
            if (y < h) {
                uint32_t res[VEC];
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    const int c = VEC * tx + k;
                    const float y00 = lds[ty * LW + c], y10 = lds[ty * LW + c + 1];
                    const float y01 = lds[(ty + 1) * LW + c], y11 = lds[(ty + 1) * LW + c + 1];
                    const float gxv = y11 - y00;
                    const float gyv = y10 - y01;
                    const float a = gxv * gxv;
                    const float b2 = gyv * gyv;
                    res[k] = mpx_px_gray(mpx_sat_u8(sqrtf(a + b2)), mpx_px_a(own[k]));
                }
                if constexpr (VEC == 4) {
                    if (xs < w) *reinterpret_cast<uint4 *>(out + (int64_t)y * w + xs) = make_uint4(res[0], res[1], res[2], res[3]);
                } else {
                    if (xs < w) out[(int64_t)y * w + xs] = res[0];
                }
            }
            __syncthreads();
        }
    }
}

Taps make_taps(int k, const float *wx, const float *wy, bool two) {
    Taps t{};
    for (int i = 0; i < k * k; ++i) {
        t.wx[i] = wx[i];
        t.wy[i] = two ? wy[i] : 0.0f;
    }
    return t;
}

// Production tile: RPT = 8 rows per wave -> 128 x 32 output tiles.
// resident workgroups per CU the chunking targets (VGPR-limited to 4 at ~100 VGPRs)
constexpr int kBlocksPerCU = 4;

template <int K, int A, int MODE, int RPT, bool FAST>
int launch_stream(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
                  const Taps &taps, bool vec, hipStream_t s, int chunk_override = 0) {
    constexpr int TH = edge::kTY * RPT;
    const int strips = (w + edge::kTW - 1) / edge::kTW;
    const int tiles_y = (oy1 - oy0 + TH - 1) / TH;
    const int64_t total = (int64_t)strips * tiles_y;
    const int64_t target = (int64_t)kNumCUs * kBlocksPerCU;
    int chunk = chunk_override > 0 ? chunk_override : (int)std::max<int64_t>(1, (total + target - 1) / target);
    chunk = std::min(chunk, tiles_y);
    const int cps = (tiles_y + chunk - 1) / chunk;
    const int64_t nblk = (int64_t)strips * cps;
    MPX_CHECK_ARG(nblk < (int64_t)1 << 31, "image too large for one launch");
    if (vec)
        hipLaunchKernelGGL((edge::conv_stream_kernel<K, A, MODE, RPT, true, FAST>), dim3((unsigned)nblk), dim3(256), 0,
                           s, in, out, w, pitch, oy0, oy1, y_lo, y_hi, tiles_y, chunk, cps, taps);
    else
        hipLaunchKernelGGL((edge::conv_stream_kernel<K, A, MODE, RPT, false, FAST>), dim3((unsigned)nblk), dim3(256), 0,
                           s, in, out, w, pitch, oy0, oy1, y_lo, y_hi, tiles_y, chunk, cps, taps);
    return MPX_OK;
}

// rows per wave segment of the wave-streaming kernel (tuned on MI355X, tools/kbench.py)
constexpr int kSegRows = 8;

template <int K, int A, int MODE, bool FAST, class F = edge::RuntimeTaps, int OWX = 0>
int launch_wave(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
                const Taps &taps, bool vec, hipStream_t s, int seg = kSegRows, int strip_minor = 1) {
    using G = edge::WaveGeom<K, A, OWX>;
    const int strips = (w + G::OW - 1) / G::OW;
    const int segs = (oy1 - oy0 + seg - 1) / seg;
    const int64_t nwaves = (int64_t)strips * segs;
    MPX_CHECK_ARG(nwaves < ((int64_t)1 << 31) - 4, "image too large for one launch");
    const unsigned nblk = (unsigned)((nwaves + 3) / 4);
    if (vec)
        hipLaunchKernelGGL((edge::conv_wave_kernel<K, A, MODE, true, FAST, F, OWX>), dim3(nblk), dim3(256), 0, s, in,
                           out, w, pitch, oy0, oy1, y_lo, y_hi, seg, segs, (int)nwaves, strips, strip_minor, taps);
    else
        hipLaunchKernelGGL((edge::conv_wave_kernel<K, A, MODE, false, FAST, F, OWX>), dim3(nblk), dim3(256), 0, s, in,
                           out, w, pitch, oy0, oy1, y_lo, y_hi, seg, segs, (int)nwaves, strips, strip_minor, taps);
    return MPX_OK;
}

// Named filters whose taps are compiled in (zero taps disappear); selected
// whenever the caller's taps are bit-identical to them.
template <class F, int N>
bool same_taps(const Taps &t) {
    for (int i = 0; i < N; ++i)
        if (__builtin_bit_cast(uint32_t, t.wx[i]) != __builtin_bit_cast(uint32_t, F::wx[i]) ||
            __builtin_bit_cast(uint32_t, t.wy[i]) != __builtin_bit_cast(uint32_t, F::wy[i]))
            return false;
    return true;
}

template <int K, int A, int MODE>
int launch_tiled(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
                 const Taps &taps, bool vec, hipStream_t s) {
    if constexpr (K == 2 && A == 0 && MODE == MPX_CONV_MAG2) {
        if (same_taps<edge::RobertsTaps, 4>(taps))
            return launch_wave<K, A, MODE, true, edge::RobertsTaps>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, vec, s);
    }
    if constexpr (K == 5 && A == 2 && MODE == MPX_CONV_MAG2) {
        if (same_taps<edge::Sobel5Taps, 25>(taps))
            return launch_wave<K, A, MODE, true, edge::Sobel5Taps>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, vec, s);
    }
    return launch_wave<K, A, MODE, true>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, vec, s);
}

// Exhaustive self-test of the fast magnitude path: every float s in
// [0, 65025] (bit patterns 0 .. 0x477E0100) must map to the same gray level as
// the correctly rounded sqrtf. Counts mismatches into *bad.
// raw = 0: the production fast path (v_sqrt + fract margin + exact fallback);
// raw = 1: bare truncation of v_sqrt_f32 with no margin test at all.
__global__ void fast_sqrt_selftest_kernel(uint32_t first, uint32_t last, unsigned long long *bad, int raw) {
    const uint32_t stride = gridDim.x * blockDim.x;
    unsigned long long nbad = 0;
    for (uint32_t u = first + blockIdx.x * blockDim.x + threadIdx.x; u <= last && u >= first; u += stride) {
        const float s = __builtin_bit_cast(float, u);
        const uint32_t exact = edge::mag_to_gray<false>(s);
        const uint32_t fast = raw ? (uint32_t)__builtin_amdgcn_sqrtf(fminf(s, 65025.0f)) : edge::mag_to_gray<true>(s);
        nbad += fast != exact;
    }
    if (nbad) atomicAdd(bad, nbad);
}

template <int MODE>
int dispatch_mode(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
                  int k, int anchor, const Taps &taps, bool vec, hipStream_t s) {
    if (k == 2 && anchor == 0) return launch_tiled<2, 0, MODE>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, vec, s);
    if (k == 3 && anchor == 1) return launch_tiled<3, 1, MODE>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, vec, s);
    if (k == 5 && anchor == 2) return launch_tiled<5, 2, MODE>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, vec, s);
    if (k == 7 && anchor == 3) return launch_tiled<7, 3, MODE>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, vec, s);
    const dim3 blk(64, 4);
    const dim3 grd((w + 63) / 64, (oy1 - oy0 + 3) / 4);
    hipLaunchKernelGGL(conv_direct_kernel<MODE>, grd, blk, 0, s, in, out, w, pitch, oy0, oy1, y_lo, y_hi, k,
                       anchor, taps);
    return MPX_OK;
}

}  // namespace

int conv_impl(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo, int y_hi, int k,
              int anchor, int mode, const float *wx, const float *wy, void *stream, bool force_direct) {
    MPX_CHECK_ARG(in && out && wx, "null pointer");
    MPX_CHECK_ARG(w > 0 && pitch >= w, "bad width/pitch");
    MPX_CHECK_ARG(k >= 1 && k <= MPX_MAX_K && anchor >= 0 && anchor < k, "bad window");
    MPX_CHECK_ARG(mode >= MPX_CONV_MAG2 && mode <= MPX_CONV_LIN1, "bad mode");
    MPX_CHECK_ARG(mode != MPX_CONV_MAG2 || wy, "MAG2 needs wy");
    MPX_CHECK_ARG(y_lo <= y_hi && oy0 >= 0, "bad row range");
    if (oy1 <= oy0) return MPX_OK;
    const Taps taps = make_taps(k, wx, wy, mode == MPX_CONV_MAG2);
    // 8-B pair loads/stores of the wave kernel: even width and pitch, 8-B aligned rows
    const bool vec = (w % 2 == 0) && (pitch % 2 == 0) && ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 7u) == 0;
    hipStream_t s = as_stream(stream);
    int rc;
    if (force_direct) {
        const dim3 blk(64, 4);
        const dim3 grd((w + 63) / 64, (oy1 - oy0 + 3) / 4);
        switch (mode) {
            case MPX_CONV_MAG2:
                hipLaunchKernelGGL(conv_direct_kernel<MPX_CONV_MAG2>, grd, blk, 0, s, in, out, w, pitch, oy0, oy1,
                                   y_lo, y_hi, k, anchor, taps);
                break;
            case MPX_CONV_ABS1:
                hipLaunchKernelGGL(conv_direct_kernel<MPX_CONV_ABS1>, grd, blk, 0, s, in, out, w, pitch, oy0, oy1,
                                   y_lo, y_hi, k, anchor, taps);
                break;
            default:
                hipLaunchKernelGGL(conv_direct_kernel<MPX_CONV_LIN1>, grd, blk, 0, s, in, out, w, pitch, oy0, oy1,
                                   y_lo, y_hi, k, anchor, taps);
        }
        rc = MPX_OK;
    } else if (mode == MPX_CONV_MAG2) {
        rc = dispatch_mode<MPX_CONV_MAG2>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, k, anchor, taps, vec, s);
    } else if (mode == MPX_CONV_ABS1) {
        rc = dispatch_mode<MPX_CONV_ABS1>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, k, anchor, taps, vec, s);
    } else {
        rc = dispatch_mode<MPX_CONV_LIN1>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, k, anchor, taps, vec, s);
    }
    if (rc != MPX_OK) return rc;
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}

static const float kRobertsX[4] = {-1.0f, 0.0f, 0.0f, 1.0f};  // Gx = Y11 - Y00
static const float kRobertsY[4] = {0.0f, 1.0f, -1.0f, 0.0f};  // Gy = Y10 - Y01

int roberts_impl(const uint32_t *in, uint32_t *out, int w, int h, int bx, int by, int gx, int gy, void *stream) {
    MPX_CHECK_ARG(in && out, "null pointer");
    MPX_CHECK_ARG(w > 0 && h > 0, "empty image");
    if (bx == 0 && by == 0 && gx == 0 && gy == 0)  // tuned path: tiled K=2 kernel
        return conv_impl(in, out, w, w, 0, h, 0, h - 1, 2, 0, MPX_CONV_MAG2, kRobertsX, kRobertsY, stream, false);
    MPX_CHECK_ARG(bx > 0 && by > 0 && gx > 0 && gy > 0, "launch geometry must be positive");
    MPX_CHECK_ARG((int64_t)bx * by <= 1024, "more than 1024 threads per block");
    const bool vec = (w % 4 == 0) && aligned16(in) && aligned16(out);
    const int VEC = vec ? 4 : 1;
    const size_t lds = sizeof(float) * (size_t)(by + 1) * (size_t)(VEC * bx + 4);
    MPX_CHECK_ARG(lds <= 64 * 1024, "tile does not fit the 64 KiB per-workgroup LDS limit");
    if (vec)
        hipLaunchKernelGGL(roberts_geom_kernel<4>, dim3(gx, gy), dim3(bx, by), lds, as_stream(stream), in, out, w, h);
    else
        hipLaunchKernelGGL(roberts_geom_kernel<1>, dim3(gx, gy), dim3(bx, by), lds, as_stream(stream), in, out, w, h);
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}

}  // namespace mpx

extern "C" int mpx_roberts(const uint32_t *in, uint32_t *out, int w, int h, int bx, int by, int gx, int gy,
                           void *stream) {
    return mpx::roberts_impl(in, out, w, h, bx, by, gx, gy, stream);
}

extern "C" int mpx_conv(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
                        int k, int anchor, int mode, const float *wx, const float *wy, void *stream) {
    return mpx::conv_impl(in, out, w, pitch, oy0, oy1, y_lo, y_hi, k, anchor, mode, wx, wy, stream, false);
}

extern "C" int mpx_conv_direct(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo,
                               int y_hi, int k, int anchor, int mode, const float *wx, const float *wy,
                               void *stream) {
    return mpx::conv_impl(in, out, w, pitch, oy0, oy1, y_lo, y_hi, k, anchor, mode, wx, wy, stream, true);
}

// Variant entry for the tuning harness (tools/kbench.py), k in {2, 5}, MAG2,
// whole image, fast magnitude path unless fast == 0:
//   kind 0: LDS streaming kernel, p1 = rows per wave (4, 8, 16), p2 = tiles per workgroup (0 = auto)
//   kind 1: wave-streaming kernel, p1 = rows per wave segment
extern "C" int mpx_conv_variant(const uint32_t *in, uint32_t *out, int w, int h, int k, int kind, int p1, int p2,
                                int fast, const float *wx, const float *wy, void *stream) {
    using namespace mpx;
    MPX_CHECK_ARG(in && out && wx && wy && w > 0 && h > 0, "bad arguments");
    MPX_CHECK_ARG(k == 2 || k == 5, "variant harness covers k = 2 and k = 5");
    const Taps taps = make_taps(k, wx, wy, true);
    hipStream_t s = as_stream(stream);
    if (kind == 1 || kind == 2) {
        // kind 1: runtime taps, kind 2: compiled-in taps of the named filter;
        // p1 = segment rows; p2 >= 1000 orders waves strip-major
        MPX_CHECK_ARG(p1 >= 1, "segment rows must be positive");
        const bool vec2 = (w % 2 == 0) && ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 7u) == 0;
        const int sm = p2 >= 1000 ? 0 : 1;
        if (k == 5) {
            if (kind == 2)
                return launch_wave<5, 2, MPX_CONV_MAG2, true, edge::Sobel5Taps>(in, out, w, w, 0, h, 0, h - 1, taps, vec2, s, p1, sm);
            return fast ? launch_wave<5, 2, MPX_CONV_MAG2, true>(in, out, w, w, 0, h, 0, h - 1, taps, vec2, s, p1, sm)
                        : launch_wave<5, 2, MPX_CONV_MAG2, false>(in, out, w, w, 0, h, 0, h - 1, taps, vec2, s, p1, sm);
        }
        if (kind == 2)
            return launch_wave<2, 0, MPX_CONV_MAG2, true, edge::RobertsTaps>(in, out, w, w, 0, h, 0, h - 1, taps, vec2, s, p1, sm);
        return fast ? launch_wave<2, 0, MPX_CONV_MAG2, true>(in, out, w, w, 0, h, 0, h - 1, taps, vec2, s, p1, sm)
                    : launch_wave<2, 0, MPX_CONV_MAG2, false>(in, out, w, w, 0, h, 0, h - 1, taps, vec2, s, p1, sm);
    }
    const bool vec = (w % 4 == 0) && aligned16(in) && aligned16(out);
#define MPX_VAR(KK, AA, R, F)                                                                                  \
    if (k == KK && p1 == R && (fast != 0) == F)                                                                 \
        return launch_stream<KK, AA, MPX_CONV_MAG2, R, F>(in, out, w, w, 0, h, 0, h - 1, taps, vec, s, p2);
    MPX_VAR(5, 2, 4, true) MPX_VAR(5, 2, 8, true) MPX_VAR(5, 2, 16, true) MPX_VAR(5, 2, 8, false)
    MPX_VAR(2, 0, 4, true) MPX_VAR(2, 0, 8, true) MPX_VAR(2, 0, 16, true) MPX_VAR(2, 0, 8, false)
#undef MPX_VAR
    set_error("unsupported variant k=%d kind=%d p1=%d fast=%d", k, kind, p1, fast);
    return MPX_ERR_ARG;
}

extern "C" int mpx_selftest_fast_sqrt(unsigned long long *bad_device, int raw, void *stream) {
    using namespace mpx;
    MPX_CHECK_ARG(bad_device, "null counter");
    hipLaunchKernelGGL(fast_sqrt_selftest_kernel, dim3(kNumCUs * 16), dim3(256), 0, as_stream(stream), 0u,
                       0x477E0100u, bad_device, raw);
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}
