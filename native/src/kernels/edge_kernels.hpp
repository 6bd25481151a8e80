// Device code of the lab2 convolution family (included by edge.hip and by the
// tools/kbench variant harness). See edge.hip for the design notes.
#pragma once

#include <type_traits>

#include "internal.hpp"
#include "peer_sync.hpp"

namespace mpx {
namespace edge {

struct Taps {
    float wx[MPX_MAX_K * MPX_MAX_K];
    float wy[MPX_MAX_K * MPX_MAX_K];
};

// Where input rows live (wave kernel). Logical rows [0, own_rows) come from
// `in`; rows < 0 from `up` and rows >= own_rows from `dn`, both biased so the
// logical row index applies unchanged (mpx_conv_peer: IPC-mapped neighbour
// slabs read over xGMI). nullptr = `in` for every row.
struct RowSrc {
    const uint32_t *up = nullptr;
    const uint32_t *dn = nullptr;
    int own_rows = 0x7fffffff;
};

// Exact magnitude -> gray level: trunc(min(sqrt_rn(s), 255)) with s = gx*gx + gy*gy.
//   FAST: hardware v_sqrt_f32 (not correctly rounded) decides the integer part
//   whenever its result is further than kSqrtMargin from an integer; otherwise
//   (and only then) the correctly rounded sqrtf runs. tests/test_gpu_kernels.py
//   checks the equivalence exhaustively for every float s in [0, 65025], and
//   the paired production form below (mag2_to_gray) for every float in [0, +inf].
constexpr float kSqrtMargin = 1.0f / 16384.0f;  // 2^-14 = 4 ulp at 255

template <bool FAST>
__device__ __forceinline__ uint32_t mag_to_gray(float s) {
    if constexpr (!FAST) {
        return mpx_sat_u8(sqrtf(s));
    } else {
        if (s >= 65025.0f) return 255u;  // sqrt_rn is monotone and sqrt_rn(255^2) == 255
        const float r = __builtin_amdgcn_sqrtf(s);
        const float n = truncf(r);
        const float fr = r - n;
        if (fr > kSqrtMargin && fr < 1.0f - kSqrtMargin) return (uint32_t)n;
        return mpx_sat_u8(sqrtf(s));
    }
}

// Fast path for two magnitudes at once: r = v_sqrt(med3(s, 0.5^2, 255.5^2)) decides
// trunc(sqrt_rn(s)) unless fract(r) is within kSqrtMargin of an integer; one
// wave-level branch then recomputes both lanes' pair exactly (rare).
__device__ __forceinline__ void mag2_to_gray(float s0, float s1, uint32_t &g0, uint32_t &g1) {
    // clamp into [0.5^2, 255.5^2] with one v_med3_f32: a zero gradient then
    // gives r = 0.5 and a saturated one r = 255.5, both half-way between
    // integers, so the margin test decides them on the fast path (trunc = 0 /
    // 255, the exact answers) instead of sending them to the fallback — a
    // plain min(s, 255^2) put both exactly on an integer. Iterated (streaming)
    // frames are full of them, random frames almost never.
    const float c0 = __builtin_amdgcn_fmed3f(s0, 0.25f, 65280.25f);
    const float c1 = __builtin_amdgcn_fmed3f(s1, 0.25f, 65280.25f);
    const float r0 = __builtin_amdgcn_sqrtf(c0), r1 = __builtin_amdgcn_sqrtf(c1);
    const float f0 = __builtin_amdgcn_fractf(r0), f1 = __builtin_amdgcn_fractf(r1);
    constexpr float kHalfOpen = 0.5f - kSqrtMargin;
    // '&', not '&&': both pixels' tests run unconditionally; a short-circuit
    // puts the second pixel's sqrt under an exec-mask branch every row
    const bool ok = (int)(fabsf(f0 - 0.5f) < kHalfOpen) & (int)(fabsf(f1 - 0.5f) < kHalfOpen);
    g0 = (uint32_t)r0;
    g1 = (uint32_t)r1;
    if (!ok) {
        g0 = mpx_sat_u8(sqrtf(s0));
        g1 = mpx_sat_u8(sqrtf(s1));
    }
}

typedef float f2_t __attribute__((ext_vector_type(2)));

// Four magnitudes at once, no float->int conversion (band kernels: 20 VALU for
// four pixels where two mag2_to_gray take 24).
// r = v_sqrt(med3(s, 0.5^2, 255.5^2)) as in mag2_to_gray; then, packed,
// x+- = (r - 0.5 +- kSqrtMargin) + 2^23. Both sums before the last are exact
// (r < 512: every operand a multiple of ulp(r)), and the last rounds to the
// nearest integer, so x+- = 2^23 + RNE(r - 0.5 +- m): equal exactly when no
// integer lies within about m of r, i.e. when v_sqrt (error < m / 4) decides
// trunc(sqrt_rn(s)) = RNE(r - 0.5 + m) — which is the low byte of x+'s bits
// (0x4B0000nn, n <= 255 since r <= 255.5 + ulp). The float compare x+ == x-
// is false on NaN, so a NaN magnitude takes the exact path as before. g[i]
// holds the gray level in its LOW BYTE only (the callers' v_perm reads byte 0).
// tests/test_gpu_kernels.py checks this form exhaustively too.
__device__ __forceinline__ void mag4_to_gray(f2_t s01, f2_t s23, uint32_t g[4]) {
    constexpr float kTwo23 = 8388608.0f;
    const f2_t c01 = {__builtin_amdgcn_fmed3f(s01.x, 0.25f, 65280.25f), __builtin_amdgcn_fmed3f(s01.y, 0.25f, 65280.25f)};
    const f2_t c23 = {__builtin_amdgcn_fmed3f(s23.x, 0.25f, 65280.25f), __builtin_amdgcn_fmed3f(s23.y, 0.25f, 65280.25f)};
    const f2_t r01 = {__builtin_amdgcn_sqrtf(c01.x), __builtin_amdgcn_sqrtf(c01.y)};
    const f2_t r23 = {__builtin_amdgcn_sqrtf(c23.x), __builtin_amdgcn_sqrtf(c23.y)};
    const f2_t kp = {-0.5f + kSqrtMargin, -0.5f + kSqrtMargin}, km = {-0.5f - kSqrtMargin, -0.5f - kSqrtMargin};
    const f2_t big = {kTwo23, kTwo23};
    const f2_t p01 = (r01 + kp) + big, m01 = (r01 + km) + big;
    const f2_t p23 = (r23 + kp) + big, m23 = (r23 + km) + big;
    const bool ok = (int)(p01.x == m01.x) & (int)(p01.y == m01.y) & (int)(p23.x == m23.x) & (int)(p23.y == m23.y);
    if (ok) {
        // whole-vector bit casts: __builtin_bit_cast of one ext_vector element
        // (p01.y) miscompiles with this ROCm clang (the other element is read)
        typedef uint32_t u2_t __attribute__((ext_vector_type(2)));
        const u2_t b01 = __builtin_bit_cast(u2_t, p01), b23 = __builtin_bit_cast(u2_t, p23);
        g[0] = b01.x;
        g[1] = b01.y;
        g[2] = b23.x;
        g[3] = b23.y;
    } else {
        g[0] = mpx_sat_u8(sqrtf(s01.x));
        g[1] = mpx_sat_u8(sqrtf(s01.y));
        g[2] = mpx_sat_u8(sqrtf(s23.x));
        g[3] = mpx_sat_u8(sqrtf(s23.y));
    }
}

template <int MODE, bool FAST>
__device__ __forceinline__ uint32_t finish_gray(float gx, float gy) {
    if constexpr (MODE == MPX_CONV_MAG2) {
        const float a = gx * gx;
        const float b = gy * gy;
        return mag_to_gray<FAST>(a + b);
    } else if constexpr (MODE == MPX_CONV_ABS1) {
        return mpx_sat_u8(fabsf(gx));
    } else {
        return mpx_sat_u8(gx);
    }
}

// ---------------------------------------------------------------------------
// Geometry shared by the tiled kernels: 256 threads = 4 waves; wave `ty`
// owns RPT output rows of the tile, lane `tx` two adjacent columns.
// ---------------------------------------------------------------------------
constexpr int kTX = 64;
constexpr int kTY = 4;
constexpr int kCPT = 2;
constexpr int kTW = kTX * kCPT;     // 128 output columns per tile
constexpr int kHL = 4;              // halo columns loaded on each side (one 16-B vector)
constexpr int kLW = kTW + 2 * kHL;  // 136 floats per LDS luminance row
constexpr int kNVROW = kLW / 4;     // 34 vectors per row

// Fetch one 16-B vector (4 pixels) of row `row` starting at column gx with
// clamp-to-edge in x. VEC: w % 4 == 0, so the vector is entirely inside,
// entirely left (gx < 0) or entirely right (gx >= w) of the image.
template <bool VEC>
__device__ __forceinline__ uint4 fetch4(const uint32_t *__restrict__ row, int gx, int w) {
    if constexpr (VEC) {
        const int gxc = mpx_clampi(gx, 0, w - 4);
        const uint4 q = *reinterpret_cast<const uint4 *>(row + gxc);
        const bool left = gx < 0, right = gx >= w;
        uint4 p;
        p.x = right ? q.w : q.x;
        p.y = left ? q.x : (right ? q.w : q.y);
        p.z = left ? q.x : (right ? q.w : q.z);
        p.w = left ? q.x : q.w;
        return p;
    } else {
        uint4 p;
        p.x = row[mpx_clampi(gx + 0, 0, w - 1)];
        p.y = row[mpx_clampi(gx + 1, 0, w - 1)];
        p.z = row[mpx_clampi(gx + 2, 0, w - 1)];
        p.w = row[mpx_clampi(gx + 3, 0, w - 1)];
        return p;
    }
}

__device__ __forceinline__ float4 luma4(uint4 p) {
    return make_float4(mpx_luma(p.x), mpx_luma(p.y), mpx_luma(p.z), mpx_luma(p.w));
}

__device__ __forceinline__ uint32_t alpha4(uint4 p) {
    return (p.x >> 24) | ((p.y >> 24) << 8) | ((p.z >> 24) << 16) | (p.w & 0xff000000u);
}

// Sliding-window compute of one tile from LDS: RPT x 2 outputs per lane, taps
// accumulated with one fmaf each in (dy, dx) order. lum rows: tile row 0 of
// the window at LDS row 0. Writes gray pixels through `emit(o, j, value)`.
template <int K, int A, int MODE, int RPT, bool FAST>
__device__ __forceinline__ void tile_compute(const float *__restrict__ lum, const Taps &taps, int tx, int ty,
                                             uint32_t (&res)[RPT][kCPT]) {
    constexpr int OFF = (kHL - A) & 1;
    constexpr int NW = (OFF + kCPT + K - 1 + 1) / 2;
    constexpr bool TWO = (MODE == MPX_CONV_MAG2);
    const int wbase = kCPT * tx + kHL - A - OFF;
    float ax[RPT][kCPT], ay[RPT][kCPT];
#pragma unroll
    for (int o = 0; o < RPT; ++o)
#pragma unroll
        for (int j = 0; j < kCPT; ++j) {
            ax[o][j] = 0.0f;
            ay[o][j] = 0.0f;
        }
#pragma unroll
    for (int r = 0; r < RPT + K - 1; ++r) {
        const float *lrow = lum + (ty * RPT + r) * kLW + wbase;
        float wnd[2 * NW];
#pragma unroll
        for (int q = 0; q < NW; ++q) {
            const float2 t = *reinterpret_cast<const float2 *>(lrow + 2 * q);
            wnd[2 * q] = t.x;
            wnd[2 * q + 1] = t.y;
        }
#pragma unroll
        for (int o = 0; o < RPT; ++o) {
            const int dy = r - o;
            if (dy < 0 || dy >= K) continue;
#pragma unroll
            for (int dx = 0; dx < K; ++dx) {
                const float cx = taps.wx[dy * K + dx];
#pragma unroll
                for (int j = 0; j < kCPT; ++j) ax[o][j] = fmaf(cx, wnd[OFF + j + dx], ax[o][j]);
                if constexpr (TWO) {
                    const float cy = taps.wy[dy * K + dx];
#pragma unroll
                    for (int j = 0; j < kCPT; ++j) ay[o][j] = fmaf(cy, wnd[OFF + j + dx], ay[o][j]);
                }
            }
        }
    }
#pragma unroll
    for (int o = 0; o < RPT; ++o)
#pragma unroll
        for (int j = 0; j < kCPT; ++j) res[o][j] = finish_gray<MODE, FAST>(ax[o][j], ay[o][j]);
}

// ---------------------------------------------------------------------------
// Streaming kernel (production path). A workgroup walks DOWN a 128-column
// strip through `chunk` consecutive tiles of TH = 4*RPT rows:
//   * luminance is computed once per input pixel and the K-1 window rows
//     shared by consecutive tiles stay resident in LDS (moved to the top of
//     the buffer) instead of being re-read from memory;
//   * the next tile's TH new rows are fetched into registers BEFORE the
//     current tile is computed, so HBM traffic overlaps the FMA work inside
//     every workgroup, not only across workgroups;
//   * workgroups of one XCD take contiguous chunk ids (xcd_remap), so strips
//     and their neighbours' halo columns share an L2.
// LDS: (TH+K-1) x 136 fp32 luminance + (TH+K-1) x 128 alpha bytes.
// ---------------------------------------------------------------------------
template <int K, int A, int MODE, int RPT, bool VEC, bool FAST>
__global__ __launch_bounds__(256) void conv_stream_kernel(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                          int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
                                                          int tiles_y, int chunk, int chunks_per_strip, Taps taps) {
    constexpr int TH = kTY * RPT;
    constexpr int LH = TH + K - 1;
    constexpr int HALO = K - 1;
    constexpr int NEWV = TH * kNVROW;   // vectors fetched per steady-state tile
    constexpr int ITN = (NEWV + 255) / 256;
    constexpr int LUMF = LH * kLW;      // floats; multiple of 4
    static_assert(A <= kHL && (K - 1 - A) <= kHL, "window exceeds loaded halo");
    static_assert(TH >= HALO, "tile shorter than the window");
    __shared__ __attribute__((aligned(16))) float smem[LUMF + LH * kTW / 4];
    float *lum = smem;
    uint8_t *alpha = reinterpret_cast<uint8_t *>(smem + LUMF);

    const int tid = threadIdx.x;
    const int tx = tid & (kTX - 1);
    const int ty = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
    const int b = xcd_remap(blockIdx.x, gridDim.x);
    const int strip = b / chunks_per_strip;
    const int t0 = (b - strip * chunks_per_strip) * chunk;
    const int t1 = min(t0 + chunk, tiles_y);
    if (t0 >= t1) return;  // uniform per workgroup
    const int x0 = strip * kTW;
    const bool full_x = (x0 + kTW <= w);

    // per-thread fetch slots: slot `it` covers vector i = tid + 256*it of a
    // block of rows, i.e. row r = i / 34 and vector v = i % 34 (fixed per thread)
    auto fetch_rows = [&](uint4 (&regs)[ITN], int gy_first, int nrows_total) {
#pragma unroll
        for (int it = 0; it < ITN; ++it) {  // unconditional (see conv_wave_kernel)
            const int i = min(tid + it * 256, nrows_total * kNVROW - 1);
            const int r = i / kNVROW;
            const int v = i - r * kNVROW;
            const int gy = mpx_clampi(gy_first + r, y_lo, y_hi);
            regs[it] = fetch4<VEC>(in + (int64_t)gy * pitch, x0 - kHL + 4 * v, w);
        }
    };
    auto store_rows = [&](const uint4 (&regs)[ITN], int lrow_first, int nrows_total) {
#pragma unroll
        for (int it = 0; it < ITN; ++it) {
            const int i = tid + it * 256;
            if (i < nrows_total * kNVROW) {
                const int r = i / kNVROW;
                const int v = i - r * kNVROW;
                const int lr = lrow_first + r;
                *reinterpret_cast<float4 *>(&lum[lr * kLW + 4 * v]) = luma4(regs[it]);
                if (v >= 1 && v <= kTW / 4) *reinterpret_cast<uint32_t *>(&alpha[lr * kTW + 4 * (v - 1)]) = alpha4(regs[it]);
            }
        }
    };

    // ---- prologue: the whole window of the first tile (LH rows) ----
    {
        constexpr int ITP = (LH * kNVROW + 255) / 256;
        uint4 pre[ITP];
        const int ytop = oy0 + t0 * TH - A;
#pragma unroll
        for (int it = 0; it < ITP; ++it) {
            const int i = min(tid + it * 256, LH * kNVROW - 1);
            const int r = i / kNVROW;
            const int v = i - r * kNVROW;
            pre[it] = fetch4<VEC>(in + (int64_t)mpx_clampi(ytop + r, y_lo, y_hi) * pitch, x0 - kHL + 4 * v, w);
        }
#pragma unroll
        for (int it = 0; it < ITP; ++it) {
            const int i = tid + it * 256;
            if (i < LH * kNVROW) {
                const int r = i / kNVROW;
                const int v = i - r * kNVROW;
                *reinterpret_cast<float4 *>(&lum[r * kLW + 4 * v]) = luma4(pre[it]);
                if (v >= 1 && v <= kTW / 4) *reinterpret_cast<uint32_t *>(&alpha[r * kTW + 4 * (v - 1)]) = alpha4(pre[it]);
            }
        }
    }
    __syncthreads();

    uint4 nxt[ITN];
    for (int t = t0; t < t1; ++t) {
        const int y0 = oy0 + t * TH;
        const bool more = (t + 1 < t1);
        // prefetch the TH new rows of tile t+1 (window rows HALO .. LH-1)
        fetch_rows(nxt, y0 + TH - A + HALO, TH);  // unconditional; unused after the last tile

        uint32_t res[RPT][kCPT];
        tile_compute<K, A, MODE, RPT, FAST>(lum, taps, tx, ty, res);

        const int gx0 = x0 + kCPT * tx;
#pragma unroll
        for (int o = 0; o < RPT; ++o) {
            const int ly = ty * RPT + o;
            const int gy = y0 + ly;
            if (gy >= oy1) break;  // wave-uniform
            const uint8_t *arow = &alpha[(ly + A) * kTW + kCPT * tx];
            const uint32_t v0 = mpx_px_gray(res[o][0], arow[0]);
            const uint32_t v1 = mpx_px_gray(res[o][1], arow[1]);
            uint32_t *orow = out + (int64_t)gy * pitch;
            if (VEC && full_x) {
                *reinterpret_cast<uint2 *>(orow + gx0) = make_uint2(v0, v1);
            } else {
                if (gx0 < w) orow[gx0] = v0;
                if (gx0 + 1 < w) orow[gx0 + 1] = v1;
            }
        }
        if (!more) break;
        // slide: window rows TH .. LH-1 become rows 0 .. HALO-1. The sources are
        // read before the barrier (nobody writes LDS until after it), written
        // after it, together with the prefetched rows HALO .. LH-1.
        static_assert(HALO * kNVROW <= 256 && HALO * (kTW / 16) <= 256, "slide must fit one pass");
        const int sr = tid / kNVROW, sv = tid - (tid / kNVROW) * kNVROW;
        const int ar = tid / (kTW / 16), ac = tid - ar * (kTW / 16);
        float4 slum;
        uint4 salp;
        if (tid < HALO * kNVROW) slum = *reinterpret_cast<const float4 *>(&lum[(TH + sr) * kLW + 4 * sv]);
        if (tid < HALO * (kTW / 16)) salp = *reinterpret_cast<const uint4 *>(&alpha[(TH + ar) * kTW + 16 * ac]);
        __syncthreads();  // every wave is done reading the window
        if (tid < HALO * kNVROW) *reinterpret_cast<float4 *>(&lum[sr * kLW + 4 * sv]) = slum;
        if (tid < HALO * (kTW / 16)) *reinterpret_cast<uint4 *>(&alpha[ar * kTW + 16 * ac]) = salp;
        store_rows(nxt, HALO, TH);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Wave-streaming kernel (production path for K in {2, 3, 5, 7}).
//
// Every wave is independent: no LDS, no barrier. A wave owns a strip of
// OW = 128 - P - R2 output columns (P = anchor rounded up to even, R2 = right
// reach rounded up to even) and a segment of SEG output rows. Lane l holds
// input columns x0 - P + 2l and +1 (one 8-B load per row), so the 64 lanes
// cover the strip plus its horizontal halo; lanes whose window would leave
// the 128 loaded columns produce no output. Per input row a lane converts its
// two pixels to luminance once and assembles the horizontal window from its
// neighbours with DPP wave shifts (pure VALU, no LDS traffic). The last K
// rows' windows stay in registers (a ring indexed statically by unrolling the
// row loop K times), and the loads run K rows ahead of their use, so each wave
// keeps K x 512 B in flight with no synchronisation at all. Registers stay low
// enough for 6-8 waves per SIMD, which is what hides HBM latency here.
// ---------------------------------------------------------------------------
constexpr int kDppShr1 = 0x138;  // wave_shr:1 -> lane i reads lane i-1
constexpr int kDppShl1 = 0x130;  // wave_shl:1 -> lane i reads lane i+1

__device__ __forceinline__ float from_prev(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), kDppShr1, 0xf, 0xf, true));
}
__device__ __forceinline__ float from_next(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), kDppShl1, 0xf, 0xf, true));
}
// Wave shift whose source-less lane (0 for shr, 63 for shl) keeps `old`
// (bound_ctrl off: that lane's write is the old value, not 0).
// (a <= b) ? n : 0 for buffer-descriptor sizes (wave-uniform operands): an
// s_cselect as long as n is not also held in a VGPR — otherwise the select
// lowers to a lane-mask v_cndmask and the descriptor in VGPRs costs a
// readfirstlane loop around every access (so no VALU value may be w * 4).
__device__ __forceinline__ int scalar_le_sel(int a, int b, int n) { return a <= b ? n : 0; }
template <int CTRL>
__device__ __forceinline__ float shift_or_old(float old, float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, v),
                                                                 CTRL, 0xf, 0xf, false));
}

template <int K, int A, int OWX = 0>
struct WaveGeom {
    static constexpr int R = K - 1 - A;            // right reach
    static constexpr int P = A + (A & 1);          // left pad, even
    static constexpr int R2 = R + (R & 1);         // right pad, even
    static constexpr int OW = OWX ? OWX : 128 - P - R2;  // output columns per strip
    static constexpr int NV = 2 + A + R;           // window values per lane and row
    static constexpr int LANE0 = P / 2;            // first producing lane
    static constexpr int NLANES = OW / 2;          // producing lanes
};

// ---- tap sources: runtime (kernel-argument SGPRs) or compile-time (named filters) ----
struct RuntimeTaps {
    static constexpr bool kConst = false;
    static constexpr bool kSep = false;
};
// Separable filter factors in the kernel-argument taps (common.h MPX_CONV_SEP layout).
struct RuntimeSepTaps {
    static constexpr bool kConst = false;
    static constexpr bool kSep = true;
};
// Separable 5x5 Sobel (filters.h "sobel5"): gx = (v (x) d) / 48, gy = (d (x) v) / 48.
struct Sobel5SepTaps {
    static constexpr bool kConst = true;
    static constexpr bool kSep = true;
    static constexpr float hx[5] = {-1, -2, 0, 2, 1};
    static constexpr float vx[5] = {1, 4, 6, 4, 1};
    static constexpr float sx = 1.0f / 48;
    static constexpr float hy[5] = {1, 4, 6, 4, 1};
    static constexpr float vy[5] = {-1, -2, 0, 2, 1};
    static constexpr float sy = 1.0f / 48;
};
// Separable 5x5 binomial blur (filters.h "gauss5").
struct Gauss5SepTaps {
    static constexpr bool kConst = true;
    static constexpr bool kSep = true;
    static constexpr float hx[5] = {1, 4, 6, 4, 1};
    static constexpr float vx[5] = {1, 4, 6, 4, 1};
    static constexpr float sx = 1.0f / 256;
    static constexpr float hy[5] = {0, 0, 0, 0, 0};
    static constexpr float vy[5] = {0, 0, 0, 0, 0};
    static constexpr float sy = 0.0f;
};
// Compile-time dense filters (filters.h named entries, matched bit-exactly by
// edgel::launch_tiled): zero taps drop out of the chains and +-1 taps fold into
// adds; kK / kA / kMode name the window and output mode they apply to.
// Reference Roberts operator (filters.h "roberts").
struct RobertsTaps {
    static constexpr bool kConst = true;
    static constexpr bool kSep = false;
    static constexpr int kK = 2, kA = 0, kMode = MPX_CONV_MAG2;
    static constexpr float wx[4] = {-1.0f, 0.0f, 0.0f, 1.0f};
    static constexpr float wy[4] = {0.0f, 1.0f, -1.0f, 0.0f};
};
// 5x5 Sobel / 48 (filters.h "sobel5"); bit-identical constants: (float)k / 48.0f
struct Sobel5Taps {
    static constexpr bool kConst = true;
    static constexpr bool kSep = false;
    static constexpr int kK = 5, kA = 2, kMode = MPX_CONV_MAG2;
    static constexpr float wx[25] = {-1.0f / 48, -2.0f / 48, 0, 2.0f / 48, 1.0f / 48,
                                     -4.0f / 48, -8.0f / 48, 0, 8.0f / 48, 4.0f / 48,
                                     -6.0f / 48, -12.0f / 48, 0, 12.0f / 48, 6.0f / 48,
                                     -4.0f / 48, -8.0f / 48, 0, 8.0f / 48, 4.0f / 48,
                                     -1.0f / 48, -2.0f / 48, 0, 2.0f / 48, 1.0f / 48};
    static constexpr float wy[25] = {-1.0f / 48, -4.0f / 48, -6.0f / 48, -4.0f / 48, -1.0f / 48,
                                     -2.0f / 48, -8.0f / 48, -12.0f / 48, -8.0f / 48, -2.0f / 48,
                                     0, 0, 0, 0, 0,
                                     2.0f / 48, 8.0f / 48, 12.0f / 48, 8.0f / 48, 2.0f / 48,
                                     1.0f / 48, 4.0f / 48, 6.0f / 48, 4.0f / 48, 1.0f / 48};
};

struct Sobel3Taps {
    static constexpr bool kConst = true;
    static constexpr bool kSep = false;
    static constexpr int kK = 3, kA = 1, kMode = MPX_CONV_MAG2;
    static constexpr float wx[9] = {-1, 0, 1, -2, 0, 2, -1, 0, 1};
    static constexpr float wy[9] = {-1, -2, -1, 0, 0, 0, 1, 2, 1};
};
struct Prewitt3Taps {
    static constexpr bool kConst = true;
    static constexpr bool kSep = false;
    static constexpr int kK = 3, kA = 1, kMode = MPX_CONV_MAG2;
    static constexpr float wx[9] = {-1, 0, 1, -1, 0, 1, -1, 0, 1};
    static constexpr float wy[9] = {-1, -1, -1, 0, 0, 0, 1, 1, 1};
};
struct Scharr3Taps {
    static constexpr bool kConst = true;
    static constexpr bool kSep = false;
    static constexpr int kK = 3, kA = 1, kMode = MPX_CONV_MAG2;
    static constexpr float wx[9] = {-3, 0, 3, -10, 0, 10, -3, 0, 3};
    static constexpr float wy[9] = {-3, -10, -3, 0, 0, 0, 3, 10, 3};
};
struct Laplace3Taps {
    static constexpr bool kConst = true;
    static constexpr bool kSep = false;
    static constexpr int kK = 3, kA = 1, kMode = MPX_CONV_ABS1;
    static constexpr float wx[9] = {0, 1, 0, 1, -4, 1, 0, 1, 0};
    static constexpr float wy[9] = {};
};
struct Sharpen3Taps {
    static constexpr bool kConst = true;
    static constexpr bool kSep = false;
    static constexpr int kK = 3, kA = 1, kMode = MPX_CONV_LIN1;
    static constexpr float wx[9] = {0, -1, 0, -1, 5, -1, 0, -1, 0};
    static constexpr float wy[9] = {};
};
struct Log5Taps {
    static constexpr bool kConst = true;
    static constexpr bool kSep = false;
    static constexpr int kK = 5, kA = 2, kMode = MPX_CONV_ABS1;
    static constexpr float wx[25] = {0, 0, -1, 0, 0, 0, -1, -2, -1, 0, -1, -2, 16, -2, -1,
                                     0, -1, -2, -1, 0, 0, 0, -1, 0, 0};
    static constexpr float wy[25] = {};
};

template <class F>
__device__ __forceinline__ float tap_x(const Taps &t, int i) {
    if constexpr (F::kConst) return F::wx[i];
    else return t.wx[i];
}
template <class F>
__device__ __forceinline__ float tap_y(const Taps &t, int i) {
    if constexpr (F::kConst) return F::wy[i];
    else return t.wy[i];
}

// Separable factors: WHICH 0 = hx, 1 = vx, 2 = hy, 3 = vy (index i < K); the
// scales through sep_scale<F, K, Y>.
template <class F, int K, int WHICH>
__device__ __forceinline__ float sep_tap(const Taps &t, int i) {
    if constexpr (F::kConst) {
        if constexpr (WHICH == 0) return F::hx[i];
        else if constexpr (WHICH == 1) return F::vx[i];
        else if constexpr (WHICH == 2) return F::hy[i];
        else return F::vy[i];
    } else {
        if constexpr (WHICH == 0) return t.wx[i];
        else if constexpr (WHICH == 1) return t.wx[K + i];
        else if constexpr (WHICH == 2) return t.wy[i];
        else return t.wy[K + i];
    }
}
template <class F, int K, bool Y>
__device__ __forceinline__ float sep_scale(const Taps &t) {
    if constexpr (F::kConst) return Y ? F::sy : F::sx;
    else return Y ? t.wy[2 * K] : t.wx[2 * K];
}

// One step of a tap chain acc = fma(c, x, acc) started at 0. With compile-time
// taps, zero taps are skipped and the first nonzero tap is a plain product
// (c = +-1 folds into the next instruction's operand): fma(c, x, 0) and c * x
// differ only in the sign of a zero result, and skipping a zero tap changes at
// most the sign of a zero sum — neither can change a gray level (squares,
// fabs and the saturating cast all map -0 and +0 alike).
template <bool CONST>
__device__ __forceinline__ void tap_step(f2_t &acc, bool &started, float c, f2_t x) {
    if constexpr (CONST) {
        if (c == 0.0f) return;
        if (!started) {
            acc = f2_t{c, c} * x;
            started = true;
            return;
        }
    }
    acc = __builtin_elementwise_fma(f2_t{c, c}, x, acc);
}

// Sequential fmaf chain from 0 over K packed operands (one of the separable
// factor passes).
template <class F, int K, int WHICH, class Get>
__device__ __forceinline__ f2_t sep_chain(const Taps &t, Get &&operand) {
    f2_t acc = {0.0f, 0.0f};
    bool started = false;
#pragma unroll
    for (int i = 0; i < K; ++i) tap_step<F::kConst>(acc, started, sep_tap<F, K, WHICH>(t, i), operand(i));
    return acc;
}

// Luminance of two pixels with packed fp32 (v_pk_mul_f32 / v_pk_add_f32): the
// same three products and two sums per pixel as mpx_luma, rounded per element.
__device__ __forceinline__ f2_t luma2(uint32_t p0, uint32_t p1) {
    const f2_t r = {(float)mpx_px_r(p0), (float)mpx_px_r(p1)};
    const f2_t g = {(float)mpx_px_g(p0), (float)mpx_px_g(p1)};
    const f2_t b = {(float)mpx_px_b(p0), (float)mpx_px_b(p1)};
    const f2_t t0 = r * f2_t{0.299f, 0.299f};
    const f2_t t1 = g * f2_t{0.587f, 0.587f};
    const f2_t t2 = b * f2_t{0.114f, 0.114f};
    return (t0 + t1) + t2;
}

template <int K, int A, int MODE, bool VEC, bool FAST, class F = RuntimeTaps, int OWX = 0, int PF = 4, int BUFLD = 1>
__global__ __launch_bounds__(256) void conv_wave_kernel(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                        int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
                                                        int seg, int segs_per_strip, int nwaves, int strips,
                                                        int strip_minor, Taps taps, RowSrc rs) {
    using G = WaveGeom<K, A, OWX>;
    static_assert(G::P + G::OW + G::R2 <= 128, "strip plus halo exceeds one wave's 128 columns");
    constexpr int NV = G::NV;
    constexpr int NE = (NV + 1) / 2;  // even-aligned pairs (w[2q], w[2q+1])
    constexpr int NO = NV / 2;        // odd pairs (w[2q+1], w[2q+2])
    constexpr bool TWO = (MODE == MPX_CONV_MAG2);
    constexpr bool SEP = F::kSep;
    const int lane = threadIdx.x & 63;
    // readfirstlane: make the wave index (and everything derived from it: the
    // segment bounds and the row-loop exits) provably wave-uniform, so the loop
    // branches are scalar and hipcc keeps counted vmcnt waits across them
    const int gw = xcd_remap(blockIdx.x, gridDim.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (gw >= nwaves) return;  // wave-uniform
    // strip_minor bit 0: consecutive waves take horizontally adjacent strips of
    // the same rows, so the waves running together stream contiguous row pieces
    // (DRAM-page friendly, like a copy); otherwise they walk one strip downwards.
    // Bit 1 (alternate): odd segments walk their rows upwards. The segments of
    // one resident round all start together, so with every segment walking
    // down, the K-1 input rows two vertical neighbours share are read at the
    // START of the lower segment and at the END of the upper one, a whole
    // segment apart — long gone from L2. Walking alternate segments up, each
    // shared band is read by both neighbours at the same moment (both ends or
    // both starts), and the second read hits L2.
    const bool minor = strip_minor & 1;
    const int strip = minor ? gw % strips : gw / segs_per_strip;
    const int sg0 = minor ? gw / strips : gw - strip * segs_per_strip;
    // both boundary segments first (strip-minor order): in a slab their halo
    // rows may come from a neighbour's HBM over xGMI (RowSrc), the slowest
    // loads of the launch, so their waves start in the first round
    const int sg = (!minor || segs_per_strip < 3 || sg0 == 0) ? sg0
                   : (sg0 == 1 ? segs_per_strip - 1 : sg0 - 1);
    const bool up = (strip_minor & 2) && (sg & 1);  // wave-uniform
    const int ys = oy0 + sg * seg;
    const int ye = min(ys + seg, oy1);
    const int x0 = strip * G::OW;
    const int cin = x0 - G::P + 2 * lane;  // this lane's first input column
    const bool producer = lane >= G::LANE0 && lane < G::LANE0 + G::NLANES;
    const int ox = cin;                    // output column of element 0 (producers only)
    const bool st0 = producer && ox < w;
    const bool st1 = producer && ox + 1 < w;
    const int iy0 = ys - A;                // first input row

    // Raw loads only: the edge fix-up (clamp-to-edge of a pair lying left or
    // right of the image) is applied when a row is CONSUMED, D rows later. Any
    // VALU use of a loaded register right after the load makes hipcc wait for it
    // there, which would drain the prefetch ring every iteration.
    const int cc = VEC ? mpx_clampi(cin, 0, w - 2) : 0;
    const bool pair_left = cin < 0, pair_right = cin >= w;
    // The sched_barrier pins every load at its program position: left alone the
    // scheduler sinks prefetches towards their first use (lower register
    // pressure), which turns the ring back into load-then-wait.
    const int iy_last = ye - 1 + (K - 1 - A);  // last input row (upward walk: input row 0)
    const int i_last = ye - ys + K - 2;          // the walk's last input row index
    auto load_row = [&](int i) -> uint2 {
        const int gy = mpx_clampi(up ? iy_last - i : iy0 + i, y_lo, y_hi);
        // wave-uniform row source select (scalar): own slab or a neighbour's
        const uint32_t *src = gy < 0 ? rs.up : (gy >= rs.own_rows ? rs.dn : in);
        const uint32_t *row = src + (int64_t)gy * pitch;
        uint2 r;
        if constexpr (VEC && BUFLD == 2) {  // non-temporal global load (A/B variant)
            typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
            const u32x2_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x2_t *>(row + cc));
            r = make_uint2(v.x, v.y);
        } else if constexpr (VEC && BUFLD == 0) {
            r = *reinterpret_cast<const uint2 *>(row + cc);
        } else if constexpr (VEC) {  // w even: the pair is entirely inside, left or right (BUFLD 1, 3)
            // buffer load: the row base lives in the (scalar) descriptor and the
            // lane's byte offset is loop-invariant — no per-row address VALU
            // (the ring's loads past the walk's last input row are never
            // consumed: out-of-range offset, dropped by the hardware)
            const __amdgpu_buffer_rsrc_t rrow = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(row), 0,
                                                                                  w * 4, 0x00020000);
            typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
            const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(rrow, i <= i_last ? cc * 4 : 0x7ffffff0, 0, 0);
            r = make_uint2(v.x, v.y);
        } else {
            r = make_uint2(row[mpx_clampi(cin, 0, w - 1)], row[mpx_clampi(cin + 1, 0, w - 1)]);
        }
        __builtin_amdgcn_sched_barrier(0);
        return r;
    };
    auto fix_pair = [&](uint2 q) -> uint2 {
        if constexpr (VEC) {
            uint2 p;
            p.x = pair_right ? q.y : q.x;
            p.y = pair_left ? q.x : q.y;
            return p;
        } else {
            return q;
        }
    };

    // Prefetch ring of D >= PF rows (a multiple of K so both rings keep
    // compile-time slots when the row loop is unrolled D times).
    constexpr int D = K * ((PF + K - 1) / K);
    uint2 pre[D];         // prefetch ring: raw pixels of input rows i .. i+D-1
    f2_t we[K][NE];       // window ring, even pairs (register-pair aligned for v_pk_fma_f32)
    f2_t wo[K][NO > 0 ? NO : 1];  // window ring, odd pairs
    f2_t hxr[K], hyr[K];  // separable filters: ring of per-row horizontal factor sums
    uint32_t alp0[K], alp1[K];  // raw source pixels of the centre row (alpha = byte 3)

    // consume the input row in window slot u: luminance (packed), alpha, and the
    // horizontal window w[0 .. NV-1] = columns cin-A .. cin+1+R from the
    // neighbouring lanes by DPP wave shifts
    auto consume = [&](int u, uint2 px) {
        const f2_t l = luma2(px.x, px.y);
        alp0[u] = px.x;  // raw pixel: v_perm takes its alpha byte at compose time
        alp1[u] = px.y;
        float wv[NV];
        wv[A] = l.x;
        wv[A + 1] = l.y;
        if constexpr (A >= 1) wv[A - 1] = from_prev(l.y);
        if constexpr (A >= 2) wv[A - 2] = from_prev(l.x);
        if constexpr (A >= 3) wv[A - 3] = from_prev(wv[A - 1]);
        if constexpr (G::R >= 1) wv[A + 2] = from_next(l.x);
        if constexpr (G::R >= 2) wv[A + 3] = from_next(l.y);
        if constexpr (G::R >= 3) wv[A + 4] = from_next(wv[A + 2]);
        if constexpr (SEP) {
            // the horizontal passes run once per input row; the K-row ring then
            // only holds their results (2 x K packed values, not the windows)
            auto pair = [&](int dx) { return f2_t{wv[dx], wv[dx + 1]}; };
            hxr[u] = sep_chain<F, K, 0>(taps, pair);
            if constexpr (TWO) hyr[u] = sep_chain<F, K, 2>(taps, pair);
        } else {
#pragma unroll
            for (int q = 0; q < NE; ++q) we[u][q] = f2_t{wv[2 * q], 2 * q + 1 < NV ? wv[2 * q + 1] : 0.0f};
#pragma unroll
            for (int q = 0; q < NO; ++q) wo[u][q] = f2_t{wv[2 * q + 1], wv[2 * q + 2]};
        }
    };

#pragma unroll
    for (int q = 0; q < D; ++q) pre[q] = load_row(q);
    // warm-up: rows 0 .. K-2 only fill the window
#pragma unroll
    for (int u = 0; u < K - 1; ++u) {
        const uint2 px = fix_pair(pre[u]);
        pre[u] = load_row(u + D);
        consume(u, px);
    }
    // steady state: every input row completes one output row. The row loop runs
    // in whole groups of D (ring slots are then compile-time constants) with no
    // branch around any memory operation; output rows past the segment end are
    // computed and dropped by the store's bounds check.
    // the ring slot of window row dy (0 = top) once input row index i (slot u)
    // is consumed: walking down the newest row is the bottom one, walking up
    // the top one; the tap chains always run top to bottom (bit-exactness)
    auto row_step = [&](auto upc, int g, int v) {
        constexpr bool UP = decltype(upc)::value;
        const int u = (K - 1 + v) % K;      // window slot of the newest row
        const int q = (K - 1 + v) % D;      // its prefetch slot
        const int i = K - 1 + g * D + v;    // its input row index
        const uint2 px = fix_pair(pre[q]);
        pre[q] = load_row(i + D);
        consume(u, px);
        const int y = UP ? ye - 1 - (g * D + v) : ys + g * D + v;  // output row completed by row i
        auto slot = [&](int dy) { return UP ? (u + K - dy) % K : (u + 1 + dy) % K; };
        // both output columns at once: packed FMAs over the (w[dx], w[dx+1]) pairs
        f2_t gx = {0.0f, 0.0f}, gy = {0.0f, 0.0f};
        if constexpr (SEP) {
            gx = sep_chain<F, K, 1>(taps, [&](int dy) { return hxr[slot(dy)]; });
            const float sx = sep_scale<F, K, false>(taps);
            gx = gx * f2_t{sx, sx};
            if constexpr (TWO) {
                gy = sep_chain<F, K, 3>(taps, [&](int dy) { return hyr[slot(dy)]; });
                const float sy = sep_scale<F, K, true>(taps);
                gy = gy * f2_t{sy, sy};
            }
        } else {
            bool sx = false, sy = false;
#pragma unroll
            for (int dy = 0; dy < K; ++dy) {
                const int r = slot(dy);
#pragma unroll
                for (int dx = 0; dx < K; ++dx) {
                    const f2_t pv = (dx & 1) ? wo[r][dx >> 1] : we[r][dx >> 1];
                    tap_step<F::kConst>(gx, sx, tap_x<F>(taps, dy * K + dx), pv);
                    if constexpr (TWO) tap_step<F::kConst>(gy, sy, tap_y<F>(taps, dy * K + dx), pv);
                }
            }
        }
        uint32_t g0, g1;
        if constexpr (TWO) {
            const f2_t sq = gx * gx + gy * gy;  // v_pk_mul x2, v_pk_add: no contraction (-ffp-contract=off)
            if constexpr (FAST) {
                mag2_to_gray(sq.x, sq.y, g0, g1);
            } else {
                g0 = mag_to_gray<false>(sq.x);
                g1 = mag_to_gray<false>(sq.y);
            }
        } else {
            g0 = finish_gray<MODE, FAST>(gx.x, 0.0f);
            g1 = finish_gray<MODE, FAST>(gx.y, 0.0f);
        }
        // (g, g, g, alpha): one v_perm_b32 per pixel — selector bytes 0-2
        // take g's low byte (g <= 255), byte 3 takes the source pixel's
        // alpha (selector 7 = byte 3 of the first operand); no alpha mask
        const uint32_t v0 = __builtin_amdgcn_perm(alp0[slot(A)], g0, 0x07000000u);
        const uint32_t v1 = __builtin_amdgcn_perm(alp1[slot(A)], g1, 0x07000000u);
        // Branch-free stores: a buffer descriptor spanning exactly this
        // output row; lanes (or padded rows) with nothing to store get an
        // out-of-range offset and the hardware bounds check drops them.
        // Stores under a branch would make the outstanding-op count
        // unknowable to hipcc and cost a vmcnt(0) drain of the ring.
        // rows past the segment get a zero-length descriptor (scalar select),
        // lanes with nothing to store a constant out-of-range offset
        const bool row_ok = UP ? y >= ys : y < ye;
        const int yc = row_ok ? y : ys;
        const __amdgpu_buffer_rsrc_t orow =
            __builtin_amdgcn_make_buffer_rsrc(out + (int64_t)yc * pitch, 0, row_ok ? w * 4 : 0, 0x00020000);
        constexpr int kDrop = 0x7ffffff0;
        if constexpr (VEC) {
            typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
            const u32x2_t pv = {v0, v1};
            // BUFLD 3 (tuning variant): non-temporal output stores (cache policy NT)
            __builtin_amdgcn_raw_buffer_store_b64(pv, orow, st0 ? ox * 4 : kDrop, 0, BUFLD == 3 ? 2 : 0);
        } else {
            __builtin_amdgcn_raw_buffer_store_b32(v0, orow, st0 ? ox * 4 : kDrop, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b32(v1, orow, st1 ? ox * 4 + 4 : kDrop, 0, 0);
        }
    };
    // whole groups with no branch between the rows (a branch there costs the
    // wait counts their precision), then the segment's last 1 .. D-1 rows with
    // a wave-uniform exit: rows past the segment are never computed
    const int nrows = ye - ys;
    const int nfull = nrows / D;
    const int rem = nrows - nfull * D;
    auto run = [&](auto upc) {
        for (int g = 0; g < nfull; ++g) {
#pragma unroll
            for (int v = 0; v < D; ++v) row_step(upc, g, v);
        }
        if (rem > 0) {
#pragma unroll
            for (int v = 0; v < D; ++v) {
                if (v >= rem) break;
                row_step(upc, nfull, v);
            }
        }
    };
    if (up) run(std::true_type{});  // wave-uniform branch
    else run(std::false_type{});
}

// ---------------------------------------------------------------------------
// Band kernel, 16-B lanes, no overlapping strips (separable and dense windows
// up to 5x5 with at most two columns of reach on each side).
//
// A 16-B-lane wave kernel with halo lanes (lanes 0 and 63 only loading halo
// columns, 248 of 256 columns produce; removed in round 2, numbers in
// profiles/lab2_conv.md) starts its strips at 992-B offsets, so every row piece
// straddles one more 128-B line than it needs. Here a wave owns exactly 256
// columns (x0 = 256 * strip): every lane loads and stores one aligned 16-B
// quad per row (the linear copy's request shape), and the four columns a strip
// needs beyond its edges come from one extra 8-B "apron" load per row that
// only lanes 0 (x0-2, x0-1) and 63 (x0+256, x0+257) issue — the other lanes'
// offsets are out of range and the hardware drops them. Waves run strip-minor
// with alternating segment directions (odd segments walk up, see
// conv_wave_kernel), which is what the row-band copy probe showed to be the
// HBM-friendly order (tools/kbench.py copy/band-*: 27.2 us rotated vs 29.1 us
// for the wave-strip copy). Clamp-to-edge needs no special code inside the
// image: quads right of the image replicate its last pixel (fix_quad), and the
// apron falls back to the lane's own edge pixel at x = 0 and x = w.
// Requires w % 4 == 0, pitch % 4 == 0 and 16-B aligned rows.
// ---------------------------------------------------------------------------
// Vertical halo sharing (conv_band16v_kernel): the LDS slots a wave exchanges
// its boundary rows through with the vertically adjacent waves of its
// workgroup (u32 offsets into the kernel's exchange array; < 0 = that side
// loads its halo rows from memory). A slot holds two raw rows (64 lanes x 16 B)
// plus the rows' 8-B aprons of lanes 0 and 63; a flag word per slot.
constexpr int kVsRowWords = 64 * 4 + 4;
constexpr int kVsSlotWords = 2 * kVsRowWords;
struct VsX {
    int take_start = -1, give_start = -1, take_end = -1, give_end = -1;  // slot offsets
    int ftake_start = 0, fgive_start = 0, ftake_end = 0, fgive_end = 0;  // flag offsets
};

// One wave's segment walk in one direction (UP: bottom row first), prologue
// included, so nothing but scalars is live across the direction branch.
// SPW (fused streaming halo, mpx_conv_stream_peer): an edge wave's walk — every
// row loads at system scope (the neighbours' mailbox rows change every step),
// and output rows 0 .. nf-1 / own_rows-nl .. own_rows-1 are also stored
// write-through into this rank's mailbox rows mbf / mbl (one extra store per
// row, dropped by the buffer bounds check on the other rows: no branch).
// VSEG > 0 (vertical halo sharing, conv_band16v_kernel): a full segment of
// exactly VSEG rows whose 2 + 2 halo rows come from the LDS slots in `vx`
// where a neighbouring wave of the workgroup owns them (those rows issue no
// memory load), and whose own first / last two rows go into the neighbours'
// slots; the walk is then fully unrolled. lds: the kernel's exchange array.
template <int K, int A, int MODE, bool FAST, class F, bool UP, int OPT, bool SPW = false, int VSEG = 0>
__device__ __forceinline__ void band4_walk(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                     int w, int pitch, int ys, int ye, int y_lo, int y_hi, int x0,
                                                     const Taps &taps, RowSrc rs, uint32_t *mbf = nullptr,
                                                     uint32_t *mbl = nullptr, int nf = 0, int nl = 0,
                                                     uint32_t *lds = nullptr, VsX vx = VsX{}) {
    constexpr int R = K - 1 - A;
    constexpr int NV = 4 + A + R;
    constexpr bool TWO = (MODE == MPX_CONV_MAG2);
    constexpr bool SEP = F::kSep;
    typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
    typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
    const int lane = threadIdx.x & 63;
    constexpr bool up = UP;
    // OPT bit 9 (HL, 248-column strips): lane l loads the quad at x0 - 4 + 4l;
    // lanes 0 and 63 only feed their neighbours through the DPP shifts (no
    // apron loads) and store nothing
    constexpr bool HL = (OPT & 512) != 0;
    const int cin = HL ? x0 - 4 + 4 * lane : x0 + 4 * lane;
    const bool st = HL ? (lane >= 1 && lane <= 62 && cin < w) : cin < w;
    const int cc = HL ? min(max(cin, 0), w - 4) : min(cin, w - 4);
    const bool q_right = cin >= w;
    const bool q_left = HL && cin < 0;  // strip 0, lane 0: clamp-to-edge replicates pixel 0
    // apron: lane 0 reads the two columns left of the strip, lane 63 the two
    // right of it; at the image edges the lane's own edge pixel stands in
    const bool ap_left = lane == 0, ap_right = lane == 63;
    // OPT bit 4 (cost probe only, wrong at strip edges): no apron loads
    const bool ap_have = !HL && !(OPT & 16) && ((ap_left && x0 > 0) || (ap_right && x0 + 256 < w));
    constexpr int kDrop = 0x7ffffff0;
    // DPP-old apron (every production instance; the HL / readlane-batched
    // (bit 3) / no-apron tuning probes keep the select form): lanes 0 / 63 feed their apron luma
    // as the `old` operand of the wave-shift DPP moves, the only lanes whose
    // shift has no source lane — no v_cndmask per window value. At the image
    // edges the lane loads its edge PAIR ((0, 1) / (w-2, w-1)) and one per-lane
    // byte select per apron pixel makes it (p0, p0) / (p[w-1], p[w-1]).
    constexpr bool kDppApron = (OPT & (8 | 16 | 512)) == 0;
    // OPT bit 11 (walks of at most 32 rows, the launcher checks): every apron
    // of the walk in ONE load up front, luma once; row i's lanes 0 / 63 then
    // fetch theirs with two ds_bpermute (the LDS crossbar, no VALU) — no
    // per-row apron load, luma or edge select. Not for the fused streaming
    // halo's edge walks (SPW): their mailbox rows need system-scope loads
    constexpr bool BPA = kDppApron && (OPT & 2048) != 0 && !SPW;
    const bool fix_l = kDppApron && ap_left && x0 == 0, fix_r = kDppApron && ap_right && x0 + 256 >= w;
    // (fix_r: lane 63's quad offset cc = w - 4 plus 8 B, not (w - 2) * 4 — a w * 4
    // in a VGPR would turn the uniform descriptor-size selects into v_cndmasks)
    const int ap_off = ap_have ? (ap_left ? x0 - 2 : x0 + 256) * 4 : (fix_l ? 0 : (fix_r ? cc * 4 + 8 : kDrop));
    const uint32_t ap_selx = fix_r ? 0x07060504u : 0x03020100u;  // perm(ap.y, ap.x, .): fix_r takes ap.y
    const uint32_t ap_sely = fix_l ? 0x03020100u : 0x07060504u;  // fix_l takes ap.x
    if constexpr (VSEG > 0) ye = ys + VSEG;  // (the caller's guarantee, made visible: every bound compile-time)
    const int iy0 = ys - A;
    const int iy_last = ye - 1 + R;
    auto row_ptr = [&](int i) {
        const int gy = mpx_clampi(up ? iy_last - i : iy0 + i, y_lo, y_hi);
        const uint32_t *src = gy < 0 ? rs.up : (gy >= rs.own_rows ? rs.dn : in);
        return src + (int64_t)gy * pitch;
    };
    // the prefetch ring runs D rows past the walk's last input row (nrows + K - 2);
    // those loads are never consumed: their descriptor is empty, so the
    // hardware drops them instead of fetching a neighbour segment's rows
    const int i_last = ye - ys + K - 2;
    static_assert(VSEG == 0 || (A == 2 && K == 5 && VSEG >= 8), "vertical sharing: 5-row windows, 2 + 2 halo rows");
    auto load_row = [&](int i, u32x2_t &ap) -> u32x4_t {
        const uint32_t *row = row_ptr(min(i, i_last));
        // wave-uniform; VSEG: rows an LDS slot delivers issue no memory access.
        // A dead row gets an empty descriptor (scalar), not dropped offsets: no
        // per-row v_cndmask on the lanes' (loop-invariant) offsets
        int nrec = scalar_le_sel(i, i_last, w * 4);
        if constexpr (VSEG > 0)
            nrec = ((i < 2 && vx.take_start >= 0) || (i >= VSEG + 2 && vx.take_end >= 0)) ? 0 : nrec;
        const __amdgpu_buffer_rsrc_t rr =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(row), 0, nrec, 0x00020000);
        const int qo = cc * 4, ao = ap_off;
        u32x4_t q;
        // OPT bit 5: rows no neighbouring segment reads (K-1 <= i < nrows) load
        // non-temporal; bit 6: every row does (probes)
        if constexpr (SPW) {  // fused streaming edge walk: mailbox rows change every step
            q = __builtin_amdgcn_raw_buffer_load_b128(rr, qo, 0, peer::kCpolSystem);
            ap = __builtin_amdgcn_raw_buffer_load_b64(rr, ao, 0, peer::kCpolSystem);
        } else if constexpr (HL) {  // no aprons
            q = __builtin_amdgcn_raw_buffer_load_b128(rr, qo, 0, 0);
            ap = u32x2_t{0u, 0u};
        } else if constexpr ((OPT & 8) != 0) {  // aprons come from the batch load
            q = __builtin_amdgcn_raw_buffer_load_b128(rr, qo, 0, (OPT & 64) ? 2 : 0);
        } else if constexpr (BPA) {  // aprons come from the batch load (bpermute form)
            if ((OPT & 32) && i >= K - 1 && i < ye - ys)
                q = __builtin_amdgcn_raw_buffer_load_b128(rr, qo, 0, 2);
            else
                q = __builtin_amdgcn_raw_buffer_load_b128(rr, qo, 0, 0);
            ap = u32x2_t{0u, 0u};
        } else if ((OPT & 64) || ((OPT & 32) && i >= K - 1 && i < ye - ys)) {
            q = __builtin_amdgcn_raw_buffer_load_b128(rr, qo, 0, 2);
            ap = __builtin_amdgcn_raw_buffer_load_b64(rr, ao, 0, (OPT & 128) ? 0 : 2);
        } else {
            q = __builtin_amdgcn_raw_buffer_load_b128(rr, qo, 0, 0);
            ap = __builtin_amdgcn_raw_buffer_load_b64(rr, ao, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        return q;
    };
    auto fix_quad = [&](u32x4_t q) -> u32x4_t {
        if constexpr ((OPT & 1024) != 0) return q;  // strip inside the image: no lane past w
        if constexpr (HL) {
            if (q_left) return u32x4_t{q.x, q.x, q.x, q.x};
        }
        return q_right ? u32x4_t{q.w, q.w, q.w, q.w} : q;
    };
    // OPT bit 3 (walks of at most 32 rows): every apron of the walk in ONE
    // load up front instead of one 8-B load per row. Lane j holds walk row
    // j >> 1's left (j even) or right (j odd) apron as two luma values; row
    // i's consumer reads lanes 2i / 2i+1 with v_readlane (wave-uniform i).
    f2_t ab = {0.0f, 0.0f};
    int bp_addr = 0;
    if constexpr (BPA) {
        const int nload = ye - ys + K - 1;  // <= 32
        const int j = lane >> 1;
        const bool side = lane & 1;  // 0: left apron (x0-2, x0-1), 1: right (x0+256, x0+257)
        const bool edge = side ? x0 + 256 >= w : x0 == 0;
        const int col = side ? (edge ? w - 2 : x0 + 256) : (edge ? 0 : x0 - 2);
        const u32x2_t v = *reinterpret_cast<const u32x2_t *>(row_ptr(min(j, nload - 1)) + col);
        // image edge: the edge pixel twice (clamp-to-edge)
        ab = luma2((edge && side) ? v.y : v.x, (edge && !side) ? v.x : v.y);
        bp_addr = ap_right ? 4 : 0;  // lane 63 reads lane 2i + 1 (right), the others lane 2i
    }
    if constexpr ((OPT & 8) != 0) {
        const int nload = ye - ys + K - 1;  // <= 32, checked by the launcher
        const int j = lane >> 1, side = lane & 1;
        const bool have = !(OPT & 16) && (side ? x0 + 256 < w : x0 > 0);
        const uint32_t *row = row_ptr(min(j, nload - 1));
        const u32x2_t v = *reinterpret_cast<const u32x2_t *>(row + (have ? (side ? x0 + 256 : x0 - 2) : 0));
        ab = luma2(v.x, v.y);
    }

    // prefetch ring of D >= 4 rows, a multiple of K (compile-time slots when
    // the row loop is unrolled D times)
    constexpr int D = K * ((4 + K - 1) / K);
    u32x4_t pre[D];
    u32x2_t apr[D];
    f2_t hxr[SEP ? K : 1][2], hyr[SEP ? K : 1][2];  // separable: per-row horizontal sums
    float win[SEP ? 1 : K][NV];                      // dense: per-row luminance windows
    // alpha bytes of each ring row, two pixels per register (byte 0 / 1: pixels
    // 0 / 1 of the lane's quad; 2 / 3 in alq): two v_perm per consumed row,
    // and the output's v_perm reads the byte straight from them
    uint32_t alp[K], alq[K];

    auto consume = [&](int u, u32x4_t px, u32x2_t ap, int ri) {
        const f2_t l01 = luma2(px.x, px.y), l23 = luma2(px.z, px.w);
        alp[u] = __builtin_amdgcn_perm(px.y, px.x, 0x0c0c0703u);
        alq[u] = __builtin_amdgcn_perm(px.w, px.z, 0x0c0c0703u);
        f2_t la;
        if constexpr ((OPT & 8) != 0) {
            auto rl = [&](float x, int l) {
                return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
            };
            const f2_t lft = {rl(ab.x, 2 * ri), rl(ab.y, 2 * ri)};
            const f2_t rgt = {rl(ab.x, 2 * ri + 1), rl(ab.y, 2 * ri + 1)};
            la = ap_left ? lft : rgt;
        } else if constexpr (BPA) {
            const int a = bp_addr + 8 * ri;
            la = f2_t{__int_as_float(__builtin_amdgcn_ds_bpermute(a, __float_as_int(ab.x))),
                      __int_as_float(__builtin_amdgcn_ds_bpermute(a, __float_as_int(ab.y)))};
        } else if constexpr (kDppApron) {
            la = luma2(__builtin_amdgcn_perm(ap.y, ap.x, ap_selx), __builtin_amdgcn_perm(ap.y, ap.x, ap_sely));
        } else {
            la = luma2(ap.x, ap.y);
        }
        float wv[NV];
        wv[A + 0] = l01.x;
        wv[A + 1] = l01.y;
        wv[A + 2] = l23.x;
        wv[A + 3] = l23.y;
        if constexpr (kDppApron) {
            // lane 0 (no lane to its left) keeps `old` = its left apron, lane
            // 63 (none to its right) its right apron
            if constexpr (A >= 1) wv[A - 1] = shift_or_old<kDppShr1>(la.y, l23.y);
            if constexpr (A >= 2) wv[A - 2] = shift_or_old<kDppShr1>(la.x, l23.x);
            if constexpr (R >= 1) wv[A + 4] = shift_or_old<kDppShl1>(la.x, l01.x);
            if constexpr (R >= 2) wv[A + 5] = shift_or_old<kDppShl1>(la.y, l01.y);
        } else {
            if constexpr (A >= 1) {
                const float d = from_prev(l23.y);
                wv[A - 1] = ap_left ? (ap_have ? la.y : l01.x) : d;
            }
            if constexpr (A >= 2) {
                const float d = from_prev(l23.x);
                wv[A - 2] = ap_left ? (ap_have ? la.x : l01.x) : d;
            }
            if constexpr (R >= 1) {
                const float d = from_next(l01.x);
                wv[A + 4] = ap_right ? (ap_have ? la.x : l23.y) : d;
            }
            if constexpr (R >= 2) {
                const float d = from_next(l01.y);
                wv[A + 5] = ap_right ? (ap_have ? la.y : l23.y) : d;
            }
        }
        if constexpr (SEP && kDppApron && A == 2 && R == 2) {
            // 5-wide windows: the seven packed operands (w[j], w[j+1]) as the
            // four aligned pairs plus three half-shifted ones (one v_pk_mov
            // each), instead of the compiler's per-element copies
            const f2_t e0 = {wv[0], wv[1]}, e3 = {wv[6], wv[7]};
            const f2_t pw[7] = {e0, __builtin_shufflevector(e0, l01, 1, 2), l01, __builtin_shufflevector(l01, l23, 1, 2),
                                l23, __builtin_shufflevector(l23, e3, 1, 2), e3};
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                auto pair = [&](int dx) { return pw[2 * e + dx]; };
                hxr[u][e] = sep_chain<F, K, 0>(taps, pair);
                if constexpr (TWO) hyr[u][e] = sep_chain<F, K, 2>(taps, pair);
            }
        } else if constexpr (SEP) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                auto pair = [&](int dx) { return f2_t{wv[2 * e + dx], wv[2 * e + dx + 1]}; };
                hxr[u][e] = sep_chain<F, K, 0>(taps, pair);
                if constexpr (TWO) hyr[u][e] = sep_chain<F, K, 2>(taps, pair);
            }
        } else {
#pragma unroll
            for (int j = 0; j < NV; ++j) win[u][j] = wv[j];
        }
    };

    // VSEG exchange: raw rows (fix_quad is applied by the reader, whose lanes
    // sit at the same columns) and lanes 0 / 63's aprons; a slot row r of a
    // walk row i: down walks keep the rows' image order, up walks reverse it
    auto vs_put = [&](int slot, int r, u32x4_t q, u32x2_t ap) {
        *reinterpret_cast<u32x4_t *>(lds + slot + r * kVsRowWords + 4 * lane) = q;
        if (ap_left || ap_right)
            *reinterpret_cast<u32x2_t *>(lds + slot + r * kVsRowWords + 256 + (ap_right ? 2 : 0)) = ap;
    };
    auto vs_get = [&](int slot, int r, u32x2_t &ap) -> u32x4_t {
        if (ap_left || ap_right)
            ap = *reinterpret_cast<const u32x2_t *>(lds + slot + r * kVsRowWords + 256 + (ap_right ? 2 : 0));
        return *reinterpret_cast<const u32x4_t *>(lds + slot + r * kVsRowWords + 4 * lane);
    };
    auto vs_flag = [&](int f) { __hip_atomic_store(lds + f, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP); };
    auto vs_wait = [&](int f) {
        while (__hip_atomic_load(lds + f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
            __builtin_amdgcn_s_sleep(1);
    };

#pragma unroll
    for (int q = 0; q < D; ++q) pre[q] = load_row(q, apr[q]);
    if constexpr (VSEG > 0) {
        // start of the walk: give this wave's first two rows (walk rows 2, 3) as
        // soon as they arrive, then take the neighbour's two (walk rows 0, 1) —
        // the neighbour does the same, so neither waits on the other's walk
        if (vx.give_start >= 0) {
            vs_put(vx.give_start, UP ? 1 : 0, pre[2], apr[2]);
            vs_put(vx.give_start, UP ? 0 : 1, pre[3], apr[3]);
            vs_flag(vx.fgive_start);
        }
        if (vx.take_start >= 0) {
            vs_wait(vx.ftake_start);
            pre[0] = vs_get(vx.take_start, UP ? 1 : 0, apr[0]);
            pre[1] = vs_get(vx.take_start, UP ? 0 : 1, apr[1]);
        }
    }
#pragma unroll
    for (int u = 0; u < K - 1; ++u) {
        const u32x4_t px = fix_quad(pre[u]);
        const u32x2_t ap = apr[u];
        pre[u] = load_row(u + D, apr[u]);
        consume(u, px, ap, u);
    }
    auto row_step = [&](int g, int v) {
        const int u = (K - 1 + v) % K;
        const int q = (K - 1 + v) % D;
        const int i = K - 1 + g * D + v;
        if constexpr (VSEG > 0) {
            // end of the walk: give the last two own rows (walk rows VSEG, VSEG+1)
            // as they are consumed, take the neighbour's two (VSEG+2, VSEG+3)
            if (vx.give_end >= 0 && (i == VSEG || i == VSEG + 1)) {
                vs_put(vx.give_end, UP ? (i == VSEG ? 1 : 0) : (i == VSEG ? 0 : 1), pre[q], apr[q]);
                if (i == VSEG + 1) vs_flag(vx.fgive_end);
            }
            if (vx.take_end >= 0 && (i == VSEG + 2 || i == VSEG + 3)) {
                if (i == VSEG + 2) vs_wait(vx.ftake_end);
                pre[q] = vs_get(vx.take_end, UP ? (i == VSEG + 2 ? 1 : 0) : (i == VSEG + 2 ? 0 : 1), apr[q]);
            }
        }
        const u32x4_t px = fix_quad(pre[q]);
        const u32x2_t ap = apr[q];
        pre[q] = load_row(i + D, apr[q]);
        consume(u, px, ap, i);
        const int y = UP ? ye - 1 - (g * D + v) : ys + g * D + v;
        auto slot = [&](int dy) { return UP ? (u + K - dy) % K : (u + 1 + dy) % K; };
        uint32_t gray[4];
        f2_t sq2[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            f2_t gx = {0.0f, 0.0f}, gy = {0.0f, 0.0f};
            if constexpr (SEP) {
                gx = sep_chain<F, K, 1>(taps, [&](int dy) { return hxr[slot(dy)][e]; });
                const float sx = sep_scale<F, K, false>(taps);
                gx = gx * f2_t{sx, sx};
                if constexpr (TWO) {
                    gy = sep_chain<F, K, 3>(taps, [&](int dy) { return hyr[slot(dy)][e]; });
                    const float sy = sep_scale<F, K, true>(taps);
                    gy = gy * f2_t{sy, sy};
                }
            } else {
                // (dy, dx) order, one fma per tap and output (conv_wave_kernel)
                bool sx = false, sy = false;
#pragma unroll
                for (int dy = 0; dy < K; ++dy) {
                    const int r = slot(dy);
#pragma unroll
                    for (int dx = 0; dx < K; ++dx) {
                        const f2_t pv = {win[r][2 * e + dx], win[r][2 * e + dx + 1]};
                        tap_step<F::kConst>(gx, sx, tap_x<F>(taps, dy * K + dx), pv);
                        if constexpr (TWO) tap_step<F::kConst>(gy, sy, tap_y<F>(taps, dy * K + dx), pv);
                    }
                }
            }
            if constexpr (TWO) {
                const f2_t sq = gx * gx + gy * gy;
                if constexpr (FAST) {
                    sq2[e] = sq;  // all four pixels at once below
                } else {
                    gray[2 * e] = mag_to_gray<false>(sq.x);
                    gray[2 * e + 1] = mag_to_gray<false>(sq.y);
                }
            } else {
                gray[2 * e] = finish_gray<MODE, FAST>(gx.x, 0.0f);
                gray[2 * e + 1] = finish_gray<MODE, FAST>(gx.y, 0.0f);
            }
        }
        if constexpr (TWO && FAST) mag4_to_gray(sq2[0], sq2[1], gray);
        const uint32_t a = alp[slot(A)], b = alq[slot(A)];
        u32x4_t o;
        o.x = __builtin_amdgcn_perm(a, gray[0], 0x04000000u);
        o.y = __builtin_amdgcn_perm(a, gray[1], 0x05000000u);
        o.z = __builtin_amdgcn_perm(b, gray[2], 0x04000000u);
        o.w = __builtin_amdgcn_perm(b, gray[3], 0x05000000u);
        const bool row_ok = UP ? y >= ys : y < ye;
        const int yc = row_ok ? y : ys;
        const __amdgpu_buffer_rsrc_t orow = __builtin_amdgcn_make_buffer_rsrc(
            out + (int64_t)yc * pitch, 0, UP ? scalar_le_sel(ys, y, w * 4) : scalar_le_sel(y, ye - 1, w * 4), 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(o, orow, st ? cin * 4 : kDrop, 0, (OPT & 2) ? 2 : 0);
        if constexpr (SPW) {
            const int own = rs.own_rows;
            const bool mf = mbf != nullptr && y < nf, ml = mbl != nullptr && y >= own - nl;  // wave-uniform
            uint32_t *mrow = mf ? mbf + (int64_t)y * w : (ml ? mbl + (int64_t)(y - (own - nl)) * w : out);
            const __amdgpu_buffer_rsrc_t mr =
                __builtin_amdgcn_make_buffer_rsrc(mrow, 0, (row_ok && (mf || ml)) ? w * 4 : 0, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(o, mr, st ? cin * 4 : kDrop, 0, peer::kCpolSystem);
        }
    };
    if constexpr (VSEG > 0) {  // ye - ys == VSEG: every row index compile-time
#pragma unroll
        for (int j = 0; j < VSEG; ++j) row_step(j / D, j % D);
        return;
    }
    const int nrows = ye - ys;
    const int nfull = nrows / D;
    const int rem = nrows - nfull * D;
    for (int g = 0; g < nfull; ++g) {
#pragma unroll
        for (int v = 0; v < D; ++v) row_step(g, v);
    }
    if (rem > 0) {
#pragma unroll
        for (int v = 0; v < D; ++v) {
            if (v >= rem) break;
            row_step(nfull, v);
        }
    }
}

// OPT (tuning variants): bit 0 caps registers for 5 waves per SIMD, bit 1
// non-temporal output stores, bit 2 16-wave workgroups (a band row's 16 strips
// of a 4096-wide image on one CU), bit 4 no apron loads (cost probe: wrong
// results at the strip edges), bit 5 non-temporal loads of rows no neighbouring
// segment reads, bit 6 non-temporal loads of every row, bit 7 keeps the apron
// loads plain under bit 5 / 6, bit 3 one batched apron load per walk (walks of
// at most 32 rows: segment + K - 1 <= 32), bit 9 248-column strips with halo
// lanes instead of aprons, bit 11 batched aprons fetched per row by
// ds_bpermute (walks of at most 32 rows; the production launch for segments
// of at most 28 rows). Bit 10 is internal (set per wave for strips inside the
// image, see the end of the kernel).
template <int K, int A, int MODE, bool FAST, class F, int OPT = 0, bool SP = false>
__global__ __launch_bounds__((OPT & 4) ? 1024 : 256) __attribute__((amdgpu_waves_per_eu((OPT & 1) ? 5 : 1))) void conv_band4_kernel(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                         int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
                                                         int seg, int nwaves, int strips, int alt, Taps taps,
                                                         RowSrc rs, mpx_conv_stream_peer sp) {
    static_assert(A <= 2 && K - 1 - A <= 2, "apron covers two columns on each side");
    constexpr int WPB = (OPT & 4) ? 16 : 4;
    const int gw = xcd_remap(blockIdx.x, gridDim.x) * WPB + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (gw >= nwaves) return;  // wave-uniform
    const int strip = gw % strips;
    const int segs = nwaves / strips;  // nwaves = strips * segs
    // alt bit 1 (slab with rows in a neighbour's HBM, RowSrc): both boundary
    // segments first — their halo loads go over xGMI, the slowest of the
    // launch, so their waves start in the first round (as in conv_wave_kernel)
    const int sg0 = gw / strips;
    const int sg = (!(alt & 2) || segs < 3 || sg0 == 0) ? sg0 : (sg0 == 1 ? segs - 1 : sg0 - 1);
    const int ys = oy0 + sg * seg;
    const int ye = min(ys + seg, oy1);
    constexpr int SW = (OPT & 512) ? 248 : 256;  // output columns per strip
    if constexpr (SP) {
        // fused streaming halo: a wave whose rows touch a slab edge that has a
        // neighbour (reads its rows, or writes rows it reads) is an edge wave
        constexpr int R = K - 1 - A;
        const bool top = sp.up_flag != nullptr && (ys - A < 0 || ys < sp.n_first);
        const bool bot = sp.dn_flag != nullptr && (ye - 1 + R >= rs.own_rows || ye > rs.own_rows - sp.n_last);
        if (top || bot) {  // wave-uniform
            // completed steps of this rank = the index of this step (bumped only after
            // every edge wave of the step has finished: no edge wave reads it bumped)
            const uint32_t c = __hip_atomic_load(sp.sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // a neighbour at >= c finished its step c - 1: its output frame c is in its
            // mailbox slot c & 1 (read-after-write), and it no longer reads this
            // rank's slot (c + 1) & 1, which this step overwrites (write-after-read)
            if (top) peer::wait_at_least(sp.up_flag, c, sp.sync + 64, sp.spin_limit);
            if (bot) peer::wait_at_least(sp.dn_flag, c, sp.sync + 64, sp.spin_limit);
            if (sp.up_flag) rs.up = sp.up_src[c & 1u];
            if (sp.dn_flag) rs.dn = sp.dn_src[c & 1u];
            uint32_t *mbf = top ? sp.mb_first[(c + 1) & 1u] : nullptr;
            uint32_t *mbl = bot ? sp.mb_last[(c + 1) & 1u] : nullptr;
            if ((alt & 1) && (sg & 1))
                band4_walk<K, A, MODE, FAST, F, true, OPT, true>(in, out, w, pitch, ys, ye, y_lo, y_hi, strip * SW,
                                                                 taps, rs, mbf, mbl, sp.n_first, sp.n_last);
            else
                band4_walk<K, A, MODE, FAST, F, false, OPT, true>(in, out, w, pitch, ys, ye, y_lo, y_hi, strip * SW,
                                                                  taps, rs, mbf, mbl, sp.n_first, sp.n_last);
            // every write-through store of this wave acknowledged, then count the
            // wave; the last edge wave of the step publishes c + 1 (release). The
            // count is acq_rel at system scope: each wave's increment
            // releases its own mailbox rows and the last wave acquires them all
            // before its publish, whatever memory kind the mailbox fell back to
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if ((threadIdx.x & 63) == 0) {
                const uint32_t n = __hip_atomic_fetch_add(sp.sync + 32, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
                if (n + 1 == (uint32_t)sp.n_edge) {
                    __hip_atomic_store(sp.sync + 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    peer::publish(sp.sync, c + 1);
                }
            }
            return;
        }
    }
    // wave-uniform: odd segments walk up; strips wholly inside the image (every
    // strip when w % 256 == 0) skip the per-row clamp of lanes past w (OPT bit
    // 10). (A fully unrolled walk for the flagship's 16-row segments cut the
    // loop-carried ring copies — 8.38M VALU per frame against 8.5M — but ran
    // the burst 2-5 % slower: 20 KB of straight-line code per walk against a
    // 5-row loop body; profiles/lab2_conv.md, round 6.)
    constexpr int OIN = (OPT & 512) ? OPT : (OPT | 1024);
    const bool inside = !(OPT & 512) && strip * SW + 256 <= w;
    const bool up = (alt & 1) && (sg & 1);
    if (up) {
        if (inside)
            band4_walk<K, A, MODE, FAST, F, true, OIN>(in, out, w, pitch, ys, ye, y_lo, y_hi, strip * SW, taps, rs);
        else
            band4_walk<K, A, MODE, FAST, F, true, OPT>(in, out, w, pitch, ys, ye, y_lo, y_hi, strip * SW, taps, rs);
    } else {
        if (inside)
            band4_walk<K, A, MODE, FAST, F, false, OIN>(in, out, w, pitch, ys, ye, y_lo, y_hi, strip * SW, taps, rs);
        else
            band4_walk<K, A, MODE, FAST, F, false, OPT>(in, out, w, pitch, ys, ye, y_lo, y_hi, strip * SW, taps, rs);
    }
}

// ---------------------------------------------------------------------------
// Band kernel with VERTICAL halo sharing (LDS): a 16-wave
// workgroup owns 16 vertically consecutive VSEG-row segments of one 256-column
// strip (one resident workgroup per CU at the band kernel's 4 waves per SIMD).
// The 2 + 2 halo rows a segment shares with the segment above / below are
// loaded ONCE, by the wave that owns them, and handed to the neighbour through
// LDS (~62 KiB of row slots; the alternating walk directions make each pair
// of neighbours reach their shared rows at the same moment: at the start of
// both walks or at the end of both). Only the workgroup's outer boundaries
// read halo rows from memory — 4 per 16 x VSEG rows instead of 4 per VSEG —
// so every row load can be non-temporal. Copy probe of this traffic
// (tools/kbench.py copy/band-seg16-f106 vs f74, NT loads): 25.25 vs 26.47 us.
// Segments that are not full (the image's last) and their neighbours fall back
// to the memory halo walk. Results are bit-identical to conv_band4_kernel (the
// same consume / tap order; only where a row's bytes come from changes).
// ---------------------------------------------------------------------------
template <int K, int A, int MODE, bool FAST, class F, int VSEG>
__global__ __launch_bounds__(1024) void conv_band16v_kernel(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                            int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
                                                            int segs, int strips, Taps taps) {
    constexpr int NB = 15;  // boundaries between the 16 waves
    __shared__ __attribute__((aligned(16))) uint32_t xlds[2 * NB * kVsSlotWords + 2 * NB];
    constexpr int kFlag0 = 2 * NB * kVsSlotWords;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < 2 * NB) xlds[kFlag0 + threadIdx.x] = 0u;
    __syncthreads();  // before any wave can exit or exchange
    const int strip = blockIdx.x % strips;
    const int sg = (blockIdx.x / strips) * 16 + wv;
    if (sg >= segs) return;  // wave-uniform; nobody exchanges with it (not full)
    const int ys = oy0 + sg * VSEG;
    const int ye = min(ys + VSEG, oy1);
    auto full = [&](int g) { return g >= 0 && g < segs && oy0 + (g + 1) * VSEG <= oy1; };
    const bool me = full(sg);
    const bool top = me && wv > 0 && full(sg - 1);    // exchange with the wave above (boundary wv - 1)
    const bool bot = me && wv < 15 && full(sg + 1);   // with the wave below (boundary wv)
    // slot (boundary b, side s): s = 0 holds the upper wave's last two rows, s = 1
    // the lower wave's first two rows; flags in the same (b, s) order
    auto slot = [](int b, int s) { return (2 * b + s) * kVsSlotWords; };
    auto flag = [](int b, int s) { return kFlag0 + 2 * b + s; };
    const bool upw = sg & 1;  // odd segments walk up (as conv_band4_kernel with alt = 1)
    VsX vx;
    // a down walk starts at its top and ends at its bottom, an up walk the reverse
    const bool st_nb = upw ? bot : top, en_nb = upw ? top : bot;
    const int bs = upw ? wv : wv - 1, be = upw ? wv - 1 : wv;  // boundaries at the start / end side
    if (st_nb) {
        // start side: down walk = the boundary above (take s = 0, give s = 1), up walk = below (take 1, give 0)
        vx.take_start = slot(bs, upw ? 1 : 0);
        vx.give_start = slot(bs, upw ? 0 : 1);
        vx.ftake_start = flag(bs, upw ? 1 : 0);
        vx.fgive_start = flag(bs, upw ? 0 : 1);
    }
    if (en_nb) {
        vx.take_end = slot(be, upw ? 0 : 1);
        vx.give_end = slot(be, upw ? 1 : 0);
        vx.ftake_end = flag(be, upw ? 0 : 1);
        vx.fgive_end = flag(be, upw ? 1 : 0);
    }
    constexpr int OPT = 2 | 64;  // NT stores, every row load non-temporal
    RowSrc rs;
    rs.up = in;  // whole-image or resident-halo launches: every row is `in`'s
    rs.dn = in;
    if (me) {
        if (upw)
            band4_walk<K, A, MODE, FAST, F, true, OPT, false, VSEG>(in, out, w, pitch, ys, ye, y_lo, y_hi, strip * 256,
                                                                    taps, rs, nullptr, nullptr, 0, 0, xlds, vx);
        else
            band4_walk<K, A, MODE, FAST, F, false, OPT, false, VSEG>(in, out, w, pitch, ys, ye, y_lo, y_hi,
                                                                     strip * 256, taps, rs, nullptr, nullptr, 0, 0,
                                                                     xlds, vx);
    } else {  // a partial segment: the memory halo walk
        if (upw)
            band4_walk<K, A, MODE, FAST, F, true, 34>(in, out, w, pitch, ys, ye, y_lo, y_hi, strip * 256, taps, rs);
        else
            band4_walk<K, A, MODE, FAST, F, false, 34>(in, out, w, pitch, ys, ye, y_lo, y_hi, strip * 256, taps, rs);
    }
}

// Gray value packing helper for the non-stream kernels.
template <int MODE, bool FAST>
__device__ __forceinline__ uint32_t gray_px(float gx, float gy, uint32_t a) {
    return mpx_px_gray(finish_gray<MODE, FAST>(gx, gy), a);
}

}  // namespace edge
}  // namespace mpx
