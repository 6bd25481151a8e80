// Tuning-only entry points of the lab2 kernels (tools/kbench.py): kernel
// variants by kind / rows per segment / fast magnitude, and the exhaustive
// fast-sqrt self-test. Built into libmpx_tune.so (make tune), never into
// libmpx: the production library exports no tuning entry points.
#include "../src/kernels/edge_launch.hpp"

namespace mpx {
using edge::Taps;
using edgel::launch_stream;
using edgel::launch_wave;
using edgel::make_taps;
namespace {

// Exhaustive self-test of the fast magnitude path: every float s in
// [0, 65025] (bit patterns 0 .. 0x477E0100) must map to the same gray level as
// the correctly rounded sqrtf. Counts mismatches into *bad.
// raw = 0: the single-pixel fast path (v_sqrt + fract margin + exact fallback);
// raw = 1: bare truncation of v_sqrt_f32 with no margin test at all;
// raw = 2: the paired production path of the band / wave kernels
// (mag2_to_gray: v_med3 clamp into [0.5^2, 255.5^2], margin test on both
// lanes, one exact fallback for the pair) — lane pairs (s, s') with s' walking
// the range backwards, so every value meets fast and fallback partners;
// raw = 3: the four-pixel production path of the band kernels (mag4_to_gray:
// no float->int conversion, the gray level in the low byte of 2^23 + n) — each
// value with three partners (walking backwards, and the two mirrors about the
// range's quarter points), only the low byte compared.
__global__ void fast_sqrt_selftest_kernel(uint32_t first, uint32_t last, unsigned long long *bad, int raw) {
    const uint32_t stride = gridDim.x * blockDim.x;
    unsigned long long nbad = 0;
    for (uint32_t u = first + blockIdx.x * blockDim.x + threadIdx.x; u <= last && u >= first; u += stride) {
        const float s = __builtin_bit_cast(float, u);
        const uint32_t exact = edge::mag_to_gray<false>(s);
        if (raw == 3) {
            const uint32_t n = last - first, k = u - first;
            const float s1 = __builtin_bit_cast(float, last - k);
            const float s2 = __builtin_bit_cast(float, first + (k + n / 4) % (n + 1));
            const float s3 = __builtin_bit_cast(float, first + (k + 3 * (n / 4)) % (n + 1));
            uint32_t g[4];
            edge::mag4_to_gray(edge::f2_t{s, s1}, edge::f2_t{s2, s3}, g);
            nbad += ((g[0] & 255u) != exact) + ((g[1] & 255u) != edge::mag_to_gray<false>(s1)) +
                    ((g[2] & 255u) != edge::mag_to_gray<false>(s2)) + ((g[3] & 255u) != edge::mag_to_gray<false>(s3));
            continue;
        }
        if (raw == 2) {
            const float s1 = __builtin_bit_cast(float, last - (u - first));
            uint32_t g0, g1;
            edge::mag2_to_gray(s, s1, g0, g1);
            nbad += (g0 != exact) + (g1 != edge::mag_to_gray<false>(s1));
            continue;
        }
        const uint32_t fast = raw ? (uint32_t)__builtin_amdgcn_sqrtf(fminf(s, 65025.0f)) : edge::mag_to_gray<true>(s);
        nbad += fast != exact;
    }
    if (nbad) atomicAdd(bad, nbad);
}

// Memory-pattern probe: the wave-strip streaming order of conv_wave_kernel with
// no arithmetic (copy in -> out). V = 32-bit pixels per lane (2: 8-B loads,
// 4: 16-B loads), ring of D rows in flight per wave.
template <int V, int D, int WPB = 4>
__global__ __launch_bounds__(64 * WPB) void strip_copy_kernel(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                         int w, int h, int seg, int nwaves, int strips) {
    typedef uint32_t vt __attribute__((ext_vector_type(V)));
    const int lane = threadIdx.x & 63;
    const int gw = xcd_remap(blockIdx.x, gridDim.x) * WPB + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (gw >= nwaves) return;
    const int strip = gw % strips, sg = gw / strips;
    const int ys = sg * seg, ye = min(ys + seg, h);
    const int col = strip * 64 * V + V * lane;
    const int cc = min(col, w - V);
    vt ring[D];
#pragma unroll
    for (int q = 0; q < D; ++q) ring[q] = *reinterpret_cast<const vt *>(in + (int64_t)min(ys + q, h - 1) * w + cc);
    const int ngroups = (ye - ys + D - 1) / D;
    for (int g = 0; g < ngroups; ++g) {
#pragma unroll
        for (int v = 0; v < D; ++v) {
            const int y = ys + g * D + v;
            const vt px = ring[v];
            ring[v] = *reinterpret_cast<const vt *>(in + (int64_t)min(y + D, h - 1) * w + cc);
            __builtin_amdgcn_sched_barrier(0);
            const bool ok = y < ye && col < w;
            const __amdgpu_buffer_rsrc_t orow =
                __builtin_amdgcn_make_buffer_rsrc(out + (int64_t)(ok ? y : ys) * w, 0, w * 4, 0x00020000);
            if constexpr (V == 2) __builtin_amdgcn_raw_buffer_store_b64(px, orow, ok ? col * 4 : 0x7ffffff0, 0, 0);
            else __builtin_amdgcn_raw_buffer_store_b128(px, orow, ok ? col * 4 : 0x7ffffff0, 0, 0);
        }
    }
}

// Linear-copy floor for the same bytes (v = 0 in the probe): one 16-B vector
// per thread like lab1's vsub (its best HBM pattern), plain or non-temporal.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ __launch_bounds__(256) void linear_copy_kernel(const u32x4_t *__restrict__ in, u32x4_t *__restrict__ out,
                                                          int64_t nvec) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nvec) return;
    if constexpr (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(in + i), out + i);
    else out[i] = in[i];
}

// Row-band probe (v = 8): a 16-wave workgroup owns a band of R rows across
// 4096 columns, one 16-B vector per thread per row (the linear copy's request
// shape), walking the band's R + 4 rows (5-row vertical window, 2 halo rows
// each side) with an 8-row register ring. out[y] = in[y-2] ^ in[y] ^ in[y+2]
// keeps every halo load live. F bit 0: per-row LDS exchange with the
// neighbouring thread + barrier (the horizontal pass's cost); bit 1: odd
// bands walk upwards; bit 2: no XCD remap; bit 3: non-temporal stores;
// bit 4: 512-thread workgroups over 2048 columns; bit 5: no halo loads;
// bit 6: non-temporal loads (the linear NT copy's load policy).
template <int F>
__global__ __launch_bounds__(1024) void band_copy_kernel(const u32x4_t *__restrict__ in, u32x4_t *__restrict__ out,
                                                         int w4, int h, int R, int nchunks) {
    __shared__ uint32_t xch[2][1025];
    const int b = (F & 4) ? (int)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
    const int band = b / nchunks, chunk = b - band * nchunks;
    const int t = threadIdx.x;
    const int c = chunk * (int)blockDim.x + t;
    const int ys = band * R, ye = min(ys + R, h);
    const bool up = (F & 2) && (band & 1);
    auto row_of = [&](int j) {  // j-th row of the walk (j = 0 .. R+3), clamped to the image
        const int y = up ? ye + 1 - j : ys - 2 + j;
        return min(max(y, 0), h - 1);
    };
    // bit 5: no halo loads (the walk's 2 + 2 halo rows read as zero): the
    // traffic of a band whose halo rows come from its neighbours through LDS
    auto ld = [&](int j) {
        if ((F & 32) && (j < 2 || j > R + 1)) return u32x4_t{0u, 0u, 0u, 0u};
        if constexpr ((F & 64) != 0) return __builtin_nontemporal_load(in + (int64_t)row_of(min(j, R + 3)) * w4 + c);
        return in[(int64_t)row_of(min(j, R + 3)) * w4 + c];
    };
    u32x4_t r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = ld(j);
    for (int g = 0; g < R; g += 8) {
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            u32x4_t o = r[v] ^ r[(v + 2) & 7] ^ r[(v + 4) & 7];
            if constexpr (F & 1) {
                xch[v & 1][t] = o.x;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                o.y ^= xch[v & 1][t + 1];
            }
            const int j = g + v + 2;  // output walk index -> row
            if (g + v < ye - ys) {
                if constexpr (F & 8) __builtin_nontemporal_store(o, out + (int64_t)row_of(j) * w4 + c);
                else out[(int64_t)row_of(j) * w4 + c] = o;
            }
            r[v] = ld(g + v + 8);
        }
    }
}

// Burst-tile probe (v = 16): a workgroup of T threads owns
// a tile of 4T columns x R output rows, every lane ONE aligned 16-B quad per
// row; it issues all R + 4 row loads of its column at once (no walking ring),
// then stores R rows (out[y] = in[y-2] ^ in[y] ^ in[y+2] keeps every halo load
// live) and exits. Tiles are many rounds deep, so the dispatcher sweeps the
// in-flight window down the image the way the linear copy does. F bit 0:
// xcd_remap (each XCD sweeps a contiguous eighth of the tiles, vertical
// neighbours share its L2), else blockIdx order (one window over all XCDs);
// bit 1: non-temporal loads; bit 2: non-temporal stores; bit 3: 96 KiB of
// (idle) LDS per workgroup, so one workgroup per CU is resident and the tiles
// run in several rounds (a compact in-flight window even at large R).
template <int R, int F>
__global__ __launch_bounds__(1024) void burst_copy_kernel(const u32x4_t *__restrict__ in, u32x4_t *__restrict__ out,
                                                          int w4, int h, int tpr) {
    if constexpr ((F & 8) != 0) {
        __shared__ uint32_t cap[96 * 256];  // residency cap only
        if (threadIdx.x == 0) cap[h & 1023] = (uint32_t)h;
        __syncthreads();
        if (cap[h & 1023] == 0xdeadbeefu) out[0] = u32x4_t{0u, 0u, 0u, 0u};  // never (h < 2^31): keeps the array
    }
    const int b = (F & 1) ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int band = b / tpr, chunk = b - band * tpr;
    const int c = chunk * (int)blockDim.x + (int)threadIdx.x;
    const int ys = band * R;
    u32x4_t r[R + 4];
#pragma unroll
    for (int j = 0; j < R + 4; ++j) {
        const int y = min(max(ys - 2 + j, 0), h - 1);
        if constexpr ((F & 2) != 0) r[j] = __builtin_nontemporal_load(in + (int64_t)y * w4 + c);
        else r[j] = in[(int64_t)y * w4 + c];
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
        if (ys + j >= h) break;
        const u32x4_t o = r[j] ^ r[j + 2] ^ r[j + 4];
        if constexpr ((F & 4) != 0) __builtin_nontemporal_store(o, out + (int64_t)(ys + j) * w4 + c);
        else out[(int64_t)(ys + j) * w4 + c] = o;
    }
}

}  // namespace

extern "C" int mpx_strip_copy_probe(const uint32_t *in, uint32_t *out, int w, int h, int v, int d, int seg,
                                    void *stream) {
    using namespace mpx;
    MPX_CHECK_ARG(in && out && w > 0 && h > 0 && w % 4 == 0, "bad arguments");
    hipStream_t s0 = as_stream(stream);
    if (v == 0) {  // linear copy: d = 0 plain, 1 non-temporal
        const int64_t nvec = (int64_t)w * h / 4;
        const dim3 g((unsigned)((nvec + 255) / 256)), b(256);
        if (d) hipLaunchKernelGGL(linear_copy_kernel<true>, g, b, 0, s0, (const u32x4_t *)in, (u32x4_t *)out, nvec);
        else hipLaunchKernelGGL(linear_copy_kernel<false>, g, b, 0, s0, (const u32x4_t *)in, (u32x4_t *)out, nvec);
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
        return MPX_OK;
    }
    MPX_CHECK_ARG(seg > 0, "seg must be > 0");
    if (v == 16) {  // burst tiles: seg = R output rows per tile, d = F | (threads code << 4)
        const int tcode = (d >> 4) & 3, F = d & 15;
        MPX_CHECK_ARG(tcode <= 2, "burst probe: threads code 0 / 1 / 2 = 256 / 512 / 1024");
        const int tpb = 256 << tcode;
        MPX_CHECK_ARG(w % (4 * tpb) == 0, "burst probe: w %% (4 * threads) == 0");
        const int tpr = w / (4 * tpb), nb = (h + seg - 1) / seg;
        const dim3 g((unsigned)(nb * tpr)), b(tpb);
        const u32x4_t *vi = (const u32x4_t *)in;
        u32x4_t *vo = (u32x4_t *)out;
#define MPX_BURST_F(RR, FF) \
    case FF: hipLaunchKernelGGL((burst_copy_kernel<RR, FF>), g, b, 0, s0, vi, vo, w / 4, h, tpr); break;
#define MPX_BURST(RR)                                                                                            \
    case RR:                                                                                                     \
        switch (F) {                                                                                             \
            MPX_BURST_F(RR, 0) MPX_BURST_F(RR, 1) MPX_BURST_F(RR, 2) MPX_BURST_F(RR, 3) MPX_BURST_F(RR, 4)       \
            MPX_BURST_F(RR, 5) MPX_BURST_F(RR, 6) MPX_BURST_F(RR, 7) MPX_BURST_F(RR, 13) MPX_BURST_F(RR, 15)     \
        }                                                                                                        \
        break;
        switch (seg) {
            MPX_BURST(2) MPX_BURST(4) MPX_BURST(8) MPX_BURST(12) MPX_BURST(16) MPX_BURST(24)
            default: set_error("unsupported burst rows %d", seg); return MPX_ERR_ARG;
        }
#undef MPX_BURST
#undef MPX_BURST_F
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
        return MPX_OK;
    }
    if (v == 8) {  // row bands: seg = rows per band (multiple of 8), d = flag bits
        MPX_CHECK_ARG(w % 4096 == 0 && seg % 4 == 0 && d >= 0 && d < 128, "band probe: w % 4096 == 0, seg % 4 == 0");
        const int tpb = (d & 16) ? 512 : 1024;
        const int nchunks = w / (4 * tpb), nb = (h + seg - 1) / seg;
        const dim3 g((unsigned)(nb * nchunks)), b(tpb);
        const u32x4_t *vi = (const u32x4_t *)in;
        u32x4_t *vo = (u32x4_t *)out;
        hipStream_t sb = as_stream(stream);
        switch (d) {
#define MPX_BAND(F) \
    case F: hipLaunchKernelGGL(band_copy_kernel<F>, g, b, 0, sb, vi, vo, w / 4, h, seg, nchunks); break;
            MPX_BAND(0) MPX_BAND(1) MPX_BAND(2) MPX_BAND(3) MPX_BAND(4) MPX_BAND(10) MPX_BAND(11) MPX_BAND(18)
            MPX_BAND(19) MPX_BAND(26) MPX_BAND(34) MPX_BAND(42) MPX_BAND(72) MPX_BAND(74) MPX_BAND(106)
            default: set_error("unsupported band flags %d", d); return MPX_ERR_ARG;
#undef MPX_BAND
        }
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
        return MPX_OK;
    }
    // d >= 100: 16 waves per workgroup (d - 100 rows in flight) instead of 4 —
    // the strips of one row band then start and advance together
    const int wpb = d >= 100 ? 16 : 4;
    if (d >= 100) d -= 100;
    const int strips = (w + 64 * v - 1) / (64 * v);
    const int nwaves = strips * ((h + seg - 1) / seg);
    const dim3 grid((nwaves + wpb - 1) / wpb), blk(64 * wpb);
    hipStream_t s = as_stream(stream);
#define MPX_PROBE(VV, DD)                                                                                             \
    if (v == VV && d == DD) {                                                                                        \
        if (wpb == 16)                                                                                              \
            hipLaunchKernelGGL((strip_copy_kernel<VV, DD, 16>), grid, blk, 0, s, in, out, w, h, seg, nwaves, strips); \
        else                                                                                                         \
            hipLaunchKernelGGL((strip_copy_kernel<VV, DD>), grid, blk, 0, s, in, out, w, h, seg, nwaves, strips);     \
        return MPX_OK;                                                                                               \
    }
    MPX_PROBE(2, 4) MPX_PROBE(2, 8) MPX_PROBE(4, 4) MPX_PROBE(4, 8) MPX_PROBE(4, 2)
#undef MPX_PROBE
    set_error("unsupported probe v=%d d=%d", v, d);
    return MPX_ERR_ARG;
}

}  // namespace mpx

// Variant entry for the tuning harness (tools/kbench.py), k in {2, 5}, MAG2,
// whole image, fast magnitude path unless fast == 0:
//   kind 0: LDS streaming kernel, p1 = rows per wave (4, 8, 16), p2 = tiles per workgroup (0 = auto)
//   kind 1: wave-streaming kernel, p1 = rows per wave segment
extern "C" int mpx_conv_variant(const uint32_t *in, uint32_t *out, int w, int h, int k, int kind, int p1, int p2,
                                int fast, const float *wx, const float *wy, void *stream) {
    using namespace mpx;
    MPX_CHECK_ARG(in && out && wx && wy && w > 0 && h > 0, "bad arguments");
    MPX_CHECK_ARG(k == 2 || k == 5, "variant harness covers k = 2 and k = 5");
    hipStream_t s = as_stream(stream);
    if (kind == 3 || kind == 4) {
        // separable sobel5 (wx / wy = MPX_CONV_SEP factors): kind 3 compiled-in
        // factors, kind 4 runtime factors; p1 = segment rows, p2 >= 1000 strip-major
        MPX_CHECK_ARG(k == 5 && p1 >= 0, "separable variants: k = 5, segment rows >= 0 (0 = auto)");
        const Taps st = make_taps(k, wx, wy, true, true);
        const bool vec2 = (w % 2 == 0) && ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 7u) == 0;
        // p2 in [1000, 2000): strip-major; [2000, 3000): strip-minor with
        // alternating segment direction (the production MAG2 order)
        const int sm = p2 >= 2000 ? 3 : p2 >= 1000 ? 0 : 1;
        // p2 % 1000 = minimum prefetch depth in rows (0 / 4: production 5, 8: 10, 12: 15)
        const int pf = p2 % 1000;
        if (kind == 3 && pf == 8)
            return launch_wave<5, 2, MPX_CONV_MAG2, true, edge::Sobel5SepTaps, 0, 8>(in, out, w, w, 0, h, 0, h - 1, st, vec2, s, p1, sm);
        if (kind == 3 && pf == 12)
            return launch_wave<5, 2, MPX_CONV_MAG2, true, edge::Sobel5SepTaps, 0, 12>(in, out, w, w, 0, h, 0, h - 1, st, vec2, s, p1, sm);
        if (kind == 3)
            return launch_wave<5, 2, MPX_CONV_MAG2, true, edge::Sobel5SepTaps>(in, out, w, w, 0, h, 0, h - 1, st, vec2, s, p1, sm);
        return launch_wave<5, 2, MPX_CONV_MAG2, true, edge::RuntimeSepTaps>(in, out, w, w, 0, h, 0, h - 1, st, vec2, s, p1, sm);
    }
    if (kind == 6 || kind == 7) {
        // A/B of the row loads: kind 6 separable sobel5, kind 7 Roberts, both
        // compiled-in taps; p2 = 1 plain global loads, 0 buffer loads (production)
        MPX_CHECK_ARG(p1 >= 0 && w % 2 == 0, "A/B variant: even width");
        const bool sep = kind == 6;
        MPX_CHECK_ARG(k == (sep ? 5 : 2), "kind 6: k = 5, kind 7: k = 2");
        const Taps st = make_taps(k, wx, wy, true, sep);
        const int seg = p1 > 0 ? p1 : (sep ? 0 : edgel::kSegRows);
        // p2: 0 buffer loads (production), 1 plain global loads, 2 non-temporal global loads
        if (sep) {
            if (p2 == 1) return launch_wave<5, 2, MPX_CONV_MAG2, true, edge::Sobel5SepTaps, 0, 4, 0>(in, out, w, w, 0, h, 0, h - 1, st, true, s, seg);
            if (p2 == 3) return launch_wave<5, 2, MPX_CONV_MAG2, true, edge::Sobel5SepTaps, 0, 4, 3>(in, out, w, w, 0, h, 0, h - 1, st, true, s, seg);
            if (p2 == 2) return launch_wave<5, 2, MPX_CONV_MAG2, true, edge::Sobel5SepTaps, 0, 4, 2>(in, out, w, w, 0, h, 0, h - 1, st, true, s, seg);
            return launch_wave<5, 2, MPX_CONV_MAG2, true, edge::Sobel5SepTaps, 0, 4, 1>(in, out, w, w, 0, h, 0, h - 1, st, true, s, seg);
        }
        if (p2 == 1) return launch_wave<2, 0, MPX_CONV_MAG2, true, edge::RobertsTaps, 0, 4, 0>(in, out, w, w, 0, h, 0, h - 1, st, true, s, seg);
        if (p2 == 2) return launch_wave<2, 0, MPX_CONV_MAG2, true, edge::RobertsTaps, 0, 4, 2>(in, out, w, w, 0, h, 0, h - 1, st, true, s, seg);
        return launch_wave<2, 0, MPX_CONV_MAG2, true, edge::RobertsTaps, 0, 4, 1>(in, out, w, w, 0, h, 0, h - 1, st, true, s, seg);
    }
    if (kind == 8) {
        // band kernel (conv_band4_kernel): p1 = segment rows (0 = auto), p2 % 100 =
        // waves per SIMD the auto segments target (0 = default), p2 / 100 % 10 == 1: no
        // alternation; p2 / 1000 = OPT (1: 5 waves per SIMD, 2: NT stores, 3: both, 6: NT + 16-wave groups,
        // 34 / 66: NT stores + NT interior / all row loads, 514: NT stores + 248-column strips with halo lanes)
        MPX_CHECK_ARG(k == 5 && p1 >= 0 && w % 4 == 0 && aligned16(in) && aligned16(out), "band variant: k = 5, w % 4 == 0");
        const Taps st = make_taps(k, wx, wy, true, true);
        const int per = p2 % 100 > 0 ? p2 % 100 : edgel::kBand4PerSimd, alt = (p2 / 100) % 10 == 1 ? 0 : 1;
        switch (p2 / 1000) {
#define MPX_BAND4(O)                                                                                          \
    case O:                                                                                                   \
        return edgel::launch_band4<5, 2, MPX_CONV_MAG2, true, edge::Sobel5SepTaps, O>(in, out, w, w, 0, h, 0, h - 1, st, s, \
                                                                                      p1, edge::RowSrc{}, per, alt);
            MPX_BAND4(0) MPX_BAND4(1) MPX_BAND4(2) MPX_BAND4(3) MPX_BAND4(6) MPX_BAND4(18) MPX_BAND4(34) MPX_BAND4(66) MPX_BAND4(162) MPX_BAND4(10) MPX_BAND4(11) MPX_BAND4(514)
#undef MPX_BAND4
        }
        set_error("unsupported band OPT %d", p2 / 1000);
        return MPX_ERR_ARG;
    }
    if (kind == 10) {
        // separable sobel5 on the vertical-halo-sharing band kernel (conv_band16v_kernel)
        MPX_CHECK_ARG(k == 5 && w % 4 == 0 && aligned16(in) && aligned16(out), "band16v variant: k = 5, w % 4 == 0");
        const Taps st = make_taps(k, wx, wy, true, true);
        return edgel::launch_band16v<5, 2, MPX_CONV_MAG2, true, edge::Sobel5SepTaps>(in, out, w, w, 0, h, 0, h - 1, st, s);
    }
    if (kind == 9) {
        // dense band kernel, compiled-in taps (k = 2 Roberts, k = 5 sobel5_dense):
        // p1 = segment rows (0 = auto), p2 % 100 = waves per SIMD for auto, p2 / 1000 = OPT
        MPX_CHECK_ARG(p1 >= 0 && w % 4 == 0 && aligned16(in) && aligned16(out), "band variant: w % 4 == 0");
        const Taps tp = make_taps(k, wx, wy, true);
        const int per = p2 % 100 > 0 ? p2 % 100 : edgel::kBand4PerSimd;
        if (k == 2) {
            if (p2 / 1000 == 2)
                return edgel::launch_band4<2, 0, MPX_CONV_MAG2, true, edge::RobertsTaps, 2>(in, out, w, w, 0, h, 0, h - 1, tp, s, p1, edge::RowSrc{}, per);
            return edgel::launch_band4<2, 0, MPX_CONV_MAG2, true, edge::RobertsTaps, 0>(in, out, w, w, 0, h, 0, h - 1, tp, s, p1, edge::RowSrc{}, per);
        }
        if (p2 / 1000 == 2)
            return edgel::launch_band4<5, 2, MPX_CONV_MAG2, true, edge::Sobel5Taps, 2>(in, out, w, w, 0, h, 0, h - 1, tp, s, p1, edge::RowSrc{}, per);
        return edgel::launch_band4<5, 2, MPX_CONV_MAG2, true, edge::Sobel5Taps, 0>(in, out, w, w, 0, h, 0, h - 1, tp, s, p1, edge::RowSrc{}, per);
    }
    const Taps taps = make_taps(k, wx, wy, true);
    if (kind == 1 || kind == 2) {
        // kind 1: runtime taps, kind 2: compiled-in taps of the named filter;
        // p1 = segment rows; p2 >= 1000 orders waves strip-major
        MPX_CHECK_ARG(p1 >= 1, "segment rows must be positive");
        const bool vec2 = (w % 2 == 0) && ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 7u) == 0;
        // p2 in [1000, 2000): strip-major; [2000, 3000): strip-minor with
        // alternating segment direction (the production MAG2 order)
        const int sm = p2 >= 2000 ? 3 : p2 >= 1000 ? 0 : 1;
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
    // raw 0 / 1: every float in [0, 65025] (255^2); raw 2 / 3: every float in
    // [0, +inf] (a squared magnitude from finite taps is never NaN)
    MPX_CHECK_ARG(raw >= 0 && raw <= 3, "raw: 0..3");
    hipLaunchKernelGGL(fast_sqrt_selftest_kernel, dim3(kNumCUs * 16), dim3(256), 0, as_stream(stream), 0u,
                       raw >= 2 ? 0x7F800000u : 0x477E0100u, bad_device, raw);
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}
