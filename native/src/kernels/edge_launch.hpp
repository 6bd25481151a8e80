// Launch helpers of the lab2 wave-streaming / LDS-streaming kernels, shared by
// the translation units that instantiate them (edge.hip: generic production
// conv; edge_roberts.hip: Roberts; edge_variants.hip: tuning entry points).
// Each TU is its own code object, loaded by HIP on first use, so a program that
// only runs Roberts loads only the Roberts kernels (cold-launch time).
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdlib>

#include "edge_kernels.hpp"

namespace mpx {
namespace edgel {
using edge::Taps;

// sep: wx / wy hold the MPX_CONV_SEP factors (2k+1 values) instead of k*k taps
inline Taps make_taps(int k, const float *wx, const float *wy, bool two, bool sep = false) {
    Taps t{};
    const int n = sep ? MPX_SEP_NTAPS(k) : k * k;
    for (int i = 0; i < n; ++i) {
        t.wx[i] = wx[i];
        t.wy[i] = two ? wy[i] : 0.0f;
    }
    return t;
}

// Production tile: RPT = 8 rows per wave -> 128 x 32 output tiles.
// resident workgroups per CU the chunking targets (VGPR-limited to 4 at ~100 VGPRs)
inline constexpr int kBlocksPerCU = 4;

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

// rows per wave segment of the wave-streaming kernel (dense filters and the
// single-filter separable passes). Tuned on MI355X with tools/named_taps_ab.py
// (4096^2, segments 6 .. 23): short segments in several rounds win for the
// dense kernels (sobel3 27.0 us, roberts 21.4-23.0, laplace3 21.8); the kernel
// leaves a segment as soon as its rows are done, so 8 need not be a multiple
// of the unrolled row group.
inline constexpr int kSegRows = 8;

// Wave order of the launches (conv_wave_kernel's strip_minor bits): 1 =
// strip-minor; 3 = strip-minor with alternating segment directions, so
// vertically adjacent segments read their shared rows at the same time (L2
// hits). Same-box A/B over 6 rotated 4096^2 slab pairs (tools/kbench.py
// --rotate 6, tools/gpu_r2_order_ab.sh, two rounds each): sobel5 33.5 -> 32.4
// us (kernel alone 31.8 -> 30.3), sobel5_dense 42.0 -> 40.0, gauss5 33.8 ->
// 33.2, Roberts 32.0 -> 31.4 — every path at least as fast, so 3 everywhere.
inline constexpr int kWaveOrder = 3;
inline constexpr int kWaveOrderAlt = 3;

// MPX_CONV_ORDER=1|3 forces the wave order of every conv launch (same-box A/B
// of the production paths with tools/kbench.py); read once per process.
inline int wave_order_override() {
    static const int v = [] {
        const char *e = std::getenv("MPX_CONV_ORDER");
        const int o = e ? std::atoi(e) : 0;
        return (o == 1 || o == 3) ? o : 0;
    }();
    return v;
}

template <int K, int A, int MODE, bool FAST, class F = edge::RuntimeTaps, int OWX = 0, int PF = 4, int BUFLD = 1>
int launch_wave(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
                const Taps &taps, bool vec, hipStream_t s, int seg = kSegRows, int strip_minor = kWaveOrder,
                edge::RowSrc rs = edge::RowSrc{}) {
    if (!rs.up) rs.up = in;
    if (!rs.dn) rs.dn = in;
    if (const int o = wave_order_override()) strip_minor = o;
    using G = edge::WaveGeom<K, A, OWX>;
    const int strips = (w + G::OW - 1) / G::OW;
    if (seg <= 0) {
        // one resident round of ~6 waves per SIMD: long segments (few warm-up
        // rows), at least 8 rows each. MI355X separable sobel5 4096^2 sweep
        // (tools/named_taps_ab.py, MPX_SSEG hook since removed): auto (seg 23)
        // 24.7 us, seg 25-30 25.0, 20 26.1, 15-16 27.1-27.6, 8-12 26.1-28.1
        const int64_t slots = (int64_t)kNumCUs * 4 * 6;
        const int64_t work = (int64_t)(oy1 - oy0) * strips;
        seg = (int)std::max<int64_t>(8, (work + slots - 1) / slots);
    }
    const int segs = (oy1 - oy0 + seg - 1) / seg;
    const int64_t nwaves = (int64_t)strips * segs;
    MPX_CHECK_ARG(nwaves < ((int64_t)1 << 31) - 4, "image too large for one launch");
    const unsigned nblk = (unsigned)((nwaves + 3) / 4);
    if (vec)
        hipLaunchKernelGGL((edge::conv_wave_kernel<K, A, MODE, true, FAST, F, OWX, PF, BUFLD>), dim3(nblk), dim3(256), 0, s, in,
                           out, w, pitch, oy0, oy1, y_lo, y_hi, seg, segs, (int)nwaves, strips, strip_minor, taps, rs);
    else
        hipLaunchKernelGGL((edge::conv_wave_kernel<K, A, MODE, false, FAST, F, OWX, PF, BUFLD>), dim3(nblk), dim3(256), 0, s, in,
                           out, w, pitch, oy0, oy1, y_lo, y_hi, seg, segs, (int)nwaves, strips, strip_minor, taps, rs);
    return MPX_OK;
}

// Band kernel (conv_band4_kernel): 256-column strips, aprons, strip-minor with
// alternating segment directions. seg <= 0: one resident round of per_simd
// waves per SIMD (104 VGPRs: 4 resident), at least 8 rows per segment.
// MI355X sobel5 4096^2, 6 rotated pairs (tools/kbench.py): auto at 4 waves
// (16-row segments) 30.1 us; 5 / 6 waves (13 / 11 rows, two rounds) 32.6 /
// 32.1; 20 / 24 rows 34.9 / 32.2; no alternation 32.4.
inline constexpr int kBand4PerSimd = 4;
inline int band4_auto_seg(int w, int rows, bool hl = false, int per_simd = kBand4PerSimd) {
    const int strips = hl ? (w + 247) / 248 : (w + 255) / 256;
    const int64_t slots = (int64_t)kNumCUs * 4 * per_simd;
    const int64_t work = (int64_t)rows * strips;
    return (int)std::max<int64_t>(8, (work + slots - 1) / slots);
}
// SP: the fused streaming-halo form (mpx_conv_stream_peer_run; *sp required, its
// n_edge filled in here).
template <int K, int A, int MODE, bool FAST, class F, int OPT = 0, bool SP = false>
int launch_band4(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
                 const Taps &taps, hipStream_t s, int seg, edge::RowSrc rs, int per_simd = kBand4PerSimd,
                 int alt = 1, mpx_conv_stream_peer *sp = nullptr) {
    MPX_CHECK_ARG(w % 4 == 0 && pitch % 4 == 0 && aligned16(in) && aligned16(out), "band kernel: 16-B aligned rows");
    if (!rs.up) rs.up = in;
    if (!rs.dn) rs.dn = in;
    if (rs.up != in || rs.dn != in || SP) alt |= 2;  // remote halo rows: boundary segments first
    const int strips = (OPT & 512) ? (w + 247) / 248 : (w + 255) / 256;
    if (seg <= 0) seg = band4_auto_seg(w, oy1 - oy0, (OPT & 512) != 0, per_simd);
    MPX_CHECK_ARG(!(OPT & (8 | 2048)) || seg + K - 1 <= 32, "batched aprons: walks of at most 32 rows");
    const int segs = (oy1 - oy0 + seg - 1) / seg;
    const int64_t nwaves = (int64_t)strips * segs;
    MPX_CHECK_ARG(nwaves < ((int64_t)1 << 31) - 4, "image too large for one launch");
    constexpr int wpb = (OPT & 4) ? 16 : 4;
    mpx_conv_stream_peer desc{};
    if constexpr (SP) {
        MPX_CHECK_ARG(sp && sp->sync && oy0 == 0 && oy1 == rs.own_rows, "fused streaming halo: whole slab, sync block");
        // edge waves (conv_band4_kernel<SP>): segments touching an edge that has a neighbour
        constexpr int R = K - 1 - A;
        int nseg = 0;
        for (int g = 0; g < segs; ++g) {
            const int ys = oy0 + g * seg, ye = std::min(ys + seg, oy1);
            nseg += (sp->up_flag && (ys - A < 0 || ys < sp->n_first)) ||
                    (sp->dn_flag && (ye - 1 + R >= rs.own_rows || ye > rs.own_rows - sp->n_last));
        }
        sp->n_edge = nseg * strips;
        desc = *sp;
    }
    hipLaunchKernelGGL((edge::conv_band4_kernel<K, A, MODE, FAST, F, OPT, SP>), dim3((unsigned)((nwaves + wpb - 1) / wpb)),
                       dim3(64 * wpb), 0,
                       s, in, out, w, pitch, oy0, oy1, y_lo, y_hi, seg, (int)nwaves, strips, alt, taps, rs, desc);
    return MPX_OK;
}

inline constexpr int kBandModeDefault = 3;

// Vertical halo sharing (conv_band16v_kernel): 16-wave workgroups of 16
// consecutive 16-row segments of one strip; the shared halo rows travel
// through LDS instead of being loaded twice. 5-row windows (A = 2) only,
// rows resident in `in` (no neighbour-slab row sources).
inline constexpr int kVSeg = 16;
template <int K, int A, int MODE, bool FAST, class F>
int launch_band16v(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
                   const Taps &taps, hipStream_t s) {
    static_assert(K == 5 && A == 2, "vertical sharing covers 5-row windows");
    MPX_CHECK_ARG(w % 4 == 0 && pitch % 4 == 0 && aligned16(in) && aligned16(out), "band kernel: 16-B aligned rows");
    const int strips = (w + 255) / 256;
    const int segs = (oy1 - oy0 + kVSeg - 1) / kVSeg;
    const int64_t nblk = (int64_t)strips * ((segs + 15) / 16);
    MPX_CHECK_ARG(nblk < ((int64_t)1 << 31), "image too large for one launch");
    hipLaunchKernelGGL((edge::conv_band16v_kernel<K, A, MODE, FAST, F, kVSeg>), dim3((unsigned)nblk), dim3(1024), 0, s,
                       in, out, w, pitch, oy0, oy1, y_lo, y_hi, segs, strips, taps);
    return MPX_OK;
}

// The band kernel serves every launch whose window reaches at most two columns
// on each side (K <= 5 except 4x4-style anchors) and whose rows (and neighbour
// rows) are 16-B aligned, with non-temporal output stores. MI355X 4096^2, 6
// rotated pairs (tools/kbench.py, µs): sobel5 separable 28.9 (30.3 with the
// 8-B-lane wave kernel; 29.4 with plain stores), sobel5_dense 32.7 (41.4),
// Roberts 27.8 (30.4). Default (MPX_CONV_BAND unset or 3): NT stores and
// non-temporal loads of the rows no neighbouring segment re-reads (OPT 34) —
// round 3, bench.py alternated on two boxes: 583 / 584 / 583 and 574 / 582
// Gpixel/s with plain loads vs 614 / 603 / 605 and 604 / 588; every named
// filter through ops.conv, two alternations (µs, plain -> NT): sobel5 28.4 ->
// 27.0, gauss5 28.0 -> 27.1, gauss5_dense 30.7 -> 27.1, sobel5_dense 32.9 ->
// 32.3, 3x3 filters -0.6 to -0.8, Roberts / sharpen3 / box3 within 0.15
// (profiles/lab2_conv.md). MPX_CONV_BAND=0: wave kernel, 1: band kernel with
// plain stores, 2: NT stores and plain loads; read once per process.
// MPX_CONV_BAND=4: the vertical-halo-sharing kernel (conv_band16v_kernel) for
// 5-row windows with resident rows, mode 3 otherwise. mpx_conv_set_band_mode()
// switches the mode at run time (tests, A/B in one process).
inline int band_mode_env() {
    const char *e = std::getenv("MPX_CONV_BAND");
    return (e && e[0] >= '0' && e[0] <= '4') ? e[0] - '0' : kBandModeDefault;
}
inline std::atomic<int> g_band_mode{band_mode_env()};
inline int band_mode() { return g_band_mode.load(std::memory_order_relaxed); }
// MPX_CONV_RESIDENT for the launch in flight on this thread: the default mode
// (3) then keeps plain interior-row loads (OPT 2), as mode 2 does
inline thread_local bool tl_conv_resident = false;
struct ResidentHint {
    bool prev;
    explicit ResidentHint(bool r) : prev(tl_conv_resident) { tl_conv_resident = r; }
    ~ResidentHint() { tl_conv_resident = prev; }
};
// Small images (below kBandMinPixels) keep the wave kernel: with one resident
// round of 16-row segments a 1-Mpx image is only a few hundred waves, and the
// reference harness's cold single launches on its 0.5-2 Mpx images measured
// 19.1 us with the band kernel vs 15.2 us with the wave kernel (lab2 large
// bucket median, tools/gpu_r2_same_method.sh).
// mpx_conv_set_band_min() moves the threshold (tests cover the band kernel's
// strip edges on small images).
inline constexpr int64_t kBandMinPixels = int64_t(1) << 22;
inline std::atomic<int64_t> g_band_min_pixels{kBandMinPixels};
inline bool band_ok(const uint32_t *in, const uint32_t *out, int w, int pitch, const edge::RowSrc &rs, int rows) {
    return band_mode() != 0 && (int64_t)w * rows >= g_band_min_pixels.load(std::memory_order_relaxed) && w % 4 == 0 && pitch % 4 == 0 && aligned16(in) && aligned16(out) &&
           (!rs.up || aligned16(rs.up)) && (!rs.dn || aligned16(rs.dn));
}

template <int K, int A>
inline constexpr bool kBandFits = A <= 2 && K - 1 - A <= 2;

template <int K, int A, int MODE, class F>
int launch_band(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
                const Taps &taps, hipStream_t s, const edge::RowSrc &rs) {
    const int m = band_mode();
    if constexpr (K == 5 && A == 2) {
        if (m == 4 && (!rs.up || rs.up == in) && (!rs.dn || rs.dn == in))
            return launch_band16v<K, A, MODE, true, F>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, s);
    }
    if (m == 1)
        return launch_band4<K, A, MODE, true, F, 0>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, s, 0, rs);
    // walks of at most 32 rows (every segment of a 4096^2 frame: 16 + 4) take
    // the batched aprons (OPT bit 11: one apron load and luma per walk, two
    // ds_bpermute per row instead of a load, a luma and two selects)
    const int seg = band4_auto_seg(w, oy1 - oy0);
    const bool bpa = seg + K - 1 <= 32;
    if (m == 2 || tl_conv_resident)
        return bpa ? launch_band4<K, A, MODE, true, F, 2 | 2048>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, s, seg, rs)
                   : launch_band4<K, A, MODE, true, F, 2>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, s, seg, rs);
    return bpa ? launch_band4<K, A, MODE, true, F, 34 | 2048>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, s, seg, rs)
               : launch_band4<K, A, MODE, true, F, 34>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, s, seg, rs);
}

// Named filters whose taps are compiled in (zero taps disappear); selected
// whenever the caller's taps are bit-identical to them.
template <class F, int N>
inline bool same_taps(const Taps &t) {
    for (int i = 0; i < N; ++i)
        if (__builtin_bit_cast(uint32_t, t.wx[i]) != __builtin_bit_cast(uint32_t, F::wx[i]) ||
            __builtin_bit_cast(uint32_t, t.wy[i]) != __builtin_bit_cast(uint32_t, F::wy[i]))
            return false;
    return true;
}

// Dense filters: the first compile-time tap class of the list whose window,
// mode and taps match (bit-exactly) the call, else runtime taps.
template <int K, int A, int MODE, class F, class... More>
int launch_named(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
                 const Taps &taps, bool vec, hipStream_t s, const edge::RowSrc &rs) {
    if constexpr (F::kK == K && F::kA == A && F::kMode == MODE) {
        if (same_taps<F, K * K>(taps)) {
            if constexpr (kBandFits<K, A>)
                if (band_ok(in, out, w, pitch, rs, oy1 - oy0))
                    return launch_band<K, A, MODE, F>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, s, rs);
            return launch_wave<K, A, MODE, true, F>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, vec, s, kSegRows, kWaveOrder, rs);
        }
    }
    if constexpr (sizeof...(More) > 0) {
        return launch_named<K, A, MODE, More...>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, vec, s, rs);
    } else {
        if constexpr (kBandFits<K, A>)
            if (band_ok(in, out, w, pitch, rs, oy1 - oy0))
                return launch_band<K, A, MODE, edge::RuntimeTaps>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, s, rs);
        return launch_wave<K, A, MODE, true>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, vec, s, kSegRows, kWaveOrder, rs);
    }
}

template <int K, int A, int MODE>
int launch_tiled(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
                 const Taps &taps, bool vec, hipStream_t s, const edge::RowSrc &rs = edge::RowSrc{}) {
    return launch_named<K, A, MODE, edge::RobertsTaps, edge::Sobel3Taps, edge::Prewitt3Taps, edge::Scharr3Taps,
                        edge::Laplace3Taps, edge::Sharpen3Taps, edge::Sobel5Taps, edge::Log5Taps>(
        in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, vec, s, rs);
}

template <class F, int K>
inline bool same_sep_taps(const Taps &t, bool two) {
    auto eq = [](float a, float b) { return __builtin_bit_cast(uint32_t, a) == __builtin_bit_cast(uint32_t, b); };
    for (int i = 0; i < K; ++i) {
        if (!eq(t.wx[i], F::hx[i]) || !eq(t.wx[K + i], F::vx[i])) return false;
        if (two && (!eq(t.wy[i], F::hy[i]) || !eq(t.wy[K + i], F::vy[i]))) return false;
    }
    return eq(t.wx[2 * K], F::sx) && (!two || eq(t.wy[2 * K], F::sy));
}

// Separable filters (MPX_CONV_SEP): the wave kernel keeps a ring of per-row
// horizontal sums instead of the K x K window. Their K-1 warm-up rows per
// segment cost a whole horizontal pass each, so the two-filter (MAG2)
// segments are longer: sized for one resident round (launch_wave, seg <= 0).
template <int K, int A, int MODE>
int launch_sep(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo, int y_hi,
               const Taps &taps, bool vec, hipStream_t s, const edge::RowSrc &rs = edge::RowSrc{}) {
    // segment rows: two-filter magnitudes one resident round (auto), the
    // lighter single-filter passes short segments (MI355X 4096^2, named_taps_ab:
    // sobel5 auto 24.7 us vs 26.1 at 8; gauss5 8 rows 23.4 us vs 25.1 auto)
    constexpr int seg = MODE == MPX_CONV_MAG2 ? 0 : kSegRows;
    constexpr int order = MODE == MPX_CONV_MAG2 ? kWaveOrderAlt : kWaveOrder;
    constexpr bool fits = kBandFits<K, A>;
    const bool band = fits && band_ok(in, out, w, pitch, rs, oy1 - oy0);
    if constexpr (K == 5 && A == 2 && MODE == MPX_CONV_MAG2) {
        if (band && same_sep_taps<edge::Sobel5SepTaps, 5>(taps, true))
            return launch_band<K, A, MODE, edge::Sobel5SepTaps>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, s, rs);
        if (same_sep_taps<edge::Sobel5SepTaps, 5>(taps, true))
            return launch_wave<K, A, MODE, true, edge::Sobel5SepTaps>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, vec, s, seg, order, rs);
    }
    if constexpr (K == 5 && A == 2 && MODE == MPX_CONV_LIN1) {
        if (band && same_sep_taps<edge::Gauss5SepTaps, 5>(taps, false))
            return launch_band<K, A, MODE, edge::Gauss5SepTaps>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, s, rs);
        if (same_sep_taps<edge::Gauss5SepTaps, 5>(taps, false))
            return launch_wave<K, A, MODE, true, edge::Gauss5SepTaps>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, vec, s, seg, order, rs);
    }
    if constexpr (fits)
        if (band)
            return launch_band<K, A, MODE, edge::RuntimeSepTaps>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, s, rs);
    return launch_wave<K, A, MODE, true, edge::RuntimeSepTaps>(in, out, w, pitch, oy0, oy1, y_lo, y_hi, taps, vec, s, seg, order, rs);
}


}  // namespace edgel
}  // namespace mpx
