/*
 * mpx common definitions shared by host C, host C++ and HIP device code.
 *
 * Pixels are carried as packed little-endian uint32 (R = bits 0..7, G = 8..15,
 * B = 16..23, A = 24..31), which is byte-identical to the reference's uchar4
 * `.data` layout (reference lab2/src/main.c:7-12, utils/converter.py:77-79)
 * but lets HIP kernels move 4 pixels per 16-byte lane load.
 */
#ifndef MPX_COMMON_H
#define MPX_COMMON_H

#include <stdint.h>

#if defined(__HIPCC__)
#define MPX_HD __host__ __device__
#else
#define MPX_HD
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* Largest convolution window supported by the generic KxK kernels. */
#define MPX_MAX_K 7
/* lab3 limit (reference lab3/src/main.cu:35). */
#define MPX_MAX_CLASSES 32

/* Output modes of the gradient-magnitude convolution family (lab2 generalisation). */
enum mpx_conv_mode {
    MPX_CONV_MAG2 = 0, /* G = sqrt(Gx^2 + Gy^2) with two filters (Roberts, Sobel) */
    MPX_CONV_ABS1 = 1, /* G = |Gx| (Laplacian-style single filter)               */
    MPX_CONV_LIN1 = 2  /* G = Gx   (blur / sharpen style single filter)           */
};

/*
 * Separable filters: OR MPX_CONV_SEP into the mode. The tap arrays then hold
 * the factors instead of k*k dense taps:
 *   wx = { hx[0..k-1], vx[0..k-1], sx }   gx = sx * sum_dy vx[dy] * (sum_dx hx[dx] * Y[y+dy-a][x+dx-a])
 *   wy = { hy[0..k-1], vy[0..k-1], sy }   (MAG2 only)
 * Both sums are sequential fmaf chains from 0 in index order (horizontal pass
 * first, clamp-to-edge in x and y), then one fp32 multiply by the scale.
 */
#define MPX_CONV_SEP 16
/*
 * Load-policy hint: OR MPX_CONV_RESIDENT into the mode when the input rows are
 * likely cache-resident (a small working set re-read across calls). The band
 * kernel then loads every row with the default cache policy instead of the
 * non-temporal interior-row loads that suit images streaming from HBM
 * (MI355X 4096^2: one resident pair 548-567 -> 580-614 Gpixel/s, 6 rotated
 * pairs 712-723 -> 654; profiles/lab2_conv.md). Results are identical.
 */
#define MPX_CONV_RESIDENT 32
#define MPX_CONV_BASE(m) ((m) & 3)
#define MPX_SEP_NTAPS(k) (2 * (k) + 1)

/* Which lab3 classifier implementation to run. */
enum mpx_classify_path {
    MPX_CLS_DIRECT = 0, /* fp64 (p-mu)^T A (p-mu), reference-exact                   */
    MPX_CLS_MFMA = 1,   /* fp32 MFMA distance GEMM, proven margin + exact fallback  */
    MPX_CLS_AUTO = 2,   /* FAST, or DIRECT when the fp32 margin cannot be proven    */
    MPX_CLS_FAST = 3,   /* fp32 packed-VALU distances, proven margin + fallback     */
    MPX_CLS_MFMA64 = 4, /* fp64 MFMA distance GEMM, proven margin + exact fallback  */
    MPX_CLS_MFMA8 = 5,  /* exact int8 MFMA distance GEMM (int32 keys), proven margin */
    MPX_CLS_MFMA16 = 6  /* f16 MFMA distance GEMM (f16 weight limbs, fp32 keys), one
                           pixel per lane, proven margin + exact fallback           */
};

/* lab5 element types (binary fixtures lab5/data/{int10,float10,uchar10}). */
enum mpx_sort_dtype {
    MPX_SORT_I32 = 0,
    MPX_SORT_F32 = 1, /* IEEE total order of the bit patterns (-NaN < -inf < -0 < +0 < +inf < +NaN) */
    MPX_SORT_U8 = 2
};

#ifdef __cplusplus
}
#endif

/* ---- pixel helpers (usable on host and device) ---- */
static inline MPX_HD uint32_t mpx_px_r(uint32_t p) { return p & 0xffu; }
static inline MPX_HD uint32_t mpx_px_g(uint32_t p) { return (p >> 8) & 0xffu; }
static inline MPX_HD uint32_t mpx_px_b(uint32_t p) { return (p >> 16) & 0xffu; }
static inline MPX_HD uint32_t mpx_px_a(uint32_t p) { return p >> 24; }
static inline MPX_HD uint32_t mpx_px_gray(uint32_t v, uint32_t a) {
    return v | (v << 8) | (v << 16) | (a << 24);
}

/*
 * Luminance exactly as the reference computes it: three fp32 products, two
 * fp32 adds, evaluated left to right with NO fused multiply-add
 * (reference lab2/src/main.cu:31-34, lab2/src/main.c:33-37). Every translation
 * unit that includes this header is built with -ffp-contract=off.
 */
static inline MPX_HD float mpx_luma(uint32_t p) {
    const float r = (float)mpx_px_r(p);
    const float g = (float)mpx_px_g(p);
    const float b = (float)mpx_px_b(p);
    const float t0 = 0.299f * r;
    const float t1 = 0.587f * g;
    const float t2 = 0.114f * b;
    return (t0 + t1) + t2;
}

/* clamp + truncating cast, reference lab2/src/main.cu:43-47 */
static inline MPX_HD uint32_t mpx_sat_u8(float g) {
    g = g < 0.0f ? 0.0f : g;
    g = g > 255.0f ? 255.0f : g;
    return (uint32_t)g;
}

static inline MPX_HD int mpx_clampi(int v, int lo, int hi) {
    return v < lo ? lo : (v > hi ? hi : v);
}

#endif /* MPX_COMMON_H */
