/*
 * Fast, exact decimal <-> double conversions for lab1's text I/O
 * (reference lab1/src/main.cu:46-52 scanf("%lf") per value, :82-84
 * printf("%.10e ") per value). Both produce exactly the bytes / bits of the
 * C library calls they replace, or report "no decision" so the caller falls
 * back to that call:
 *
 *  - fast_e10(v, out): "%.10e" of a finite double. The 11 significant digits
 *    come from one 64 x 128-bit product with a truncated 128-bit power of ten
 *    (pow10_table.h); the true product lies in [z, z + 2^64) units of z's low
 *    word, so the rounding decision is exact unless the discarded bits sit
 *    within that slack of an integer or a half — then 0 is returned;
 *  - fast_strtod(s, lim, &v, &end): decimal tokens [+-]digits[.digits][e[+-]digits]
 *    with at most 19 significant digits: Clinger's exact fast path
 *    (w <= 2^53, |q| <= 22), else the Eisel-Lemire 64 x 128-bit product with
 *    the same ambiguity guard; anything else (hex, inf, nan, long mantissas,
 *    subnormal or overflowing results) returns 0.
 *
 * tests/test_host_io.py checks both against glibc on millions of values,
 * including random bit patterns over the whole double range.
 */
#ifndef MPX_FASTFLOAT_H
#define MPX_FASTFLOAT_H

#include <stdint.h>
#include <string.h>

#include "pow10_table.h"

typedef unsigned __int128 mpx_u128;

/* z = a * (hi:lo) as 192 bits (z2:z1:z0) */
static inline void mpx_mul_64x128(uint64_t a, uint64_t hi, uint64_t lo, uint64_t *z2, uint64_t *z1, uint64_t *z0) {
    const mpx_u128 t1 = (mpx_u128)a * hi, t0 = (mpx_u128)a * lo;
    const mpx_u128 mid = (t0 >> 64) + (uint64_t)t1;
    *z0 = (uint64_t)t0;
    *z1 = (uint64_t)mid;
    *z2 = (uint64_t)(t1 >> 64) + (uint64_t)(mid >> 64);
}

/* floor(v * 10^k) split as N and a rounding verdict: returns 1 with *n = the
 * round-half-even result when the decision is certain, 0 otherwise.
 * v = m * 2^e2 with m > 0. */
static inline int mpx_scaled_round(uint64_t m, int e2, int k, uint64_t *n) {
    if (k < MPX_POW10_MIN || k > MPX_POW10_MAX) return 0;
    const int lz = __builtin_clzll(m);
    const uint64_t mn = m << lz;
    const int pe = mpx_pow10_tab[k - MPX_POW10_MIN].e;
    uint64_t z2, z1, z0;
    mpx_mul_64x128(mn, mpx_pow10_tab[k - MPX_POW10_MIN].hi, mpx_pow10_tab[k - MPX_POW10_MIN].lo, &z2, &z1, &z0);
    const int s = -(pe + e2 - lz);  /* value = z * 2^-s */
    if (s <= 128 || s >= 192) return 0;
    const int sh = s - 128;
    const uint64_t mask = ((uint64_t)1 << sh) - 1, half = (uint64_t)1 << (sh - 1);
    const uint64_t fh = z2 & mask;
    /* the true product is z + eps, 0 <= eps < 2^64 (z0 units): undecidable only
     * next to the carry into N or next to the half */
    if (fh == mask && z1 == UINT64_MAX) return 0;
    if ((fh == half && z1 == 0) || (fh == half - 1 && z1 == UINT64_MAX)) return 0;
    uint64_t q = z2 >> sh;
    if (fh >= half) ++q;  /* strictly above the half (the tie zone was excluded) */
    *n = q;
    return 1;
}

static const uint64_t mpx_p10u[20] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull, 10000000ull,
                                      100000000ull, 1000000000ull, 10000000000ull, 100000000000ull,
                                      1000000000000ull, 10000000000000ull, 100000000000000ull,
                                      1000000000000000ull, 10000000000000000ull, 100000000000000000ull,
                                      1000000000000000000ull, 10000000000000000000ull};

/* "%.10e" of v into out (>= 32 bytes, no terminator written); returns the
 * length, or 0 when the caller must use snprintf (non-finite, undecided). */
static inline int mpx_fast_e10(double v, char *out) {
    uint64_t bits;
    memcpy(&bits, &v, 8);
    const int neg = (int)(bits >> 63);
    const int ex = (int)((bits >> 52) & 0x7ff);
    const uint64_t frac = bits & (((uint64_t)1 << 52) - 1);
    if (ex == 0x7ff) return 0;
    char *p = out;
    if (neg) *p++ = '-';
    if (ex == 0 && frac == 0) {
        memcpy(p, "0.0000000000e+00", 16);
        return (int)(p - out) + 16;
    }
    const uint64_t m = ex ? (frac | ((uint64_t)1 << 52)) : frac;
    const int e2 = ex ? ex - 1075 : -1074;
    /* decimal exponent estimate from the bit length, corrected below */
    const int b = 63 - __builtin_clzll(m) + e2;  /* floor(log2 v) */
    int e10 = (int)((b * 78913LL) >> 18);        /* ~floor(b * log10(2)) (arithmetic shift floors) */
    uint64_t n = 0;
    for (int tries = 0; tries < 3; ++tries) {
        if (!mpx_scaled_round(m, e2, 10 - e10, &n)) return 0;
        if (n < mpx_p10u[10]) {
            --e10;
            continue;
        }
        if (n > mpx_p10u[11]) {
            ++e10;
            continue;
        }
        break;
    }
    if (n == mpx_p10u[11]) {  /* rounded up to the next power of ten */
        n = mpx_p10u[10];
        ++e10;
    }
    if (n < mpx_p10u[10] || n >= mpx_p10u[11]) return 0;
    char d[11];
    for (int i = 10; i >= 0; --i) {
        d[i] = (char)('0' + n % 10);
        n /= 10;
    }
    *p++ = d[0];
    *p++ = '.';
    memcpy(p, d + 1, 10);
    p += 10;
    *p++ = 'e';
    int ee = e10;
    *p++ = ee < 0 ? '-' : '+';
    if (ee < 0) ee = -ee;
    if (ee >= 100) {
        *p++ = (char)('0' + ee / 100);
        ee %= 100;
    }
    *p++ = (char)('0' + ee / 10);
    *p++ = (char)('0' + ee % 10);
    return (int)(p - out);
}

static const double mpx_p10d[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                    1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

static inline int mpx_is_ws(char c) { return c == ' ' || c == '\n' || c == '\t' || c == '\r' || c == '\f' || c == '\v'; }

/* Decimal token at s (s < lim, not whitespace) -> *val and *end (first byte
 * after the token, which must be whitespace or lim). Returns 1, or 0 when the
 * caller must use strtod (any other syntax or an undecided rounding). */
static inline int mpx_fast_strtod(const char *s, const char *lim, double *val, const char **end) {
    const char *p = s;
    int neg = 0;
    if (p < lim && (*p == '-' || *p == '+')) neg = *p++ == '-';
    uint64_t w = 0;
    int nd = 0, drop = 0, frac_digits = 0, any = 0;
    while (p < lim && *p == '0') {  /* leading zeros */
        ++p;
        any = 1;
    }
    while (p < lim && (unsigned)(*p - '0') < 10) {
        if (nd < 19) w = w * 10 + (uint64_t)(*p - '0'), ++nd;
        else if (*p != '0') return 0;
        else ++drop;
        ++p;
        any = 1;
    }
    if (p < lim && *p == '.') {
        ++p;
        if (nd == 0)
            while (p < lim && *p == '0') ++p, ++frac_digits, any = 1;
        while (p < lim && (unsigned)(*p - '0') < 10) {
            if (nd < 19) w = w * 10 + (uint64_t)(*p - '0'), ++nd, ++frac_digits;
            else if (*p != '0') return 0;
            ++p;
            any = 1;
        }
    }
    if (!any) return 0;
    int64_t q = (int64_t)drop - frac_digits;
    if (p < lim && (*p == 'e' || *p == 'E')) {
        const char *e = p + 1;
        int eneg = 0;
        if (e < lim && (*e == '-' || *e == '+')) eneg = *e++ == '-';
        if (!(e < lim && (unsigned)(*e - '0') < 10)) return 0;  /* "1e" : let strtod decide */
        int64_t x = 0;
        while (e < lim && (unsigned)(*e - '0') < 10) {
            if (x < 100000) x = x * 10 + (*e - '0');
            ++e;
        }
        q += eneg ? -x : x;
        p = e;
    }
    if (p < lim && !mpx_is_ws(*p)) return 0;
    *end = p;
    if (w == 0) {
        *val = neg ? -0.0 : 0.0;
        return 1;
    }
    if (w <= ((uint64_t)1 << 53) && q >= -22 && q <= 22) {  /* Clinger: one correctly rounded op */
        double d = (double)w;
        d = q < 0 ? d / mpx_p10d[-q] : d * mpx_p10d[q];
        *val = neg ? -d : d;
        return 1;
    }
    if (q < MPX_POW10_MIN || q > MPX_POW10_MAX) return 0;
    const int lz = __builtin_clzll(w);
    const uint64_t wn = w << lz;
    uint64_t z2, z1, z0;
    mpx_mul_64x128(wn, mpx_pow10_tab[q - MPX_POW10_MIN].hi, mpx_pow10_tab[q - MPX_POW10_MIN].lo, &z2, &z1, &z0);
    (void)z0;
    const int upper = (int)(z2 >> 63);  /* product msb at bit 191 (1) or 190 (0) */
    const int cut = upper + 9;          /* keep 54 bits: 53 + the round bit */
    const uint64_t lowmask = ((uint64_t)1 << cut) - 1;
    const uint64_t rest = z2 & lowmask;
    if (rest == lowmask && z1 == UINT64_MAX) return 0;  /* a carry could reach the round bit */
    uint64_t mant = z2 >> cut;
    if ((mant & 1) && rest == 0 && z1 == 0) return 0;   /* possibly an exact tie */
    int x = 128 + cut + mpx_pow10_tab[q - MPX_POW10_MIN].e - lz + 1;  /* value ~ (mant >> 1) * 2^x */
    mant = (mant >> 1) + (mant & 1);
    if (mant == ((uint64_t)1 << 53)) {
        mant >>= 1;
        ++x;
    }
    const int biased = x + 52 + 1023;
    if (biased <= 0 || biased >= 0x7ff) return 0;  /* subnormal or overflow: strtod */
    const uint64_t bits = ((uint64_t)neg << 63) | ((uint64_t)biased << 52) | (mant & (((uint64_t)1 << 52) - 1));
    memcpy(val, &bits, 8);
    return 1;
}

#endif
