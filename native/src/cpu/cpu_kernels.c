/*
 * CPU reference operators (see cpu_kernels.h). OpenMP pragmas are inert in the
 * serial -O0 build (no -fopenmp), which reproduces the reference's single-thread
 * methodology; the library build uses -O3 -fopenmp.
 */
#include "cpu_kernels.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fastfloat.h"
#include "mpx/common.h"

#ifdef _OPENMP
#include <omp.h>
#endif

/* On x86-64 gcc only emits a hardware FMA for fmaf() inside an "fma" target
 * clone; the default clone calls libm's correctly rounded fmaf. Both give the
 * same bits, the clone is just faster. */
#if defined(__GNUC__) && !defined(__clang__) && defined(__x86_64__) && !defined(MPX_NO_CLONES)
#define MPX_FMA_CLONES __attribute__((target_clones("fma", "default")))
#else
#define MPX_FMA_CLONES
#endif

int mpx_cpu_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ---- lab1 text I/O ---- */
static int is_ws(char c) { return c == ' ' || c == '\n' || c == '\t' || c == '\r' || c == '\f' || c == '\v'; }

int64_t mpx_parse_doubles(const char *buf, size_t len, size_t pos, int64_t count, double *out, size_t *end) {
    *end = pos;
    if (count <= 0) return 0;
    while (pos < len && is_ws(buf[pos])) ++pos;
    int T = 1;
#ifdef _OPENMP
    T = omp_get_max_threads();
    if ((int64_t)(len - pos) < ((int64_t)1 << 16)) T = 1;
#endif
    /* chunk k starts at a token start (or len): cut evenly, then move each cut
     * past the token it lands in and the whitespace after it */
    size_t *start = (size_t *)malloc(sizeof(size_t) * (size_t)(T + 1));
    int64_t *ntok = (int64_t *)calloc((size_t)T + 1, sizeof(int64_t));
    if (!start || !ntok) {
        free(start);
        free(ntok);
        return 0;
    }
    start[0] = pos;
    start[T] = len;
    for (int k = 1; k < T; ++k) {
        size_t c = pos + (len - pos) / (size_t)T * (size_t)k;
        if (c < start[k - 1]) c = start[k - 1];
        if (c > pos && !is_ws(buf[c - 1]))
            while (c < len && !is_ws(buf[c])) ++c;
        while (c < len && is_ws(buf[c])) ++c;
        start[k] = c;
    }
    /* pass 1: tokens per chunk */
#ifdef _OPENMP
#pragma omp parallel for schedule(static, 1) num_threads(T)
#endif
    for (int k = 0; k < T; ++k) {
        int64_t c = 0;
        int in_tok = 0;
        for (size_t i = start[k]; i < start[k + 1]; ++i) {
            const int w = is_ws(buf[i]);
            if (!w && !in_tok) ++c;
            in_tok = !w;
        }
        ntok[k + 1] = c;
    }
    for (int k = 0; k < T; ++k) ntok[k + 1] += ntok[k];
    /* pass 2: strtod each token whose index is < count */
    int64_t bad = count;  /* first malformed token index */
    size_t last_end = pos;
#ifdef _OPENMP
#pragma omp parallel for schedule(static, 1) num_threads(T) reduction(min : bad)
#endif
    for (int k = 0; k < T; ++k) {
        int64_t idx = ntok[k];
        size_t i = start[k];
        while (idx < count && i < start[k + 1]) {
            while (i < start[k + 1] && is_ws(buf[i])) ++i;
            if (i >= start[k + 1]) break;
            const char *fe = NULL;
            size_t j;
            if (mpx_fast_strtod(buf + i, buf + start[k + 1], &out[idx], &fe)) {  /* exact fast path */
                j = (size_t)(fe - buf);
            } else {  /* anything the fast path does not decide: the C library */
                char *e = NULL;
                out[idx] = strtod(buf + i, &e);
                if (e == buf + i) {  /* not a number */
                    if (idx < bad) bad = idx;
                    break;
                }
                j = i;
                while (j < start[k + 1] && !is_ws(buf[j])) ++j;
                if ((size_t)(e - buf) != j) {  /* trailing junk in the token */
                    if (idx < bad) bad = idx;
                    break;
                }
            }
            if (idx == count - 1) last_end = j;
            i = j;
            ++idx;
        }
    }
    const int64_t got = ntok[T] < count ? ntok[T] : count;
    free(start);
    free(ntok);
    const int64_t n = bad < got ? bad : got;
    if (n == count) *end = last_end;
    return n;
}

char *mpx_format_e10(const double *v, int64_t n, size_t *len) {
    int T = 1;
#ifdef _OPENMP
    T = omp_get_max_threads();
    if (n < 4096) T = 1;
#endif
    char **part = (char **)calloc((size_t)T, sizeof(char *));
    size_t *plen = (size_t *)calloc((size_t)T + 1, sizeof(size_t));
    int fail = 0;
    char *outb = NULL;
    size_t total = 0;
    if (!part || !plen) goto out;
    /* pass 1: each thread formats its slice (exact fast path, snprintf when
     * the fast path cannot decide) */
#ifdef _OPENMP
#pragma omp parallel for schedule(static, 1) num_threads(T) reduction(| : fail)
#endif
    for (int k = 0; k < T; ++k) {
        const int64_t a = n * k / T, b = n * (k + 1) / T;
        char *buf = (char *)malloc((size_t)(b - a) * 32 + 1);
        if (!buf) {
            fail |= 1;
            continue;
        }
        size_t o = 0;
        for (int64_t i = a; i < b; ++i) {
            const int l = mpx_fast_e10(v[i], buf + o);
            o += l ? (size_t)l : (size_t)snprintf(buf + o, 32, "%.10e", v[i]);
            buf[o++] = ' ';
        }
        part[k] = buf;
        plen[k + 1] = o;
    }
    for (int k = 0; k < T; ++k) plen[k + 1] += plen[k];
    total = plen[T];
    outb = fail ? NULL : (char *)malloc(total + 1);
    /* pass 2: the slices land at their prefix offsets in parallel */
    if (outb) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static, 1) num_threads(T)
#endif
        for (int k = 0; k < T; ++k) memcpy(outb + plen[k], part[k], plen[k + 1] - plen[k]);
        outb[total] = 0;
    }
out:
    if (part)
        for (int k = 0; k < T; ++k) free(part[k]);
    free(part);
    free(plen);
    *len = outb ? total : 0;
    return outb;
}

void mpx_cpu_vsub_f64(const double *a, const double *b, double *c, int64_t n) {
    int64_t i;
#pragma omp parallel for schedule(static)
    for (i = 0; i < n; ++i) c[i] = a[i] - b[i];
}

void mpx_cpu_vsub_f32(const float *a, const float *b, float *c, int64_t n) {
    int64_t i;
#pragma omp parallel for schedule(static)
    for (i = 0; i < n; ++i) c[i] = a[i] - b[i];
}

/* Roberts cross exactly as the reference CPU program evaluates it, including
 * recomputing luminance four times per pixel (reference lab2/src/main.c:23-59). */
void mpx_cpu_roberts(const uint32_t *in, uint32_t *out, int w, int h) {
    int y;
#pragma omp parallel for schedule(static)
    for (y = 0; y < h; ++y) {
        const int y1 = y + 1 < h ? y + 1 : h - 1;
        for (int x = 0; x < w; ++x) {
            const int x1 = x + 1 < w ? x + 1 : w - 1;
            const uint32_t p00 = in[(int64_t)y * w + x];
            const float y00 = mpx_luma(p00);
            const float y10 = mpx_luma(in[(int64_t)y * w + x1]);
            const float y01 = mpx_luma(in[(int64_t)y1 * w + x]);
            const float y11 = mpx_luma(in[(int64_t)y1 * w + x1]);
            const float gx = y11 - y00;
            const float gy = y10 - y01;
            const float g2 = gx * gx + gy * gy;
            const float g = sqrtf(g2);
            out[(int64_t)y * w + x] = mpx_px_gray(mpx_sat_u8(g), mpx_px_a(p00));
        }
    }
}

/* Per-channel Roberts cross, L1 magnitude: every colour channel c of
 * pixel (x, y) becomes min(255, |c(x,y) - c(x+1,y+1)| + |c(x+1,y) - c(x,y+1)|)
 * with clamp-to-edge neighbours, alpha kept. The operator behind the
 * reference's lab2/test_data/lenna_out.data (byte-exact on all 512 x 512
 * pixels; no reference program computes it). Integer arithmetic. */
void mpx_cpu_roberts_rgb(const uint32_t *in, uint32_t *out, int w, int h) {
    int y;
#pragma omp parallel for schedule(static)
    for (y = 0; y < h; ++y) {
        const int y1 = y + 1 < h ? y + 1 : h - 1;
        for (int x = 0; x < w; ++x) {
            const int x1 = x + 1 < w ? x + 1 : w - 1;
            const uint32_t a = in[(int64_t)y * w + x], b = in[(int64_t)y * w + x1];
            const uint32_t c = in[(int64_t)y1 * w + x], d = in[(int64_t)y1 * w + x1];
            uint32_t o = a & 0xff000000u;
            for (int ch = 0; ch < 24; ch += 8) {
                const int va = (int)((a >> ch) & 255u), vb = (int)((b >> ch) & 255u);
                const int vc = (int)((c >> ch) & 255u), vd = (int)((d >> ch) & 255u);
                int g = abs(va - vd) + abs(vb - vc);
                g = g > 255 ? 255 : g;
                o |= (uint32_t)g << ch;
            }
            out[(int64_t)y * w + x] = o;
        }
    }
}

static inline float conv_finish(int mode, float gx, float gy) {
    if (mode == MPX_CONV_MAG2) {
        const float a = gx * gx;
        const float b = gy * gy;
        return sqrtf(a + b);
    }
    if (mode == MPX_CONV_ABS1) return fabsf(gx);
    return gx;
}

MPX_FMA_CLONES
static void conv_rows(const float *lum, int lum_y0, const uint32_t *in, uint32_t *out, int w,
                      int pitch, int oy0, int oy1, int y_lo, int y_hi, int k, int anchor, int mode,
                      const float *wx, const float *wy) {
    int y;
#pragma omp parallel for schedule(static)
    for (y = oy0; y < oy1; ++y) {
        for (int x = 0; x < w; ++x) {
            float ax = 0.0f, ay = 0.0f;
            for (int dy = 0; dy < k; ++dy) {
                const int yy = mpx_clampi(y + dy - anchor, y_lo, y_hi);
                const float *row = lum + (int64_t)(yy - lum_y0) * w;
                for (int dx = 0; dx < k; ++dx) {
                    const int xx = mpx_clampi(x + dx - anchor, 0, w - 1);
                    ax = fmaf(wx[dy * k + dx], row[xx], ax);
                    if (mode == MPX_CONV_MAG2) ay = fmaf(wy[dy * k + dx], row[xx], ay);
                }
            }
            const float g = conv_finish(mode, ax, ay);
            out[(int64_t)y * pitch + x] = mpx_px_gray(mpx_sat_u8(g), mpx_px_a(in[(int64_t)y * pitch + x]));
        }
    }
}

/* Separable form (MPX_CONV_SEP, common.h): per input row the horizontal
 * factor sums, then per output the vertical sum of those, then the scale.
 * Every sum is a sequential fmaf chain from 0 in index order. */
MPX_FMA_CLONES
static void conv_rows_sep(const float *lum, int lum_y0, int nrows, const uint32_t *in, uint32_t *out,
                          int w, int pitch, int oy0, int oy1, int y_lo, int y_hi, int k, int anchor,
                          int mode, const float *wx, const float *wy) {
    const int two = mode == MPX_CONV_MAG2;
    /* horizontal pass: hs[0] (gx factor) and hs[1] (gy factor) of every row */
    float *hs = (float *)malloc(sizeof(float) * (size_t)nrows * (size_t)w * (two ? 2 : 1));
    if (!hs) return;
    float *hsy = two ? hs + (size_t)nrows * (size_t)w : 0;
    int r;
#pragma omp parallel for schedule(static)
    for (r = 0; r < nrows; ++r) {
        const float *row = lum + (int64_t)r * w;
        for (int x = 0; x < w; ++x) {
            float ax = 0.0f, ay = 0.0f;
            for (int dx = 0; dx < k; ++dx) {
                const float l = row[mpx_clampi(x + dx - anchor, 0, w - 1)];
                ax = fmaf(wx[dx], l, ax);
                if (two) ay = fmaf(wy[dx], l, ay);
            }
            hs[(int64_t)r * w + x] = ax;
            if (two) hsy[(int64_t)r * w + x] = ay;
        }
    }
    int y;
#pragma omp parallel for schedule(static)
    for (y = oy0; y < oy1; ++y) {
        for (int x = 0; x < w; ++x) {
            float ax = 0.0f, ay = 0.0f;
            for (int dy = 0; dy < k; ++dy) {
                const int64_t rr = (int64_t)(mpx_clampi(y + dy - anchor, y_lo, y_hi) - lum_y0) * w + x;
                ax = fmaf(wx[k + dy], hs[rr], ax);
                if (two) ay = fmaf(wy[k + dy], hsy[rr], ay);
            }
            const float gx = ax * wx[2 * k];
            const float gy = two ? ay * wy[2 * k] : 0.0f;
            const float g = conv_finish(mode, gx, gy);
            out[(int64_t)y * pitch + x] = mpx_px_gray(mpx_sat_u8(g), mpx_px_a(in[(int64_t)y * pitch + x]));
        }
    }
    free(hs);
}

void mpx_cpu_conv(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo,
                  int y_hi, int k, int anchor, int mode, const float *wx, const float *wy) {
    if (oy1 <= oy0 || w <= 0) return;
    /* luminance plane for every input row the requested outputs touch */
    const int r0 = mpx_clampi(oy0 - anchor, y_lo, y_hi);
    const int r1 = mpx_clampi(oy1 - 1 + (k - 1 - anchor), y_lo, y_hi);
    const int nrows = r1 - r0 + 1;
    float *lum = (float *)malloc(sizeof(float) * (size_t)nrows * (size_t)w);
    if (!lum) return;
    int r;
#pragma omp parallel for schedule(static)
    for (r = 0; r < nrows; ++r) {
        const uint32_t *src = in + (int64_t)(r0 + r) * pitch;
        float *dst = lum + (int64_t)r * w;
        for (int x = 0; x < w; ++x) dst[x] = mpx_luma(src[x]);
    }
    if (mode & MPX_CONV_SEP)
        conv_rows_sep(lum, r0, nrows, in, out, w, pitch, oy0, oy1, y_lo, y_hi, k, anchor, MPX_CONV_BASE(mode), wx, wy);
    else
        conv_rows(lum, r0, in, out, w, pitch, oy0, oy1, y_lo, y_hi, k, anchor, mode, wx, wy);
    free(lum);
}

/* lab3 per-pixel quadratic form, FMA chain of the reference GPU kernel
 * (reference lab3/src/main.cu:49-72): strict '<' keeps the lowest class on
 * ties, an all-NaN pixel keeps class -1 which is stored as 255. */
MPX_FMA_CLONES
void mpx_cpu_classify(uint32_t *img, int64_t npix, int nc, const double *mu, const double *inv) {
    int64_t i;
#pragma omp parallel for schedule(static)
    for (i = 0; i < npix; ++i) {
        const uint32_t p = img[i];
        const double pr = (double)mpx_px_r(p), pg = (double)mpx_px_g(p), pb = (double)mpx_px_b(p);
        double best = DBL_MAX;
        int cls = -1;
        for (int c = 0; c < nc; ++c) {
            const double d0 = pr - mu[3 * c + 0];
            const double d1 = pg - mu[3 * c + 1];
            const double d2 = pb - mu[3 * c + 2];
            const double *A = inv + 9 * c;
            double t0 = fma(d0, A[0], 0.0), t1 = fma(d0, A[1], 0.0), t2 = fma(d0, A[2], 0.0);
            t0 = fma(d1, A[3], t0);
            t1 = fma(d1, A[4], t1);
            t2 = fma(d1, A[5], t2);
            t0 = fma(d2, A[6], t0);
            t1 = fma(d2, A[7], t1);
            t2 = fma(d2, A[8], t2);
            double dist = fma(t0, d0, 0.0);
            dist = fma(t1, d1, dist);
            dist = fma(t2, d2, dist);
            if (dist < best) {
                best = dist;
                cls = c;
            }
        }
        img[i] = (p & 0x00ffffffu) | ((uint32_t)(uint8_t)cls << 24);
    }
}

double mpx_cpu_jacobi_f64(const double *u, double *un, int cols, int pitch, int r0, int r1) {
    double res = 0.0;
    int i;
#pragma omp parallel for schedule(static) reduction(max : res)
    for (i = r0; i < r1; ++i) {
        const double *up = u + (int64_t)(i - 1) * pitch;
        const double *uc = u + (int64_t)i * pitch;
        const double *ud = u + (int64_t)(i + 1) * pitch;
        double *o = un + (int64_t)i * pitch;
        o[0] = uc[0];
        o[cols - 1] = uc[cols - 1];
        for (int j = 1; j < cols - 1; ++j) {
            const double s = ((up[j] + ud[j]) + (uc[j - 1] + uc[j + 1])) * 0.25;
            const double d = fabs(s - uc[j]);
            res = d > res ? d : res;
            o[j] = s;
        }
    }
    return res;
}

/* Host statistics with the reference's exact operation order
 * (reference lab3/src/main.cu:102-152): mean, unbiased covariance, cofactor
 * determinant and the modular-index adjugate inverse. */
int mpx_cpu_class_stats(const uint32_t *img, int w, int h, int nc, const int *np,
                        const int *coords, double *mu, double *inv) {
    const int *pts = coords;
    for (int c = 0; c < nc; ++c) {
        const int n = np[c];
        double sum[3] = {0.0, 0.0, 0.0};
        for (int i = 0; i < n; ++i) {
            const int x = pts[2 * i], y = pts[2 * i + 1];
            if (x < 0 || y < 0 || x >= w || y >= h) return -1;
            const uint32_t px = img[(int64_t)y * w + x];
            sum[0] += (double)mpx_px_r(px);
            sum[1] += (double)mpx_px_g(px);
            sum[2] += (double)mpx_px_b(px);
        }
        double avg[3] = {sum[0] / n, sum[1] / n, sum[2] / n};
        double cov[3][3];
        memset(cov, 0, sizeof(cov));
        for (int i = 0; i < n; ++i) {
            const uint32_t px = img[(int64_t)pts[2 * i + 1] * w + pts[2 * i]];
            const double d[3] = {(double)mpx_px_r(px) - avg[0], (double)mpx_px_g(px) - avg[1],
                                 (double)mpx_px_b(px) - avg[2]};
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) {
                    const double prod = d[a] * d[b];
                    cov[a][b] += prod;
                }
        }
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) cov[a][b] /= (n - 1);
        const double m0 = cov[1][1] * cov[2][2] - cov[2][1] * cov[1][2];
        const double m1 = cov[1][0] * cov[2][2] - cov[1][2] * cov[2][0];
        const double m2 = cov[1][0] * cov[2][1] - cov[1][1] * cov[2][0];
        const double det = cov[0][0] * m0 - cov[0][1] * m1 + cov[0][2] * m2;
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                const double p1 = cov[(b + 1) % 3][(a + 1) % 3] * cov[(b + 2) % 3][(a + 2) % 3];
                const double p2 = cov[(b + 1) % 3][(a + 2) % 3] * cov[(b + 2) % 3][(a + 1) % 3];
                inv[9 * c + 3 * a + b] = (p1 - p2) / det;
            }
        mu[3 * c + 0] = avg[0];
        mu[3 * c + 1] = avg[1];
        mu[3 * c + 2] = avg[2];
        pts += 2 * n;
    }
    return 0;
}

/* ---- lab5 sort: order-preserving uint32 keys (floats: IEEE total order of
 * the bit patterns), the same key map as native/src/kernels/sort.hip ---- */
static int cmp_u32(const void *a, const void *b) {
    const uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return (x > y) - (x < y);
}

#ifdef _OPENMP
/* OpenMP build: T sorted runs (qsort per thread), then log2(T) rounds of
 * pairwise merges, each round's merges in parallel. */
static void merge_u32(const uint32_t *a, int64_t na, const uint32_t *b, int64_t nb, uint32_t *out) {
    int64_t i = 0, j = 0, o = 0;
    while (i < na && j < nb) out[o++] = b[j] < a[i] ? b[j++] : a[i++];
    while (i < na) out[o++] = a[i++];
    while (j < nb) out[o++] = b[j++];
}

static int sort_u32_parallel(uint32_t *x, int64_t n) {
    int runs = omp_get_max_threads();
    if (runs < 2 || n < (1 << 16)) return 0;
    uint32_t *tmp = (uint32_t *)malloc((size_t)n * sizeof(uint32_t));
    int64_t *bound = (int64_t *)malloc((size_t)(runs + 1) * sizeof(int64_t));
    if (!tmp || !bound) {
        free(tmp);
        free(bound);
        return 0;
    }
    for (int r = 0; r <= runs; ++r) bound[r] = n * r / runs;
#pragma omp parallel for schedule(static)
    for (int r = 0; r < runs; ++r) qsort(x + bound[r], (size_t)(bound[r + 1] - bound[r]), sizeof(uint32_t), cmp_u32);
    uint32_t *src = x, *dst = tmp;
    for (int width = 1; width < runs; width *= 2) {
#pragma omp parallel for schedule(dynamic, 1)
        for (int r = 0; r < runs; r += 2 * width) {
            const int mid = r + width < runs ? r + width : runs;
            const int end = r + 2 * width < runs ? r + 2 * width : runs;
            merge_u32(src + bound[r], bound[mid] - bound[r], src + bound[mid], bound[end] - bound[mid], dst + bound[r]);
        }
        uint32_t *t = src;
        src = dst;
        dst = t;
    }
    if (src != x) memcpy(x, src, (size_t)n * sizeof(uint32_t));
    free(tmp);
    free(bound);
    return 1;
}
#endif

void mpx_cpu_sort(void *data, int64_t n, int dtype) {
    if (n < 2) return;
    if (dtype == MPX_SORT_U8) { /* counting sort (per-thread histograms in the OpenMP build) */
        uint8_t *x = (uint8_t *)data;
        int64_t cnt[256] = {0};
#ifdef _OPENMP
#pragma omp parallel
        {
            int64_t local[256] = {0};
#pragma omp for schedule(static) nowait
            for (int64_t i = 0; i < n; ++i) local[x[i]]++;
#pragma omp critical
            for (int v = 0; v < 256; ++v) cnt[v] += local[v];
        }
        int64_t start[257];
        start[0] = 0;
        for (int v = 0; v < 256; ++v) start[v + 1] = start[v] + cnt[v];
#pragma omp parallel for schedule(dynamic, 8)
        for (int v = 0; v < 256; ++v) memset(x + start[v], v, (size_t)cnt[v]);
#else
        for (int64_t i = 0; i < n; ++i) cnt[x[i]]++;
        int64_t o = 0;
        for (int v = 0; v < 256; ++v)
            for (int64_t c = 0; c < cnt[v]; ++c) x[o++] = (uint8_t)v;
#endif
        return;
    }
    uint32_t *x = (uint32_t *)data;
    const int is_float = dtype == MPX_SORT_F32;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t i = 0; i < n; ++i) {
        const uint32_t v = x[i];
        x[i] = is_float ? (v ^ ((uint32_t)((int32_t)v >> 31) | 0x80000000u)) : (v ^ 0x80000000u);
    }
#ifdef _OPENMP
    if (!sort_u32_parallel(x, n))
#endif
        qsort(x, (size_t)n, sizeof(uint32_t), cmp_u32);
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t i = 0; i < n; ++i) {
        const uint32_t k = x[i];
        x[i] = is_float ? (k ^ ((k >> 31) ? 0x80000000u : 0xffffffffu)) : (k ^ 0x80000000u);
    }
}
