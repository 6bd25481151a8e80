/*
 * Host (CPU) implementations of every mpx operator. They define the numerics
 * the HIP kernels are tested against bit for bit:
 *   - luminance without FMA (mpx_luma), Roberts/conv gradient without FMA,
 *     conv taps accumulated with one fmaf per tap in (dy, dx) row-major order;
 *   - lab3 quadratic form with the FMA chain the reference GPU kernel compiles to
 *     (nvcc contracts `temp += d*A`; reference lab3/src/main.cu:57-67).
 * The same file is built twice: serial -O0 (reproduces the reference CPU
 * methodology, README.md:11) and OpenMP -O3 (honest multi-core baseline).
 */
#ifndef MPX_CPU_KERNELS_H
#define MPX_CPU_KERNELS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int mpx_cpu_threads(void);
void mpx_cpu_vsub_f64(const double *a, const double *b, double *c, int64_t n);
void mpx_cpu_vsub_f32(const float *a, const float *b, float *c, int64_t n);
void mpx_cpu_roberts(const uint32_t *in, uint32_t *out, int w, int h);
void mpx_cpu_roberts_rgb(const uint32_t *in, uint32_t *out, int w, int h);
void mpx_cpu_conv(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo,
                  int y_hi, int k, int anchor, int mode, const float *wx, const float *wy);
void mpx_cpu_classify(uint32_t *img, int64_t npix, int nc, const double *mu, const double *inv);
double mpx_cpu_jacobi_f64(const double *u, double *un, int cols, int pitch, int r0, int r1);
/* lab5: ascending sort in place, same order as mpx_sort (dtype: enum mpx_sort_dtype). */
void mpx_cpu_sort(void *data, int64_t n, int dtype);

/* lab1 host text I/O (reference lab1/src/main.cu:46-52 scanf per value,
 * :82-84 printf per value), parallel over OpenMP threads in the -fopenmp builds
 * and serial otherwise; byte-identical to the serial strtod / "%.10e " path.
 * mpx_parse_doubles: the next `count` whitespace-separated numbers of
 * buf[pos, len) (buf NUL-terminated at len) into out[]; returns how many were
 * parsed (< count: missing or malformed token at that index) and sets *end to
 * the offset just past the last parsed token.
 * mpx_format_e10: "%.10e " for each of n values, as one malloc'd buffer of
 * *len bytes (caller frees). */
int64_t mpx_parse_doubles(const char *buf, size_t len, size_t pos, int64_t count, double *out, size_t *end);
char *mpx_format_e10(const double *v, int64_t n, size_t *len);

/* lab3 host statistics H1 (reference lab3/src/main.cu:102-152). Returns 0, or
 * -1 when a coordinate lies outside the image. */
int mpx_cpu_class_stats(const uint32_t *img, int w, int h, int nc, const int *np,
                        const int *coords, double *mu, double *inv);

#ifdef __cplusplus
}
#endif

#endif
