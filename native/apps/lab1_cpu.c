/*
 * lab1 CPU reference: c = a - b over fp64 vectors.
 *   stdin  "<n>\n<a0 ..>\n<b0 ..>"   stdout "CPU execution time: <X ms>\n" + n x "%.10e "
 * Built twice (Makefile): cpu_exe = serial -O0 with clock() timing, the
 * published methodology (reference lab1/src/main.c:54-58, README.md:11);
 * cpu_omp_exe = -O3 -fopenmp with wall-clock timing.
 */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "../src/cpu/cpu_kernels.h"
#ifdef _OPENMP
#include <omp.h>
#endif

static double now_ms(void) {
#ifdef _OPENMP
    return omp_get_wtime() * 1000.0;
#else
    return (double)clock() / CLOCKS_PER_SEC * 1000.0;
#endif
}

#ifdef _OPENMP
/* OpenMP build: the rest of stdin read once, both vectors parsed in parallel
 * (mpx_parse_doubles: one strtod per token, the values scanf("%lf") yields) */
static char *g_in = NULL;
static size_t g_len = 0, g_pos = 0;

static int slurp_stdin(void) {
    size_t cap = 1 << 20;
    g_in = (char *)malloc(cap + 1);
    if (!g_in) return 1;
    size_t got;
    while ((got = fread(g_in + g_len, 1, cap - g_len, stdin)) > 0) {
        g_len += got;
        if (g_len == cap) {
            char *p = (char *)realloc(g_in, 2 * cap + 1);
            if (!p) return 1;
            g_in = p;
            cap *= 2;
        }
    }
    g_in[g_len] = 0;
    return 0;
}

static int read_vec(double *v, int n, const char *what) {
    size_t end = g_pos;
    const int64_t got = mpx_parse_doubles(g_in, g_len, g_pos, n, v, &end);
    if (got != n) {
        fprintf(stderr, "[ERROR CPU] %s: expected %d values, got %lld\n", what, n, (long long)got);
        return 1;
    }
    g_pos = end;
    return 0;
}
#else
/* serial build: scanf per value, the reference's host loop (lab1/src/main.c) */
static int read_vec(double *v, int n, const char *what) {
    for (int i = 0; i < n; ++i)
        if (scanf("%lf", &v[i]) != 1) {
            fprintf(stderr, "[ERROR CPU] %s: expected %d values, got %d\n", what, n, i);
            return 1;
        }
    return 0;
}
#endif

int main(void) {
    int n;
    if (scanf("%d", &n) != 1 || n < 0) {
        fprintf(stderr, "[ERROR CPU] expected vector size\n");
        return 1;
    }
    int rc = 1;
    double *a = (double *)malloc(sizeof(double) * (n ? n : 1));
    double *b = (double *)malloc(sizeof(double) * (n ? n : 1));
    double *c = (double *)malloc(sizeof(double) * (n ? n : 1));
    if (!a || !b || !c) {
        fprintf(stderr, "[ERROR CPU] allocation failed\n");
        goto done;
    }
#ifdef _OPENMP
    const int io_timing = getenv("MPX_IO_TIMING") != NULL;
    double ts[5];
    ts[0] = now_ms();
    if (slurp_stdin()) {
        fprintf(stderr, "[ERROR CPU] out of memory reading stdin\n");
        goto done;
    }
#endif
#ifdef _OPENMP
    ts[1] = now_ms();
#endif
    if (read_vec(a, n, "first vector") || read_vec(b, n, "second vector")) goto done;
#ifdef _OPENMP
    ts[2] = now_ms();
#endif
    const double t0 = now_ms();
    mpx_cpu_vsub_f64(a, b, c, n);
    const double t1 = now_ms();
    printf("CPU execution time: <%f ms>\n", t1 - t0);
#ifdef _OPENMP
    {
        size_t len = 0;
        char *txt = mpx_format_e10(c, n, &len);
        if (!txt && n) {
            fprintf(stderr, "[ERROR CPU] out of memory formatting the result\n");
            goto done;
        }
        ts[3] = now_ms();
        fflush(stdout);
        if (len) fwrite(txt, 1, len, stdout);
        fflush(stdout);
        ts[4] = now_ms();
        free(txt);
        if (io_timing)
            fprintf(stderr, "[io] read %.1f ms, parse %.1f ms, format %.1f ms, write %.1f ms\n", ts[1] - ts[0],
                    ts[2] - ts[1], ts[3] - t1, ts[4] - ts[3]);
    }
#else
    for (int i = 0; i < n; ++i) printf("%.10e ", c[i]);
#endif
    rc = 0;
done:  /* one exit path: the host sanitizer build checks for leaks */
#ifdef _OPENMP
    free(g_in);
#endif
    free(a);
    free(b);
    free(c);
    return rc;
}
