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

static int read_vec(double *v, int n, const char *what) {
    for (int i = 0; i < n; ++i)
        if (scanf("%lf", &v[i]) != 1) {
            fprintf(stderr, "[ERROR CPU] %s: expected %d values, got %d\n", what, n, i);
            return 1;
        }
    return 0;
}

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
    if (read_vec(a, n, "first vector") || read_vec(b, n, "second vector")) goto done;
    const double t0 = now_ms();
    mpx_cpu_vsub_f64(a, b, c, n);
    const double t1 = now_ms();
    printf("CPU execution time: <%f ms>\n", t1 - t0);
    for (int i = 0; i < n; ++i) printf("%.10e ", c[i]);
    rc = 0;
done:  /* one exit path: the host sanitizer build checks for leaks */
    free(a);
    free(b);
    free(c);
    return rc;
}
