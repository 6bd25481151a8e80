/*
 * lab3 CPU classifier — NEW: the reference ships no CPU version of lab3
 * (SURVEY §2.4 "No C3"), so GPU/CPU speedups for lab3 were never reported.
 *   stdin "<in.data>\n<out.data>\n<nc>\n<np x y ...>\n..."   stdout "CPU execution time: <X ms>\n"
 * Same statistics and FMA chain as the GPU kernel, so outputs are identical.
 */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "../src/cpu/cpu_kernels.h"
#include "mpx/cio.h"
#include "mpx/common.h"
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

int main(void) {
    char in_path[4096], out_path[4096];
    if (scanf("%4095s", in_path) != 1 || scanf("%4095s", out_path) != 1) {
        fprintf(stderr, "[ERROR CPU] expected input and output paths\n");
        return 1;
    }
    int w, h, nc, rc = 1;
    int *coords = NULL;
    uint32_t *img = mpx_read_data_image(in_path, &w, &h);
    if (!img) return 1;
    if (scanf("%d", &nc) != 1 || nc < 1 || nc > MPX_MAX_CLASSES) {
        fprintf(stderr, "[ERROR CPU] expected 1 <= nc <= %d\n", MPX_MAX_CLASSES);
        goto done;
    }
    int np[MPX_MAX_CLASSES];
    int cap = 1024, used = 0;
    coords = (int *)malloc(sizeof(int) * cap);
    if (!coords) goto done;
    for (int c = 0; c < nc; ++c) {
        if (scanf("%d", &np[c]) != 1 || np[c] < 1) {
            fprintf(stderr, "[ERROR CPU] class %d: expected a positive point count\n", c);
            goto done;
        }
        for (int i = 0; i < 2 * np[c]; ++i) {
            if (used == cap) {
                int *grown = (int *)realloc(coords, sizeof(int) * cap * 2);
                if (!grown) goto done;
                coords = grown;
                cap *= 2;
            }
            if (scanf("%d", &coords[used++]) != 1) {
                fprintf(stderr, "[ERROR CPU] class %d: truncated coordinate list\n", c);
                goto done;
            }
        }
    }
    double mu[3 * MPX_MAX_CLASSES], inv[9 * MPX_MAX_CLASSES];
    if (mpx_cpu_class_stats(img, w, h, nc, np, coords, mu, inv) != 0) {
        fprintf(stderr, "[ERROR CPU] class point outside the %dx%d image\n", w, h);
        goto done;
    }
    const double t0 = now_ms();
    mpx_cpu_classify(img, (int64_t)w * h, nc, mu, inv);
    const double t1 = now_ms();
    rc = mpx_write_data_image(out_path, img, w, h);
    printf("CPU execution time: <%f ms>\n", t1 - t0);
done:  /* one exit path: the host sanitizer build checks for leaks */
    free(coords);
    free(img);
    return rc;
}
