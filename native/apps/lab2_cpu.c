/*
 * lab2 CPU reference: Roberts cross (or any named filter via MPX_LAB2_OP / --op).
 *   stdin "<in.data>\n<out.data>"   stdout "CPU execution time: <X ms>\n"
 * cpu_exe = serial -O0 + clock() (reference lab2/src/main.c methodology),
 * cpu_omp_exe = -O3 -fopenmp + wall clock.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../src/cpu/cpu_kernels.h"
#include "mpx/cio.h"
#include "mpx/filters.h"
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

int main(int argc, char **argv) {
    const char *op = getenv("MPX_LAB2_OP");
    if (!op) op = "roberts";
    for (int i = 1; i + 1 < argc; ++i)
        if (strcmp(argv[i], "--op") == 0) op = argv[i + 1];
    const mpx_filter *f = mpx_find_filter(op);
    if (!f) {
        fprintf(stderr, "[ERROR CPU] unknown filter '%s'\n", op);
        return 1;
    }
    char in_path[4096], out_path[4096];
    if (scanf("%4095s", in_path) != 1 || scanf("%4095s", out_path) != 1) {
        fprintf(stderr, "[ERROR CPU] expected input and output paths\n");
        return 1;
    }
    int w, h;
    uint32_t *img = mpx_read_data_image(in_path, &w, &h);
    if (!img) return 1;
    uint32_t *out = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)w * h);
    if (!out) {
        fprintf(stderr, "Error allocating memory for output image.\n");
        free(img);
        return 1;
    }
    const double t0 = now_ms();
    if (strcmp(op, "roberts") == 0)
        mpx_cpu_roberts(img, out, w, h);
    else
        mpx_cpu_conv(img, out, w, w, 0, h, 0, h - 1, f->k, f->anchor, f->mode, f->wx, f->wy);
    const double t1 = now_ms();
    printf("CPU execution time: <%f ms>\n", t1 - t0);
    const int rc = mpx_write_data_image(out_path, out, w, h);
    free(img);
    free(out);
    return rc;
}
