/*
 * lab5 CPU reference: ascending sort of a binary lab5 array (reference
 * lab5/data/{int10,float10,uchar10}; no reference program exists).
 *   stdin  int32 n + n binary elements   stdout "CPU execution time: <X ms>\n" + n sorted elements
 *   element type: argv[1] or MPX_LAB5_TYPE = int (default) | float | uchar
 * Same order as the GPU program (mpx_cpu_sort: IEEE total order for floats).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../src/cpu/cpu_kernels.h"
#include "mpx/common.h"
#ifdef _OPENMP
#include <omp.h>
#endif

static double now_ms(void) {
#ifdef _OPENMP
    return omp_get_wtime() * 1000.0;
#else
    return (double)clock() * 1000.0 / CLOCKS_PER_SEC;
#endif
}

int main(int argc, char **argv) {
    const char *kind = argc > 1 ? argv[1] : getenv("MPX_LAB5_TYPE");
    if (!kind) kind = "int";
    int dtype = -1;
    size_t elem = 0;
    if (!strcmp(kind, "int")) dtype = MPX_SORT_I32, elem = 4;
    else if (!strcmp(kind, "float")) dtype = MPX_SORT_F32, elem = 4;
    else if (!strcmp(kind, "uchar")) dtype = MPX_SORT_U8, elem = 1;
    if (dtype < 0) {
        fprintf(stderr, "[ERROR CPU] element type must be int, float or uchar (got '%s')\n", kind);
        return 1;
    }
    int32_t n = 0;
    if (fread(&n, sizeof(n), 1, stdin) != 1 || n < 0) {
        fprintf(stderr, "[ERROR CPU] expected a binary int32 element count on stdin\n");
        return 1;
    }
    unsigned char *buf = (unsigned char *)malloc(elem * (size_t)n + 1);
    if (!buf) {
        fprintf(stderr, "[ERROR CPU] allocation failed\n");
        return 1;
    }
    int rc = 1;
    if (n && fread(buf, elem, (size_t)n, stdin) != (size_t)n) {
        fprintf(stderr, "[ERROR CPU] expected %d binary elements on stdin\n", n);
        goto done;
    }
    const double t0 = now_ms();
    mpx_cpu_sort(buf, n, dtype);
    const double t1 = now_ms();
    printf("CPU execution time: <%f ms>\n", t1 - t0);
    fflush(stdout);
    if (n && fwrite(buf, elem, (size_t)n, stdout) != (size_t)n) {
        fprintf(stderr, "[ERROR CPU] write failed\n");
        goto done;
    }
    rc = 0;
done:
    free(buf);
    return rc;
}
