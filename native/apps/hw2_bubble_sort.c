/*
 * hw2: ascending bubble sort of n fp32 values (reference hw2/src/main.c).
 *   stdin "<n> v0 v1 ..."   stdout "%.6e " per value, then a newline.
 * Same pass structure as the reference (n-1 passes, adjacent swaps), plus an
 * early exit once a pass swaps nothing, which leaves the output unchanged.
 */
#include <stdio.h>
#include <stdlib.h>

static void bubble_sort(float *v, int n) {
    for (int pass = 0; pass + 1 < n; ++pass) {
        int swapped = 0;
        for (int j = 0; j + 1 < n - pass; ++j) {
            if (v[j] > v[j + 1]) {
                const float t = v[j];
                v[j] = v[j + 1];
                v[j + 1] = t;
                swapped = 1;
            }
        }
        if (!swapped) break;
    }
}

int main(void) {
    int n;
    if (scanf("%d", &n) != 1 || n < 0) {
        fprintf(stderr, "expected element count\n");
        return 1;
    }
    float *v = (float *)malloc(sizeof(float) * (n > 0 ? n : 1));
    if (!v) {
        fprintf(stderr, "allocation failed\n");
        return 1;
    }
    for (int i = 0; i < n; ++i)
        if (scanf("%f", &v[i]) != 1) {
            fprintf(stderr, "expected %d values\n", n);
            free(v);
            return 1;
        }
    bubble_sort(v, n);
    for (int i = 0; i < n; ++i) printf("%.6e ", v[i]);
    putchar('\n');
    free(v);
    return 0;
}
