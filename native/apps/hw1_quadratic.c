/*
 * hw1: real roots of a*x^2 + b*x + c = 0 in fp32 (reference hw1/src/main.c).
 * Output contract: "any" (0 = 0), "incorrect" (c = 0 with c != 0), one root,
 * two roots "%.6f %.6f", or "imaginary".
 */
#include <math.h>
#include <stdio.h>

typedef enum { ROOTS_ANY, ROOTS_NONE_DEGENERATE, ROOTS_ONE, ROOTS_TWO, ROOTS_COMPLEX } roots_kind;

static roots_kind solve(float a, float b, float c, float *r1, float *r2) {
    if (a == 0) {
        if (b == 0) return c == 0 ? ROOTS_ANY : ROOTS_NONE_DEGENERATE;
        *r1 = -c / b;
        return ROOTS_ONE;
    }
    const float disc = b * b - 4 * a * c;
    if (disc > 0) {
        const float s = sqrtf(disc);
        *r1 = (-b + s) / (2 * a);
        *r2 = (-b - s) / (2 * a);
        return ROOTS_TWO;
    }
    if (disc == 0) {
        *r1 = -b / (2 * a);
        return ROOTS_ONE;
    }
    return ROOTS_COMPLEX; /* negative or NaN discriminant */
}

int main(void) {
    float a, b, c, r1 = 0, r2 = 0;
    if (scanf("%f %f %f", &a, &b, &c) != 3) {
        fprintf(stderr, "expected three coefficients\n");
        return 1;
    }
    switch (solve(a, b, c, &r1, &r2)) {
        case ROOTS_ANY: puts("any"); break;
        case ROOTS_NONE_DEGENERATE: puts("incorrect"); break;
        case ROOTS_ONE: printf("%.6f\n", r1); break;
        case ROOTS_TWO: printf("%.6f %.6f\n", r1, r2); break;
        case ROOTS_COMPLEX: puts("imaginary"); break;
    }
    return 0;
}
