/*
 * Named filters of the lab2 convolution family. Single source of truth for the
 * CLIs (C and C++) and, through mpx_filter_lookup(), for the Python package.
 *
 * "roberts" reproduces the reference operator exactly (lab2/src/main.cu:37-38:
 * Gx = Y11 - Y00, Gy = Y10 - Y01, taps row-major [dy][dx], anchor 0); with the
 * fixed fmaf accumulation order a zero tap contributes exactly nothing, so the
 * generic kernel is bit-identical to the dedicated Roberts kernel.
 * "sobel5" is the 5x5 configuration named by BASELINE.json (gradient
 * magnitude of the 5x5 Sobel pair, normalised by 1/48 so that an ideal 255-step
 * maps to 255 instead of saturating). Both 5x5 Sobel kernels are rank 1, so
 * "sobel5" (and "gauss5") are stored factored (MPX_CONV_SEP, common.h): 18
 * fmaf per pixel instead of 40. "sobel5_dense" / "gauss5_dense" keep the
 * 25-tap direct sums of the same operators.
 */
#ifndef MPX_FILTERS_H
#define MPX_FILTERS_H

#include <string.h>

#include "mpx/common.h"

typedef struct {
    const char *name;
    int k;
    int anchor;
    int mode;
    float wx[MPX_MAX_K * MPX_MAX_K];
    float wy[MPX_MAX_K * MPX_MAX_K];
} mpx_filter;

#define MPX_F48(v) ((float)(v) / 48.0f)

static const mpx_filter mpx_filters[] = {
    {"roberts", 2, 0, MPX_CONV_MAG2, {-1, 0, 0, 1}, {0, 1, -1, 0}},
    {"sobel3", 3, 1, MPX_CONV_MAG2, {-1, 0, 1, -2, 0, 2, -1, 0, 1}, {-1, -2, -1, 0, 0, 0, 1, 2, 1}},
    {"prewitt3", 3, 1, MPX_CONV_MAG2, {-1, 0, 1, -1, 0, 1, -1, 0, 1}, {-1, -1, -1, 0, 0, 0, 1, 1, 1}},
    {"scharr3", 3, 1, MPX_CONV_MAG2, {-3, 0, 3, -10, 0, 10, -3, 0, 3}, {-3, -10, -3, 0, 0, 0, 3, 10, 3}},
    {"laplace3", 3, 1, MPX_CONV_ABS1, {0, 1, 0, 1, -4, 1, 0, 1, 0}, {0}},
    {"box3", 3, 1, MPX_CONV_LIN1,
     {1.0f / 9, 1.0f / 9, 1.0f / 9, 1.0f / 9, 1.0f / 9, 1.0f / 9, 1.0f / 9, 1.0f / 9, 1.0f / 9}, {0}},
    {"sharpen3", 3, 1, MPX_CONV_LIN1, {0, -1, 0, -1, 5, -1, 0, -1, 0}, {0}},
    /* separable 5x5 Sobel: gx = (v (x) d) / 48, gy = (d (x) v) / 48 with
       d = [-1 -2 0 2 1], v = [1 4 6 4 1]; the same operator as sobel5_dense,
       evaluated as a 1x5 then a 5x1 pass (fp32 rounding differs) */
    {"sobel5", 5, 2, MPX_CONV_MAG2 | MPX_CONV_SEP,
     {-1, -2, 0, 2, 1, 1, 4, 6, 4, 1, 1.0f / 48},
     {1, 4, 6, 4, 1, -1, -2, 0, 2, 1, 1.0f / 48}},
    {"gauss5", 5, 2, MPX_CONV_LIN1 | MPX_CONV_SEP, {1, 4, 6, 4, 1, 1, 4, 6, 4, 1, 1.0f / 256}, {0}},
    {"sobel5_dense", 5, 2, MPX_CONV_MAG2,
     {MPX_F48(-1), MPX_F48(-2), 0, MPX_F48(2), MPX_F48(1),
      MPX_F48(-4), MPX_F48(-8), 0, MPX_F48(8), MPX_F48(4),
      MPX_F48(-6), MPX_F48(-12), 0, MPX_F48(12), MPX_F48(6),
      MPX_F48(-4), MPX_F48(-8), 0, MPX_F48(8), MPX_F48(4),
      MPX_F48(-1), MPX_F48(-2), 0, MPX_F48(2), MPX_F48(1)},
     {MPX_F48(-1), MPX_F48(-4), MPX_F48(-6), MPX_F48(-4), MPX_F48(-1),
      MPX_F48(-2), MPX_F48(-8), MPX_F48(-12), MPX_F48(-8), MPX_F48(-2),
      0, 0, 0, 0, 0,
      MPX_F48(2), MPX_F48(8), MPX_F48(12), MPX_F48(8), MPX_F48(2),
      MPX_F48(1), MPX_F48(4), MPX_F48(6), MPX_F48(4), MPX_F48(1)}},
    {"gauss5_dense", 5, 2, MPX_CONV_LIN1,
     {1.0f / 256, 4.0f / 256, 6.0f / 256, 4.0f / 256, 1.0f / 256,
      4.0f / 256, 16.0f / 256, 24.0f / 256, 16.0f / 256, 4.0f / 256,
      6.0f / 256, 24.0f / 256, 36.0f / 256, 24.0f / 256, 6.0f / 256,
      4.0f / 256, 16.0f / 256, 24.0f / 256, 16.0f / 256, 4.0f / 256,
      1.0f / 256, 4.0f / 256, 6.0f / 256, 4.0f / 256, 1.0f / 256},
     {0}},
    {"log5", 5, 2, MPX_CONV_ABS1,
     {0, 0, -1, 0, 0, 0, -1, -2, -1, 0, -1, -2, 16, -2, -1, 0, -1, -2, -1, 0, 0, 0, -1, 0, 0}, {0}},
};

#define MPX_NUM_FILTERS ((int)(sizeof(mpx_filters) / sizeof(mpx_filters[0])))

static inline const mpx_filter *mpx_find_filter(const char *name) {
    for (int i = 0; i < MPX_NUM_FILTERS; ++i)
        if (strcmp(mpx_filters[i].name, name) == 0) return &mpx_filters[i];
    return 0;
}

#endif
