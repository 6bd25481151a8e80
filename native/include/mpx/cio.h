/*
 * Checked `.data` image I/O and tiny stdin helpers for the C programs (CPU
 * references, hw1/hw2). Format: little-endian int32 w, int32 h, then w*h RGBA8
 * pixels row-major (reference lab2/src/main.c:73-91). Messages follow the
 * reference CPU program (lab2/src/main.c:67-131); unlike the reference GPU
 * programs every fopen/fread/fwrite is checked.
 */
#ifndef MPX_CIO_H
#define MPX_CIO_H

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

/* Returns a malloc'd pixel array (caller frees) or NULL after printing why. */
static inline uint32_t *mpx_read_data_image(const char *path, int *w, int *h) {
    FILE *fp = fopen(path, "rb");
    if (fp == NULL) {
        fprintf(stderr, "Error opening input file.\n");
        return NULL;
    }
    if (fread(w, sizeof(int), 1, fp) != 1 || fread(h, sizeof(int), 1, fp) != 1) {
        fprintf(stderr, "Error reading image dimensions.\n");
        fclose(fp);
        return NULL;
    }
    if (*w <= 0 || *h <= 0 || (int64_t)(*w) * (*h) > (int64_t)1 << 31) {
        fprintf(stderr, "Error: bad image dimensions %d x %d.\n", *w, *h);
        fclose(fp);
        return NULL;
    }
    const size_t n = (size_t)(*w) * (size_t)(*h);
    uint32_t *data = (uint32_t *)malloc(sizeof(uint32_t) * n);
    if (data == NULL) {
        fprintf(stderr, "Error allocating memory for input image.\n");
        fclose(fp);
        return NULL;
    }
    if (fread(data, sizeof(uint32_t), n, fp) != n) {
        fprintf(stderr, "Error reading image data.\n");
        free(data);
        fclose(fp);
        return NULL;
    }
    fclose(fp);
    return data;
}

static inline int mpx_write_data_image(const char *path, const uint32_t *data, int w, int h) {
    FILE *fp = fopen(path, "wb");
    if (fp == NULL) {
        fprintf(stderr, "Error opening output file.\n");
        return 1;
    }
    const size_t n = (size_t)w * (size_t)h;
    if (fwrite(&w, sizeof(int), 1, fp) != 1 || fwrite(&h, sizeof(int), 1, fp) != 1) {
        fprintf(stderr, "Error writing image dimensions.\n");
        fclose(fp);
        return 1;
    }
    if (fwrite(data, sizeof(uint32_t), n, fp) != n) {
        fprintf(stderr, "Error writing image data.\n");
        fclose(fp);
        return 1;
    }
    if (fclose(fp) != 0) {
        fprintf(stderr, "Error closing output file.\n");
        return 1;
    }
    return 0;
}

#endif
