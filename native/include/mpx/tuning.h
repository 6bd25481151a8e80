/* Tuning entry points exported by libmpx_tune.so (native/tune/, `make tune`),
 * not by libmpx.so and not part of the production C API in capi.h. Declared
 * here for the sort (native/tune/sort_variants.hip, kernels shared with the
 * production sort through src/kernels/sort_radix.hpp); the conv, Jacobi and
 * vsub variants (mpx_conv_variant, mpx_jacobi_variant, mpx_vsub_variant) are
 * bound by name from Python (_native.tune_lib). Used by
 * tools/experiments/{lab5_bench,sort_probe,jbench,vsub_sweep}.py, tools/kbench.py
 * and the GPU suites. */
#ifndef MPX_TUNING_H
#define MPX_TUNING_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The sort with a fixed radix schedule (sort_variants.hip): 0 = AUTO,
 * 1 onesweep (look-back), 2 reduce-then-scan, 4 / 7 / 8 persistent scatters
 * (round 2-3), 9-13 the returning-add ranking (8192 / 4096-key tiles, 3 blocks
 * per CU, two tiles in flight), 14 the lean onesweep, 15 the same at one block per CU. */
int mpx_sort_variant(void *data, int64_t n, int dtype, void *workspace, int64_t workspace_bytes, int variant,
                     void *stream);

/* Count + scan + lean scatter for each digit of the unchanged keys with step
 * knock-outs (radix_scatter_lean_kernel KNOCK: 0, 1, 6, 12, 14, 16, 31); the
 * workspace holds garbage afterwards, `data` is not modified. */
int mpx_sort_scatter_probe(const void *data, int64_t n, void *workspace, int64_t workspace_bytes, int knock,
                           void *stream);

#ifdef __cplusplus
}
#endif

#endif
