// libmpx C ABI glue: error reporting, device queries, host statistics.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "../cpu/cpu_kernels.h"
#include "../kernels/internal.hpp"
#include "mpx/capi.h"
#include "mpx/filters.h"

namespace mpx {

static thread_local std::string g_last_error;

void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

}  // namespace mpx

namespace mpx {
const void *module_anchor_vsub();
const void *module_anchor_jacobi();
const void *module_anchor_classify();
const void *module_anchor_edge();
const void *module_anchor_edge_roberts();
const void *module_anchor_sort();
const void *module_anchor_edge_stream();
}  // namespace mpx

extern "C" int mpx_preload_modules(void) {
    const void *anchors[] = {mpx::module_anchor_vsub(),         mpx::module_anchor_jacobi(),
                             mpx::module_anchor_classify(),     mpx::module_anchor_edge(),
                             mpx::module_anchor_edge_roberts(), mpx::module_anchor_sort(),
                             mpx::module_anchor_edge_stream()};
    for (const void *k : anchors) {
        hipFuncAttributes attr;
        MPX_RETURN_IF_HIP_ERROR(hipFuncGetAttributes(&attr, k));
    }
    return MPX_OK;
}

extern "C" const char *mpx_last_error(void) { return mpx::g_last_error.c_str(); }

extern "C" const char *mpx_version(void) { return "mpx 0.1.0 (gfx950)"; }

extern "C" int mpx_device_count(int *count) {
    MPX_CHECK_ARG(count, "null count");
    *count = 0;
    MPX_RETURN_IF_HIP_ERROR(hipGetDeviceCount(count));
    return MPX_OK;
}

extern "C" int mpx_stream_sync(void *stream) {
    MPX_RETURN_IF_HIP_ERROR(hipStreamSynchronize(mpx::as_stream(stream)));
    return MPX_OK;
}

// gpu_info equivalent (reference gpu_info/src/main.cu:4-18), with the CDNA
// facts a kernel author needs: gfx arch, wave size, LDS, L2, clocks.
extern "C" int mpx_device_report(int device, char *buf, size_t len) {
    MPX_CHECK_ARG(buf && len > 0, "null buffer");
    hipDeviceProp_t p;
    MPX_RETURN_IF_HIP_ERROR(hipGetDeviceProperties(&p, device));
    int lds_per_cu = 0;
    (void)hipDeviceGetAttribute(&lds_per_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device);
    std::snprintf(buf, len,
                  "Compute capability : %d.%d\n"
                  "Name : %s\n"
                  "Arch : %s\n"
                  "Total Global Memory : %zu\n"
                  "Shared memory per block : %zu\n"
                  "Shared memory (LDS) per CU : %d\n"
                  "Max threads per block : (%d, %d, %d)\n"
                  "Max block : (%d, %d, %d)\n"
                  "Total constant memory : %zu\n"
                  "Multiprocessors count : %d\n"
                  "Wavefront size : %d\n"
                  "L2 cache size : %d\n"
                  "Clock rate (kHz) : %d\n"
                  "Memory clock rate (kHz) : %d\n"
                  "Memory bus width (bits) : %d\n",
                  p.major, p.minor, p.name, p.gcnArchName, (size_t)p.totalGlobalMem, (size_t)p.sharedMemPerBlock,
                  lds_per_cu, p.maxThreadsDim[0], p.maxThreadsDim[1], p.maxThreadsDim[2], p.maxGridSize[0],
                  p.maxGridSize[1], p.maxGridSize[2], (size_t)p.totalConstMem, p.multiProcessorCount, p.warpSize,
                  p.l2CacheSize, p.clockRate, p.memoryClockRate, p.memoryBusWidth);
    return MPX_OK;
}

extern "C" int mpx_filter_lookup(const char *name, int *k, int *anchor, int *mode, float *wx, float *wy) {
    MPX_CHECK_ARG(name && k && anchor && mode && wx && wy, "null pointer");
    const mpx_filter *f = mpx_find_filter(name);
    if (!f) {
        mpx::set_error("unknown filter '%s'", name);
        return MPX_ERR_ARG;
    }
    *k = f->k;
    *anchor = f->anchor;
    *mode = f->mode;
    const int n = (f->mode & MPX_CONV_SEP) ? MPX_SEP_NTAPS(f->k) : f->k * f->k;
    for (int i = 0; i < n; ++i) {
        wx[i] = f->wx[i];
        wy[i] = f->wy[i];
    }
    return MPX_OK;
}

extern "C" const char *mpx_filter_name(int i) { return (i >= 0 && i < MPX_NUM_FILTERS) ? mpx_filters[i].name : nullptr; }

extern "C" int mpx_class_stats(const uint32_t *img, int w, int h, int nc, const int *np, const int *coords,
                               double *mu, double *inv) {
    MPX_CHECK_ARG(img && np && coords && mu && inv, "null pointer");
    MPX_CHECK_ARG(nc >= 1 && nc <= MPX_MAX_CLASSES, "need 1 <= nc <= 32");
    for (int c = 0; c < nc; ++c) MPX_CHECK_ARG(np[c] >= 1, "every class needs at least one point");
    if (mpx_cpu_class_stats(img, w, h, nc, np, coords, mu, inv) != 0) {
        mpx::set_error("class point outside the %dx%d image", w, h);
        return MPX_ERR_ARG;
    }
    return MPX_OK;
}
