// Inter-process device memory sharing between the ranks of one node (one
// process per MI355X): a rank exports an IPC handle of its slab allocation,
// its neighbours map it and read the halo rows straight over xGMI
// (mpx_conv_peer). Handles are dmabuf-backed on this stack
// (HSA_ENABLE_IPC_MODE_LEGACY=0). The reference has no multi-GPU code at all
// (SURVEY §2.6); this is the one-sided transport of the halo exchange.
#include <hip/hip_runtime.h>

#include <cstring>

#include "../kernels/internal.hpp"

extern "C" int mpx_ipc_handle_size(void) { return (int)sizeof(hipIpcMemHandle_t); }

// handle: mpx_ipc_handle_size() bytes; offset: ptr - base of its allocation
// (a caching allocator hands out sub-ranges of larger hipMalloc blocks).
extern "C" int mpx_ipc_get_handle(const void *ptr, void *handle, int64_t *offset) {
    MPX_CHECK_ARG(ptr && handle && offset, "null pointer");
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    MPX_RETURN_IF_HIP_ERROR(hipMemGetAddressRange(&base, &size, const_cast<void *>(ptr)));
    hipIpcMemHandle_t h;
    MPX_RETURN_IF_HIP_ERROR(hipIpcGetMemHandle(&h, base));
    std::memcpy(handle, &h, sizeof(h));
    *offset = reinterpret_cast<const char *>(ptr) - reinterpret_cast<const char *>(base);
    return MPX_OK;
}

// Maps a peer's allocation on the current device; *base is what
// mpx_ipc_close takes back (add the exporter's offset to reach its tensor).
extern "C" int mpx_ipc_open(const void *handle, void **base) {
    MPX_CHECK_ARG(handle && base, "null pointer");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle, sizeof(h));
    MPX_RETURN_IF_HIP_ERROR(hipIpcOpenMemHandle(base, h, hipIpcMemLazyEnablePeerAccess));
    return MPX_OK;
}

// Same on an explicit device: for callers that map from a helper thread
// (a deadline-bounded open), whose current device is not the rank's.
extern "C" int mpx_ipc_open_dev(int device, const void *handle, void **base) {
    MPX_RETURN_IF_HIP_ERROR(hipSetDevice(device));
    return mpx_ipc_open(handle, base);
}

extern "C" int mpx_ipc_close(void *base) {
    MPX_CHECK_ARG(base, "null pointer");
    MPX_RETURN_IF_HIP_ERROR(hipIpcCloseMemHandle(base));
    return MPX_OK;
}

// Stream-ordered device-to-device copy (also from an IPC-mapped peer range):
// fills halo rows for verification and for callers that want a local copy.
extern "C" int mpx_memcpy_d2d(void *dst, const void *src, int64_t bytes, void *stream) {
    MPX_CHECK_ARG(dst && src && bytes >= 0, "bad arguments");
    if (bytes == 0) return MPX_OK;
    MPX_RETURN_IF_HIP_ERROR(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, mpx::as_stream(stream)));
    return MPX_OK;
}
