/*
 * C ABI of libmpx.so — the one native library behind every lab CLI, the
 * multi-GPU tools and the Python package (loaded with ctypes).
 *
 * Conventions
 *   - every function returns 0 on success, a non-zero mpx error code otherwise;
 *     mpx_last_error() returns a thread-local human readable message;
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream), so a
 *     PyTorch caller passes torch.cuda.current_stream().cuda_stream;
 *   - GPU entry points never allocate, free or synchronise (graph-capturable);
 *   - grid/block arguments of 0 mean "choose for MI355X" (256 CUs, wave64).
 *
 * The reference has no library at all (its library.cu is an empty kernel,
 * reference library.cu:3-4); every lab re-declared its own macros.
 */
#ifndef MPX_CAPI_H
#define MPX_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum mpx_status {
    MPX_OK = 0,
    MPX_ERR_ARG = 1,
    MPX_ERR_HIP = 2,
    MPX_ERR_UNSUPPORTED = 3,
    MPX_ERR_IO = 4
};

const char *mpx_last_error(void);
const char *mpx_version(void);
/* Loads every libmpx code object on the current device now instead of at the
 * first launch of one of its kernels (HIP loads them lazily, ~0.25 ms each). */
int mpx_preload_modules(void);

/* ---------------- device queries ---------------- */
int mpx_device_count(int *count);
/* Writes a multi-line report like the reference gpu_info (gpu_info/src/main.cu:9-16). */
int mpx_device_report(int device, char *buf, size_t len);
int mpx_stream_sync(void *stream);

/* ---------------- lab1: element-wise vector subtraction ---------------- */
/* c[i] = a[i] - b[i]; reference lab1/src/main.cu:22-29 */
int mpx_vsub_f64(const double *a, const double *b, double *c, int64_t n, int grid, int block,
                 void *stream);
int mpx_vsub_f32(const float *a, const float *b, float *c, int64_t n, int grid, int block,
                 void *stream);

/* ---------------- lab2: Roberts cross (launch-geometry faithful) ---------------- */
/* block (bx,by) and grid (gx,gy) exactly as the harness passes them
 * (reference lab2/src/to_plot.cu:57-64,106). Each thread owns 4 pixels of a row. */
int mpx_roberts(const uint32_t *in, uint32_t *out, int w, int h, int bx, int by, int gx, int gy,
                void *stream);
/* Per-channel Roberts cross, L1 magnitude, saturated to 255, alpha kept (the
 * operator of the reference's lab2/test_data samples; mpx_cpu_roberts_rgb). */
int mpx_roberts_rgb(const uint32_t *in, uint32_t *out, int w, int h, void *stream);

/* ---------------- lab2 generalisation: KxK convolution on luminance ---------------- */
/*
 * Output rows [oy0, oy1) of a (possibly slab-local) image.
 *   in/out   point at row 0 of the local slab, `pitch` pixels per row;
 *   y_lo/y_hi are the rows (relative to row 0, may be negative / >= rows when
 *            halo rows are resident) that input reads are clamped into;
 *   k, anchor  window size (2..7) and its anchor (taps at y+dy-anchor);
 *   wx, wy   k*k row-major taps (wy ignored unless mode == MPX_CONV_MAG2).
 * Accumulation order is fixed: dy ascending, dx ascending, one fmaf per tap.
 */
int mpx_conv(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo,
             int y_hi, int k, int anchor, int mode, const float *wx, const float *wy,
             void *stream);

/* mpx_conv with peer-sourced halo rows (one-sided xGMI loads): input rows with
 * logical index < 0 are read at in_up + row*pitch, rows >= own_rows at
 * in_dn + row*pitch (pointers into IPC-mapped neighbour slabs, biased so the
 * logical row index applies unchanged), rows [0, own_rows) from `in`. */
int mpx_conv_peer(const uint32_t *in, const uint32_t *in_up, const uint32_t *in_dn, int own_rows,
                  uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo, int y_hi, int k, int anchor,
                  int mode, const float *wx, const float *wy, void *stream);

/* Generic direct (untiled, one pixel per thread) variant of mpx_conv: any
 * anchor, naive global loads; the baseline the tiled kernel is measured against. */
int mpx_conv_direct(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo,
                    int y_hi, int k, int anchor, int mode, const float *wx, const float *wy,
                    void *stream);

/* Minimum image size in pixels for the band kernel (smaller aligned images take
 * the wave kernel); returns the previous value, n < 0 only queries. */
long long mpx_conv_set_band_min(long long n);
/* band kernel mode (as MPX_CONV_BAND: 0 wave kernel, 1 plain stores, 2 NT stores,
 * 3 NT stores + NT interior loads (default), 4 vertical halo sharing through LDS
 * for 5-row windows); returns the previous mode, m < 0 queries */
int mpx_conv_set_band_mode(int m);

/* Tuning-harness entry (tools/kbench.py): kernel variants for k in {2, 5}, MAG2,
 * whole image. kind 0 = LDS streaming kernel (p1 = rows per wave 4/8/16,
 * p2 = tiles per workgroup, 0 = auto); kind 1 = wave-streaming kernel
 * (p1 = rows per wave segment). fast selects the fast magnitude path. */
int mpx_conv_variant(const uint32_t *in, uint32_t *out, int w, int h, int k, int kind, int p1, int p2, int fast,
                     const float *wx, const float *wy, void *stream);
/* Exhaustive check of the fast magnitude path over every float in [0, 65025];
 * adds the number of disagreements with correctly rounded sqrtf to *bad_device. */
int mpx_selftest_fast_sqrt(unsigned long long *bad_device, int raw, void *stream);

/* Named filter table (native/include/mpx/filters.h). Returns MPX_ERR_ARG for an
 * unknown name; wx/wy receive k*k taps (wy zero-filled for one-filter modes).
 * mpx_filter_name(i) enumerates the table (NULL past the end). */
int mpx_filter_lookup(const char *name, int *k, int *anchor, int *mode, float *wx, float *wy);
const char *mpx_filter_name(int i);

/* ---------------- lab3: Mahalanobis maximum-likelihood classifier ---------------- */
/*
 * Per-class statistics from training points (reference lab3/src/main.cu:102-152).
 * coords holds (x, y) pairs for every class back to back; np[c] points per class.
 * mu: nc*3, inv: nc*9 (row-major inverse covariance), computed in fp64 on the host.
 */
int mpx_class_stats(const uint32_t *img, int w, int h, int nc, const int *np, const int *coords,
                    double *mu, double *inv);
/* img[i].a = argmin_c (p - mu_c)^T inv_c (p - mu_c), in place (alpha = 255 if all NaN). */
int mpx_classify(uint32_t *img, int64_t npix, int nc, const double *mu, const double *inv,
                 int grid, int block, int path, void *stream);
/* Same; when `ambiguous` (device uint32) is non-NULL it is incremented once per
 * pixel whose fp32 margin was too small and that took the exact fp64 chain. */
int mpx_classify_ex(uint32_t *img, int64_t npix, int nc, const double *mu, const double *inv,
                    int grid, int block, int path, uint32_t *ambiguous, void *stream);
/* Host-side plan: the path `path` resolves to for these statistics (DIRECT when
 * the fp32 decision cannot be proven) and the fp32 decision margin. <0 = error. */
int mpx_classify_plan(int nc, const double *mu, const double *inv, int path, float *margin);
/* MFMA8 integer weights as the kernel uses them (CPU emulation in the tests):
 * a, b: 32 x 16 int8 limbs per class and slot; c: 32 accumulator constants;
 * *t2: decision margin in key units. MPX_ERR_UNSUPPORTED when no bound exists. */
int mpx_classify_i8_params(int nc, const double *mu, const double *inv, int8_t *a, int8_t *b, int32_t *c,
                           int32_t *t2);

/* ---------------- native RCCL tier (inter-GPU transport) ---------------- */
/*
 * The ncclXxx entry points are bound with dlsym from `path` (the librccl torch
 * loaded; RTLD_NOLOAD first so one RCCL serves the whole process).
 * A communicator owns a non-blocking comm stream and two events:
 * p2p_start orders a grouped send/recv list after the work queued on `stream`
 * and runs it on the comm stream; p2p_wait makes `stream` wait for it.
 */
int mpx_comm_load(const char *path);
int mpx_comm_version(void);
int mpx_comm_unique_id(void *out, int nbytes); /* returns the id size */
int mpx_comm_init(void **comm, int nranks, int rank, const void *id, int nbytes, int device);
int mpx_comm_destroy(void *comm);
int mpx_comm_rank(void *comm);
int mpx_comm_size(void *comm);
int mpx_comm_p2p_start(void *comm, int n, const int *kind, void *const *ptr, const int64_t *bytes,
                       const int *peer, void *stream); /* kind 0 send, 1 recv */
int mpx_comm_p2p_wait(void *comm, void *stream);
/* the same op list in order on `stream` itself (no comm stream, no events) */
int mpx_comm_p2p(void *comm, int n, const int *kind, void *const *ptr, const int64_t *bytes, const int *peer,
                 void *stream);
/* dtype 0 f64, 1 f32, 2 i32, 3 u64; op 0 sum, 1 max, 2 min; on `stream` */
int mpx_comm_allreduce(void *comm, const void *send, void *recv, int64_t count, int dtype, int op,
                       void *stream);
int mpx_comm_check(void *comm);
/* ncclCommAbort: release a communicator whose peers hung or died (watchdog) */
int mpx_comm_abort(void *comm);
/* the communicator's comm stream (for caller-managed cross-step pipelining) */
void *mpx_comm_stream(void *comm);

/* ---------------- device memory shared between the processes of a node ---------------- */
int mpx_ipc_handle_size(void);
/* handle: mpx_ipc_handle_size() bytes; *offset = ptr - base of ptr's allocation */
int mpx_ipc_get_handle(const void *ptr, void *handle, int64_t *offset);
/* maps a peer's allocation on the current device (peer access enabled lazily) */
int mpx_ipc_open(const void *handle, void **base);
/* the same with hipSetDevice(device) first (mapping from a helper thread) */
int mpx_ipc_open_dev(int device, const void *handle, void **base);
int mpx_ipc_close(void *base);
/* stream-ordered device-to-device copy (either side may be IPC-mapped) */
int mpx_memcpy_d2d(void *dst, const void *src, int64_t bytes, void *stream);

/* ---------------- one-sided transports: probes, streaming halo fetch (peer.hip) ---------------- */
/* *out += position-sensitive checksum of nrows rows read with the kernels' 16-byte
 * buffer loads (sys != 0: system-scope cache policy); zero *out first. */
int mpx_rows_checksum(const void *rows, int64_t row_bytes, int nrows, int64_t pitch_bytes, int sys,
                      unsigned long long *out, void *stream);
/* Signalled start-up probe (one workgroup): write a (rank, buffer)-pattern into
 * own_rows[0..3] (buffer = index / 2; NULL = skip) with system-scope stores,
 * publish sync[0] = magic (release), then for each side s with flag[s]: wait
 * flag[s] >= magic (bounded; sync[64] = 1 on give-up) and compare
 * nb_rows[s][0..1] with the neighbour's pattern; mismatching words are added
 * to sync[96]. row_bytes: a multiple of 4 (16-byte accesses when every row is
 * 16-byte aligned and row_bytes a multiple of 16, 4-byte ones otherwise). */
typedef struct mpx_peer_probe {
    void *own_rows[4];
    const void *nb_rows[2][2];
    const unsigned int *flag[2];
    unsigned int *sync;
    int64_t row_bytes;
    int rank;
    unsigned int magic;
    unsigned int spin_limit;
} mpx_peer_probe;
int mpx_peer_probe_run(const mpx_peer_probe *p, void *stream);
/* Streaming halo fetch (filters the fused band kernel does not cover): block s
 * first copies this rank's own boundary rows own_src[s] into its mailbox rows
 * mb_dst[s] (mb_bytes[s], system-scope write-through stores); once BOTH blocks'
 * copies are acknowledged the later one publishes sync[0] = step (release).
 * Then per side s with a neighbour (flag[s] != NULL): wait flag[s] >= step
 * (bounded), and when src[s] is set copy bytes[s] from it (the neighbour's
 * mailbox rows, system-scope loads) to dst[s] (this rank's halo rows). A side
 * without rows to copy still waits: the neighbour reads this rank's mailbox
 * (write-after-read order). */
typedef struct mpx_halo_fetch {
    const void *src[2];
    void *dst[2];
    int64_t bytes[2];
    const unsigned int *flag[2];
    unsigned int *sync;
    unsigned int step;
    unsigned int spin_limit;
    const void *own_src[2];
    void *mb_dst[2];
    int64_t mb_bytes[2];
} mpx_halo_fetch;
int mpx_halo_fetch_run(const mpx_halo_fetch *f, void *stream);
/* Streaming convolution with the halo exchange fused into the band kernel (one
 * launch per step, no fetch kernel): the waves whose rows touch the slab edges
 * read their halo rows straight from the neighbours' mailboxes (system-scope
 * loads) after a bounded wait on the neighbour's step word, write their first
 * n_first / last n_last output rows into this rank's mailbox as well
 * (write-through), and the last of the n_edge edge waves publishes the step;
 * interior waves never wait. The step index c = this rank's sync[0] (completed
 * steps, read on the device): the halo rows come from slot c & 1 of the
 * neighbours' mailboxes, the output rows go to slot (c + 1) & 1 of this one.
 * up_src[p] / dn_src[p]: biased row-source pointers (logical row g < 0 at
 * up_src[p] + g * w, g >= own_rows at dn_src[p] + g * w); NULL flag = global
 * edge (the clamp rows then come from `in` itself). Requires the band kernel:
 * k <= 5 with at most two columns of reach per side, w % 4 == 0, pitch == w,
 * 16-byte aligned rows. */
typedef struct mpx_conv_stream_peer {
    const uint32_t *up_src[2];
    const uint32_t *dn_src[2];
    const unsigned int *up_flag;
    const unsigned int *dn_flag;
    uint32_t *mb_first[2];
    uint32_t *mb_last[2];
    unsigned int *sync;
    int n_first;
    int n_last;
    int n_edge; /* filled in by the launcher */
    unsigned int spin_limit;
} mpx_conv_stream_peer;
int mpx_conv_stream_peer_run(const uint32_t *in, uint32_t *out, int w, int pitch, int own_rows, int y_lo, int y_hi,
                         int k, int anchor, int mode, const float *wx, const float *wy,
                         const mpx_conv_stream_peer *sp, void *stream);
/* 1 when mpx_conv_stream_peer can run this launch shape, else 0 */
int mpx_conv_stream_peer_ok(int w, int pitch, int own_rows, int k, int anchor, int mode);
/* IPC-exportable sync block: uncached (kind 2), fine-grained (1) or coarse (0) memory, zeroed */
int mpx_sync_alloc(int64_t bytes, void **ptr, int *kind);
int mpx_sync_free(void *ptr);
/* synchronous host access to word `word` (0..127) of a sync block */
int mpx_sync_write(unsigned int *sync, int word, unsigned int value);
int mpx_sync_read(const unsigned int *sync, int word, unsigned int *value);
int mpx_sync_clear(unsigned int *sync, int64_t bytes);

/* ---------------- 2-D Jacobi (distributed stencil tier) ---------------- */
/*
 * One sweep over rows [r0, r1) of a slab stored with one halo row above and
 * below: `u`/`un` point at the first halo row, rows 1..rows are owned, the row
 * pitch is `pitch` elements, columns 0 and cols-1 are Dirichlet boundary.
 *   un[i][j] = 0.25*(u[i-1][j] + u[i+1][j] + u[i][j-1] + u[i][j+1])  (j in 1..cols-2)
 * Rows listed in [r0, r1) are 1-based owned rows. When `resid` is non-NULL the
 * kernel folds max|un-u| over the swept points into *resid (atomic max, bit
 * pattern of a non-negative double), so callers zero it first.
 */
/* One-sided, device-signalled halo sweep of a whole slab (rows 1..rows of a
 * (rows + 2) x pitch buffer): the halo rows are read from the neighbours'
 * IPC-mapped buffers, ordered by completed-iteration counters (see jacobi.hip).
 * up_row[k] / dn_row[k]: the neighbour's last / first owned row of u at even
 * (k = 0) / odd (k = 1) iterations — rows of its MAILBOX (a small exported
 * allocation, so slabs of any size keep the one-sided transport), or of its
 * slab buffers when mb_first / mb_last are NULL; NULL (with a NULL flag) at
 * the global boundary, where the local halo row is the boundary row.
 * sync: this rank's mpx_jacobi_sync_bytes() block; word 0 = completed
 * iterations (the neighbours' *_flag points at theirs), word 64 != 0 after a
 * bounded wait gave up. */
typedef struct mpx_jacobi_peer {
    const void *up_row[2];
    const void *dn_row[2];
    const unsigned int *up_flag;
    const unsigned int *dn_flag;
    unsigned int *sync;
    unsigned int spin_limit; /* polls before a wait gives up (0 = default, ~seconds) */
    /* this rank's mailbox rows (one row each; slot p receives the edge row of
     * u^(t) for t % 2 == p, written during sweep t - 1 with write-through
     * stores): mb_first = its first owned row (read by the upper neighbour),
     * mb_last = its last (read by the lower one); NULL at a global edge */
    void *mb_first[2];
    void *mb_last[2];
} mpx_jacobi_peer;
int mpx_jacobi_sync_bytes(void);
int mpx_jacobi_peer_sweep(int fp64, void *u, void *un, int cols, int pitch, int rows, void *resid,
                          const mpx_jacobi_peer *p, void *stream);
int mpx_jacobi_f64(const double *u, double *un, int cols, int pitch, int r0, int r1,
                   double *resid, void *stream);
int mpx_jacobi_f32(const float *u, float *un, int cols, int pitch, int r0, int r1, float *resid,
                   void *stream);

/* ---------------- lab5: ascending sort (no reference program) ---------------- */
/* In place on the device; dtype is an mpx_sort_dtype. int32/float32: LSD radix sort
 * (onesweep, 8-bit digits) on order-preserving uint32 keys, bitonic network for
 * n <= 4096 or n >= 2^30; uint8: counting sort.
 * mpx_sort_ws takes the scratch from the caller (>= mpx_sort_workspace_bytes(n, dtype)
 * bytes, 16-byte aligned, stream-ordered with `stream`; may be NULL when that size is 0).
 * mpx_sort allocates and frees its own scratch and synchronises the stream. */
int64_t mpx_sort_workspace_bytes(int64_t n, int dtype);
int mpx_sort_ws(void *data, int64_t n, int dtype, void *workspace, int64_t workspace_bytes, void *stream);
/* After the sort's stream drained: non-zero if a bounded look-back wait of the
 * sort that last used `workspace` gave up (hardware-fault detector). */
int mpx_sort_ws_status(const void *workspace, int64_t n, int dtype);
int mpx_sort(void *data, int64_t n, int dtype, void *stream);
/* 1 when the current device applies same-address returning LDS adds in
 * ascending lane order (the stability premise of the production radix
 * ranking; probed once per device, synchronising the stream), 0 when not,
 * negative when the probe could not run. AUTO falls back to the peer-mask
 * ranking unless 1. */
int mpx_sort_lane_order_ok(void *stream);

/* ---------------- CPU references (OpenMP, -O3, same numerics) ---------------- */
int mpx_cpu_threads(void);
void mpx_cpu_vsub_f64(const double *a, const double *b, double *c, int64_t n);
void mpx_cpu_vsub_f32(const float *a, const float *b, float *c, int64_t n);
void mpx_cpu_roberts(const uint32_t *in, uint32_t *out, int w, int h);
void mpx_cpu_roberts_rgb(const uint32_t *in, uint32_t *out, int w, int h);
void mpx_cpu_conv(const uint32_t *in, uint32_t *out, int w, int pitch, int oy0, int oy1, int y_lo,
                  int y_hi, int k, int anchor, int mode, const float *wx, const float *wy);
void mpx_cpu_classify(uint32_t *img, int64_t npix, int nc, const double *mu, const double *inv);
double mpx_cpu_jacobi_f64(const double *u, double *un, int cols, int pitch, int r0, int r1);
void mpx_cpu_sort(void *data, int64_t n, int dtype);

#ifdef __cplusplus
}
#endif

#endif /* MPX_CAPI_H */
