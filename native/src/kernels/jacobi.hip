// 2-D Jacobi sweep for the distributed stencil tier (the MPI north star of
// BASELINE.json, re-expressed over RCCL): slab rows with one halo row above
// and below, Dirichlet columns 0 and cols-1, fused L-infinity residual.
//
// MI355X design: HBM-bound 5-point stencil (2 x 8 B per fp64 point).
//   * wave strips: a wave owns a strip of 62 16-B column vectors (lanes 1..62
//     compute, lanes 0 and 63 only load the strip's halo vectors) and walks
//     R rows down it, so every input row is fetched once per sweep and the
//     left/right neighbours of a vector come from the adjacent lanes through
//     DPP wave shifts (v_mov_dpp wave_shr:1 / wave_shl:1) — one 16-B load per
//     lane and row, nothing re-read through L1;
//   * a 5-slot row ring of unconditional (clamped) loads, unrolled by 5 so the
//     slots are compile-time registers, keeps three rows of HBM requests in
//     flight per wave; stores are raw buffer stores whose
//     masked-off lanes get an out-of-range offset, so there is no divergent
//     store branch to break the compiler's vmcnt accounting;
//   * the residual is reduced wave -> lane 0 -> one device-scope atomic max per
//     wave on the bit pattern (non-negative IEEE values order like unsigned
//     integers), so no second kernel is needed.
// Pitches or widths that are not a multiple of the vector width use the
// generic per-lane kernel below.
#include "jacobi_wave.hpp"

namespace mpx {
namespace {

template <typename T>
int launch_jacobi(const T *u, T *un, int cols, int pitch, int r0, int r1, T *resid, void *stream) {
    MPX_CHECK_ARG(u && un, "null pointer");
    MPX_CHECK_ARG(cols >= 1 && pitch >= cols && r0 >= 1 && r1 >= r0, "bad slab geometry");
    if (r1 == r0) return MPX_OK;
    constexpr int NV = JVec<T>::n;
    if ((pitch % NV == 0) && (cols % NV == 0) && aligned16(u) && aligned16(un)) {
        const int strips = (cols / NV + kStripVec - 1) / kStripVec;
        const int rows = r1 - r0;
        // 8 rows per wave, odd row blocks walking up (ALT: two vertically
        // adjacent blocks read their shared halo rows at the same moment) —
        // tools/jbench.py, profiles/jacobi.md: 16384^2 fp64 R8+alt 728 us vs
        // 763 (R5, all down) / 767 (R8, all down); fp32 363 vs 370 / 396.
        // Stores nontemporal (aux NT): the next sweep reads u_new from HBM
        // anyway, and keeping it out of L2 leaves L2 to the shared halo rows
        int R = kJacobiRows;
        while (R > 1 && (int64_t)strips * ((rows + R - 1) / R) < 16384) R >>= 1;
        const int nwaves = strips * ((rows + R - 1) / R);
        hipLaunchKernelGGL((jacobi_wave_kernel<T, 2, 0, true, false, true>), dim3((nwaves + 3) / 4), dim3(256), 0,
                           as_stream(stream), u, un, cols, pitch, r0, r1, strips, R, nwaves, resid, mpx_jacobi_peer{});
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
        return MPX_OK;
    }
    const bool vec = (pitch % NV == 0) && aligned16(u) && aligned16(un);
    const int lanes = vec ? (cols + NV - 1) / NV : cols;
    const dim3 blk(256);
    const dim3 grd((lanes + 255) / 256, (r1 - r0 + kRows - 1) / kRows);
    if (vec)
        hipLaunchKernelGGL((jacobi_kernel<T, true>), grd, blk, 0, as_stream(stream), u, un, cols, pitch, r0, r1, resid);
    else
        hipLaunchKernelGGL((jacobi_kernel<T, false>), grd, blk, 0, as_stream(stream), u, un, cols, pitch, r0, r1,
                           resid);
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}

template <typename T>
int launch_jacobi_peer(const T *u, T *un, int cols, int pitch, int rows, T *resid, const mpx_jacobi_peer &pr,
                       void *stream) {
    MPX_CHECK_ARG(u && un && pr.sync, "null pointer");
    MPX_CHECK_ARG(cols >= 1 && pitch >= cols && rows >= 1, "bad slab geometry");
    MPX_CHECK_ARG(!pr.up_flag == !pr.up_row[0] && !pr.up_row[0] == !pr.up_row[1], "up neighbour: rows and flag together");
    MPX_CHECK_ARG(!pr.dn_flag == !pr.dn_row[0] && !pr.dn_row[0] == !pr.dn_row[1], "down neighbour: rows and flag together");
    constexpr int NV = JVec<T>::n;
    MPX_CHECK_ARG(pitch % NV == 0 && cols % NV == 0 && aligned16(u) && aligned16(un),
                  "peer halos need the 16-byte vector layout (cols and pitch multiples of the vector width)");
    for (const void *q : {pr.up_row[0], pr.up_row[1], pr.dn_row[0], pr.dn_row[1], (const void *)pr.mb_first[0],
                          (const void *)pr.mb_first[1], (const void *)pr.mb_last[0], (const void *)pr.mb_last[1]})
        MPX_CHECK_ARG(!q || aligned16(q), "neighbour and mailbox rows must be 16-byte aligned");
    MPX_CHECK_ARG(!pr.mb_first[0] == !pr.mb_first[1] && !pr.mb_last[0] == !pr.mb_last[1],
                  "mailbox rows come in slot pairs");
    MPX_CHECK_ARG((!pr.mb_first[0] || pr.up_flag) && (!pr.mb_last[0] || pr.dn_flag),
                  "a mailbox side needs the neighbour that reads it");
    const int strips = (cols / NV + kStripVec - 1) / kStripVec;
    int R = kJacobiRows;
    while (R > 1 && (int64_t)strips * ((rows + R - 1) / R) < 16384) R >>= 1;
    const int nwaves = strips * ((rows + R - 1) / R);
    hipLaunchKernelGGL((jacobi_wave_kernel<T, 2, 0, true, true, true>), dim3((nwaves + 3) / 4), dim3(256), 0,
                       as_stream(stream), u, un, cols, pitch, 1, rows + 1, strips, R, nwaves, resid, pr);
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}

}  // namespace
MPX_MODULE_ANCHOR(jacobi)

}  // namespace mpx

extern "C" int mpx_jacobi_f64(const double *u, double *un, int cols, int pitch, int r0, int r1, double *resid,
                              void *stream) {
    return mpx::launch_jacobi<double>(u, un, cols, pitch, r0, r1, resid, stream);
}

extern "C" int mpx_jacobi_f32(const float *u, float *un, int cols, int pitch, int r0, int r1, float *resid,
                              void *stream) {
    return mpx::launch_jacobi<float>(u, un, cols, pitch, r0, r1, resid, stream);
}

extern "C" int mpx_jacobi_peer_sweep(int fp64, void *u, void *un, int cols, int pitch, int rows, void *resid,
                                     const mpx_jacobi_peer *p, void *stream) {
    using namespace mpx;
    MPX_CHECK_ARG(p, "null peer descriptor");
    if (fp64)
        return launch_jacobi_peer<double>((const double *)u, (double *)un, cols, pitch, rows, (double *)resid, *p,
                                          stream);
    return launch_jacobi_peer<float>((const float *)u, (float *)un, cols, pitch, rows, (float *)resid, *p, stream);
}

extern "C" int mpx_jacobi_sync_bytes(void) { return 4 * 128; }
