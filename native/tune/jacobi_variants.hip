// Tuning entry point of the Jacobi wave kernel (tools/experiments/jbench.py):
// explicit rows per wave R and the A/B forms of round 2-3 (buffer-store cache
// policy, non-temporal loads, no tail exit, alternating walks, 16-wave
// workgroups). Built into libmpx_tune.so only; production launches are in
// native/src/kernels/jacobi.hip.
#include "../src/kernels/jacobi_wave.hpp"

// Tuning entry point (tools/jbench.py): wave kernel with an explicit rows-per-
// wave R and buffer-store cache policy aux (0 default, 2 = nontemporal).
extern "C" int mpx_jacobi_variant(void *u, void *un, int cols, int pitch, int r0, int r1, void *resid, int fp64,
                                  int R, int aux, void *stream) {
    using namespace mpx;
    MPX_CHECK_ARG(u && un && cols >= 1 && pitch >= cols && r0 >= 1 && r1 >= r0 && R >= 1, "bad arguments");
    MPX_CHECK_ARG(aux == 0 || aux == 2 || aux == 6 || aux == 10 || aux == 18 || aux == 22 || aux == 50,
                  "aux must be 0, 2, 6 (2 + non-temporal loads), 10 (2 without the tail exit) or 18 (2 + "
                  "alternating walk directions), 22 (18 + non-temporal interior row loads), 50 (18 with 16-wave "
                  "workgroups)");
    const int NV = fp64 ? 2 : 4;
    MPX_CHECK_ARG(pitch % NV == 0 && cols % NV == 0 && aligned16(u) && aligned16(un), "needs the vector layout");
    const int strips = (cols / NV + kStripVec - 1) / kStripVec;
    const int nwaves = strips * ((r1 - r0 + R - 1) / R);
    const dim3 g((nwaves + 3) / 4), b(256);
    hipStream_t s = as_stream(stream);
#define MPX_JV(T, A)                                                                                          \
    hipLaunchKernelGGL((jacobi_wave_kernel<T, A>), g, b, 0, s, (const T *)u, (T *)un, cols, pitch, r0, r1, strips, \
                       R, nwaves, (T *)resid, mpx_jacobi_peer{})
#define MPX_JVN(T)                                                                                             \
    hipLaunchKernelGGL((jacobi_wave_kernel<T, 2, 1>), g, b, 0, s, (const T *)u, (T *)un, cols, pitch, r0, r1,    \
                       strips, R, nwaves, (T *)resid, mpx_jacobi_peer{})
#define MPX_JVA(T)                                                                                             \
    hipLaunchKernelGGL((jacobi_wave_kernel<T, 2, 0, true, false, true>), g, b, 0, s, (const T *)u, (T *)un, cols,  \
                       pitch, r0, r1, strips, R, nwaves, (T *)resid, mpx_jacobi_peer{})
#define MPX_JVW(T)                                                                                             \
    hipLaunchKernelGGL((jacobi_wave_kernel<T, 2, 0, true, false, true, 16>), dim3((nwaves + 15) / 16), dim3(1024),  \
                       0, s, (const T *)u, (T *)un, cols, pitch, r0, r1, strips, R, nwaves, (T *)resid, mpx_jacobi_peer{})
#define MPX_JVI(T)                                                                                             \
    hipLaunchKernelGGL((jacobi_wave_kernel<T, 2, 2, true, false, true>), g, b, 0, s, (const T *)u, (T *)un, cols,  \
                       pitch, r0, r1, strips, R, nwaves, (T *)resid, mpx_jacobi_peer{})
#define MPX_JVX(T)                                                                                             \
    hipLaunchKernelGGL((jacobi_wave_kernel<T, 2, 0, false>), g, b, 0, s, (const T *)u, (T *)un, cols, pitch, r0, \
                       r1, strips, R, nwaves, (T *)resid, mpx_jacobi_peer{})
    if (fp64) {
        if (aux == 22) MPX_JVI(double); else if (aux == 50) MPX_JVW(double); else if (aux == 18) MPX_JVA(double); else if (aux == 10) MPX_JVX(double); else if (aux == 6) MPX_JVN(double); else if (aux) MPX_JV(double, 2); else MPX_JV(double, 0);
    } else {
        if (aux == 22) MPX_JVI(float); else if (aux == 50) MPX_JVW(float); else if (aux == 18) MPX_JVA(float); else if (aux == 10) MPX_JVX(float); else if (aux == 6) MPX_JVN(float); else if (aux) MPX_JV(float, 2); else MPX_JV(float, 0);
    }
#undef MPX_JV
#undef MPX_JVN
#undef MPX_JVX
#undef MPX_JVI
#undef MPX_JVA
#undef MPX_JVW
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}
