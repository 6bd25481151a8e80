// lab3: per-pixel Mahalanobis maximum-likelihood classification.
//
// Reference: lab3/src/main.cu:40-76 — for every pixel p, argmin over classes of
// (p - mu_c)^T A_c (p - mu_c) in fp64 with class statistics in __constant__
// memory; strict '<' keeps the lowest class on ties, an all-NaN pixel keeps
// class -1 (stored as 255); alpha is written in place.
//
// MI355X design
//   * class parameters travel as a kernel-argument block (3 KiB, < 4 KiB
//     kernarg limit): the class loop index is wave-uniform, so every mu/A load
//     is a scalar s_load into SGPRs — the CDNA equivalent of a constant-cache
//     broadcast, without a hipMemcpyToSymbol in the launch path;
//   * each lane classifies 4 pixels from one 16-B load and writes them back with
//     one 16-B store (the reference does a 4-B load and a 1-B store per pixel);
//   * DIRECT path: the same FMA chain the reference GPU kernel compiles to, so
//     results are bit-identical to mpx_cpu_classify;
//   * MFMA path: dist = phi(p) . w_c with phi = [r^2 g^2 b^2 rg rb gb r g b 1],
//     evaluated as a (16 pixels x 12) x (12 x 16 classes) fp64 GEMM per wave on
//     v_mfma_f64_16x16x4_f64, then a top-2 argmin; any pixel whose best/second
//     margin is within a rigorous rounding bound is recomputed with the DIRECT
//     chain, so the chosen class is identical to the reference's.
#include "internal.hpp"

#include <cmath>

namespace mpx {
namespace {

struct ClassParams {
    double mu[MPX_MAX_CLASSES * 3];
    double A[MPX_MAX_CLASSES * 9];
};

__device__ __forceinline__ uint32_t classify_direct(uint32_t p, int nc, const ClassParams &cp) {
    const double pr = (double)mpx_px_r(p), pg = (double)mpx_px_g(p), pb = (double)mpx_px_b(p);
    double best = 1.7976931348623157e308;  // DBL_MAX
    int cls = -1;
    for (int c = 0; c < nc; ++c) {
        const double d0 = pr - cp.mu[3 * c + 0];
        const double d1 = pg - cp.mu[3 * c + 1];
        const double d2 = pb - cp.mu[3 * c + 2];
        const double *A = cp.A + 9 * c;
        double t0 = fma(d0, A[0], 0.0), t1 = fma(d0, A[1], 0.0), t2 = fma(d0, A[2], 0.0);
        t0 = fma(d1, A[3], t0);
        t1 = fma(d1, A[4], t1);
        t2 = fma(d1, A[5], t2);
        t0 = fma(d2, A[6], t0);
        t1 = fma(d2, A[7], t1);
        t2 = fma(d2, A[8], t2);
        double dist = fma(t0, d0, 0.0);
        dist = fma(t1, d1, dist);
        dist = fma(t2, d2, dist);
        if (dist < best) {
            best = dist;
            cls = c;
        }
    }
    return (p & 0x00ffffffu) | ((uint32_t)(uint8_t)cls << 24);
}

__global__ void classify_direct_kernel(uint32_t *__restrict__ img, int64_t npix, int nc, ClassParams cp,
                                       int vec) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t done = 0;
    if (vec) {
        const int64_t nvec = npix / 4;
        uint4 *v = reinterpret_cast<uint4 *>(img);
        for (int64_t i = tid; i < nvec; i += stride) {
            uint4 q = v[i];
            q.x = classify_direct(q.x, nc, cp);
            q.y = classify_direct(q.y, nc, cp);
            q.z = classify_direct(q.z, nc, cp);
            q.w = classify_direct(q.w, nc, cp);
            v[i] = q;
        }
        done = nvec * 4;
    }
    for (int64_t i = done + tid; i < npix; i += stride) img[i] = classify_direct(img[i], nc, cp);
}

// ---------------------------------------------------------------------------
// MFMA path. Geometry: 256-thread workgroups, each wave handles 16-pixel
// groups; D[class][pixel] = sum_k W[k][class] * PHI[k][pixel] so that after
// the MFMA lane l holds pixel (l & 15) for classes (l >> 4) + 4*reg.
// v_mfma_f64_16x16x4_f64 operand maps (cdna_hip_programming.md §3):
//   A[i][k]: lane l holds A[l & 15][k = l >> 4];  B[k][j]: lane l holds B[k = l >> 4][l & 15]
//   C/D:     lane l, reg r holds D[row = (l >> 4) + 4 r][col = l & 15]
// Here A = W^T (16 classes x 4 k), B = PHI (4 k x 16 pixels).
// ---------------------------------------------------------------------------
typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kPhi = 12;  // 10 features padded to 3 k-steps of 4

struct QuadParams {
    double w[kPhi][32];  // w[k][class]: expanded quadratic-form weights (class padded to 32)
    double tol[32];      // per-class rounding tolerance; +inf for padded classes
};

// feature k = 4*ks + kq of phi for this lane's pixel, as selects (no divergent
// switch, no runtime-indexed array that would spill to scratch)
template <int KS>
__device__ __forceinline__ double phi_of(int kq, double r, double g, double b) {
    if constexpr (KS == 0) return kq == 0 ? r * r : (kq == 1 ? g * g : (kq == 2 ? b * b : r * g));
    else if constexpr (KS == 1) return kq == 0 ? r * b : (kq == 1 ? g * b : (kq == 2 ? r : g));
    else return kq == 0 ? b : (kq == 1 ? 1.0 : 0.0);
}

__global__ __launch_bounds__(256) void classify_mfma_kernel(uint32_t *__restrict__ img, int64_t npix, int nc,
                                                            ClassParams cp, QuadParams qp) {
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * (blockDim.x >> 6)) + (threadIdx.x >> 6);
    const int nwaves = gridDim.x * (blockDim.x >> 6);
    const int col = lane & 15;  // pixel within the 16-pixel group
    const int kq = lane >> 4;   // k row this lane feeds, and class row-block of the result
    const int ncb = (nc + 15) >> 4;  // 16-class blocks (1 or 2)
    const int64_t ngroups = (npix + 15) >> 4;
    for (int64_t g = wave; g < ngroups; g += nwaves) {
        const int64_t pi = g * 16 + col;
        const bool valid = pi < npix;
        const uint32_t p = valid ? img[pi] : 0u;
        const double r = (double)mpx_px_r(p), gg = (double)mpx_px_g(p), b = (double)mpx_px_b(p);
        double best = 1.7976931348623157e308, second = 1.7976931348623157e308;
        double best_tol = 0.0, second_tol = 0.0;
        int cls = -1;
        for (int cb = 0; cb < ncb; ++cb) {
            f64x4 acc = {0.0, 0.0, 0.0, 0.0};
            // A operand: class (lane & 15), k (lane >> 4); B operand: k (lane >> 4), pixel (lane & 15)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(qp.w[0 + kq][cb * 16 + col], phi_of<0>(kq, r, gg, b), acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(qp.w[4 + kq][cb * 16 + col], phi_of<1>(kq, r, gg, b), acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(qp.w[8 + kq][cb * 16 + col], phi_of<2>(kq, r, gg, b), acc, 0, 0, 0);
            // lane holds classes cb*16 + kq + 4*reg for pixel col
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const int c = cb * 16 + kq + 4 * reg;
                const double d = acc[reg];
                const double t = qp.tol[c];
                if (c < nc) {
                    if (d < best) {
                        second = best;
                        second_tol = best_tol;
                        best = d;
                        best_tol = t;
                        cls = c;
                    } else if (d < second) {
                        second = d;
                        second_tol = t;
                    }
                }
            }
        }
        // merge the 4 lanes (kq = 0..3) that share this pixel: xor 16, xor 32
#pragma unroll
        for (int m = 16; m <= 32; m <<= 1) {
            const double ob = __shfl_xor(best, m), os = __shfl_xor(second, m);
            const double obt = __shfl_xor(best_tol, m), ost = __shfl_xor(second_tol, m);
            const int oc = __shfl_xor(cls, m);
            // keep lowest class index on exact ties (reference strict '<' order)
            const bool take = (ob < best) || (ob == best && oc < cls && oc >= 0);
            double nb, nbt, ns, nst;
            int nc2;
            if (take) {
                nb = ob; nbt = obt; nc2 = oc;
                // new second = min(best, os)
                if (best < os) { ns = best; nst = best_tol; } else { ns = os; nst = ost; }
            } else {
                nb = best; nbt = best_tol; nc2 = cls;
                if (ob < second) { ns = ob; nst = obt; } else { ns = second; nst = second_tol; }
            }
            best = nb; best_tol = nbt; cls = nc2; second = ns; second_tol = nst;
        }
        if (valid && kq == 0) {
            // ambiguous (margin within rounding bounds) or non-finite: exact direct chain
            const bool ambiguous = !(second - best > best_tol + second_tol) || !(best == best);
            uint32_t res;
            if (ambiguous || cls < 0)
                res = classify_direct(p, nc, cp);
            else
                res = (p & 0x00ffffffu) | ((uint32_t)cls << 24);
            img[pi] = res;
        }
    }
}

bool build_quad(int nc, const double *mu, const double *inv, QuadParams &qp) {
    const double u = 1.1102230246251565e-16;  // 2^-53
    for (int k = 0; k < kPhi; ++k)
        for (int c = 0; c < 32; ++c) qp.w[k][c] = 0.0;
    for (int c = 0; c < 32; ++c) qp.tol[c] = INFINITY;
    for (int c = 0; c < nc; ++c) {
        const double *A = inv + 9 * c;
        double S[3][3], Sa[3][3];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                S[i][j] = 0.5 * (A[3 * i + j] + A[3 * j + i]);
                Sa[i][j] = 0.5 * (std::fabs(A[3 * i + j]) + std::fabs(A[3 * j + i]));
            }
        const double m[3] = {mu[3 * c], mu[3 * c + 1], mu[3 * c + 2]};
        for (int i = 0; i < 3; ++i)
            if (!std::isfinite(m[i])) return false;
        for (int i = 0; i < 9; ++i)
            if (!std::isfinite(A[i])) return false;
        double Sm[3], Sam[3];
        for (int i = 0; i < 3; ++i) {
            Sm[i] = S[i][0] * m[0] + S[i][1] * m[1] + S[i][2] * m[2];
            Sam[i] = Sa[i][0] * std::fabs(m[0]) + Sa[i][1] * std::fabs(m[1]) + Sa[i][2] * std::fabs(m[2]);
        }
        const double mSm = m[0] * Sm[0] + m[1] * Sm[1] + m[2] * Sm[2];
        const double mSam = std::fabs(m[0]) * Sam[0] + std::fabs(m[1]) * Sam[1] + std::fabs(m[2]) * Sam[2];
        qp.w[0][c] = S[0][0];
        qp.w[1][c] = S[1][1];
        qp.w[2][c] = S[2][2];
        qp.w[3][c] = 2.0 * S[0][1];
        qp.w[4][c] = 2.0 * S[0][2];
        qp.w[5][c] = 2.0 * S[1][2];
        qp.w[6][c] = -2.0 * Sm[0];
        qp.w[7][c] = -2.0 * Sm[1];
        qp.w[8][c] = -2.0 * Sm[2];
        qp.w[9][c] = mSm;
        // |terms| bound for any pixel with channels in [0, 255]: sum over the
        // absolute expanded weights times max|phi| = 255^2 (phi_9 = 1 <= 255^2).
        // Both the expanded MFMA sum and the reference's direct chain stay
        // within a few ulps of this bound; 64 u is a wide safety factor, and an
        // asymmetric A (adjugate rounding) is covered by the |A - A^T| term.
        double asym = 0.0;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) asym += std::fabs(A[3 * i + j] - A[3 * j + i]);
        const double wsum = Sa[0][0] + Sa[1][1] + Sa[2][2] + 2.0 * (Sa[0][1] + Sa[0][2] + Sa[1][2]) +
                            2.0 * (Sam[0] + Sam[1] + Sam[2]) + mSam;
        const double pmax = 255.0 + std::fabs(m[0]) + std::fabs(m[1]) + std::fabs(m[2]);
        qp.tol[c] = 64.0 * u * wsum * 65025.0 + 64.0 * u * asym * pmax * pmax + 1e-300;
    }
    return true;
}

}  // namespace

int classify_impl(uint32_t *img, int64_t npix, int nc, const double *mu, const double *inv, int grid, int block,
                  int path, void *stream) {
    MPX_CHECK_ARG(npix >= 0, "npix must be >= 0");
    MPX_CHECK_ARG(nc >= 1 && nc <= MPX_MAX_CLASSES, "need 1 <= nc <= 32");
    MPX_CHECK_ARG(mu && inv, "null class parameters");
    MPX_CHECK_ARG(grid >= 0 && block >= 0 && block <= 1024, "bad launch geometry");
    MPX_CHECK_ARG(path >= MPX_CLS_DIRECT && path <= MPX_CLS_AUTO, "bad path");
    if (npix == 0) return MPX_OK;
    MPX_CHECK_ARG(img, "null image");
    ClassParams cp{};
    for (int i = 0; i < 3 * nc; ++i) cp.mu[i] = mu[i];
    for (int i = 0; i < 9 * nc; ++i) cp.A[i] = inv[i];
    hipStream_t s = as_stream(stream);
    bool use_mfma = (path == MPX_CLS_MFMA) || (path == MPX_CLS_AUTO && nc >= 4);
    QuadParams qp;
    if (use_mfma && !build_quad(nc, mu, inv, qp)) use_mfma = false;  // non-finite stats: exact path only
    if (use_mfma) {
        int blk = 256;
        int64_t waves_needed = (npix + 15) / 16;
        int g = grid > 0 ? grid : (int)std::min<int64_t>((waves_needed + 3) / 4, (int64_t)kNumCUs * 8);
        if (g < 1) g = 1;
        hipLaunchKernelGGL(classify_mfma_kernel, dim3(g), dim3(blk), 0, s, img, npix, nc, cp, qp);
    } else {
        const int vec = aligned16(img) ? 1 : 0;
        if (block == 0) block = 256;
        if (grid == 0) {
            int64_t g = (npix / 4 + block - 1) / block;
            grid = (int)std::max<int64_t>(1, std::min<int64_t>(g, (int64_t)kNumCUs * 8));
        }
        hipLaunchKernelGGL(classify_direct_kernel, dim3(grid), dim3(block), 0, s, img, npix, nc, cp, vec);
    }
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}

}  // namespace mpx

extern "C" int mpx_classify(uint32_t *img, int64_t npix, int nc, const double *mu, const double *inv, int grid,
                            int block, int path, void *stream) {
    return mpx::classify_impl(img, npix, nc, mu, inv, grid, block, path, stream);
}
