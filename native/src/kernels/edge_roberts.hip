// lab2 Roberts cross (reference lab2/src/main.cu:15-52, to_plot.cu:101-122):
//   * geometry-faithful LDS kernel for the harness's [[bx, by], [gx, gy]] launch
//     shapes (the reference's block/grid semantics: grid-stride over the image);
//   * geometry 0/0/0/0: the tuned wave-streaming kernel with the Roberts taps
//     compiled in (bit-identical: zero taps contribute exactly nothing).
// Its own translation unit so a Roberts-only program loads a small code object
// on its first launch (the reference's published times are cold launches).
#include "edge_launch.hpp"

namespace mpx {
using edge::Taps;
namespace {

// ---------------------------------------------------------------------------
// Roberts with the caller's launch geometry (harness contract). Block (bx, by)
// threads, each thread VEC horizontally adjacent pixels of one row, so a tile
// is (VEC*bx) x by pixels; grid (gx, gy) grid-strides over tiles. Luminance of
// the tile plus its 1-pixel right/bottom halo is staged in LDS once.
// ---------------------------------------------------------------------------
template <int VEC>
__global__ void roberts_geom_kernel(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, int w,
                                    int h) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int bx = blockDim.x, by = blockDim.y;
    const int tx = threadIdx.x, ty = threadIdx.y;
    const int TW = VEC * bx, TH = by;
    const int LW = TW + 4;  // 16-B aligned rows; column TW holds the right halo
    const int tiles_x = (w + TW - 1) / TW, tiles_y = (h + TH - 1) / TH;
    for (int tyt = blockIdx.y; tyt < tiles_y; tyt += gridDim.y) {
        for (int txt = blockIdx.x; txt < tiles_x; txt += gridDim.x) {
            const int x0 = txt * TW, y0 = tyt * TH;
            const int xs = x0 + VEC * tx;
            const int yrow = min(y0 + ty, h - 1);
            uint32_t own[VEC];
            // own pixels (clamped copies beyond the right/bottom edge)
            if constexpr (VEC == 4) {
                const uint4 q = *reinterpret_cast<const uint4 *>(in + (int64_t)yrow * w + min(xs, w - 4));
                const bool right = xs >= w;
                own[0] = right ? q.w : q.x;
                own[1] = right ? q.w : q.y;
                own[2] = right ? q.w : q.z;
                own[3] = q.w;
                *reinterpret_cast<float4 *>(&lds[ty * LW + VEC * tx]) =
                    make_float4(mpx_luma(own[0]), mpx_luma(own[1]), mpx_luma(own[2]), mpx_luma(own[3]));
            } else {
                own[0] = in[(int64_t)yrow * w + min(xs, w - 1)];
                lds[ty * LW + tx] = mpx_luma(own[0]);
            }
            const int ybot = min(y0 + TH, h - 1);
            if (ty == 0) {  // bottom halo row
                if constexpr (VEC == 4) {
                    const uint4 q = *reinterpret_cast<const uint4 *>(in + (int64_t)ybot * w + min(xs, w - 4));
                    const bool right = xs >= w;
                    *reinterpret_cast<float4 *>(&lds[TH * LW + VEC * tx]) =
                        make_float4(mpx_luma(right ? q.w : q.x), mpx_luma(right ? q.w : q.y),
                                    mpx_luma(right ? q.w : q.z), mpx_luma(q.w));
                } else {
                    lds[TH * LW + tx] = mpx_luma(in[(int64_t)ybot * w + min(xs, w - 1)]);
                }
            }
            if (tx == 0) {  // right halo column
                const int xr = min(x0 + TW, w - 1);
                lds[ty * LW + TW] = mpx_luma(in[(int64_t)yrow * w + xr]);
                if (ty == 0) lds[TH * LW + TW] = mpx_luma(in[(int64_t)ybot * w + xr]);
            }
            __syncthreads();
            const int y = y0 + ty;
            if (y < h) {
                uint32_t res[VEC];
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    const int c = VEC * tx + k;
                    const float y00 = lds[ty * LW + c], y10 = lds[ty * LW + c + 1];
                    const float y01 = lds[(ty + 1) * LW + c], y11 = lds[(ty + 1) * LW + c + 1];
                    const float gxv = y11 - y00;
                    const float gyv = y10 - y01;
                    const float a = gxv * gxv;
                    const float b2 = gyv * gyv;
                    res[k] = mpx_px_gray(edge::mag_to_gray<true>(a + b2), mpx_px_a(own[k]));  // == trunc(sqrtf), see mag_to_gray
                }
                if constexpr (VEC == 4) {
                    if (xs < w) *reinterpret_cast<uint4 *>(out + (int64_t)y * w + xs) = make_uint4(res[0], res[1], res[2], res[3]);
                } else {
                    if (xs < w) out[(int64_t)y * w + xs] = res[0];
                }
            }
            __syncthreads();
        }
    }
}
// ---------------------------------------------------------------------------
// The same geometry contract for THIN launches (fewer than 16K threads, e.g.
// the harness's [[2, 2], [16, 16]]: 1024 threads for a whole image). There
// each thread walks hundreds of tiles, so the LDS kernel's load -> barrier ->
// compute round trip per tile is pure latency. Here a thread reads its own 4+1
// pixels of rows y and y+1 straight from global memory (L2-resident
// neighbours, no LDS, no barrier) and keeps U tiles' loads in flight.
// Identical tile walk and arithmetic, so identical pixels.
// ---------------------------------------------------------------------------
template <int U, bool VEC>
__global__ void roberts_thin_kernel(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, int w, int h) {
    const int bx = blockDim.x, by = blockDim.y;
    const int TW = 4 * bx, TH = by;
    const int tiles_x = (w + TW - 1) / TW, tiles_y = (h + TH - 1) / TH;
    const int nx = blockIdx.x < tiles_x ? (tiles_x - blockIdx.x + gridDim.x - 1) / gridDim.x : 0;
    const int ny = blockIdx.y < tiles_y ? (tiles_y - blockIdx.y + gridDim.y - 1) / gridDim.y : 0;
    const int ntiles = nx * ny;  // this block's tiles, row-major as the LDS kernel walks them
    int k = 0, m = 0;            // (column, row) index of tile j0 in that walk — block-uniform, no division
    for (int j0 = 0; j0 < ntiles; j0 += U) {
        uint32_t a[U][5], b[U][5];  // pixels x .. x+4 (clamped) of rows y and y+1
        int xs[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            // tiles past the end repeat the last one (loaded, never stored)
            const int tyt = blockIdx.y + m * gridDim.y, txt = blockIdx.x + k * gridDim.x;
            if (j0 + u + 1 < ntiles && ++k == nx) {
                k = 0;
                ++m;
            }
            xs[u] = txt * TW + 4 * threadIdx.x;
            y[u] = tyt * TH + threadIdx.y;
            const uint32_t *ra = in + (int64_t)min(y[u], h - 1) * w;
            const uint32_t *rb = in + (int64_t)min(y[u] + 1, h - 1) * w;
            if constexpr (VEC) {  // w % 4 == 0: the quad is inside the row or the thread has no output
                const int xc = min(xs[u], w - 4);
                const uint4 qa = *reinterpret_cast<const uint4 *>(ra + xc);
                const uint4 qb = *reinterpret_cast<const uint4 *>(rb + xc);
                a[u][0] = qa.x; a[u][1] = qa.y; a[u][2] = qa.z; a[u][3] = qa.w;
                b[u][0] = qb.x; b[u][1] = qb.y; b[u][2] = qb.z; b[u][3] = qb.w;
                a[u][4] = ra[min(xs[u] + 4, w - 1)];
                b[u][4] = rb[min(xs[u] + 4, w - 1)];
            } else {
#pragma unroll
                for (int k = 0; k < 5; ++k) {
                    a[u][k] = ra[min(xs[u] + k, w - 1)];
                    b[u][k] = rb[min(xs[u] + k, w - 1)];
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);  // all U tiles' loads in flight before the first use
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (j0 + u >= ntiles || y[u] >= h || xs[u] >= w) continue;
            // packed fp32 (v_pk_mul / v_pk_add): each element takes the same
            // products and sums as mpx_luma and the scalar magnitude, so the
            // bytes are unchanged; a wave here often has 4 live lanes, so its
            // time is instruction issue and the pairs halve it
            using edge::f2_t;
            const f2_t la01 = edge::luma2(a[u][0], a[u][1]), la23 = edge::luma2(a[u][2], a[u][3]);
            const f2_t lb01 = edge::luma2(b[u][0], b[u][1]), lb23 = edge::luma2(b[u][2], b[u][3]);
            const f2_t l4 = edge::luma2(a[u][4], b[u][4]);  // (row a, row b) at x + 4
            uint32_t res[4];
            auto pair = [&](f2_t y00, f2_t y10, f2_t y01, f2_t y11, int k) {
                const f2_t gxv = y11 - y00;
                const f2_t gyv = y10 - y01;
                const f2_t s0 = gxv * gxv;
                const f2_t s1 = gyv * gyv;
                const f2_t sq = s0 + s1;
                uint32_t g0, g1;
                edge::mag2_to_gray(sq.x, sq.y, g0, g1);  // == trunc(sqrtf) each, see mag2_to_gray
                res[k] = mpx_px_gray(g0, mpx_px_a(a[u][k]));
                res[k + 1] = mpx_px_gray(g1, mpx_px_a(a[u][k + 1]));
            };
            pair(la01, f2_t{la01.y, la23.x}, lb01, f2_t{lb01.y, lb23.x}, 0);
            pair(la23, f2_t{la23.y, l4.x}, lb23, f2_t{lb23.y, l4.y}, 2);
            uint32_t *o = out + (int64_t)y[u] * w + xs[u];
            if (VEC) {
                *reinterpret_cast<uint4 *>(o) = make_uint4(res[0], res[1], res[2], res[3]);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (xs[u] + k < w) o[k] = res[k];
            }
        }
    }
}

// Internal-linkage tag for the tuned instantiation (band kernel when the rows
// are 16-B aligned, else wave kernel). conv_wave_kernel<...,
// edge::RobertsTaps> is also instantiated by the production and variants TUs;
// a kernel name registered from several fat binaries may resolve to one of the
// large code objects, whose first launch then costs ~1 ms more than this 43 KB
// one (measured cold: 1.25 ms vs 0.25 ms).
struct RobertsTuned : edge::RobertsTaps {};
}  // namespace

static const float kRobertsX[4] = {-1.0f, 0.0f, 0.0f, 1.0f};  // Gx = Y11 - Y00
static const float kRobertsY[4] = {0.0f, 1.0f, -1.0f, 0.0f};  // Gy = Y10 - Y01

int roberts_impl(const uint32_t *in, uint32_t *out, int w, int h, int bx, int by, int gx, int gy, void *stream) {
    MPX_CHECK_ARG(in && out, "null pointer");
    MPX_CHECK_ARG(w > 0 && h > 0, "empty image");
    if (bx == 0 && by == 0 && gx == 0 && gy == 0) {  // tuned path: wave kernel with compiled-in Roberts taps
        const Taps taps = edgel::make_taps(2, kRobertsX, kRobertsY, true);
        const bool vec2 = (w % 2 == 0) && ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 7u) == 0;
        const int rc = edgel::band_ok(in, out, w, w, edge::RowSrc{}, h)
                           ? edgel::launch_band<2, 0, MPX_CONV_MAG2, RobertsTuned>(in, out, w, w, 0, h, 0, h - 1, taps,
                                                                                   as_stream(stream), edge::RowSrc{})
                           : edgel::launch_wave<2, 0, MPX_CONV_MAG2, true, RobertsTuned>(in, out, w, w, 0, h, 0, h - 1,
                                                                                         taps, vec2, as_stream(stream));
        if (rc != MPX_OK) return rc;
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
        return MPX_OK;
    }
    MPX_CHECK_ARG(bx > 0 && by > 0 && gx > 0 && gy > 0, "launch geometry must be positive");
    MPX_CHECK_ARG((int64_t)bx * by <= 1024, "more than 1024 threads per block");
    const bool vec = (w % 4 == 0) && aligned16(in) && aligned16(out);
    const int VEC = vec ? 4 : 1;
    const size_t lds = sizeof(float) * (size_t)(by + 1) * (size_t)(VEC * bx + 4);
    MPX_CHECK_ARG(lds <= 64 * 1024, "tile does not fit the 64 KiB per-workgroup LDS limit");
    // empty workgroups dropped (useful_grid): a block whose first tile column
    // (row) lies past the image owns none, and with gx >= tiles_x every block
    // owns exactly its own column either way. Tiles: (4 bx) x by pixels in the
    // vector and thin kernels, bx x by in the scalar LDS kernel.
    // The kernel is chosen from the caller's geometry before the clamp.
    const bool thin = (int64_t)bx * by * gx * gy < 16384;
    {
        const int64_t tw = (vec || thin) ? 4 * bx : bx;
        gx = (int)useful_grid(gx, (w + tw - 1) / tw, 1);
        gy = (int)useful_grid(gy, (h + by - 1) / by, 1);
    }
    // (16 tiles in flight for launches of <= 2048 threads measured no faster
    // than 8: [[2, 2], [16, 16]] 200 us either way, profiles/harness_vs_baseline.md)
    if (thin && vec)
        hipLaunchKernelGGL((roberts_thin_kernel<8, true>), dim3(gx, gy), dim3(bx, by), 0, as_stream(stream), in, out, w, h);
    else if (thin)
        hipLaunchKernelGGL((roberts_thin_kernel<4, false>), dim3(gx, gy), dim3(bx, by), 0, as_stream(stream), in, out, w, h);
    else if (vec)
        hipLaunchKernelGGL(roberts_geom_kernel<4>, dim3(gx, gy), dim3(bx, by), lds, as_stream(stream), in, out, w, h);
    else
        hipLaunchKernelGGL(roberts_geom_kernel<1>, dim3(gx, gy), dim3(bx, by), lds, as_stream(stream), in, out, w, h);
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}

// Per-channel Roberts cross, L1 magnitude (mpx_cpu_roberts_rgb; the operator
// of the reference's lab2/test_data samples). Byte-exact integer math. One
// thread per aligned 16-B quad of 4 pixels (w % 4 == 0) or per pixel (VEC 1):
// the quad, the pixel right of it, and the same from the row below (clamped).
__device__ __forceinline__ uint32_t roberts_rgb_px(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    uint32_t o = a & 0xff000000u;
#pragma unroll
    for (int ch = 0; ch < 24; ch += 8) {
        const int va = (int)__builtin_amdgcn_ubfe(a, ch, 8), vb = (int)__builtin_amdgcn_ubfe(b, ch, 8);
        const int vc = (int)__builtin_amdgcn_ubfe(c, ch, 8), vd = (int)__builtin_amdgcn_ubfe(d, ch, 8);
        o |= (uint32_t)min(abs(va - vd) + abs(vb - vc), 255) << ch;
    }
    return o;
}

template <int VEC>
__global__ __launch_bounds__(256) void roberts_rgb_kernel(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                          int w, int h) {
    const int per_row = w / VEC;
    const int64_t total = (int64_t)per_row * h;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(t / per_row), x = (int)(t - (int64_t)y * per_row) * VEC;
        const int y1 = min(y + 1, h - 1), xr = min(x + VEC, w - 1);
        const uint32_t *r0 = in + (int64_t)y * w, *r1 = in + (int64_t)y1 * w;
        if constexpr (VEC == 4) {
            const uint4 q0 = *reinterpret_cast<const uint4 *>(r0 + x), q1 = *reinterpret_cast<const uint4 *>(r1 + x);
            const uint32_t e0 = r0[xr], e1 = r1[xr];
            uint4 o;
            o.x = roberts_rgb_px(q0.x, q0.y, q1.x, q1.y);
            o.y = roberts_rgb_px(q0.y, q0.z, q1.y, q1.z);
            o.z = roberts_rgb_px(q0.z, q0.w, q1.z, q1.w);
            o.w = roberts_rgb_px(q0.w, e0, q1.w, e1);
            *reinterpret_cast<uint4 *>(out + (int64_t)y * w + x) = o;
        } else {
            out[(int64_t)y * w + x] = roberts_rgb_px(r0[x], r0[xr], r1[x], r1[xr]);
        }
    }
}

int roberts_rgb_impl(const uint32_t *in, uint32_t *out, int w, int h, void *stream) {
    MPX_CHECK_ARG(in && out && w > 0 && h > 0, "bad image");
    MPX_CHECK_ARG(in != out, "in-place is not supported (neighbours are read after the write)");
    const bool vec = w % 4 == 0 && aligned16(in) && aligned16(out);
    const int64_t work = (int64_t)w * h / (vec ? 4 : 1);
    const int grid = (int)std::min<int64_t>((work + 255) / 256, (int64_t)kNumCUs * 16);
    if (vec)
        hipLaunchKernelGGL(roberts_rgb_kernel<4>, dim3(grid), dim3(256), 0, as_stream(stream), in, out, w, h);
    else
        hipLaunchKernelGGL(roberts_rgb_kernel<1>, dim3(grid), dim3(256), 0, as_stream(stream), in, out, w, h);
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}

MPX_MODULE_ANCHOR(edge_roberts)

}  // namespace mpx

extern "C" int mpx_roberts(const uint32_t *in, uint32_t *out, int w, int h, int bx, int by, int gx, int gy,
                           void *stream) {
    return mpx::roberts_impl(in, out, w, h, bx, by, gx, gy, stream);
}

extern "C" int mpx_roberts_rgb(const uint32_t *in, uint32_t *out, int w, int h, void *stream) {
    return mpx::roberts_rgb_impl(in, out, w, h, stream);
}
