// Tuning-only entry points of the lab2 kernels (tools/kbench.py): kernel
// variants by kind / rows per segment / fast magnitude, and the exhaustive
// fast-sqrt self-test. Kept out of the production code objects.
#include "edge_launch.hpp"

namespace mpx {
using edge::Taps;
using edgel::launch_stream;
using edgel::launch_wave;
using edgel::make_taps;
namespace {

// Exhaustive self-test of the fast magnitude path: every float s in
// [0, 65025] (bit patterns 0 .. 0x477E0100) must map to the same gray level as
// the correctly rounded sqrtf. Counts mismatches into *bad.
// raw = 0: the production fast path (v_sqrt + fract margin + exact fallback);
// raw = 1: bare truncation of v_sqrt_f32 with no margin test at all.
__global__ void fast_sqrt_selftest_kernel(uint32_t first, uint32_t last, unsigned long long *bad, int raw) {
    const uint32_t stride = gridDim.x * blockDim.x;
    unsigned long long nbad = 0;
    for (uint32_t u = first + blockIdx.x * blockDim.x + threadIdx.x; u <= last && u >= first; u += stride) {
        const float s = __builtin_bit_cast(float, u);
        const uint32_t exact = edge::mag_to_gray<false>(s);
        const uint32_t fast = raw ? (uint32_t)__builtin_amdgcn_sqrtf(fminf(s, 65025.0f)) : edge::mag_to_gray<true>(s);
        nbad += fast != exact;
    }
    if (nbad) atomicAdd(bad, nbad);
}

}  // namespace
MPX_MODULE_ANCHOR(edge_variants)

}  // namespace mpx

// Variant entry for the tuning harness (tools/kbench.py), k in {2, 5}, MAG2,
// whole image, fast magnitude path unless fast == 0:
//   kind 0: LDS streaming kernel, p1 = rows per wave (4, 8, 16), p2 = tiles per workgroup (0 = auto)
//   kind 1: wave-streaming kernel, p1 = rows per wave segment
extern "C" int mpx_conv_variant(const uint32_t *in, uint32_t *out, int w, int h, int k, int kind, int p1, int p2,
                                int fast, const float *wx, const float *wy, void *stream) {
    using namespace mpx;
    MPX_CHECK_ARG(in && out && wx && wy && w > 0 && h > 0, "bad arguments");
    MPX_CHECK_ARG(k == 2 || k == 5, "variant harness covers k = 2 and k = 5");
    hipStream_t s = as_stream(stream);
    if (kind == 3 || kind == 4) {
        // separable sobel5 (wx / wy = MPX_CONV_SEP factors): kind 3 compiled-in
        // factors, kind 4 runtime factors; p1 = segment rows, p2 >= 1000 strip-major
        MPX_CHECK_ARG(k == 5 && p1 >= 0, "separable variants: k = 5, segment rows >= 0 (0 = auto)");
        const Taps st = make_taps(k, wx, wy, true, true);
        const bool vec2 = (w % 2 == 0) && ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 7u) == 0;
        const int sm = p2 >= 1000 ? 0 : 1;
        if (kind == 3)
            return launch_wave<5, 2, MPX_CONV_MAG2, true, edge::Sobel5SepTaps>(in, out, w, w, 0, h, 0, h - 1, st, vec2, s, p1, sm);
        return launch_wave<5, 2, MPX_CONV_MAG2, true, edge::RuntimeSepTaps>(in, out, w, w, 0, h, 0, h - 1, st, vec2, s, p1, sm);
    }
    const Taps taps = make_taps(k, wx, wy, true);
    if (kind == 1 || kind == 2) {
        // kind 1: runtime taps, kind 2: compiled-in taps of the named filter;
        // p1 = segment rows; p2 >= 1000 orders waves strip-major
        MPX_CHECK_ARG(p1 >= 1, "segment rows must be positive");
        const bool vec2 = (w % 2 == 0) && ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 7u) == 0;
        const int sm = p2 >= 1000 ? 0 : 1;
        if (k == 5) {
            if (kind == 2)
                return launch_wave<5, 2, MPX_CONV_MAG2, true, edge::Sobel5Taps>(in, out, w, w, 0, h, 0, h - 1, taps, vec2, s, p1, sm);
            return fast ? launch_wave<5, 2, MPX_CONV_MAG2, true>(in, out, w, w, 0, h, 0, h - 1, taps, vec2, s, p1, sm)
                        : launch_wave<5, 2, MPX_CONV_MAG2, false>(in, out, w, w, 0, h, 0, h - 1, taps, vec2, s, p1, sm);
        }
        if (kind == 2)
            return launch_wave<2, 0, MPX_CONV_MAG2, true, edge::RobertsTaps>(in, out, w, w, 0, h, 0, h - 1, taps, vec2, s, p1, sm);
        return fast ? launch_wave<2, 0, MPX_CONV_MAG2, true>(in, out, w, w, 0, h, 0, h - 1, taps, vec2, s, p1, sm)
                    : launch_wave<2, 0, MPX_CONV_MAG2, false>(in, out, w, w, 0, h, 0, h - 1, taps, vec2, s, p1, sm);
    }
    const bool vec = (w % 4 == 0) && aligned16(in) && aligned16(out);
#define MPX_VAR(KK, AA, R, F)                                                                                  \
    if (k == KK && p1 == R && (fast != 0) == F)                                                                 \
        return launch_stream<KK, AA, MPX_CONV_MAG2, R, F>(in, out, w, w, 0, h, 0, h - 1, taps, vec, s, p2);
    MPX_VAR(5, 2, 4, true) MPX_VAR(5, 2, 8, true) MPX_VAR(5, 2, 16, true) MPX_VAR(5, 2, 8, false)
    MPX_VAR(2, 0, 4, true) MPX_VAR(2, 0, 8, true) MPX_VAR(2, 0, 16, true) MPX_VAR(2, 0, 8, false)
#undef MPX_VAR
    set_error("unsupported variant k=%d kind=%d p1=%d fast=%d", k, kind, p1, fast);
    return MPX_ERR_ARG;
}

extern "C" int mpx_selftest_fast_sqrt(unsigned long long *bad_device, int raw, void *stream) {
    using namespace mpx;
    MPX_CHECK_ARG(bad_device, "null counter");
    hipLaunchKernelGGL(fast_sqrt_selftest_kernel, dim3(kNumCUs * 16), dim3(256), 0, as_stream(stream), 0u,
                       0x477E0100u, bad_device, raw);
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}
