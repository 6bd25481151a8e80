// lab5: sort of the binary arrays in the reference's lab5/data fixtures
// (int10, float10, uchar10: int32 n, then n elements). The reference ships the
// inputs only — no program consumes them — so the contract here is
// ours: ascending order, in place on the device.
//
// MI355X design
//   * int32 and float32 become order-preserving uint32 keys in place (sign
//     flip; floats flip every bit when negative), so one network sorts both.
//     Float order is the IEEE total order on the bit patterns: -NaN < -inf <
//     ... < -0 < +0 < ... < +inf < +NaN.
//   * The network is the all-ascending bitonic form: the first step of stage k
//     compares i with i ^ (k - 1), later steps with i ^ j, and the lower index
//     always keeps the minimum. Elements past n act as +inf and never move, so
//     any n sorts without padding or scratch.
//   * Stages up to kTile (4096 keys) run entirely in LDS, 16 keys per thread,
//     in one launch. Larger stages issue one global compare-exchange pass per
//     step with j >= kTile; the steps j < kTile of the same stage run in one
//     LDS launch per tile. N = 2^26 takes 105 global passes + 15 LDS passes.
//   * uint8 uses a counting sort instead: 256 LDS histogram bins per block
//     stored to a per-block row (no global atomics), one block reduces the
//     rows and scans them into 257 bucket starts, and every block writes its
//     output range by binary search over those starts staged in LDS.
#include <mutex>

#include "internal.hpp"

namespace mpx {
namespace {

constexpr int kSortThreads = 256;
constexpr int kPerThread = 16;
constexpr int kTile = kSortThreads * kPerThread;  // 4096 keys = 16 KiB of LDS

__global__ void to_keys_kernel(uint32_t *__restrict__ x, int64_t n, int is_float) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t v = x[i];
        x[i] = is_float ? (v ^ ((uint32_t)((int32_t)v >> 31) | 0x80000000u)) : (v ^ 0x80000000u);
    }
}

__global__ void from_keys_kernel(uint32_t *__restrict__ x, int64_t n, int is_float) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t k = x[i];
        x[i] = is_float ? (k ^ ((k >> 31) ? 0x80000000u : 0xffffffffu)) : (k ^ 0x80000000u);
    }
}

__device__ __forceinline__ void cmpx(uint32_t *s, int i, int p) {
    const uint32_t a = s[i], b = s[p];
    if (b < a) {
        s[i] = b;
        s[p] = a;
    }
}

// one LDS pass over a tile: either the whole network up to kTile (full = 1),
// or the steps j = kTile/2 .. 1 of a larger stage (full = 0)
__global__ __launch_bounds__(kSortThreads) void sort_tile_kernel(uint32_t *__restrict__ x, int64_t n, int full) {
    __shared__ uint32_t s[kTile];
    const int64_t base = (int64_t)blockIdx.x * kTile;
    const int t = threadIdx.x;
#pragma unroll
    for (int e = 0; e < kPerThread; ++e) {
        const int i = e * kSortThreads + t;
        s[i] = base + i < n ? x[base + i] : 0xffffffffu;
    }
    __syncthreads();
    // each of the kTile/2 compare pairs per step is owned by one (thread, e)
    if (full) {
        for (int k = 2; k <= kTile; k <<= 1) {
            for (int e = 0; e < kPerThread / 2; ++e) {  // flip step of stage k
                const int q = e * kSortThreads + t;
                const int h = k >> 1;
                const int i = (q / h) * k + (q % h);
                cmpx(s, i, (i / k) * k + (k - 1) - (q % h));
            }
            __syncthreads();
            for (int j = k >> 2; j >= 1; j >>= 1) {
                for (int e = 0; e < kPerThread / 2; ++e) {
                    const int q = e * kSortThreads + t;
                    const int i = (q / j) * 2 * j + (q % j);
                    cmpx(s, i, i + j);
                }
                __syncthreads();
            }
        }
    } else {
        for (int j = kTile >> 1; j >= 1; j >>= 1) {
            for (int e = 0; e < kPerThread / 2; ++e) {
                const int q = e * kSortThreads + t;
                const int i = (q / j) * 2 * j + (q % j);
                cmpx(s, i, i + j);
            }
            __syncthreads();
        }
    }
#pragma unroll
    for (int e = 0; e < kPerThread; ++e) {
        const int i = e * kSortThreads + t;
        if (base + i < n) x[base + i] = s[i];
    }
}

// one global compare-exchange step of stage k: flip (j == k/2, first step) or half-cleaner
__global__ void sort_step_kernel(uint32_t *__restrict__ x, int64_t n, int64_t npairs, int64_t k, int64_t j,
                                 int flip) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < npairs; q += stride) {
        const int64_t i = (q / j) * 2 * j + (q % j);
        const int64_t p = flip ? (i / k) * k + (k - 1) - (q % j) : i + j;
        if (p >= n) continue;  // partner past the end is +inf: no exchange
        const uint32_t a = x[i], b = x[p];
        if (b < a) {
            x[i] = b;
            x[p] = a;
        }
    }
}

// L consecutive half-cleaner steps (j = 2^(L-1) h, ..., 2h, h) fused into one
// global pass: each thread owns the 2^L slots i + e*h (i has the L bits from h
// up clear), so the array is read and written once instead of L times.
// Power-of-two index math with shifts. Slots past the end read as +inf and are
// never stored (an ascending network never moves +inf down).
template <int L>
__global__ void sort_stepn_kernel(uint32_t *__restrict__ x, int64_t n, int64_t ngroups, int lh) {
    constexpr int G = 1 << L;
    const int64_t h = (int64_t)1 << lh;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < ngroups; q += stride) {
        const int64_t i = ((q >> lh) << (lh + L)) | (q & (h - 1));
        if (i + h >= n) continue;  // only slot 0 is real: nothing moves
        uint32_t v[G];
#pragma unroll
        for (int e = 0; e < G; ++e) v[e] = i + e * h < n ? x[i + e * h] : 0xffffffffu;
#pragma unroll
        for (int d = G / 2; d >= 1; d >>= 1)
#pragma unroll
            for (int e = 0; e < G; ++e)
                if ((e & d) == 0) {
                    const uint32_t lo = min(v[e], v[e + d]), hi = max(v[e], v[e + d]);
                    v[e] = lo;
                    v[e + d] = hi;
                }
#pragma unroll
        for (int e = 0; e < G; ++e)
            if (i + e * h < n) x[i + e * h] = v[e];
    }
}

// Per-block LDS histogram written to its own row of `partial` (no global
// atomics), then one block reduces the rows column-wise (coalesced, four row
// groups in parallel) and scans them into the 257 bucket starts the fill
// kernel reads. The body of the array moves as 16-B vectors (one uint4 per
// thread and iteration); the unaligned head (< 16 B) and the tail go bytewise.
__device__ inline int64_t u8_scalar_pos(int64_t i, int64_t head, int64_t tail0) {
    return i < head ? i : tail0 + (i - head);
}

__global__ __launch_bounds__(256) void hist_u8_kernel(const uint8_t *__restrict__ x, int64_t n, int64_t head,
                                                      int64_t nvec, uint32_t *__restrict__ partial) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint4 *v = reinterpret_cast<const uint4 *>(x + head);
    for (int64_t i = gid; i < nvec; i += stride) {
        const uint4 q = v[i];
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int b = 0; b < 4; ++b) atomicAdd(&h[(w[k] >> (8 * b)) & 255u], 1u);
    }
    const int64_t tail0 = head + 16 * nvec;
    for (int64_t i = gid; i < head + (n - tail0); i += stride) atomicAdd(&h[x[u8_scalar_pos(i, head, tail0)]], 1u);
    __syncthreads();
    partial[(int64_t)blockIdx.x * 256 + threadIdx.x] = h[threadIdx.x];
}

__global__ __launch_bounds__(1024) void scan_u8_kernel(const uint32_t *__restrict__ partial, int nblocks,
                                                       int64_t *__restrict__ start) {
    __shared__ int64_t acc[4][256];
    const int col = threadIdx.x & 255, grp = threadIdx.x >> 8;
    int64_t sum = 0;
#pragma unroll 8
    for (int b = grp; b < nblocks; b += 4) sum += partial[(int64_t)b * 256 + col];
    acc[grp][col] = sum;
    __syncthreads();
    // inclusive Hillis-Steele scan of the 256 column totals (8 steps)
    __shared__ int64_t scan[2][256];
    int64_t tot = 0;
    if (threadIdx.x < 256) {
        tot = acc[0][col] + acc[1][col] + acc[2][col] + acc[3][col];
        scan[0][col] = tot;
    }
    __syncthreads();
    int cur = 0;
    for (int off = 1; off < 256; off <<= 1) {
        if (threadIdx.x < 256) scan[cur ^ 1][col] = scan[cur][col] + (col >= off ? scan[cur][col - off] : 0);
        __syncthreads();
        cur ^= 1;
    }
    if (threadIdx.x < 256) {
        start[col] = scan[cur][col] - tot;
        if (col == 255) start[256] = scan[cur][col];
    }
}

__device__ inline int u8_value_at(const int64_t *start, int64_t o) {
    int lo = 0, hi = 255;  // largest v with start[v] <= o
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (start[mid] <= o) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__global__ __launch_bounds__(256) void fill_u8_kernel(uint8_t *__restrict__ x, int64_t n, int64_t head,
                                                      int64_t nvec, const int64_t *__restrict__ gstart) {
    __shared__ int64_t start[257];
    start[threadIdx.x] = gstart[threadIdx.x];
    if (threadIdx.x == 0) start[256] = gstart[256];
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint4 *v = reinterpret_cast<uint4 *>(x + head);
    for (int64_t i = gid; i < nvec; i += stride) {
        const int64_t o = head + 16 * i;
        int val = u8_value_at(start, o);
        uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            while (start[val + 1] <= o + k) ++val;  // start[256] = n > o + k: stops at 255
            w[k >> 2] |= (uint32_t)val << (8 * (k & 3));
        }
        v[i] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    const int64_t tail0 = head + 16 * nvec;
    for (int64_t i = gid; i < head + (n - tail0); i += stride) {
        const int64_t o = u8_scalar_pos(i, head, tail0);
        x[o] = (uint8_t)u8_value_at(start, o);
    }
}

int grid_for(int64_t work, int block) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((work + block - 1) / block, (int64_t)kNumCUs * 16));
}

// The uint8 path's scratch (257 bucket starts + kHistBlocks histogram rows,
// 1 MiB) is allocated once per device and kept: a stream-ordered
// hipMallocAsync/hipFreeAsync pair per call returned corrupted output when a
// plain HIP program (labs/lab5 CLI, null stream) sorted the same buffer twice
// (tools/lab5_u8_diag.py), while the torch process did not. Sorts of uint8
// data on one device therefore share the scratch and must run on one stream.
constexpr int kHistBlocks = 256;  // one per CU
constexpr int kMaxDevices = 64;

int u8_scratch(void **out) {
    static std::mutex mu;
    static void *bufs[kMaxDevices] = {};
    int dev = 0;
    MPX_RETURN_IF_HIP_ERROR(hipGetDevice(&dev));
    MPX_CHECK_ARG(dev >= 0 && dev < kMaxDevices, "device index out of range");
    std::lock_guard<std::mutex> lock(mu);
    if (!bufs[dev]) {
        const size_t bytes = 257 * sizeof(int64_t) + (size_t)kHistBlocks * 256 * sizeof(uint32_t);
        MPX_RETURN_IF_HIP_ERROR(hipMalloc(&bufs[dev], bytes));
    }
    *out = bufs[dev];
    return MPX_OK;
}

int sort_keys(uint32_t *x, int64_t n, hipStream_t s) {
    if (n < 2) return MPX_OK;
    const int64_t tiles = (n + kTile - 1) / kTile;
    MPX_CHECK_ARG(tiles <= INT32_MAX, "array too large");
    hipLaunchKernelGGL(sort_tile_kernel, dim3((unsigned)tiles), dim3(kSortThreads), 0, s, x, n, 1);
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    int64_t npow = kTile;
    while (npow < n) npow <<= 1;
    const int64_t npairs = npow / 2;
    for (int64_t k = 2 * (int64_t)kTile; k <= npow; k <<= 1) {
        hipLaunchKernelGGL(sort_step_kernel, dim3(grid_for(npairs, 256)), dim3(256), 0, s, x, n, npairs, k, k / 2, 1);
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
        int64_t j = k / 4;
        while (j >= kTile) {  // remaining half-cleaners j, j/2, ..., kTile: up to 3 per pass
            int steps = 1;
            while (steps < 3 && (j >> steps) >= kTile) ++steps;
            int lh = 0;
            while (((int64_t)1 << lh) < (j >> (steps - 1))) ++lh;
            const int64_t groups = npow >> steps;
            if (steps == 3)
                hipLaunchKernelGGL(sort_stepn_kernel<3>, dim3(grid_for(groups, 256)), dim3(256), 0, s, x, n, groups, lh);
            else if (steps == 2)
                hipLaunchKernelGGL(sort_stepn_kernel<2>, dim3(grid_for(groups, 256)), dim3(256), 0, s, x, n, groups, lh);
            else
                hipLaunchKernelGGL(sort_stepn_kernel<1>, dim3(grid_for(groups, 256)), dim3(256), 0, s, x, n, groups, lh);
            MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
            j >>= steps;
        }
        hipLaunchKernelGGL(sort_tile_kernel, dim3((unsigned)tiles), dim3(kSortThreads), 0, s, x, n, 0);
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    }
    return MPX_OK;
}

}  // namespace

int sort_impl(void *data, int64_t n, int dtype, void *stream) {
    MPX_CHECK_ARG(n >= 0, "n must be >= 0");
    MPX_CHECK_ARG(dtype == MPX_SORT_I32 || dtype == MPX_SORT_F32 || dtype == MPX_SORT_U8, "bad dtype");
    if (n == 0) return MPX_OK;
    MPX_CHECK_ARG(data, "null data");
    hipStream_t s = as_stream(stream);
    if (dtype == MPX_SORT_U8) {
        const int64_t head = std::min<int64_t>(n, (16 - (int64_t)(reinterpret_cast<uintptr_t>(data) & 15u)) & 15);
        const int64_t nvec = (n - head) / 16;
        const int hblocks = std::min(grid_for(std::max<int64_t>(nvec, 1), 256), kHistBlocks);
        void *scratch = nullptr;
        if (const int rc = u8_scratch(&scratch)) return rc;
        int64_t *start = static_cast<int64_t *>(scratch);
        uint32_t *partial = reinterpret_cast<uint32_t *>(start + 257);
        uint8_t *x = static_cast<uint8_t *>(data);
        hipLaunchKernelGGL(hist_u8_kernel, dim3(hblocks), dim3(256), 0, s, x, n, head, nvec, partial);
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
        hipLaunchKernelGGL(scan_u8_kernel, dim3(1), dim3(1024), 0, s, partial, hblocks, start);
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
        hipLaunchKernelGGL(fill_u8_kernel, dim3(grid_for(std::max<int64_t>(nvec, 1), 256)), dim3(256), 0, s, x, n, head,
                           nvec, start);
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
        return MPX_OK;
    }
    MPX_CHECK_ARG((reinterpret_cast<uintptr_t>(data) & 3u) == 0, "int32/float32 data must be 4-byte aligned");
    uint32_t *x = static_cast<uint32_t *>(data);
    const int is_float = dtype == MPX_SORT_F32;
    hipLaunchKernelGGL(to_keys_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, x, n, is_float);
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    const int rc = sort_keys(x, n, s);
    if (rc != MPX_OK) return rc;
    hipLaunchKernelGGL(from_keys_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, x, n, is_float);
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}

MPX_MODULE_ANCHOR(sort)

}  // namespace mpx

extern "C" int mpx_sort(void *data, int64_t n, int dtype, void *stream) { return mpx::sort_impl(data, n, dtype, stream); }
