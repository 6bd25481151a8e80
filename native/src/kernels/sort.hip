// lab5: sort of the binary arrays in the reference's lab5/data fixtures
// (int10, float10, uchar10: int32 n, then n elements). The reference ships the
// inputs only — no program consumes them — so the contract here is
// ours: ascending order, in place on the device.
//
// MI355X design
//   * int32 and float32 become order-preserving uint32 keys (sign flip; floats
//     flip every bit when negative). Float order is the IEEE total order on the
//     bit patterns: -NaN < -inf < ... < -0 < +0 < ... < +inf < +NaN.
//   * n > kTile: LSD radix sort, 8-bit digits, 4 passes (radix_sort32), in
//     one of two forms chosen by n:
//       - onesweep (tuning variant 1; AUTO up to 2^18 keys before round 5): one histogram pass builds all
//         four 256-bin digit histograms at once; each digit pass is ONE kernel
//         in which a block takes the next 8192-key tile from an atomic tile
//         counter, ranks its keys stably in LDS (per-wave peer masks of equal
//         digits from an LDS OR table, mbcnt for the rank among lower lanes,
//         per-wave digit counters), resolves its global digit offsets by
//         decoupled look-back (flag + count in one 32-bit word), then stages
//         the tile in LDS in digit order and writes it out in runs per digit;
//       - AUTO, reduce-then-scan: per pass a count kernel (per-tile digit
//         counts), a scan kernel (per-tile offsets and digit totals) and a
//         persistent scatter kernel (radix_scatter_lean_kernel: 2 blocks per
//         CU walking XCD-local tiles, next tile prefetched while this one is
//         ranked as above, buffer loads / stores, one counter add per
//         distinct digit). It
//         re-reads each tile once more but never waits on a look-back chain,
//         whose cross-XCD round trips bound onesweep at large n.
//     The key transform rides on the first pass's loads and the inverse on
//     the last pass's stores; 4 passes ping-pong data -> ws -> data.
//   * n <= kTile (4096 keys): the whole bitonic network in LDS, one launch;
//     n >= 2^30 (beyond the 30-bit counts): the global bitonic network
//     (stages > kTile as fused global half-cleaner passes, up to 3 per pass).
//   * uint8 uses a counting sort: a per-block LDS histogram folded into 256
//     global bin counts by one atomic per bin and block (hist_u8_kernel), then
//     every block scans the 256 counts itself and writes one contiguous run of
//     16-B pieces of the output, a piece's value searched only among the
//     buckets its run overlaps (fill_u8_kernel).
//   * Scratch comes from a caller-provided workspace (mpx_sort_workspace_bytes
//     / mpx_sort_ws): the Python op takes it from torch's caching allocator on
//     the tensor's stream, so concurrent sorts on different streams or devices
//     never share scratch.
#include <atomic>
#include <mutex>
#include <type_traits>

#include "mpx/tuning.h"
#include "sort_radix.hpp"

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
    // k, h and j are powers of two: index arithmetic by shifts and masks (the
    // variable-divisor integer divisions made 4096 keys take 0.1 ms)
    if (full) {
        for (int lk = 1; (1 << lk) <= kTile; ++lk) {
            const int k = 1 << lk, lh = lk - 1;
            for (int e = 0; e < kPerThread / 2; ++e) {  // flip step of stage k
                const int q = e * kSortThreads + t;
                const int r = q & ((1 << lh) - 1);
                const int i = ((q >> lh) << lk) + r;
                cmpx(s, i, ((i >> lk) << lk) + (k - 1) - r);
            }
            __syncthreads();
            for (int lj = lk - 2; lj >= 0; --lj) {
                for (int e = 0; e < kPerThread / 2; ++e) {
                    const int q = e * kSortThreads + t;
                    const int i = ((q >> lj) << (lj + 1)) + (q & ((1 << lj) - 1));
                    cmpx(s, i, i + (1 << lj));
                }
                __syncthreads();
            }
        }
    } else {
        for (int lj = __builtin_ctz(kTile) - 1; lj >= 0; --lj) {
            for (int e = 0; e < kPerThread / 2; ++e) {
                const int q = e * kSortThreads + t;
                const int i = ((q >> lj) << (lj + 1)) + (q & ((1 << lj) - 1));
                cmpx(s, i, i + (1 << lj));
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

// uint8 counting sort. The body of the array moves as 16-B vectors; the
// unaligned head (< 16 B) and the tail go bytewise. (Round 1 wrote per-block
// histogram rows and reduced them in a single-block scan kernel: 18.6 us of a
// 72 us sort at 2^26; the rows are now folded by global atomics.)
__device__ inline int64_t u8_scalar_pos(int64_t i, int64_t head, int64_t tail0) {
    return i < head ? i : tail0 + (i - head);
}

// Counting sort, step 1: per-block LDS histogram of the bytes, then one
// global atomic per non-empty bin (ghist zeroed beforehand). Each thread keeps
// four 16-B loads in flight. The histogram has 32 copies of every bin, copy
// lane % 32 at word bin * 32 + lane % 32: each 32-lane half of an atomic then
// touches 32 distinct banks. (One shared 256-word histogram put random bytes
// ~3.5 deep on the busiest bank: 22.9 us at 2^26, LDS-bound.)
__global__ __launch_bounds__(1024) void hist_u8_kernel(const uint8_t *__restrict__ x, int64_t n, int64_t head,
                                                       int64_t nvec, uint32_t *__restrict__ ghist) {
    __shared__ uint32_t h[256 * 32];
    for (int k = threadIdx.x; k < 256 * 32; k += 1024) h[k] = 0;
    __syncthreads();
    const uint32_t lane32 = threadIdx.x & 31u;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint4 *v = reinterpret_cast<const uint4 *>(x + head);
    auto count = [&](const uint4 q) {
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int b = 0; b < 4; ++b) atomicAdd(&h[(((w[k] >> (8 * b)) & 255u) << 5) | lane32], 1u);
    };
    int64_t i = gid;
    for (; i + 3 * stride < nvec; i += 4 * stride) {
        const uint4 q0 = v[i], q1 = v[i + stride], q2 = v[i + 2 * stride], q3 = v[i + 3 * stride];
        count(q0);
        count(q1);
        count(q2);
        count(q3);
    }
    for (; i < nvec; i += stride) count(v[i]);
    const int64_t tail0 = head + 16 * nvec;
    for (int64_t j = gid; j < head + (n - tail0); j += stride)
        atomicAdd(&h[((uint32_t)x[u8_scalar_pos(j, head, tail0)] << 5) | lane32], 1u);
    __syncthreads();
    if (threadIdx.x < 256) {
        const int t = threadIdx.x;
        uint32_t c = 0;
#pragma unroll 8
        for (int j = 0; j < 32; ++j) c += h[(t << 5) | ((j + t) & 31)];  // rotated: 32 banks per half
        if (c) atomicAdd(&ghist[t], c);
    }
}

__device__ inline int u8_value_at(const int64_t *start, int64_t o, int lo = 0, int hi = 255) {
    // largest v in [lo, hi] with start[v] <= o (start[lo] <= o given)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (start[mid] <= o) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// step 2: every block scans the 256 global bin counts itself (exclusive
// prefix in LDS: no separate scan launch), then writes one contiguous run of
// 16-B pieces of the sorted output, 4 KiB per block-wide store. A piece's
// value is searched only between the buckets of the run's first and last
// byte: no search at all when one bucket covers the run (a bucket spans
// n / 256 bytes of uniform input, a run nvec / grid pieces).
__global__ __launch_bounds__(256) void fill_u8_kernel(uint8_t *__restrict__ x, int64_t n, int64_t head,
                                                      int64_t nvec, const uint32_t *__restrict__ ghist) {
    __shared__ int64_t start[257];
    __shared__ int64_t s_wsum[4];
    {
        const int t = threadIdx.x, lane = t & 63;
        const int64_t c = ghist[t];
        int64_t xs = c;  // inclusive wave scan
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t y = __shfl_up(xs, o);
            if (lane >= o) xs += y;
        }
        if (lane == 63) s_wsum[t >> 6] = xs;
        __syncthreads();
        int64_t add = 0;
        for (int w = 0; w < (t >> 6); ++w) add += s_wsum[w];
        start[t] = xs - c + add;
        if (t == 255) start[256] = xs + add;
        __syncthreads();
    }
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint4 *v = reinterpret_cast<uint4 *>(x + head);
    const int64_t per = (nvec + gridDim.x - 1) / gridDim.x;
    const int64_t c0 = (int64_t)blockIdx.x * per, c1 = min(c0 + per, nvec);
    const int b0 = c0 < c1 ? u8_value_at(start, head + 16 * c0) : 0;
    const int b1 = c0 < c1 ? u8_value_at(start, head + 16 * c1 - 1, b0) : 0;
    for (int64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
        const int64_t o = head + 16 * i;
        int val = u8_value_at(start, o, b0, b1);
        if (start[val + 1] > o + 15) {  // the whole 16-B piece lies in one bucket (all but ~256 pieces)
            const uint32_t r = (uint32_t)val * 0x01010101u;
            v[i] = make_uint4(r, r, r, r);
            continue;
        }
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


// Lane order of same-address returning LDS adds. The RANK >= 1
// scatters (variants 9-21, AUTO above 2^18 keys) are stable only because one
// ds_add_rtn_u32 applies its same-address lanes in ascending lane order —
// observed on gfx950, not promised by the ISA. This probe checks it once per
// device before the first such sort, in the scatter's widest shape (1024
// threads, 16 waves, as variant 22 ranks), with four address patterns: every
// lane on one counter, lane % 3, a scattered 5-way split, and most lanes on
// one counter with a few elsewhere. Every address comes from a per-lane value
// the compiler cannot prove uniform (`zero[lane]`, all 0 at run time), so the
// atomic optimizer cannot turn the one-counter pattern into one add plus an
// mbcnt prefix (ascending by construction: that would test the compiler, not
// the LDS). Each lane's returned count must equal the number of
// lower lanes on its counter. On a failure AUTO falls back to the peer-mask
// ranking (variants 7 / 8, which rank with explicit lane masks) and the
// explicit RANK variants refuse.
__device__ __forceinline__ int probe_addr(int k, int lane) {
    return k == 0 ? 0 : k == 1 ? lane % 3 : k == 2 ? (lane * 7) % 5 : (lane % 9 == 4 ? 1 + lane % 5 : 0);
}

__global__ __launch_bounds__(1024) void lds_rtn_order_probe_kernel(uint32_t *bad, const uint32_t *zero) {
    constexpr int kPat = 4;
    __shared__ uint32_t cnt[16][kPat][8];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = lane; i < kPat * 8; i += 64) (&cnt[w][0][0])[i] = 0;
    __syncthreads();
    const uint32_t z = zero[lane];  // 0, but per lane and from memory
    uint32_t err = 0;
#pragma unroll
    for (int k = 0; k < kPat; ++k) {
        const uint32_t got = atomicAdd(&cnt[w][k][probe_addr(k, lane) + z], 1u);
        uint32_t want = 0;
        for (int j = 0; j < lane; ++j) want += probe_addr(k, j) == probe_addr(k, lane);
        err |= got != want;
    }
    if (err) bad[0] = 1u;  // vector store; any lane of any wave
}

// 1 = ascending lane order holds on the current device, 0 = it does not,
// negative = the probe could not run (treated as "does not hold")
int lds_rtn_order_ok(hipStream_t s) {
    static std::atomic<int> cache[64];
    static std::once_flag init;
    std::call_once(init, [] {
        for (auto &c : cache) c.store(-2);
    });
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
    int v = cache[dev].load();
    if (v != -2) return v;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone)
        return -1;  // no synchronous probe inside a graph capture (not cached: the next eager sort probes)
    uint32_t *d = nullptr, h = 1u;
    int ok = -1;
    if (hipMalloc(&d, 65 * sizeof(uint32_t)) == hipSuccess) {  // [0] = the flag, [1..64] = per-lane zeros
        if (hipMemsetAsync(d, 0, 65 * sizeof(uint32_t), s) == hipSuccess) {
            hipLaunchKernelGGL(lds_rtn_order_probe_kernel, dim3(1), dim3(1024), 0, s, d, d + 1);
            if (hipGetLastError() == hipSuccess && hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, s) == hipSuccess &&
                hipStreamSynchronize(s) == hipSuccess)
                ok = h == 0u ? 1 : 0;
        }
        (void)hipFree(d);
    }
    cache[dev].store(ok);
    return ok;
}

int radix_sort32(uint32_t *x, int64_t n, int mode, void *ws, int variant, hipStream_t s) {
    const RadixWs r = radix_layout(ws, n);
    const bool auto_variant = variant == 0;
    // AUTO (round 5, profiles/lab5_sort.md): the returning-add ranking with
    // two tiles of keys in flight and the two hottest digits of a skewed pass
    // ranked by compare masks (RANK 4), on 4096-key tiles up to 2^23 keys
    // (21; also below 2^18 since round 5: 0.059-0.062 vs onesweep's
    // 0.068-0.082 ms from 2^14 to 2^18 keys), on 8192-key tiles below 2^26
    // (20), on 16384-key tiles from 2^26 (22: longer digit runs, fewer partial
    // output lines; 2^26 int32 0.689-0.697 vs 0.706 ms, but 10 % slower at 2^24
    // with one block per CU); uniform passes run the RANK 1 loop. Every other
    // variant lives in the tuning library (mpx_sort_variant).
    if (variant == 0) variant = n <= kTile4kMaxN ? 21 : n < kTile16kMinN ? 20 : 22;
    if (variant != 7 && variant != 8 && (variant < 20 || variant > 22)) return MPX_ERR_UNSUPPORTED;
    // the returning-add ranking needs ascending lane order (probe above); the
    // fallback ranks with explicit lane masks (7 / 8)
    if (variant >= 20 && lds_rtn_order_ok(s) != 1) {
        if (!auto_variant) return MPX_ERR_UNSUPPORTED;
        variant = n <= kTile4kMaxN ? 8 : 7;
    }
    const bool small_tiles = variant == 8 || variant == 21;  // 4096-key tiles (256-thread scatter, 4 blocks per CU)
    const bool big_tiles = variant == 22;                     // 16384-key tiles (1024 threads, 1 block per CU)
    const int ntiles = small_tiles ? (int)((n + kRTileSmall - 1) / kRTileSmall)
                       : big_tiles ? (int)((n + kRTileBig - 1) / kRTileBig)
                                   : (int)r.tiles;
    // the give-up flag sort_ws_status reads: reduce-then-scan never waits,
    // but the caller's workspace may hold anything (recycled allocations)
    MPX_RETURN_IF_HIP_ERROR(hipMemsetAsync(r.err, 0, sizeof(uint32_t), s));
    for (int p = 0; p < 4; ++p) {
        const uint32_t *src = (p & 1) ? r.tmp : x;
        uint32_t *dst = (p & 1) ? x : r.tmp;
        const int in_mode = p == 0 ? mode : (int)kRawKeys;
        // offsets in status[0 .. 256 * ntiles), digit totals in hist[0 .. 256)
        if (small_tiles)
            hipLaunchKernelGGL(radix_count_kernel<kRTileSmall>, dim3((unsigned)ntiles), dim3(kCThreads), 0, s, src, n,
                               8 * p, in_mode, r.status, ntiles);
        else if (big_tiles)
            hipLaunchKernelGGL(radix_count_kernel<kRTileBig>, dim3((unsigned)ntiles), dim3(kCThreads), 0, s, src, n,
                               8 * p, in_mode, r.status, ntiles);
        else
            hipLaunchKernelGGL(radix_count_kernel<kRTile>, dim3((unsigned)ntiles), dim3(kCThreads), 0, s, src, n,
                               8 * p, in_mode, r.status, ntiles);
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
        hipLaunchKernelGGL(radix_scan1024_kernel, dim3(256), dim3(kScanThreads), 0, s, r.status, ntiles, r.hist);
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
        const int rounded = (ntiles + kNumXCDs - 1) / kNumXCDs * kNumXCDs;
        if (variant == 7)
            launch_lean(p, mode, std::min(kNumCUs * 2, rounded), s, src, dst, n, r.hist, r.status, ntiles);
        else if (variant == 8)
            launch_lean<kRThreads / 2>(p, mode, std::min(kNumCUs * 4, rounded), s, src, dst, n, r.hist, r.status,
                                       ntiles);
        else if (variant == 20)  // RANK 4, two tiles of keys in flight
            launch_lean<kRThreads, 4, 4, 2>(p, mode, std::min(kNumCUs * 2, rounded), s, src, dst, n, r.hist, r.status,
                                            ntiles);
        else if (variant == 21)  // 20 on 4096-key tiles
            launch_lean<kRThreads / 2, 4, 4, 2>(p, mode, std::min(kNumCUs * 4, rounded), s, src, dst, n, r.hist,
                                                r.status, ntiles);
        else  // 22: 20 on 16384-key tiles: longer digit runs, fewer partial output lines
            launch_lean<kRThreads * 2, 4, 4, 2>(p, mode, std::min(kNumCUs, rounded), s, src, dst, n, r.hist, r.status,
                                                ntiles);
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    }
    return MPX_OK;
}

int grid_for(int64_t work, int block) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((work + block - 1) / block, (int64_t)kNumCUs * 16));
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

size_t u8_ws_bytes() { return 256 * sizeof(uint32_t); }  // the global bin counts

bool use_radix(int64_t n) { return n > kTile && n < kRadixMaxN; }

}  // namespace

int64_t sort_workspace_bytes(int64_t n, int dtype) {
    if (n < 2) return 0;
    if (dtype == MPX_SORT_U8) return (int64_t)u8_ws_bytes();
    return use_radix(n) ? (int64_t)radix_ws_bytes(n) : 0;
}

int sort_impl(void *data, int64_t n, int dtype, void *ws, int64_t ws_bytes, void *stream, int variant,
              SortRadixFn radix) {
    MPX_CHECK_ARG(n >= 0, "n must be >= 0");
    MPX_CHECK_ARG(dtype == MPX_SORT_I32 || dtype == MPX_SORT_F32 || dtype == MPX_SORT_U8, "bad dtype");
    if (n < 2) return MPX_OK;
    MPX_CHECK_ARG(data, "null data");
    MPX_CHECK_ARG(ws_bytes >= sort_workspace_bytes(n, dtype) && (ws || sort_workspace_bytes(n, dtype) == 0),
                  "workspace smaller than mpx_sort_workspace_bytes(n, dtype)");
    MPX_CHECK_ARG(!ws || aligned16(ws), "workspace must be 16-byte aligned");
    hipStream_t s = as_stream(stream);
    if (dtype == MPX_SORT_U8) {
        const int64_t head = std::min<int64_t>(n, (16 - (int64_t)(reinterpret_cast<uintptr_t>(data) & 15u)) & 15);
        const int64_t nvec = (n - head) / 16;
        // one 16-wave block per CU (each block ends with 256 global atomics: 8
        // blocks per CU measured 45 us for the histogram at 2^26), two loads in
        // flight per thread
        const int hblocks = (int)std::min<int64_t>(grid_for(std::max<int64_t>((nvec + 1) / 2, 1), 1024), kNumCUs);
        uint32_t *ghist = static_cast<uint32_t *>(ws);
        uint8_t *x = static_cast<uint8_t *>(data);
        MPX_RETURN_IF_HIP_ERROR(hipMemsetAsync(ghist, 0, 256 * sizeof(uint32_t), s));
        hipLaunchKernelGGL(hist_u8_kernel, dim3(hblocks), dim3(1024), 0, s, x, n, head, nvec, ghist);
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
        hipLaunchKernelGGL(fill_u8_kernel, dim3(grid_for(std::max<int64_t>(nvec, 1), 256)), dim3(256), 0, s, x, n, head,
                           nvec, ghist);
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
        return MPX_OK;
    }
    MPX_CHECK_ARG((reinterpret_cast<uintptr_t>(data) & 3u) == 0, "int32/float32 data must be 4-byte aligned");
    uint32_t *x = static_cast<uint32_t *>(data);
    const int is_float = dtype == MPX_SORT_F32;
    if (use_radix(n)) return (radix ? radix : radix_sort32)(x, n, is_float ? kRawF32 : kRawI32, ws, variant, s);
    hipLaunchKernelGGL(to_keys_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, x, n, is_float);
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    const int rc = sort_keys(x, n, s);
    if (rc != MPX_OK) return rc;
    hipLaunchKernelGGL(from_keys_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, x, n, is_float);
    MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    return MPX_OK;
}

// Convenience form without a caller workspace (tools, one-off sorts): the
// scratch is allocated for this call and freed after the stream drains.
// Did a look-back wait of the last sort in `ws` give up (kSpinLimit)? Only
// the onesweep schedule (variant 1, on request) waits; its predecessors are
// always resident (tile ids in launch order), so this is a hardware-fault
// detector. Synchronous: call after the sort's stream has drained.
int sort_ws_status(const void *ws, int64_t n, int dtype) {
    if (dtype == MPX_SORT_U8 || !ws || !use_radix(n)) return MPX_OK;
    const RadixWs r = radix_layout(const_cast<void *>(ws), n);
    uint32_t err = 0;
    MPX_RETURN_IF_HIP_ERROR(hipMemcpy(&err, r.err, sizeof(err), hipMemcpyDeviceToHost));
    if (err) {
        set_error("sort: a decoupled look-back wait gave up (a predecessor tile never published)");
        return MPX_ERR_HIP;
    }
    return MPX_OK;
}

int sort_alloc(void *data, int64_t n, int dtype, void *stream) {
    const int64_t bytes = sort_workspace_bytes(std::max<int64_t>(n, 0), dtype);
    void *ws = nullptr;
    if (bytes > 0) MPX_RETURN_IF_HIP_ERROR(hipMalloc(&ws, (size_t)bytes));
    int rc = sort_impl(data, n, dtype, ws, bytes, stream, 0, nullptr);
    if (ws) {
        const hipError_t e = hipStreamSynchronize(as_stream(stream));
        if (rc == MPX_OK && e == hipSuccess) rc = sort_ws_status(ws, n, dtype);
        (void)hipFree(ws);
        MPX_RETURN_IF_HIP_ERROR(e);
    }
    return rc;
}

MPX_MODULE_ANCHOR(sort)

}  // namespace mpx

extern "C" int mpx_sort(void *data, int64_t n, int dtype, void *stream) { return mpx::sort_alloc(data, n, dtype, stream); }

extern "C" int64_t mpx_sort_workspace_bytes(int64_t n, int dtype) { return mpx::sort_workspace_bytes(n, dtype); }

extern "C" int mpx_sort_ws_status(const void *workspace, int64_t n, int dtype) {
    return mpx::sort_ws_status(workspace, n, dtype);
}

extern "C" int mpx_sort_ws(void *data, int64_t n, int dtype, void *workspace, int64_t workspace_bytes, void *stream) {
    return mpx::sort_impl(data, n, dtype, workspace, workspace_bytes, stream, 0, nullptr);
}

extern "C" int mpx_sort_lane_order_ok(void *stream) { return mpx::lds_rtn_order_ok(mpx::as_stream(stream)); }
