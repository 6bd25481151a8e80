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
//       - onesweep (variant 1; AUTO up to 2^18 keys before round 5): one histogram pass builds all
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

#include "internal.hpp"
#include "mpx/tuning.h"

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


// ---------------------------------------------------------------------------
// LSD radix sort (onesweep)
// ---------------------------------------------------------------------------
constexpr int kRThreads = 512;                 // 8 waves
constexpr int kRWaves = kRThreads / 64;
constexpr int kRPer = 16;                      // keys per thread
constexpr int kRTile = kRThreads * kRPer;      // 8192 keys per tile
constexpr int kRWaveKeys = kRTile / kRWaves;   // 1024 contiguous keys per wave
constexpr int kHotMax = 4;                     // RANK 3: hot digits ranked by ballot (RANK 4: 2)
constexpr int kHotShare = 16;                  // hot: at least 1 / kHotShare of the keys
constexpr uint32_t kFlagA = 1u << 30;          // tile aggregate published
constexpr uint32_t kFlagP = 2u << 30;          // inclusive prefix published
constexpr uint32_t kCountMask = (1u << 30) - 1;
constexpr int64_t kRadixMaxN = (int64_t)1 << 30;
constexpr uint32_t kSpinLimit = 1u << 26;      // exit guarantee; never reached with resident predecessors

enum { kRawKeys = 0, kRawI32 = 1, kRawF32 = 2 };

__device__ __forceinline__ uint32_t to_key(uint32_t v, int mode) {
    return mode == kRawF32 ? (v ^ ((uint32_t)((int32_t)v >> 31) | 0x80000000u))
                           : mode == kRawI32 ? (v ^ 0x80000000u) : v;
}
__device__ __forceinline__ uint32_t from_key(uint32_t k, int mode) {
    return mode == kRawF32 ? (k ^ ((k >> 31) ? 0x80000000u : 0xffffffffu))
                           : mode == kRawI32 ? (k ^ 0x80000000u) : k;
}

// all four digit histograms of the (transformed) keys in one read
__global__ __launch_bounds__(256) void radix_hist_kernel(const uint32_t *__restrict__ x, int64_t n, int mode,
                                                         uint32_t *__restrict__ hist) {
    __shared__ uint32_t h[4 * 256];
    for (int i = threadIdx.x; i < 4 * 256; i += 256) h[i] = 0;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t k = to_key(x[i], mode);
        atomicAdd(&h[k & 255u], 1u);
        atomicAdd(&h[256 + ((k >> 8) & 255u)], 1u);
        atomicAdd(&h[512 + ((k >> 16) & 255u)], 1u);
        atomicAdd(&h[768 + (k >> 24)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 4 * 256; i += 256)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

// All four digit histograms in one read for the lean onesweep (variant 14):
// per-wave LDS tables (no cross-wave contention on a digit's counter),
// 16-B non-temporal key loads where the array is 16-B aligned, one global add
// per (block, digit, non-zero count); 2 persistent blocks per CU.
__global__ __launch_bounds__(256) void radix_hist4_kernel(const uint32_t *__restrict__ x, int64_t n, int mode,
                                                          uint32_t *__restrict__ hist) {
    __shared__ uint32_t h[4][4 * 256];
    const int t = threadIdx.x;
    for (int i = t; i < 4 * 4 * 256; i += 256) (&h[0][0])[i] = 0;
    __syncthreads();
    uint32_t *hw = h[t >> 6];
    auto add = [&](uint32_t v) {
        const uint32_t k = to_key(v, mode);
        atomicAdd(&hw[k & 255u], 1u);
        atomicAdd(&hw[256 + ((k >> 8) & 255u)], 1u);
        atomicAdd(&hw[512 + ((k >> 16) & 255u)], 1u);
        atomicAdd(&hw[768 + (k >> 24)], 1u);
    };
    const int64_t stride = (int64_t)gridDim.x * 256;
    const int64_t gt = (int64_t)blockIdx.x * 256 + t;
    int64_t done = 0;
    if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 *xv = reinterpret_cast<const u32x4 *>(x);
        const int64_t nv = n / 4;
        for (int64_t i = gt; i < nv; i += stride) {
            const u32x4 q = __builtin_nontemporal_load(xv + i);
            add(q[0]);
            add(q[1]);
            add(q[2]);
            add(q[3]);
        }
        done = nv * 4;
    }
    for (int64_t i = done + gt; i < n; i += stride) add(x[i]);
    __syncthreads();
    for (int i = t; i < 4 * 256; i += 256) {
        const uint32_t c = h[0][i] + h[1][i] + h[2][i] + h[3][i];
        if (c) atomicAdd(&hist[i], c);
    }
}

// exclusive scan of one value per thread over threads 0..255 (waves 0-3);
// every thread of the block must call it (two barriers)
__device__ __forceinline__ uint32_t scan256_excl(uint32_t v, uint32_t *s_wsum) {
    const int t = threadIdx.x, lane = t & 63;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (t < 256 && lane == 63) s_wsum[t >> 6] = x;
    __syncthreads();
    uint32_t add = 0;
    for (int w = 0; w < (t >> 6) && w < 4; ++w) add += s_wsum[w];
    __syncthreads();  // s_wsum may be reused by the caller
    return x - v + add;
}

// Peer mask of equal digits within a wave through a wave-private LDS table of
// 256 lane masks: every lane ORs its bit into its digit's slot, reads the slot
// back and clears it (LDS ops of one wave execute in order; OR commutes, so
// the mask is deterministic whatever order the lanes land in). Three LDS ops
// per 64 keys instead of an 8-ballot VALU match (~50 VALU per 64 keys), which
// made the rank instruction-bound.
// Each lane ORs and clears only its half-wave's 32-bit word of the slot
// (ds_or_b32 / ds_write_b32: half the bytes and bank slots of a 64-bit
// access); the read-back takes both words.
// All three accesses go through uint32_t: a 64-bit read of the slot would not
// alias the 32-bit OR and clear for the compiler (type-based alias analysis),
// which may then move the clear above the read.
__device__ __forceinline__ uint64_t match_digit_lds(uint32_t d, int lane, uint64_t *tbl) {
    uint32_t *slot = reinterpret_cast<uint32_t *>(tbl) + 2 * d;
    uint32_t *word = slot + (lane >> 5);
    atomicOr(word, 1u << (lane & 31));
    const uint32_t lo = slot[0], hi = slot[1];
    *word = 0;
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// (A ballot form of the peer mask — 8 x (bfe + cmp + 2 bitop3) VALU per 64
// keys, no LDS — ran the round-3 scatter at 85.3M VALU instructions and 214 us
// per pass against 190 us with the LDS table; retired, profiles/lab5_sort.md.)

// Digit pass. LOOKBACK (onesweep): the tile id comes from an atomic counter
// and the global digit offsets from decoupled look-back over `status`.
// !LOOKBACK (reduce-then-scan): the tile id is the XCD-remapped block id and
// the offsets were scanned beforehand (radix_count_kernel + radix_scan_kernel:
// offs[d][tile] = keys of digit d in the tiles before this one, tot[d] = keys
// of digit d in the array).
template <bool LOOKBACK>
__global__ __launch_bounds__(kRThreads) __attribute__((amdgpu_waves_per_eu(6))) void radix_pass_kernel(const uint32_t *__restrict__ in,
                                                               uint32_t *__restrict__ out, int64_t n, int shift,
                                                               int in_mode, int out_mode,
                                                               const uint32_t *__restrict__ hist,
                                                               uint32_t *__restrict__ status,
                                                               uint32_t *__restrict__ tile_ctr,
                                                               uint32_t *__restrict__ err, int ntiles) {
    // s_keys (scatter staging) doubles as the per-wave peer-mask tables
    // (8 x 256 x 8 B) used only while ranking: 43 KB of LDS per block
    __shared__ uint32_t s_keys[kRTile];
    __shared__ uint32_t s_cnt[kRWaves][256];  // per-wave digit counts, then exclusive offsets
    __shared__ uint32_t s_dstart[256];        // tile-local start of each digit
    __shared__ uint32_t s_gbase[256];         // global position of digit d's run minus s_dstart[d]
    __shared__ uint32_t s_wsum[4];
    __shared__ uint32_t s_tile;
    static_assert(kRWaves * 256 * 2 <= kRTile, "peer-mask tables must fit in the staging buffer");
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint64_t *tbl = reinterpret_cast<uint64_t *>(s_keys) + w * 256;
    if constexpr (LOOKBACK) {
        if (t == 0) s_tile = atomicAdd(tile_ctr, 1u);
    }
    for (int i = t; i < kRWaves * 256; i += kRThreads) {
        (&s_cnt[0][0])[i] = 0;
        reinterpret_cast<uint64_t *>(s_keys)[i] = 0;
    }
    __syncthreads();
    const uint32_t tile = LOOKBACK ? s_tile : (uint32_t)xcd_remap(blockIdx.x, gridDim.x);
    const int64_t base = (int64_t)tile * kRTile + w * kRWaveKeys + lane;

    uint32_t key[kRPer], rank[kRPer];
#pragma unroll
    for (int e = 0; e < kRPer; ++e) {
        const int64_t i = base + e * 64;
        key[e] = i < n ? to_key(in[i], in_mode) : 0xffffffffu;  // pads rank last and are never stored
    }
    // reduce-then-scan: this tile's offsets and the digit totals are known
    // up front — issue their loads now, under the ranking
    uint32_t pre_excl = 0, pre_tot = 0;
    if constexpr (!LOOKBACK) {
        if (t < 256) {
            pre_excl = status[(size_t)t * ntiles + tile];  // offs[d][tile]
            pre_tot = hist[t];
        }
    }
    // Stable rank within the wave (slices in index order, lanes in order),
    // batched so the LDS round trips overlap: (1) every slice's peer mask,
    // (2) one leader per digit and slice adds the slice's count to the wave
    // counter (ds_add_rtn; same-wave LDS ops land in program order, so slice
    // e sees exactly slices < e), (3) peers take the leader's old count.
    // groups of kRG slices bound the live peer masks (VGPR pressure)
    constexpr int kRG = 4;
#pragma unroll
    for (int g = 0; g < kRPer; g += kRG) {
        uint64_t m[kRG];
#pragma unroll
        for (int e = 0; e < kRG; ++e) m[e] = match_digit_lds((key[g + e] >> shift) & 255u, lane, tbl);
        uint32_t old[kRG], pre[kRG];
#pragma unroll
        for (int e = 0; e < kRG; ++e) {
            pre[e] = lanes_below(m[e]);
            old[e] = 0;
            if (pre[e] == 0) old[e] = atomicAdd(&s_cnt[w][(key[g + e] >> shift) & 255u], (uint32_t)__popcll(m[e]));
        }
#pragma unroll
        for (int e = 0; e < kRG; ++e) {
            const int leader = (int)__builtin_ctzll(m[e]);
            rank[g + e] = (uint32_t)__builtin_amdgcn_ds_bpermute(leader << 2, (int)old[e]) + pre[e];
        }
    }
    __syncthreads();
    uint32_t tot = 0;
    if (t < 256) {
#pragma unroll
        for (int ww = 0; ww < kRWaves; ++ww) {
            const uint32_t c = s_cnt[ww][t];
            s_cnt[ww][t] = tot;
            tot += c;
        }
        uint32_t excl = 0;
        if constexpr (LOOKBACK) {
            // publish this tile's count, then look back for the preceding tiles' sum
            uint32_t *st = status + (size_t)tile * 256 + t;
            if (tile == 0) {
                __hip_atomic_store(st, kFlagP | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                __hip_atomic_store(st, kFlagA | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                int64_t j = (int64_t)tile - 1;
                uint32_t spins = 0;
                while (true) {
                    const uint32_t v = __hip_atomic_load(status + (size_t)j * 256 + t, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
                    if ((v & ~kCountMask) == 0) {
                        if (++spins > kSpinLimit) {
                            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                        continue;
                    }
                    excl += v & kCountMask;
                    if (v & kFlagP) break;
                    --j;
                }
                __hip_atomic_store(st, kFlagP | (excl + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            excl = pre_excl;
        }
        s_gbase[t] = excl;  // + digit base - tile-local start, below
    }
    const uint32_t dstart = scan256_excl(tot, s_wsum);
    const uint32_t dbase = scan256_excl(t < 256 ? (LOOKBACK ? hist[t] : pre_tot) : 0u, s_wsum);
    if (t < 256) {
        s_dstart[t] = dstart;
        s_gbase[t] += dbase - dstart;
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < kRPer; ++e) {
        const uint32_t d = (key[e] >> shift) & 255u;
        s_keys[s_dstart[d] + s_cnt[w][d] + rank[e]] = key[e];
    }
    __syncthreads();
#pragma unroll 4
    for (int i = t; i < kRTile; i += kRThreads) {
        const uint32_t k = s_keys[i];
        const int64_t pos = (int64_t)s_gbase[(k >> shift) & 255u] + i;
        if (pos < n) out[pos] = from_key(k, out_mode);
    }
}

// LDS-only workgroup barrier: orders LDS accesses without waiting for the
// block's global loads (the next tile's prefetch stays in flight across it)
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// scan256_excl with LDS-only barriers
__device__ __forceinline__ uint32_t scan256_excl_lds(uint32_t v, uint32_t *s_wsum) {
    const int t = threadIdx.x, lane = t & 63;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (t < 256 && lane == 63) s_wsum[t >> 6] = x;
    lds_barrier();
    uint32_t add = 0;
    for (int w = 0; w < (t >> 6) && w < 4; ++w) add += s_wsum[w];
    lds_barrier();
    return x - v + add;
}

// reduce-then-scan scatter, persistent: kPersistBlocksPerCU blocks per CU walk
// the tiles of their XCD's contiguous range (consecutive tiles stay XCD-local
// so their output runs merge in L2) and load the next tile's keys while the
// current one is ranked, scanned, staged and written — the per-tile phases
// that left the memory system idle in the one-tile-per-block kernel. Barriers
// are LDS-only so the prefetch stays in flight across them.
constexpr int kPersistBlocksPerCU = 2;

// The round-2 production scatter (LDS peer-mask table, leader ds_add_rtn +
// bpermute ranking), kept as tuning variant 4 for same-process A/B against
// the lean kernel below.
__global__ __launch_bounds__(kRThreads) __attribute__((amdgpu_waves_per_eu(4))) void radix_scatter_kernel(
    const uint32_t *__restrict__ in, uint32_t *__restrict__ out, int64_t n, int shift, int in_mode, int out_mode,
    const uint32_t *__restrict__ tot, const uint32_t *__restrict__ offs, int ntiles) {
    __shared__ uint32_t s_keys[kRTile];
    __shared__ uint32_t s_cnt[kRWaves][256];
    __shared__ uint32_t s_gbase[256];
    __shared__ uint32_t s_wsum[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint64_t *tbl = reinterpret_cast<uint64_t *>(s_keys) + w * 256;
    const int xcd = blockIdx.x % kNumXCDs, per = gridDim.x / kNumXCDs;  // gridDim.x: a multiple of 8
    const int t1 = (int)((int64_t)ntiles * (xcd + 1) / kNumXCDs);
    const int t0 = (int)((int64_t)ntiles * xcd / kNumXCDs);
    int tile = t0 + (int)blockIdx.x / kNumXCDs;
    if (tile >= t1) return;  // block-uniform
    // digit bases of the whole array (the same for every tile of the pass)
    const uint32_t dbase = scan256_excl_lds(t < 256 ? tot[t] : 0u, s_wsum);

    uint32_t raw[kRPer], nxt[kRPer];
    auto load_tile = [&](uint32_t (&dst)[kRPer], int tl) {
        const int64_t base = (int64_t)tl * kRTile + w * kRWaveKeys + lane;
#pragma unroll
        for (int e = 0; e < kRPer; ++e) {
            const int64_t i = base + e * 64;
            dst[e] = i < n ? in[i] : 0u;
        }
    };
    load_tile(raw, tile);
    for (; tile < t1; tile += per) {
        const int ptile = tile;
        const int64_t tile0 = (int64_t)ptile * kRTile;
        if (tile + per < t1) load_tile(nxt, tile + per);  // in flight under this tile's work
        const uint32_t excl = t < 256 ? offs[(size_t)t * ntiles + ptile] : 0u;
        for (int i = t; i < kRWaves * 256; i += kRThreads) {
            (&s_cnt[0][0])[i] = 0;
            reinterpret_cast<uint64_t *>(s_keys)[i] = 0;
        }
        lds_barrier();
        uint32_t key[kRPer], rank[kRPer];
#pragma unroll
        for (int e = 0; e < kRPer; ++e)  // pads (past n) rank last and are never stored
            key[e] = tile0 + w * kRWaveKeys + lane + e * 64 < n ? to_key(raw[e], in_mode) : 0xffffffffu;
#ifndef MPX_SORT_RG  // slices ranked per batch (A/B builds override)
#define MPX_SORT_RG 4
#endif
        constexpr int kRG = MPX_SORT_RG;
#pragma unroll
        for (int g = 0; g < kRPer; g += kRG) {
            uint64_t m[kRG];
#pragma unroll
            for (int e = 0; e < kRG; ++e)
                m[e] = match_digit_lds((key[g + e] >> shift) & 255u, lane, tbl);
            uint32_t old[kRG], pre[kRG];
#pragma unroll
            for (int e = 0; e < kRG; ++e) {
                pre[e] = lanes_below(m[e]);
                old[e] = 0;
                if (pre[e] == 0) old[e] = atomicAdd(&s_cnt[w][(key[g + e] >> shift) & 255u], (uint32_t)__popcll(m[e]));
            }
#pragma unroll
            for (int e = 0; e < kRG; ++e) {
                const int leader = (int)__builtin_ctzll(m[e]);
                rank[g + e] = (uint32_t)__builtin_amdgcn_ds_bpermute(leader << 2, (int)old[e]) + pre[e];
            }
        }
        lds_barrier();
        uint32_t cnt = 0, wexcl[kRWaves];
        if (t < 256) {
#pragma unroll
            for (int ww = 0; ww < kRWaves; ++ww) {
                wexcl[ww] = cnt;
                cnt += s_cnt[ww][t];
            }
        }
        const uint32_t dstart = scan256_excl_lds(cnt, s_wsum);
        if (t < 256) {
            // one table per wave holding tile-local digit start + the wave's
            // offset: the staging scatter below gathers once per key, not twice
#pragma unroll
            for (int ww = 0; ww < kRWaves; ++ww) s_cnt[ww][t] = dstart + wexcl[ww];
            s_gbase[t] = excl + dbase - dstart;
        }
        lds_barrier();
#pragma unroll
        for (int e = 0; e < kRPer; ++e) {
            const uint32_t d = (key[e] >> shift) & 255u;
            s_keys[s_cnt[w][d] + rank[e]] = key[e];
        }
        lds_barrier();
#pragma unroll 4
        for (int i = t; i < kRTile; i += kRThreads) {
            const uint32_t k = s_keys[i];
            const int64_t pos = (int64_t)s_gbase[(k >> shift) & 255u] + i;
            if (pos < n) out[pos] = from_key(k, out_mode);
        }
        lds_barrier();  // s_keys / s_gbase are rewritten by the next tile
#pragma unroll
        for (int e = 0; e < kRPer; ++e) raw[e] = nxt[e];
    }
}

// Inclusive scan over the 64 lanes of a wave on DPP (row shifts within
// 16-lane rows, then the row-15 / row-31 broadcasts): six VALU ops, no LDS
// round trip (the __shfl_up form is six dependent ds_bpermute).
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// scan256_excl_lds on DPP, without the trailing barrier: the caller orders
// the next write of s_wsum behind a later block barrier
__device__ __forceinline__ uint32_t scan256_excl_dpp(uint32_t v, uint32_t *s_wsum) {
    const int t = threadIdx.x, lane = t & 63;
    const uint32_t x = wave_incl_scan_dpp(v);
    if (t < 256 && lane == 63) s_wsum[t >> 6] = x;
    lds_barrier();
    uint32_t add = 0;
    for (int w = 0; w < (t >> 6) && w < 4; ++w) add += s_wsum[w];
    return x - v + add;
}

template <int MODE>
__device__ __forceinline__ uint32_t to_key_t(uint32_t v) { return to_key(v, MODE); }
template <int MODE>
__device__ __forceinline__ uint32_t from_key_t(uint32_t k) { return from_key(k, MODE); }

// Lean persistent scatter (variants 7 / 8, production). The same schedule and
// ranking as radix_scatter_kernel (LDS peer-mask table), with the
// per-key VALU cut — the round-3 counters put the scatter on its VALU pipe
// (51.6M VALU per pass with the LDS table, 85.3M with ballots; 4 cycles each
// per SIMD ~ 88 / 145 us of a 190 / 214 us pass):
//   * key loads and output stores are buffer instructions: one lane offset
//     register, the 16 slices in the instruction's immediate field, the tile
//     in the scalar offset, and the array bound in the descriptor (pads and
//     past-the-end stores are dropped by the hardware, no 64-bit address or
//     compare per key);
//   * the key transform is a template parameter (only the first pass reads
//     raw int32 / float32, only the last writes them);
//   * a slice's digit counter is read before its lowest lane adds the peer
//     count (ds_add, no return): a wave's LDS operations execute in program
//     order, so the read returns the count of the slices before it, and
//     lanes_below(peer mask) the rank among its peers — no find-first-bit or
//     bpermute;
//   * the next tile's keys load into a second register set while this tile is
//     ranked, staged and written.
//   * four block barriers per tile instead of six (the retired variant 6) — each
//     wave zeroes its own counter row after its own staging reads (no other
//     wave writes that row before the next tile's first barrier), the 256-digit
//     scan runs on DPP row shifts / broadcasts with one barrier for the four
//     wave sums, and nothing needs the closing barrier: the next tile's first
//     barrier orders its staging / scan writes after this tile's write-out.
// TPB = 512: 8192-key tiles, 2 blocks per CU (4 waves per SIMD; 3 blocks = 6
// waves per SIMD fit the LDS but not the registers: 80 VGPRs spill 280 B per
// lane). TPB = 256 (variant 8): 4096-key tiles, 4 blocks per CU — twice the
// independent barrier domains per CU for the same waves.
// RANK 1 (variants 9 / 10, production above 2^18 keys): every lane takes its
// rank straight from a returning LDS add on its wave's digit counter
// (ds_add_rtn_u32: one LDS instruction per slice instead of the table's
// or / read / clear plus the counter read and the leaders' add; per 2^26-key
// pass 9.7M -> 5.5M LDS instructions, 38.4M -> 15.2M bank-conflict cycles,
// 21.4M -> 10.9M VALU). The sort is stable because the LDS applies one
// instruction's same-address lanes in ascending lane order: a pass that broke
// that order would scramble keys equal in this digit and already ordered by
// the lower ones, which the GPU sort suite's uniform, few-distinct, sorted and
// reversed inputs (every variant, 4097 .. 2^26 keys) would catch.
// RANK 3 / 4 (variants 18 / 19 and 20 / 21, AUTO): RANK 1 plus hot digits
// ranked without LDS. A digit holding at least 1/kHotShare of the pass's keys
// (tot[], known before the pass) puts many lanes of one returning add on one
// counter, and those lanes serialise (the float32 top byte: 28.1M conflict
// cycles against 15.2M for uniform digits, 136 vs 120 us; small-range ints:
// every lane on one counter). The largest kHotMax (RANK 3) or 2 (RANK 4) such
// digits keep a wave-uniform count in scalar registers instead: one compare
// mask per hot digit per slice, rank = count + lanes below in the mask; the
// remaining lanes take the returning add as before. The order is the same
// (slice-major, lane-minor), so the pass stays stable. A pass without hot
// digits (uniform data) runs the RANK 1 loop: the tile loop is instantiated
// twice and the block picks one. Per 2^26-key float32 last pass
// (profiles/lab5_sort.md): RANK 1 135.9 us, RANK 3 118.6 (8.3M conflicts,
// 35.8M VALU), RANK 4 114.2 (16.0M, 25.2M VALU).
// KNOCK (tuning probe, mpx_sort_scatter_probe; output NOT sorted): bit 1 stages
// at lane-linear positions, 2 skips the counter read, 4 the leaders' add, 8 the
// peer-mask table (own-lane masks), 16 the write-out's digit lookup — same
// loads and stores, so the counters attribute LDS conflicts and time per step.
template <int IN_MODE, int OUT_MODE, int TPB = kRThreads, int RANK = 0, int KNOCK = 0, int WPE = 4, int PF = 1>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(WPE))) void radix_scatter_lean_kernel(
    const uint32_t *__restrict__ in, uint32_t *__restrict__ out, int64_t n, int shift,
    const uint32_t *__restrict__ tot, const uint32_t *__restrict__ offs, int ntiles) {
    constexpr int NW = TPB / 64, TILE = TPB * kRPer;  // kRWaveKeys keys per wave either way
    __shared__ uint32_t s_keys[TILE];  // staging
    // per-wave peer-mask tables, separate from the staging buffer: every
    // slice clears the words it set, so the tables are zero again after each
    // tile and are cleared only once, here
    __shared__ uint32_t s_tbl[NW * 512];
    // digit counters: one row per wave (RANK 0 / 1) or per half-wave (RANK 2,
    // rows padded so a half-wave pair's rows start 32 banks apart)
    constexpr int NR = RANK == 2 ? 2 * NW : NW, CW = RANK == 2 ? 256 + 32 : 256;
    __shared__ uint32_t s_cnt[NR][CW];
    __shared__ uint32_t s_gbase[256];
    __shared__ uint32_t s_wsum[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int crow = RANK == 2 ? 2 * w + (lane >> 5) : w;  // this lane's counter row
    if constexpr (RANK == 0)  // the returning-add rankings never touch the tables (no LDS kept for them)
        for (int i = t; i < NW * 512; i += TPB) s_tbl[i] = 0;
    for (int i = t; i < NR * CW; i += TPB) (&s_cnt[0][0])[i] = 0;
    const int xcd = blockIdx.x % kNumXCDs, per = gridDim.x / kNumXCDs;  // gridDim.x: a multiple of 8
    const int t1 = (int)((int64_t)ntiles * (xcd + 1) / kNumXCDs);
    const int t0 = (int)((int64_t)ntiles * xcd / kNumXCDs);
    int tile = t0 + (int)blockIdx.x / kNumXCDs;
    if (tile >= t1) return;  // block-uniform
    const uint32_t n32 = (uint32_t)n;           // n < 2^30
    const int nbytes = (int)(n32 * 4u);          // the byte bound fits the descriptor's 32 bits
    const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(in), 0, nbytes,
                                                                         0x00020000);
    const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(out, 0, nbytes, 0x00020000);
    // RANK 2: each half-wave owns a contiguous half of its wave's keys (slice
    // e of lane l is key 512 (l >> 5) + 32 e + (l & 31)), so ranking each half
    // on its own counter row keeps the order stable; otherwise slice e of lane
    // l is key 64 e + l
    constexpr uint32_t kSlice = RANK == 2 ? 32u : 64u;  // keys between a lane's slices
    const int klane = RANK == 2 ? (lane >> 5) * (kRWaveKeys / 2) + (lane & 31) : lane;
    const int vlane = (w * kRWaveKeys + klane) * 4;
    // peer-mask table: slot d = two words (lanes 0-31, 32-63) at tbl + 2d.
    // (A split layout — the lanes 0-31 words at tbl[d], the 32-63 words at
    // tbl[256 + d], so a half-wave's OR / clear spreads over 32 banks instead
    // of 16 — measured neutral: 37.6M vs 38.4M conflict cycles per pass, the
    // same time; profiles/lab5_sort.md.)
    uint32_t *tbl = s_tbl + w * 512;
    uint32_t *const myword = tbl + (lane >> 5);
    const uint32_t mybit = 1u << (lane & 31);
    const uint32_t mytot = t < 256 ? tot[t] : 0u;
    const uint32_t dbase = scan256_excl_lds(mytot, s_wsum);  // + the barrier after the zeroing
    // RANK 3 / 4: the pass's hot digits, the HN largest (ties: lower digit
    // first) of those with at least 1/kHotShare of the keys — at most
    // kHotShare candidates; once per block
    constexpr bool HOT = RANK == 3 || RANK == 4;
    constexpr int HN = RANK == 4 ? 2 : kHotMax;  // hot-digit slots
    int nh = 0;
    uint32_t hd[HN] = {};
    if constexpr (HOT) {
        __shared__ uint32_t s_hotc[4], s_cd[kHotShare], s_cc[kHotShare], s_hd[HN];
        const bool hot = t < 256 && (uint64_t)mytot * kHotShare >= (uint64_t)n;
        const uint64_t hm = __builtin_amdgcn_ballot_w64(hot);
        if (t < 256 && lane == 0) s_hotc[w] = (uint32_t)__popcll(hm);
        lds_barrier();
        uint32_t pos = lanes_below(hm), all = 0;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) {
            const uint32_t c = s_hotc[ww];
            pos += ww < w ? c : 0u;
            all += c;
        }
        if (hot) {  // pos < kHotShare: the candidates hold more than all keys otherwise
            s_cd[pos] = (uint32_t)t;
            s_cc[pos] = mytot;
        }
        lds_barrier();
        if (hot) {
            uint32_t order = 0;
            for (uint32_t c = 0; c < all; ++c)
                order += s_cc[c] > mytot || (s_cc[c] == mytot && s_cd[c] < (uint32_t)t);
            if (order < (uint32_t)HN) s_hd[order] = (uint32_t)t;
        }
        lds_barrier();
        nh = (int)__builtin_amdgcn_readfirstlane(all < (uint32_t)HN ? all : (uint32_t)HN);
#pragma unroll
        for (int j = 0; j < HN; ++j) hd[j] = j < nh ? __builtin_amdgcn_readfirstlane(s_hd[j]) : 256u;
    }

    // whole tiles: one offset register (tile base + lane), slices in the
    // immediate field; the partial last tile (block-uniform) loads and stores
    // under explicit index checks, so correctness never rests on the
    // descriptor's range check
    auto load_tile = [&](uint32_t (&dst)[kRPer], int tl) {
        const int64_t tile0 = (int64_t)tl * TILE;
        if (tile0 + TILE <= n) {
            const uint32_t voff = (uint32_t)tile0 * 4u + (uint32_t)vlane;  // < n * 4 < 2^32
#pragma unroll
            for (int e = 0; e < kRPer; ++e)
                // non-temporal: the keys are read once, and L2 stays free to merge
                // the partial-line digit runs this tile and its XCD neighbours
                // write (2^26 int32 0.828 -> 0.769 ms; NT output stores instead
                // lose those merges: 1.28 ms; profiles/lab5_sort.md)
                dst[e] = __builtin_amdgcn_raw_buffer_load_b32(rin, (int)(voff + e * kSlice * 4u), 0, 2);
        } else {  // 32-bit indices (n < 2^30) keep the partial path's registers small
            const uint32_t i0 = (uint32_t)tile0 + (uint32_t)(w * kRWaveKeys + klane);
#pragma unroll
            for (int e = 0; e < kRPer; ++e) {
                const uint32_t i = i0 + e * kSlice;
                dst[e] = i < n32 ? __builtin_amdgcn_raw_buffer_load_b32(rin, (int)(i * 4u), 0, 0) : 0u;
            }
        }
    };
    // HOTP (RANK 3 / 4 with hot digits in this pass): a separate instance of the
    // tile loop, so a pass without hot digits runs RANK 1's code unchanged
    auto do_tile = [&](uint32_t (&key)[kRPer], int ptile, auto hotp) {
        constexpr bool HOTP = decltype(hotp)::value;
        // s_cnt and the tables are zero here (kernel start / previous write-out)
        const uint32_t excl = t < 256 ? offs[(size_t)t * ntiles + ptile] : 0u;
        const int64_t tile0 = (int64_t)ptile * TILE;
        const bool full = tile0 + TILE <= n;  // block-uniform
#pragma unroll
        for (int e = 0; e < kRPer; ++e) key[e] = to_key_t<IN_MODE>(key[e]);
        if (!full) {  // pads rank last (digit 255 in every pass) and are never stored
            const uint32_t i0 = (uint32_t)tile0 + (uint32_t)(w * kRWaveKeys + klane);
#pragma unroll
            for (int e = 0; e < kRPer; ++e)
                if (i0 + e * kSlice >= n32) key[e] = 0xffffffffu;
        }
        uint32_t rank[kRPer];
        if constexpr (HOTP) {
            // every slot is compared (unused slots hold 256, which no digit
            // matches): straight-line code keeps the counts in scalar registers
            uint32_t hc[HN] = {};  // wave-uniform counts of the hot digits
#pragma unroll
            for (int e = 0; e < kRPer; ++e) {
                const uint32_t d = (key[e] >> shift) & 255u;
                uint32_t r = 0;
                bool hit = false;
#pragma unroll
                for (int j = 0; j < HN; ++j) {
                    const bool is = d == hd[j];
                    const uint64_t m = __builtin_amdgcn_uicmp(d, hd[j], 32);  // ICMP_EQ: the compare's lane mask
                    // hc[j] + the lanes below in m: mbcnt accumulates onto its operand
                    const uint32_t rj =
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, hc[j]));
                    r = is ? rj : r;
                    hc[j] += (uint32_t)__popcll(m);
                    hit = hit || is;
                }
                if (!hit) r = atomicAdd(&s_cnt[crow][d], 1u);
                rank[e] = r;
            }
            // no returning add touched a hot digit's counter
            if (lane == 0) {
                const int wrow = __builtin_amdgcn_readfirstlane(crow);  // scalar addresses: no VGPRs held for them
#pragma unroll
                for (int j = 0; j < HN; ++j)
                    if (j < nh) s_cnt[wrow][hd[j]] = hc[j];
            }
        } else if constexpr (RANK >= 1) {
#pragma unroll
            for (int e = 0; e < kRPer; ++e) rank[e] = atomicAdd(&s_cnt[crow][(key[e] >> shift) & 255u], 1u);
        } else {
#pragma unroll
            for (int g = 0; g < kRPer; g += 4) {  // 4 slices in flight: bounds the live LDS results
                uint32_t lo[4], hi[4], before[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t d = (key[g + e] >> shift) & 255u;
                    if constexpr (KNOCK & 8) {
                        lo[e] = lane < 32 ? mybit : 0u;
                        hi[e] = lane < 32 ? 0u : mybit;
                    } else {
                        atomicOr(myword + 2 * d, mybit);
                        lo[e] = tbl[2 * d];
                        hi[e] = tbl[2 * d + 1];
                        myword[2 * d] = 0;
                    }
                    before[e] = (KNOCK & 2) ? 0u : s_cnt[w][d];
                    // one add per distinct digit (its lowest lane): 64 lanes adding
                    // to one counter would serialise on skewed digits (the top byte
                    // of normally distributed floats takes a handful of values)
                    const uint64_t m = ((uint64_t)hi[e] << 32) | lo[e];
                    if (!(KNOCK & 4) && lanes_below(m) == 0) atomicAdd(&s_cnt[w][d], (uint32_t)__popcll(m));
                }
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    rank[g + e] = before[e] + __builtin_amdgcn_mbcnt_hi(hi[e], __builtin_amdgcn_mbcnt_lo(lo[e], 0u));
            }
        }
        lds_barrier();
        uint32_t cnt = 0, wexcl[NR];
        if (t < 256) {
#pragma unroll
            for (int ww = 0; ww < NR; ++ww) {
                wexcl[ww] = cnt;
                cnt += s_cnt[ww][t];
            }
        }
        const uint32_t dstart = scan256_excl_dpp(cnt, s_wsum);
        if (t < 256) {
#pragma unroll
            for (int ww = 0; ww < NR; ++ww) s_cnt[ww][t] = dstart + wexcl[ww];
            s_gbase[t] = excl + dbase - dstart;
        }
        lds_barrier();
#pragma unroll
        for (int e = 0; e < kRPer; ++e) {
            const uint32_t rk = rank[e];
            if constexpr (KNOCK & 1)
                s_keys[w * kRWaveKeys + e * 64 + lane] = key[e] + (s_cnt[crow][0] + rk == ~0u);  // keeps rank live
            else
                s_keys[s_cnt[crow][(key[e] >> shift) & 255u] + rk] = key[e];
        }
        lds_barrier();
        // this wave's staging reads of its own row(s) are done (program order)
#pragma unroll
        for (int i = lane; i < 256; i += 64) {
            if constexpr (RANK == 2) {
                s_cnt[2 * w][i] = 0;
                s_cnt[2 * w + 1][i] = 0;
            } else {
                s_cnt[w][i] = 0;
            }
        }
        if (full) {
#pragma unroll
            for (int j = 0; j < TILE / TPB; ++j) {
                const int i = t + j * TPB;
                const uint32_t k = s_keys[i];
                const uint32_t gd = (KNOCK & 16) ? s_gbase[0] : s_gbase[(k >> shift) & 255u];
                __builtin_amdgcn_raw_buffer_store_b32(from_key_t<OUT_MODE>(k), rout, (int)((gd + (uint32_t)i) * 4u), 0, 0);
            }
        } else {
            for (int j = 0; j < TILE / TPB; ++j) {
                const int i = t + j * TPB;
                const uint32_t k = s_keys[i];
                const uint32_t pos = s_gbase[(k >> shift) & 255u] + (uint32_t)i;  // < n + TILE < 2^31
                if (pos < n32) __builtin_amdgcn_raw_buffer_store_b32(from_key_t<OUT_MODE>(k), rout, (int)(pos * 4u), 0, 0);
            }
        }
    };

    auto run_tiles = [&](auto hotp) {
        if constexpr (PF == 2) {
            // two tiles in flight: three register sets in fixed roles (an
            // unrolled rotation — a copy between sets would wait for the copied
            // loads and shorten the prefetch back to one tile)
            uint32_t a[kRPer], b[kRPer], c[kRPer];
            load_tile(a, tile);
            if (tile + per < t1) load_tile(b, tile + per);
            for (;;) {
                if (tile + 2 * per < t1) load_tile(c, tile + 2 * per);
                do_tile(a, tile, hotp);
                if ((tile += per) >= t1) break;
                if (tile + 2 * per < t1) load_tile(a, tile + 2 * per);
                do_tile(b, tile, hotp);
                if ((tile += per) >= t1) break;
                if (tile + 2 * per < t1) load_tile(b, tile + 2 * per);
                do_tile(c, tile, hotp);
                if ((tile += per) >= t1) break;
            }
        } else {
            uint32_t a[kRPer], b[kRPer];
            load_tile(a, tile);
            for (; tile < t1; tile += per) {
                if (tile + per < t1) load_tile(b, tile + per);  // in flight under this tile's work
                do_tile(a, tile, hotp);
#pragma unroll
                for (int e = 0; e < kRPer; ++e) a[e] = b[e];
            }
        }
    };
    if constexpr (HOT) {
        if (nh > 0)  // block-uniform
            run_tiles(std::true_type{});
        else
            run_tiles(std::false_type{});
    } else {
        run_tiles(std::false_type{});
    }
}

// Lean onesweep (variant 14): the returning-add ranking of the lean scatter
// with decoupled look-back instead of a count pass per digit. One histogram
// kernel reads the keys once for all four digits; each digit pass then moves
// the keys once. Persistent blocks (2 per CU, all resident) take tiles from an
// atomic counter in increasing order and hold at most three ids (the tile
// being ranked, the prefetched next one, and the id whose counter add is in
// flight); every wait is on a smaller tile id, whose holder ranks its tiles
// in increasing order, so the smallest unfinished tile always progresses.
// Per tile: rank into LDS (one ds_add_rtn per key) -> publish the tile's
// digit counts (flag A, agent-scope store) -> stage in LDS -> threads 0-255
// look back over the predecessors' status words, kLbWin at a time (one
// round trip covers kLbWin tiles), until an inclusive prefix (flag P) ->
// publish this tile's inclusive prefix -> write out.
// STATIC (variant 16, experiment): block b takes tiles b, b + G, b + 2G ... in
// order, no tile counter (one atomic word saturates near 88 adds per us on
// this chip, MI355X_MICROARCH.md). Deadlock-free only while every block of
// the grid is resident at once (2 per CU here); a block that never starts
// leaves its tiles' successors spinning to kSpinLimit, the error word set.
template <int IN_MODE, int OUT_MODE, int kLbWin = 8, bool STATIC = false>
__global__ __launch_bounds__(kRThreads) __attribute__((amdgpu_waves_per_eu(4))) void radix_onesweep_lean_kernel(
    const uint32_t *__restrict__ in, uint32_t *__restrict__ out, int64_t n, int shift,
    const uint32_t *__restrict__ tot, uint32_t *__restrict__ status, uint32_t *__restrict__ tile_ctr,
    uint32_t *__restrict__ err, int ntiles) {
    constexpr int TPB = kRThreads, NW = TPB / 64, TILE = kRTile;
    __shared__ uint32_t s_keys[TILE];
    __shared__ uint32_t s_cnt[NW][256];
    __shared__ uint32_t s_gbase[256];
    __shared__ uint32_t s_wsum[4];
    __shared__ int s_next;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (int i = t; i < NW * 256; i += TPB) (&s_cnt[0][0])[i] = 0;
    if (!STATIC && t == 0) s_next = (int)atomicAdd(tile_ctr, 1u);
    const uint32_t dbase = scan256_excl_lds(t < 256 ? tot[t] : 0u, s_wsum);  // its barrier publishes s_next
    int tile = STATIC ? (int)blockIdx.x : s_next;
    if (tile >= ntiles) return;  // block-uniform
    const uint32_t n32 = (uint32_t)n;
    const int nbytes = (int)(n32 * 4u);
    const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(in), 0, nbytes,
                                                                         0x00020000);
    const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc(out, 0, nbytes, 0x00020000);
    const int vlane = (w * kRWaveKeys + lane) * 4;

    auto load_tile = [&](uint32_t (&dst)[kRPer], int tl) {
        const int64_t tile0 = (int64_t)tl * TILE;
        if (tile0 + TILE <= n) {
            const uint32_t voff = (uint32_t)tile0 * 4u + (uint32_t)vlane;
#pragma unroll
            for (int e = 0; e < kRPer; ++e) dst[e] = __builtin_amdgcn_raw_buffer_load_b32(rin, (int)(voff + e * 256u), 0, 2);
        } else {
            const uint32_t i0 = (uint32_t)tile0 + (uint32_t)(w * kRWaveKeys + lane);
#pragma unroll
            for (int e = 0; e < kRPer; ++e) {
                const uint32_t i = i0 + e * 64u;
                dst[e] = i < n32 ? __builtin_amdgcn_raw_buffer_load_b32(rin, (int)(i * 4u), 0, 0) : 0u;
            }
        }
    };
    auto do_tile = [&](uint32_t (&key)[kRPer], int ptile) {
        const int64_t tile0 = (int64_t)ptile * TILE;
        const bool full = tile0 + TILE <= n;  // block-uniform
#pragma unroll
        for (int e = 0; e < kRPer; ++e) key[e] = to_key_t<IN_MODE>(key[e]);
        if (!full) {  // pads rank last (digit 255 in every pass) and are never stored
            const uint32_t i0 = (uint32_t)tile0 + (uint32_t)(w * kRWaveKeys + lane);
#pragma unroll
            for (int e = 0; e < kRPer; ++e)
                if (i0 + e * 64u >= n32) key[e] = 0xffffffffu;
        }
        uint32_t rank[kRPer];
#pragma unroll
        for (int e = 0; e < kRPer; ++e) rank[e] = atomicAdd(&s_cnt[w][(key[e] >> shift) & 255u], 1u);
        lds_barrier();
        uint32_t cnt = 0, wexcl[NW];
        if (t < 256) {
#pragma unroll
            for (int ww = 0; ww < NW; ++ww) {
                wexcl[ww] = cnt;
                cnt += s_cnt[ww][t];
            }
            // the tile's count of digit t, visible to the successors' look-back
            __hip_atomic_store(status + (size_t)ptile * 256 + t, (ptile == 0 ? kFlagP : kFlagA) | cnt, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        const uint32_t dstart = scan256_excl_dpp(cnt, s_wsum);
        if (t < 256) {
#pragma unroll
            for (int ww = 0; ww < NW; ++ww) s_cnt[ww][t] = dstart + wexcl[ww];
        }
        lds_barrier();
#pragma unroll
        for (int e = 0; e < kRPer; ++e) s_keys[s_cnt[w][(key[e] >> shift) & 255u] + rank[e]] = key[e];
        if (t < 256) {
            uint32_t excl = 0;
            if (ptile > 0) {
                int j = ptile - 1;  // next predecessor to consume
                uint32_t spins = 0;
                bool found = false;
                while (!found) {
                    uint32_t v[kLbWin];
#pragma unroll
                    for (int k = 0; k < kLbWin; ++k)
                        v[k] = j - k >= 0 ? __hip_atomic_load(status + (size_t)(j - k) * 256 + t, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT)
                                          : kFlagP;  // never reached: tile 0 publishes a prefix
                    int used = 0;
                    bool stalled = false;
#pragma unroll
                    for (int k = 0; k < kLbWin; ++k) {
                        if (found || stalled) continue;
                        if ((v[k] & ~kCountMask) == 0) {
                            stalled = true;
                            continue;
                        }
                        excl += v[k] & kCountMask;
                        ++used;
                        if (v[k] & kFlagP) found = true;
                    }
                    j -= used;
                    if (stalled && !found) {
                        if (++spins > kSpinLimit) {
                            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                __hip_atomic_store(status + (size_t)ptile * 256 + t, kFlagP | (excl + cnt), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
            s_gbase[t] = excl + dbase - dstart;
        }
        lds_barrier();
        // this wave's staging reads of its own counter row are done (program order)
#pragma unroll
        for (int i = lane; i < 256; i += 64) s_cnt[w][i] = 0;
        if (full) {
#pragma unroll
            for (int jj = 0; jj < TILE / TPB; ++jj) {
                const int i = t + jj * TPB;
                const uint32_t k = s_keys[i];
                __builtin_amdgcn_raw_buffer_store_b32(from_key_t<OUT_MODE>(k), rout,
                                                      (int)((s_gbase[(k >> shift) & 255u] + (uint32_t)i) * 4u), 0, 0);
            }
        } else {
            for (int jj = 0; jj < TILE / TPB; ++jj) {
                const int i = t + jj * TPB;
                const uint32_t k = s_keys[i];
                const uint32_t pos = s_gbase[(k >> shift) & 255u] + (uint32_t)i;
                if (pos < n32) __builtin_amdgcn_raw_buffer_store_b32(from_key_t<OUT_MODE>(k), rout, (int)(pos * 4u), 0, 0);
            }
        }
    };

    uint32_t a[kRPer], b[kRPer];
    load_tile(a, tile);
    if constexpr (STATIC) {
        for (int next = tile + (int)gridDim.x;; next += (int)gridDim.x) {
            if (next < ntiles) load_tile(b, next);
            do_tile(a, tile);
            if (next >= ntiles) break;
            tile = next;
#pragma unroll
            for (int e = 0; e < kRPer; ++e) a[e] = b[e];
        }
        return;
    }
    lds_barrier();  // every thread has read s_next
    if (t == 0) s_next = (int)atomicAdd(tile_ctr, 1u);
    lds_barrier();
    int next = s_next;
    for (;;) {
        // the id after next: its counter add is in flight under this tile's work
        int grabbed = 0;
        if (t == 0 && next < ntiles) grabbed = (int)atomicAdd(tile_ctr, 1u);
        if (next < ntiles) load_tile(b, next);
        do_tile(a, tile);  // ends after a barrier: every thread has read s_next
        if (next >= ntiles) break;
        tile = next;
#pragma unroll
        for (int e = 0; e < kRPer; ++e) a[e] = b[e];
        if (t == 0) s_next = grabbed;
        lds_barrier();
        next = s_next;
    }
}

// reduce-then-scan, step 1: the tile's digit counts (per-wave LDS atomics,
// order irrelevant), digit-major
// (cnt[d][tile]); consecutive tiles share an XCD so their L2 merges the
// 4-byte stores into whole lines
constexpr int kCThreads = 256;
// VEC (16-B aligned input, whole tile in range): counting ignores order, so
// each lane reads 16-B pieces (8 loads of 1 KiB per wave instead of 32 of
// 256 B); the partial last tile keeps the 4-B form.
// One key per lane into the wave's histogram row. The lanes holding the first
// active lane's digit add through that lane alone (one add of their count): a
// pass whose digits are skewed (one value for small-range ints, a few for
// floats' top byte) otherwise serialises up to 32 same-address lanes per add.
__device__ __forceinline__ void count_add(uint32_t *hw, uint32_t d) {
    const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
    const bool is = d == d0;
    const uint64_t m = __builtin_amdgcn_ballot_w64(is);
    const bool lead = (int)(threadIdx.x & 63) == __builtin_ctzll(m);  // the first active lane
    if (!is || lead) atomicAdd(&hw[d], is ? (uint32_t)__popcll(m) : 1u);
}

typedef uint32_t sort_u32x4 __attribute__((ext_vector_type(4)));  // the nontemporal builtins take clang vectors

// NT: non-temporal key loads (the count pass reads every key once; tuning
// A/B, MPX_SORT_COUNT_NT)
template <bool VEC, int TILE, bool NT = false>
__device__ __forceinline__ void count_tile_keys(const uint32_t *__restrict__ in, int64_t n, int shift, int mode,
                                                int tile, uint32_t *hw) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    constexpr int kCPer = TILE / kCThreads;              // 32 keys per thread (16 for 4096-key tiles)
    constexpr int kWaveKeys = TILE / (kCThreads / 64);  // 2048 contiguous keys per wave
    if constexpr (VEC) {
        const uint4 *src = reinterpret_cast<const uint4 *>(in + (int64_t)tile * TILE + w * kWaveKeys) + lane;
        uint4 q[kCPer / 4];
#pragma unroll
        for (int e = 0; e < kCPer / 4; ++e) {
            if constexpr (NT) {
                const sort_u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const sort_u32x4 *>(src + e * 64));
                q[e] = make_uint4(x[0], x[1], x[2], x[3]);
            } else {
                q[e] = src[e * 64];
            }
        }
#pragma unroll
        for (int e = 0; e < kCPer / 4; ++e) {
            count_add(hw, (to_key(q[e].x, mode) >> shift) & 255u);
            count_add(hw, (to_key(q[e].y, mode) >> shift) & 255u);
            count_add(hw, (to_key(q[e].z, mode) >> shift) & 255u);
            count_add(hw, (to_key(q[e].w, mode) >> shift) & 255u);
        }
    } else {
        const int64_t base = (int64_t)tile * TILE + w * kWaveKeys + lane;
        uint32_t key[kCPer];
#pragma unroll
        for (int e = 0; e < kCPer; ++e) {
            const int64_t i = base + e * 64;
            key[e] = i < n ? in[i] : 0u;
        }
#pragma unroll
        for (int e = 0; e < kCPer; ++e)
            if (base + e * 64 < n) count_add(hw, (to_key(key[e], mode) >> shift) & 255u);
    }
}

template <int TILE = kRTile, bool NT = false>
__global__ __launch_bounds__(kCThreads) void radix_count_kernel(const uint32_t *__restrict__ in, int64_t n, int shift,
                                                                int mode, uint32_t *__restrict__ cnt, int ntiles) {
    __shared__ uint32_t h[kCThreads / 64][256];
    const int t = threadIdx.x, w = t >> 6;
    for (int i = t; i < (kCThreads / 64) * 256; i += kCThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    // block-uniform: whole tile in range and the input 16-B aligned
    if (((int64_t)tile + 1) * TILE <= n && (reinterpret_cast<uintptr_t>(in) & 15) == 0)
        count_tile_keys<true, TILE, NT>(in, n, shift, mode, tile, h[w]);
    else
        count_tile_keys<false, TILE>(in, n, shift, mode, tile, h[w]);
    __syncthreads();
    uint32_t c = 0;
#pragma unroll
    for (int ww = 0; ww < kCThreads / 64; ++ww) c += h[ww][t];
    cnt[(size_t)t * ntiles + tile] = c;
}

// reduce-then-scan, step 2 (production): one 1024-thread block per digit
// turns its row of tile counts into exclusive offsets in place and records
// the digit total. 8192 counts per round (2^26 keys: one round); a thread owns
// 8 consecutive counts, read from LDS as two 16-byte pieces. The 256-thread
// form below took 15.3 us per pass at 2^26 in two dependent rounds.
constexpr int kScanThreads = 1024;
__device__ __forceinline__ uint32_t scan1024_excl(uint32_t v, uint32_t *s_wsum) {
    const int t = threadIdx.x, lane = t & 63;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_wsum[t >> 6] = x;
    __syncthreads();
    uint32_t add = 0;
    for (int w = 0; w < (t >> 6); ++w) add += s_wsum[w];
    __syncthreads();  // s_wsum may be reused by the caller
    return x - v + add;
}

__global__ __launch_bounds__(kScanThreads) void radix_scan1024_kernel(uint32_t *__restrict__ cnt, int ntiles,
                                                                      uint32_t *__restrict__ tot) {
    constexpr int kChunk = kScanThreads * 8;
    __shared__ uint4 v4[kChunk / 4];
    __shared__ uint32_t s_wsum[kScanThreads / 64];
    uint32_t *v = reinterpret_cast<uint32_t *>(v4);
    const int t = threadIdx.x;
    uint32_t *row = cnt + (size_t)blockIdx.x * ntiles;
    uint32_t carry = 0;
    for (int c0 = 0; c0 < ntiles; c0 += kChunk) {
        const int m = min(kChunk, ntiles - c0);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = t + k * kScanThreads;
            v[i] = i < m ? row[c0 + i] : 0u;
        }
        __syncthreads();
        const uint4 a = v4[2 * t], b = v4[2 * t + 1];
        const uint32_t own = a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
        uint32_t run = carry + scan1024_excl(own, s_wsum);
        uint4 ea, eb;
        ea.x = run, run += a.x, ea.y = run, run += a.y, ea.z = run, run += a.z, ea.w = run, run += a.w;
        eb.x = run, run += b.x, eb.y = run, run += b.y, eb.z = run, run += b.z, eb.w = run, run += b.w;
        v4[2 * t] = ea, v4[2 * t + 1] = eb;
        if (t == kScanThreads - 1) s_wsum[0] = run;  // carry for the next round
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = t + k * kScanThreads;
            if (i < m) row[c0 + i] = v[i];
        }
        carry = s_wsum[0];
        __syncthreads();
    }
    if (t == 0) tot[blockIdx.x] = carry;
}

// the round-2 scan (256 threads, 4096 counts per round): tuning variant 4
__global__ __launch_bounds__(256) void radix_scan_kernel(uint32_t *__restrict__ cnt, int ntiles,
                                                         uint32_t *__restrict__ tot) {
    constexpr int kChunk = 256 * 16;
    __shared__ uint32_t v[kChunk];
    __shared__ uint32_t s_wsum[4];
    const int t = threadIdx.x;
    uint32_t *row = cnt + (size_t)blockIdx.x * ntiles;
    uint32_t carry = 0;
    for (int c0 = 0; c0 < ntiles; c0 += kChunk) {
        const int m = min(kChunk, ntiles - c0);
        for (int i = t; i < kChunk; i += 256) v[i] = i < m ? row[c0 + i] : 0u;
        __syncthreads();
        uint32_t own = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) own += v[t * 16 + k];
        uint32_t run = carry + scan256_excl(own, s_wsum);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t x = v[t * 16 + k];
            v[t * 16 + k] = run;
            run += x;
        }
        if (t == 255) s_wsum[0] = run;  // carry for the next chunk
        __syncthreads();
        for (int i = t; i < m; i += 256) row[c0 + i] = v[i];
        carry = s_wsum[0];
        __syncthreads();
    }
    if (t == 0) tot[blockIdx.x] = carry;
}

struct RadixWs {
    uint32_t *tmp, *hist, *ctr, *err, *status;
    int64_t tiles;
    size_t zero_bytes;
};

int64_t radix_tiles(int64_t n) { return (n + kRTile - 1) / kRTile; }
constexpr int kRTileSmall = kRTile / 2;  // the 256-thread lean scatter's tile (variant 8)
constexpr int kRTileBig = kRTile * 2;    // the 1024-thread lean scatter's tile (variant 22)

size_t radix_ws_bytes(int64_t n) {  // status sized for the smaller tile (twice the tiles)
    const size_t keys = ((size_t)n * 4 + 255) / 256 * 256;
    return keys + (4 * 256 + 64) * 4 + (size_t)4 * ((n + kRTileSmall - 1) / kRTileSmall) * 256 * 4;
}

RadixWs radix_layout(void *ws, int64_t n) {
    RadixWs r;
    char *p = static_cast<char *>(ws);
    const size_t keys = ((size_t)n * 4 + 255) / 256 * 256;
    r.tmp = reinterpret_cast<uint32_t *>(p);
    r.hist = reinterpret_cast<uint32_t *>(p + keys);
    r.ctr = r.hist + 4 * 256;
    r.err = r.ctr + 4;
    r.status = r.ctr + 64;
    r.tiles = radix_tiles(n);
    r.zero_bytes = (4 * 256 + 64) * 4 + (size_t)4 * r.tiles * 256 * 4;
    return r;
}

// Radix variants: 1 = onesweep (decoupled look-back), 2 = reduce-then-scan
// (one tile per block), 4 = reduce-then-scan with the round-2 persistent
// scatter (radix_scatter_kernel, 256-thread scan; same-process A/B), 7 = the
// lean persistent scatter (radix_scatter_lean_kernel, 8192-key tiles), 8 = 7
// on 4096-key tiles (256-thread blocks, 4 per CU), 9 = 7 ranked by returning
// LDS adds (RANK 1), 10 = 9 on 4096-key tiles, 11 = 9 with 3 blocks per CU,
// 12 / 13 = 9 / 10 with two tiles of keys in flight (PF 2), 14 = the lean
// onesweep (one histogram read, then decoupled look-back per digit pass):
// correct, and 1.2 ms at 2^26 against 0.70 (profiles/lab5_sort.md); 15 / 16 its
// one-block-per-CU and static-order experiments; 17 = 12 with one counter row
// per half-wave (RANK 2: skewed digits contend half as much); 18 / 19 = 12 / 13
// with up to four hot digits ranked by ballot (RANK 3), 20 / 21 the same with
// two (RANK 4); 22 = 20 on 16384-key tiles (1024 threads, one block per CU).
// Retired after round-3
// measurements (profiles/lab5_sort.md): 3 (ballot peer masks), 5 (reverse
// tile walk), 6 (lean with six barriers per tile).
// Look-back resolves one predecessor tile per memory round trip and the
// cross-XCD round trip on MI355X is long (agent-scope loads miss the per-XCD
// L2), so once many tiles are in flight the chain, not HBM, bounds onesweep;
// reduce-then-scan re-reads each tile once more but never waits.
constexpr int64_t kOnesweepMaxN = (int64_t)1 << 18;  // onesweep's AUTO range before round 5; the probe's lower bound
constexpr int64_t kTile4kMaxN = (int64_t)1 << 23;    // 4096-key tiles up to here (2^24: 0.187 ms both ways)
constexpr int64_t kTile16kMinN = (int64_t)1 << 26;   // 16384-key tiles from here (variant 22)

// pass p of the lean scatter: the first pass reads raw int32 / float32, the
// last writes them back, the middle passes move keys
template <int TPB = kRThreads, int RANK = 0, int WPE = 4, int PF = 1>
void launch_lean(int p, int mode, int blocks, hipStream_t s, const uint32_t *src, uint32_t *dst, int64_t n,
                 const uint32_t *tot, const uint32_t *offs, int ntiles) {
    const dim3 g((unsigned)blocks), b(TPB);
    const int sh = 8 * p;
    const bool f = mode == kRawF32;
#define MPX_LEAN(I, O) \
    hipLaunchKernelGGL((radix_scatter_lean_kernel<I, O, TPB, RANK, 0, WPE, PF>), g, b, 0, s, src, dst, n, sh, tot, offs, ntiles)
    if (p == 0 && f)
        MPX_LEAN(kRawF32, kRawKeys);
    else if (p == 0)
        MPX_LEAN(kRawI32, kRawKeys);
    else if (p == 3 && f)
        MPX_LEAN(kRawKeys, kRawF32);
    else if (p == 3)
        MPX_LEAN(kRawKeys, kRawI32);
    else
        MPX_LEAN(kRawKeys, kRawKeys);
#undef MPX_LEAN
}

// Lane order of same-address returning LDS adds. The RANK >= 1
// scatters (variants 9-21, AUTO above 2^18 keys) are stable only because one
// ds_add_rtn_u32 applies its same-address lanes in ascending lane order —
// observed on gfx950, not promised by the ISA. This probe checks it once per
// device before the first such sort: four waves, three address patterns
// (every lane on one counter; lane % 3; a scattered 5-way split), each lane's
// returned count must equal the number of lower lanes on its counter. On a
// failure AUTO falls back to the peer-mask ranking (variants 7 / 8, which
// rank with explicit lane masks) and the explicit RANK variants refuse.
__global__ __launch_bounds__(256) void lds_rtn_order_probe_kernel(uint32_t *bad) {
    __shared__ uint32_t cnt[4][3][8];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = lane; i < 24; i += 64) (&cnt[w][0][0])[i] = 0;
    __syncthreads();
    uint32_t err = 0;
    const int addr[3] = {0, lane % 3, (lane * 7) % 5};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t got = atomicAdd(&cnt[w][k][addr[k]], 1u);
        uint32_t want = 0;
        for (int j = 0; j < lane; ++j) {
            const int aj = k == 0 ? 0 : k == 1 ? j % 3 : (j * 7) % 5;
            want += aj == addr[k];
        }
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
    if (hipMalloc(&d, sizeof(uint32_t)) == hipSuccess) {
        if (hipMemsetAsync(d, 0, sizeof(uint32_t), s) == hipSuccess) {
            hipLaunchKernelGGL(lds_rtn_order_probe_kernel, dim3(1), dim3(256), 0, s, d);
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
    // 4096-key tiles win up to 2^24 keys (2^20: 0.070 vs 0.075 ms, 2^24: 0.221
    // vs 0.229) and lose at 2^26 (0.987 vs 0.828; not yet explained — a
    // candidate: with 16 tiles per block the 64-B digit runs of neighbouring
    // tiles stop meeting in L2; profiles/lab5_sort.md)
    // AUTO (round 5, profiles/lab5_sort.md): the returning-add ranking with
    // two tiles of keys in flight and the two hottest digits of a skewed pass
    // ranked by compare masks (RANK 4), on 4096-key tiles up to 2^23 keys
    // (21), on 8192-key tiles below 2^26 (20), on 16384-key tiles from 2^26
    // (22: longer digit runs, fewer partial output lines; 2^26 int32 0.689-0.697
    // vs 0.706 ms, but 10 % slower at 2^24 with one block per CU); uniform
    // passes run the round-4 code (12 / 13)
    // (21 also below 2^18 since round 5: 0.059-0.062 vs onesweep's 0.068-0.082 ms
    // from 2^14 to 2^18 keys, profiles/raw/r5/l5small/)
    if (variant == 0) variant = n <= kTile4kMaxN ? 21 : n < kTile16kMinN ? 20 : 22;
    // the returning-add ranking needs ascending lane order (probe above)
    const bool rtn_rank = (variant >= 9 && variant <= 22);
    if (rtn_rank && lds_rtn_order_ok(s) != 1) {
        if (!auto_variant) return MPX_ERR_UNSUPPORTED;
        variant = n <= kTile4kMaxN ? 8 : 7;
    }
    // variant 8: 4096-key tiles (256-thread lean scatter, 4 blocks per CU)
    const bool small_tiles = variant == 8 || variant == 10 || variant == 13 || variant == 19 || variant == 21;
    const bool big_tiles = variant == 22;  // 16384-key tiles (1024-thread lean scatter, 1 block per CU)
    static const bool count_nt = [] {  // MPX_SORT_COUNT_NT=1: non-temporal count-pass loads (A/B, read once)
        const char *e = std::getenv("MPX_SORT_COUNT_NT");
        return e && e[0] == '1';
    }();
    const int ntiles = small_tiles ? (int)((n + kRTileSmall - 1) / kRTileSmall)
                       : big_tiles ? (int)((n + kRTileBig - 1) / kRTileBig)
                                   : (int)r.tiles;
    const bool onesweep = variant >= 14 && variant <= 16;
    if (variant == 1 || onesweep) {
        MPX_RETURN_IF_HIP_ERROR(hipMemsetAsync(r.hist, 0, r.zero_bytes, s));
        if (variant != 1)
            hipLaunchKernelGGL(radix_hist4_kernel,
                               dim3(std::max<int64_t>(1, std::min<int64_t>((n + 1023) / 1024, kNumCUs * 2))), dim3(256),
                               0, s, x, n, mode, r.hist);
        else
            hipLaunchKernelGGL(radix_hist_kernel,
                               dim3(std::max<int64_t>(1, std::min<int64_t>((n + 4095) / 4096, kNumCUs * 8))), dim3(256),
                               0, s, x, n, mode, r.hist);
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    } else {
        // the give-up flag sort_ws_status reads: reduce-then-scan never waits,
        // but the caller's workspace may hold anything (recycled allocations)
        MPX_RETURN_IF_HIP_ERROR(hipMemsetAsync(r.err, 0, sizeof(uint32_t), s));
    }
    for (int p = 0; p < 4; ++p) {
        const uint32_t *src = (p & 1) ? r.tmp : x;
        uint32_t *dst = (p & 1) ? x : r.tmp;
        const int in_mode = p == 0 ? mode : (int)kRawKeys, out_mode = p == 3 ? mode : (int)kRawKeys;
        if (onesweep) {
            // 15: one block per CU — half the tiles in flight, so half the
            // predecessors a look-back walks before it meets an inclusive prefix;
            // 16: static tile order (no counter), all blocks co-resident
            const dim3 g((unsigned)std::min(kNumCUs * (variant == 15 ? 1 : 2), ntiles)), b(kRThreads);
            uint32_t *st = r.status + (size_t)p * ntiles * 256;
            const bool f = mode == kRawF32;
#define MPX_OS1(I, O, W, ST) \
    hipLaunchKernelGGL((radix_onesweep_lean_kernel<I, O, W, ST>), g, b, 0, s, src, dst, n, 8 * p, r.hist + 256 * p, st, r.ctr + p, r.err, ntiles)
#define MPX_OS(I, O)                   \
    do {                               \
        if (variant == 16)             \
            MPX_OS1(I, O, 8, true);    \
        else                           \
            MPX_OS1(I, O, 8, false);   \
    } while (0)
            if (p == 0 && f)
                MPX_OS(kRawF32, kRawKeys);
            else if (p == 0)
                MPX_OS(kRawI32, kRawKeys);
            else if (p == 3 && f)
                MPX_OS(kRawKeys, kRawF32);
            else if (p == 3)
                MPX_OS(kRawKeys, kRawI32);
            else
                MPX_OS(kRawKeys, kRawKeys);
#undef MPX_OS
#undef MPX_OS1
        } else if (variant == 1) {
            hipLaunchKernelGGL(radix_pass_kernel<true>, dim3((unsigned)ntiles), dim3(kRThreads), 0, s, src, dst, n,
                               8 * p, in_mode, out_mode, r.hist + 256 * p, r.status + (size_t)p * ntiles * 256,
                               r.ctr + p, r.err, ntiles);
        } else {
            // offsets in status[0 .. 256 * ntiles), digit totals in hist[0 .. 256)
            if (small_tiles)
                hipLaunchKernelGGL(radix_count_kernel<kRTileSmall>, dim3((unsigned)ntiles), dim3(kCThreads), 0, s, src,
                                   n, 8 * p, in_mode, r.status, ntiles);
            else if (big_tiles && count_nt)
                hipLaunchKernelGGL((radix_count_kernel<kRTileBig, true>), dim3((unsigned)ntiles), dim3(kCThreads), 0, s,
                                   src, n, 8 * p, in_mode, r.status, ntiles);
            else if (big_tiles)
                hipLaunchKernelGGL(radix_count_kernel<kRTileBig>, dim3((unsigned)ntiles), dim3(kCThreads), 0, s, src,
                                   n, 8 * p, in_mode, r.status, ntiles);
            else
                hipLaunchKernelGGL(radix_count_kernel<kRTile>, dim3((unsigned)ntiles), dim3(kCThreads), 0, s, src, n,
                                   8 * p, in_mode, r.status, ntiles);
            MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
            if (variant == 4)
                hipLaunchKernelGGL(radix_scan_kernel, dim3(256), dim3(256), 0, s, r.status, ntiles, r.hist);
            else
                hipLaunchKernelGGL(radix_scan1024_kernel, dim3(256), dim3(kScanThreads), 0, s, r.status, ntiles,
                                   r.hist);
            MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
            if (variant >= 7) {
                const int rounded = (ntiles + kNumXCDs - 1) / kNumXCDs * kNumXCDs;
                if (variant == 7)
                    launch_lean(p, mode, std::min(kNumCUs * 2, rounded), s, src, dst, n, r.hist, r.status, ntiles);
                else if (variant == 9)
                    launch_lean<kRThreads, 1>(p, mode, std::min(kNumCUs * 2, rounded), s, src, dst, n, r.hist, r.status,
                                              ntiles);
                else if (variant == 10)
                    launch_lean<kRThreads / 2, 1>(p, mode, std::min(kNumCUs * 4, rounded), s, src, dst, n, r.hist,
                                                  r.status, ntiles);
                else if (variant == 11)  // 3 blocks (24 waves) per CU: the returning-add ranking frees the table's LDS
                    launch_lean<kRThreads, 1, 6>(p, mode, std::min(kNumCUs * 3, rounded), s, src, dst, n, r.hist,
                                                 r.status, ntiles);
                else if (variant == 12)  // 9 with two tiles of keys in flight
                    launch_lean<kRThreads, 1, 4, 2>(p, mode, std::min(kNumCUs * 2, rounded), s, src, dst, n, r.hist,
                                                    r.status, ntiles);
                else if (variant == 17)  // 12 with a counter row per half-wave (skewed digits contend half as much)
                    launch_lean<kRThreads, 2, 4, 2>(p, mode, std::min(kNumCUs * 2, rounded), s, src, dst, n, r.hist,
                                                    r.status, ntiles);
                else if (variant == 13)  // 10 with two tiles of keys in flight
                    launch_lean<kRThreads / 2, 1, 4, 2>(p, mode, std::min(kNumCUs * 4, rounded), s, src, dst, n,
                                                        r.hist, r.status, ntiles);
                else if (variant == 18)  // 12 with hot digits ranked by ballot (RANK 3)
                    launch_lean<kRThreads, 3, 4, 2>(p, mode, std::min(kNumCUs * 2, rounded), s, src, dst, n, r.hist,
                                                    r.status, ntiles);
                else if (variant == 19)  // 13 with hot digits ranked by ballot
                    launch_lean<kRThreads / 2, 3, 4, 2>(p, mode, std::min(kNumCUs * 4, rounded), s, src, dst, n,
                                                        r.hist, r.status, ntiles);
                else if (variant == 20)  // 18 with two hot-digit slots (RANK 4)
                    launch_lean<kRThreads, 4, 4, 2>(p, mode, std::min(kNumCUs * 2, rounded), s, src, dst, n, r.hist,
                                                    r.status, ntiles);
                else if (variant == 21)  // 19 with two hot-digit slots
                    launch_lean<kRThreads / 2, 4, 4, 2>(p, mode, std::min(kNumCUs * 4, rounded), s, src, dst, n,
                                                        r.hist, r.status, ntiles);
                else if (variant == 22)  // 20 on 16384-key tiles: longer digit runs, fewer partial output lines
                    launch_lean<kRThreads * 2, 4, 4, 2>(p, mode, std::min(kNumCUs, rounded), s, src, dst, n, r.hist,
                                                        r.status, ntiles);
                else
                    launch_lean<kRThreads / 2>(p, mode, std::min(kNumCUs * 4, rounded), s, src, dst, n, r.hist,
                                               r.status, ntiles);
            } else if (variant == 4) {
                const int blocks = std::min(kNumCUs * kPersistBlocksPerCU, (ntiles + kNumXCDs - 1) / kNumXCDs * kNumXCDs);
                hipLaunchKernelGGL(radix_scatter_kernel, dim3((unsigned)blocks), dim3(kRThreads), 0, s, src, dst, n,
                                   8 * p, in_mode, out_mode, r.hist, r.status, ntiles);
            } else {
                hipLaunchKernelGGL(radix_pass_kernel<false>, dim3((unsigned)ntiles), dim3(kRThreads), 0, s, src, dst,
                                   n, 8 * p, in_mode, out_mode, r.hist, r.status, r.ctr, r.err, ntiles);
            }
        }
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

int sort_impl(void *data, int64_t n, int dtype, void *ws, int64_t ws_bytes, void *stream, int variant = 0) {
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
    if (use_radix(n)) return radix_sort32(x, n, is_float ? kRawF32 : kRawI32, ws, variant, s);
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
    int rc = sort_impl(data, n, dtype, ws, bytes, stream);
    if (ws) {
        const hipError_t e = hipStreamSynchronize(as_stream(stream));
        if (rc == MPX_OK && e == hipSuccess) rc = sort_ws_status(ws, n, dtype);
        (void)hipFree(ws);
        MPX_RETURN_IF_HIP_ERROR(e);
    }
    return rc;
}

// Scatter probe (tools/experiments/sort_probe.py): count + scan + one lean
// scatter per digit on the UNCHANGED input (every pass sees the same uniform
// keys, src -> workspace), with the KNOCK bits of radix_scatter_lean_kernel.
// The output is not sorted; only the counters and the kernel times matter.
template <int KNOCK>
int scatter_probe_k(const uint32_t *x, int64_t n, void *ws, hipStream_t s) {
    const RadixWs r = radix_layout(ws, n);
    const int ntiles = (int)r.tiles;
    const int blocks = std::min(kNumCUs * 2, (ntiles + kNumXCDs - 1) / kNumXCDs * kNumXCDs);
    for (int p = 0; p < 4; ++p) {
        hipLaunchKernelGGL(radix_count_kernel<kRTile>, dim3((unsigned)ntiles), dim3(kCThreads), 0, s, x, n, 8 * p,
                           (int)kRawKeys, r.status, ntiles);
        hipLaunchKernelGGL(radix_scan1024_kernel, dim3(256), dim3(kScanThreads), 0, s, r.status, ntiles, r.hist);
        hipLaunchKernelGGL((radix_scatter_lean_kernel<kRawKeys, kRawKeys, kRThreads, 0, KNOCK>), dim3((unsigned)blocks),
                           dim3(kRThreads), 0, s, x, r.tmp, n, 8 * p, r.hist, r.status, ntiles);
        MPX_RETURN_IF_HIP_ERROR(hipGetLastError());
    }
    return MPX_OK;
}

int scatter_probe(const void *x, int64_t n, void *ws, int64_t ws_bytes, int knock, void *stream) {
    MPX_CHECK_ARG(x && ws && n > kOnesweepMaxN && n < kRadixMaxN, "probe: 2^18 < n < 2^30 keys and a workspace");
    MPX_CHECK_ARG(ws_bytes >= (int64_t)radix_ws_bytes(n), "probe: workspace smaller than mpx_sort_workspace_bytes");
    const uint32_t *k = static_cast<const uint32_t *>(x);
    hipStream_t s = as_stream(stream);
    switch (knock) {
        case 0: return scatter_probe_k<0>(k, n, ws, s);
        case 1: return scatter_probe_k<1>(k, n, ws, s);
        case 6: return scatter_probe_k<6>(k, n, ws, s);
        case 12: return scatter_probe_k<12>(k, n, ws, s);
        case 14: return scatter_probe_k<14>(k, n, ws, s);
        case 16: return scatter_probe_k<16>(k, n, ws, s);
        case 31: return scatter_probe_k<31>(k, n, ws, s);
        default: set_error("probe knock %d: 0, 1, 6, 12, 14, 16 or 31", knock); return MPX_ERR_ARG;
    }
}

MPX_MODULE_ANCHOR(sort)

}  // namespace mpx

extern "C" int mpx_sort(void *data, int64_t n, int dtype, void *stream) { return mpx::sort_alloc(data, n, dtype, stream); }

extern "C" int64_t mpx_sort_workspace_bytes(int64_t n, int dtype) { return mpx::sort_workspace_bytes(n, dtype); }

extern "C" int mpx_sort_ws_status(const void *workspace, int64_t n, int dtype) {
    return mpx::sort_ws_status(workspace, n, dtype);
}

extern "C" int mpx_sort_ws(void *data, int64_t n, int dtype, void *workspace, int64_t workspace_bytes, void *stream) {
    return mpx::sort_impl(data, n, dtype, workspace, workspace_bytes, stream);
}

// Tuning entry (tools/experiments/lab5_bench.py): radix variant 0 = auto, 1 = onesweep
// (decoupled look-back), 2 = reduce-then-scan, 4 / 7 / 8 = reduce-then-scan
// with a persistent scatter (see radix_sort32).
extern "C" int mpx_sort_variant(void *data, int64_t n, int dtype, void *workspace, int64_t workspace_bytes, int variant,
                                void *stream) {
    if (variant < 0 || variant > 22 || variant == 3 || variant == 5 || variant == 6) {
        mpx::set_error("sort variant %d: 0 (auto), 1, 2, 4, 7 .. 22", variant);
        return MPX_ERR_ARG;
    }
    return mpx::sort_impl(data, n, dtype, workspace, workspace_bytes, stream, variant);
}

extern "C" int mpx_sort_scatter_probe(const void *data, int64_t n, void *workspace, int64_t workspace_bytes, int knock,
                                      void *stream) {
    return mpx::scatter_probe(data, n, workspace, workspace_bytes, knock, stream);
}

extern "C" int mpx_sort_lane_order_ok(void *stream) { return mpx::lds_rtn_order_ok(mpx::as_stream(stream)); }
