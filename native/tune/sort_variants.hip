// lab5 radix-sort variants for A/B measurement (tools/experiments/lab5_bench.py,
// sort_probe.py; tests/test_lab5_sort.py): the tuning library, not libmpx
// (VERDICT r5 Next #3). Production keeps AUTO (20 / 21 / 22) and the
// lane-order fallback (7 / 8) in native/src/kernels/sort.hip; the kernels both
// use are in sort_radix.hpp. mpx_sort_variant runs any variant below through
// libmpx's sort_impl (the same key transforms, small-n and uint8 paths).
//
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
#include <algorithm>

#include "../src/kernels/sort_radix.hpp"

extern "C" int mpx_sort_lane_order_ok(void *stream);

namespace mpx {
namespace {

int lane_order_ok(hipStream_t s) { return ::mpx_sort_lane_order_ok(reinterpret_cast<void *>(s)); }

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

int tune_radix_sort32(uint32_t *x, int64_t n, int mode, void *ws, int variant, hipStream_t s) {
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
    if (rtn_rank && lane_order_ok(s) != 1) {
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

}  // namespace
}  // namespace mpx

// Tuning entry: radix variant 0 = auto, 1 = onesweep (decoupled look-back),
// 2 = reduce-then-scan, 4 / 7 .. 22 = reduce-then-scan with a persistent
// scatter (the table above). AUTO's own variants run libmpx's radix body.
extern "C" int mpx_sort_variant(void *data, int64_t n, int dtype, void *workspace, int64_t workspace_bytes, int variant,
                                void *stream) {
    if (variant < 0 || variant > 22 || variant == 3 || variant == 5 || variant == 6) {
        mpx::set_error("sort variant %d: 0 (auto), 1, 2, 4, 7 .. 22", variant);
        return MPX_ERR_ARG;
    }
    const bool production = variant == 0 || variant == 7 || variant == 8 || variant >= 20;
    return mpx::sort_impl(data, n, dtype, workspace, workspace_bytes, stream, variant,
                          production ? nullptr : &mpx::tune_radix_sort32);
}

extern "C" int mpx_sort_scatter_probe(const void *data, int64_t n, void *workspace, int64_t workspace_bytes, int knock,
                                      void *stream) {
    return mpx::scatter_probe(data, n, workspace, workspace_bytes, knock, stream);
}
