// Radix-sort kernels shared by libmpx (native/src/kernels/sort.hip: the
// AUTO variants 20 / 21 / 22 and their lane-order fallback 7 / 8) and the
// tuning library (native/tune/sort_variants.hip: every other variant and the
// scatter probe, VERDICT r5 Next #3). Each translation unit that includes it
// gets its own copies (anonymous namespace) and instantiates only the
// template configurations it launches: libmpx carries no experiment kernels.
// The variant table is in sort_variants.hip.
#pragma once

#include <algorithm>

#include "internal.hpp"

namespace mpx {

// the four-pass radix body behind sort_impl (production: radix_sort32 in
// sort.hip; the tuning library passes its own for the experimental variants)
using SortRadixFn = int (*)(uint32_t *x, int64_t n, int mode, void *ws, int variant, hipStream_t s);
int sort_impl(void *data, int64_t n, int dtype, void *ws, int64_t ws_bytes, void *stream, int variant,
              SortRadixFn radix);

namespace {

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

}  // namespace
}  // namespace mpx
