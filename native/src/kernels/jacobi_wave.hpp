// Jacobi sweep kernels shared by jacobi.hip (production launches) and
// native/tune/jacobi_variants.hip (tuning entry point, libmpx_tune.so). The
// design notes are at the top of jacobi.hip.
#pragma once
#include "internal.hpp"
#include "peer_sync.hpp"

#include <type_traits>

namespace mpx {
namespace {

template <typename T> struct JVec;
template <> struct JVec<double> {
    using type = double2;
    using bits = unsigned long long;
    static constexpr int n = 2;
};
template <> struct JVec<float> {
    using type = float4;
    using bits = unsigned int;
    static constexpr int n = 4;
};

constexpr int kRows = 16;  // rows swept per lane (vertical register reuse)

// Fold one wave's residual into the global max. Read first, atomic only when
// this wave raises the max: with hundreds of thousands of short waves per
// sweep, unconditional device-scope atomics on one word serialise (16384^2
// fp64 with R = 4: 6.2 ms instead of 0.8 ms); after the first few waves the
// max has settled and almost every wave skips the atomic.
template <typename B>
__device__ __forceinline__ void residual_max(B *p, B v) {
    const B cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v > cur) atomicMax(p, v);
}

template <typename T>
__device__ __forceinline__ T lane_of(const typename JVec<T>::type &v, int i) {
    if constexpr (JVec<T>::n == 2) return i == 0 ? v.x : v.y;
    else return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void jacobi_kernel(const T *__restrict__ u, T *__restrict__ un, int cols,
                                                     int pitch, int r0, int r1, T *__restrict__ resid) {
    using V = typename JVec<T>::type;
    constexpr int NV = VEC ? JVec<T>::n : 1;
    const int j0 = NV * (blockIdx.x * blockDim.x + threadIdx.x);
    const int i0 = r0 + blockIdx.y * kRows;
    const int i1 = min(i0 + kRows, r1);
    T rmax = (T)0;
    if (j0 < cols && i0 < i1) {
        T up[NV], cen[NV], dn[NV];
        auto load_row = [&](int i, T (&dst)[NV]) {
            const T *row = u + (int64_t)i * pitch;
            if constexpr (VEC) {
                if (j0 + NV <= cols) {
                    const V q = *reinterpret_cast<const V *>(row + j0);
#pragma unroll
                    for (int k = 0; k < NV; ++k) dst[k] = lane_of<T>(q, k);
                    return;
                }
            }
#pragma unroll
            for (int k = 0; k < NV; ++k) dst[k] = (j0 + k < cols) ? row[j0 + k] : (T)0;
        };
        load_row(i0 - 1, up);
        load_row(i0, cen);
        for (int i = i0; i < i1; ++i) {
            load_row(i + 1, dn);
            const T *crow = u + (int64_t)i * pitch;
            const T left = j0 > 0 ? crow[j0 - 1] : (T)0;
            const T right = (j0 + NV < cols) ? crow[j0 + NV] : (T)0;
            T res[NV];
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                const int j = j0 + k;
                const T l = k == 0 ? left : cen[k - 1];
                const T r = k == NV - 1 ? right : cen[k + 1];
                const T s = ((up[k] + dn[k]) + (l + r)) * (T)0.25;
                const bool interior = j > 0 && j < cols - 1;
                res[k] = interior ? s : cen[k];
                if (interior && j < cols) {
                    const T d = s > cen[k] ? s - cen[k] : cen[k] - s;
                    rmax = d > rmax ? d : rmax;
                }
            }
            T *orow = un + (int64_t)i * pitch;
            bool stored = false;
            if constexpr (VEC) {
                if (j0 + NV <= cols) {
                    if constexpr (JVec<T>::n == 2)
                        *reinterpret_cast<double2 *>(orow + j0) = make_double2(res[0], res[1]);
                    else
                        *reinterpret_cast<float4 *>(orow + j0) = make_float4(res[0], res[1], res[2], res[3]);
                    stored = true;
                }
            }
            if (!stored) {
#pragma unroll
                for (int k = 0; k < NV; ++k)
                    if (j0 + k < cols) orow[j0 + k] = res[k];
            }
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                up[k] = cen[k];
                cen[k] = dn[k];
            }
        }
    }
    if (resid) {
        using B = typename JVec<T>::bits;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            const T o = __shfl_xor(rmax, m);
            rmax = o > rmax ? o : rmax;
        }
        if ((threadIdx.x & 63) == 0 && rmax > (T)0) residual_max(reinterpret_cast<B *>(resid), __builtin_bit_cast(B, rmax));
    }
}

// ---------------------------------------------------------------------------
// wave-strip kernel (16-B vectors, cols % NV == 0, pitch % NV == 0)
// ---------------------------------------------------------------------------
constexpr int kStripVec = 62;             // output vectors per wave
constexpr int kJacobiRows = 8;            // rows per wave (row block) of the production sweeps
constexpr uint32_t kDrop = 0x7ffffff0u;   // buffer offset past any range: store dropped

template <typename T> struct JWide;
template <> struct JWide<double> { typedef double type __attribute__((ext_vector_type(2))); };
template <> struct JWide<float> { typedef float type __attribute__((ext_vector_type(4))); };

template <typename T>
__device__ __forceinline__ T dpp_shift(T v, int ctrl) {
    if constexpr (sizeof(T) == 8) {
        const uint2 b = __builtin_bit_cast(uint2, v);
        uint2 r;
        if (ctrl == 0x138) {
            r.x = __builtin_amdgcn_mov_dpp((int)b.x, 0x138, 0xf, 0xf, true);
            r.y = __builtin_amdgcn_mov_dpp((int)b.y, 0x138, 0xf, 0xf, true);
        } else {
            r.x = __builtin_amdgcn_mov_dpp((int)b.x, 0x130, 0xf, 0xf, true);
            r.y = __builtin_amdgcn_mov_dpp((int)b.y, 0x130, 0xf, 0xf, true);
        }
        return __builtin_bit_cast(T, r);
    } else {
        const int b = __builtin_bit_cast(int, v);
        return __builtin_bit_cast(T, ctrl == 0x138 ? __builtin_amdgcn_mov_dpp(b, 0x138, 0xf, 0xf, true)
                                                   : __builtin_amdgcn_mov_dpp(b, 0x130, 0xf, 0xf, true));
    }
}

// ---------------------------------------------------------------------------
// one-sided, device-signalled halos (PEER): the neighbours' slab rows are read
// straight from their IPC-mapped buffers over xGMI, and per-iteration order
// comes from completed-iteration counters in device memory — no host round
// trip, no exchange kernel, no RCCL: one launch per iteration, as on one GPU.
//
// Only the slab-edge waves (row block 0: reads halo row 0, writes row 1; the
// last row block: writes row n, reads halo row n+1) take part. At iteration t
// an edge wave waits until the neighbour's counter is >= t — the neighbour has
// finished iteration t-1, so (a) its edge row of u^(t) is written and (b) it
// is done reading this rank's edge row of u^(t-1), the buffer this sweep
// overwrites. After its stores, an edge wave waits for their acknowledgement
// and bumps this rank's edge-wave counter; the last one publishes counter
// value t+1 with a system-scope RELEASE store (peer_sync.hpp: one L2
// write-back per sweep, by that one wave). No per-wave cache maintenance (an
// L2 write-back or invalidate per edge wave cost ~40 us per sweep): the rows
// a neighbour reads are stored at system scope (write-through) and
// acknowledged before the count goes up, and halo rows are loaded at system
// scope (never a stale cached line), so the consumer needs no acquire fence
// after its wait. Interior waves never wait. Edge waves are dispatched first so the
// counter is published early in the sweep. Waits are bounded (pr.spin_limit):
// a wave that gives up sets sync[kSyncErr] and the host raises.
// ---------------------------------------------------------------------------
constexpr int kSyncIter = 0, kSyncCtr = 32, kSyncErr = 64;  // uint32 slots, 128 B apart
constexpr int kCpolSystem = peer::kCpolSystem;               // gfx950 cache policy SC0 | SC1: system scope

// Max over the wave of non-negative values through DPP (row_shr 1/2/4/8 within
// each 16-lane row, then row_bcast 15/31 across rows; lanes with no source
// read +0, the identity here), read from lane 63. VALU only, in place of a
// 6 (fp32) / 12 (fp64) step __shfl_xor tree through the LDS crossbar.
template <int CTRL, int RMASK, typename T>
__device__ __forceinline__ T dpp_max_step(T v) {
    T o;
    if constexpr (sizeof(T) == 8) {
        const uint2 b = __builtin_bit_cast(uint2, v);
        uint2 r;
        r.x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b.x, CTRL, RMASK, 0xf, true);
        r.y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b.y, CTRL, RMASK, 0xf, true);
        o = __builtin_bit_cast(T, r);
    } else {
        o = __builtin_bit_cast(T, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, RMASK, 0xf, true));
    }
    return o > v ? o : v;
}

template <typename T>
__device__ __forceinline__ T wave_max_dpp(T v) {
    v = dpp_max_step<0x111, 0xf>(v);  // row_shr:1
    v = dpp_max_step<0x112, 0xf>(v);  // row_shr:2
    v = dpp_max_step<0x114, 0xf>(v);  // row_shr:4
    v = dpp_max_step<0x118, 0xf>(v);  // row_shr:8 -> lane 15 of each row holds its row's max
    v = dpp_max_step<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
    v = dpp_max_step<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3 -> lane 63 holds the max
    if constexpr (sizeof(T) == 8) {
        const uint2 b = __builtin_bit_cast(uint2, v);
        return __builtin_bit_cast(T, make_uint2((uint32_t)__builtin_amdgcn_readlane((int)b.x, 63),
                                                (uint32_t)__builtin_amdgcn_readlane((int)b.y, 63)));
    } else {
        return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
    }
}

// LNT: 0 plain loads, 1 every row non-temporal (tuning), 2 only the rows no
// neighbouring row block reads (i0 + 1 .. i1 - 2), the conv band kernel's
// round-3 default for separable windows
template <typename T, int AUX = 0, int LNT = 0, bool TAIL_EXIT = true, bool PEER = false, bool ALT = false,
          int WPB = 4>
__global__ __launch_bounds__(64 * WPB) void jacobi_wave_kernel(const T *__restrict__ u, T *__restrict__ un, int cols,
                                                          int pitch, int r0, int r1, int strips, int rows_per_wave,
                                                          int nwaves, T *__restrict__ resid, mpx_jacobi_peer pr) {
    using V = typename JWide<T>::type;
    constexpr int NV = JVec<T>::n;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    T rmax = (T)0;
    if (wave < nwaves) {
        const int strip = wave % strips;  // consecutive waves: adjacent strips of the same rows
        int rb = wave / strips;
        const int nrb = nwaves / strips;
        if (PEER && nrb > 1) rb = rb == 0 ? 0 : rb == 1 ? nrb - 1 : rb - 1;  // both edge blocks first
        const int nvec = cols / NV;
        const int cv = strip * kStripVec - 1 + lane;  // this lane's column vector
        const bool out_lane = lane >= 1 && lane <= kStripVec && cv < nvec;
        const int cvc = min(max(cv, 0), nvec - 1);
        const int i0 = r0 + rb * rows_per_wave;
        const int i1 = min(i0 + rows_per_wave, r1);
        const T *base = u + (int64_t)cvc * NV;
        const bool edge = PEER && (rb == 0 || i1 == r1);
        const T *up_row = nullptr, *dn_row = nullptr;
        T *mbf = nullptr, *mbl = nullptr;  // this sweep's mailbox rows (slot of u^(it+1))
        const bool mbx = PEER && (pr.mb_first[0] != nullptr || pr.mb_last[0] != nullptr);
        uint32_t it = 0;
        if constexpr (PEER) {
            if (edge) {
                // this rank's completed iterations = the index of this sweep (bumped only
                // after every edge wave of the sweep has finished)
                it = __hip_atomic_load(pr.sync + kSyncIter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (rb == 0 && pr.up_flag) {
                    peer::wait_at_least(pr.up_flag, it, pr.sync + kSyncErr, pr.spin_limit);
                    up_row = static_cast<const T *>(pr.up_row[it & 1u]) + (int64_t)cvc * NV;
                }
                if (i1 == r1 && pr.dn_flag) {
                    peer::wait_at_least(pr.dn_flag, it, pr.sync + kSyncErr, pr.spin_limit);
                    dn_row = static_cast<const T *>(pr.dn_row[it & 1u]) + (int64_t)cvc * NV;
                }
                // the waits above also order the mailbox writes: a neighbour at >= it
                // has finished sweep it - 1, the last reader of slot (it + 1) & 1
                if (rb == 0) mbf = static_cast<T *>(pr.mb_first[(it + 1) & 1u]);
                if (i1 == r1) mbl = static_cast<T *>(pr.mb_last[(it + 1) & 1u]);
            }
        }
        auto ld = [&](int i) {
            const V *p = reinterpret_cast<const V *>(base + (int64_t)i * pitch);
            if constexpr (PEER) {  // wave-uniform row select: halo rows come from the neighbours,
                const T *q = nullptr;  // loaded at system scope (sc0 sc1): never a stale cached line
                if (i == r0 - 1 && up_row) q = up_row;
                if (i == r1 && dn_row) q = dn_row;
                if (q) {
                    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T *>(q), 0, 16,
                                                                                       0x00020000);
                    return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(rs, 0, 0, kCpolSystem));
                }
            }
            if constexpr (LNT == 1) return __builtin_nontemporal_load(p);  // tuning variant
            if constexpr (LNT == 2) {
                if (i > i0 && i < i1 - 1) return __builtin_nontemporal_load(p);  // wave-uniform
            }
            return *p;
        };
        const uint32_t soff = out_lane ? (uint32_t)(cv * NV * sizeof(T)) : kDrop;
        const int j0 = cv * NV;
        // One walk over the block's rows, prologue included (each direction its
        // own inlined body: nothing but scalars is live across the branch).
        // UPW (ALT, odd row blocks): bottom row first, so two vertically
        // adjacent blocks read the halo rows they share at the same moment.
        // ring: row x_{i0-1+t} (x_{i1-t} walking up) lives in slot t % 5; the
        // loop advances 5 rows so every slot index is a compile-time constant
        // (no register rotation, whose moves would force a wait on the
        // in-flight prefetch)
        auto walk = [&](auto upc) {
            constexpr bool UPW = decltype(upc)::value;
            V S[5];
            if constexpr (UPW) {
                S[0] = ld(i1);
                S[1] = ld(i1 - 1);
                S[2] = ld(max(i1 - 2, i0 - 1));
                S[3] = ld(max(i1 - 3, i0 - 1));
            } else {
                S[0] = ld(i0 - 1);
                S[1] = ld(i0);
                S[2] = ld(min(i0 + 1, i1));
                S[3] = ld(min(i0 + 2, i1));
            }
            S[4] = V{};  // first written by step 0; a copy of S[3] would wait on its load
            __builtin_amdgcn_sched_barrier(0);
            auto step = [&](auto kc, int i) {
                constexpr int k = decltype(kc)::value;
                const int r = UPW ? i - k : i + k;  // row computed in this step
                // x_{r+3} replaces x_{r-2} (walking up: x_{r-3} replaces x_{r+2})
                S[(k + 4) % 5] = UPW ? ld(max(r - 3, i0 - 1)) : ld(min(r + 3, i1));
                const V up = S[(UPW ? k + 2 : k) % 5], cen = S[(k + 1) % 5], dn = S[(UPW ? k : k + 2) % 5];
                const T left = dpp_shift<T>(cen[NV - 1], 0x138);  // lane - 1's last element
                const T right = dpp_shift<T>(cen[0], 0x130);      // lane + 1's first element
                V res;
#pragma unroll
                for (int e = 0; e < NV; ++e) {
                    const int j = j0 + e;
                    const T l = e == 0 ? left : cen[e - 1];
                    const T rr = e == NV - 1 ? right : cen[e + 1];
                    const T sm = ((up[e] + dn[e]) + (l + rr)) * (T)0.25;
                    const bool interior = j > 0 && j < cols - 1;
                    res[e] = interior ? sm : cen[e];
                    const T d = sm > cen[e] ? sm - cen[e] : cen[e] - sm;
                    rmax = fmax(rmax, (interior && out_lane) ? d : (T)0);  // select + v_max: no exec branch
                }
                // rows outside the block (tail group) store nowhere: offset out of range
                const bool rok = UPW ? r >= i0 : r < i1;
                const __amdgpu_buffer_rsrc_t orow = __builtin_amdgcn_make_buffer_rsrc(
                    un + (int64_t)(UPW ? max(r, i0) : min(r, i1 - 1)) * pitch, 0, cols * (int)sizeof(T), 0x00020000);
                typedef uint32_t u4 __attribute__((ext_vector_type(4)));
                if constexpr (PEER) {
                    // mailbox mode: every row stores to un with the sweep's policy, and
                    // a second, write-through store copies the two edge rows into this
                    // rank's mailbox slot for u^(it+1) (dropped — out-of-range offset —
                    // everywhere else: two stores per row on every path, so the wait
                    // counts stay exact without a branch); slab mode (no mailbox): the
                    // edge rows themselves are stored write-through
                    const bool first = edge && r == r0 && mbf != nullptr;
                    const bool last = edge && r == r1 - 1 && mbl != nullptr;
                    if (!mbx && edge && (r == r0 || r == r1 - 1))
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, res), orow, rok ? soff : kDrop, 0,
                                                               kCpolSystem);
                    else
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, res), orow, rok ? soff : kDrop, 0,
                                                               AUX);
                    const __amdgpu_buffer_rsrc_t mrow = __builtin_amdgcn_make_buffer_rsrc(
                        first ? mbf : (last ? mbl : un), 0, (first || last) ? cols * (int)sizeof(T) : 0, 0x00020000);
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, res), mrow,
                                                           (rok && (first || last)) ? soff : kDrop, 0, kCpolSystem);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, res), orow, rok ? soff : kDrop, 0, AUX);
                }
                // keep each step's prefetch at its start: the scheduler otherwise sinks
                // loads past the next step's use and the wait counts collapse to 0
                __builtin_amdgcn_sched_barrier(0);
            };
            using I0 = std::integral_constant<int, 0>;
            using I1 = std::integral_constant<int, 1>;
            using I2 = std::integral_constant<int, 2>;
            using I3 = std::integral_constant<int, 3>;
            using I4 = std::integral_constant<int, 4>;
            // straight-line groups of 5 rows with no branch inside a group (a branch
            // between the steps costs the wait counts their precision: 10-rows-per-
            // wave sweeps measured 9% slower with per-step exits), then the 1-4 tail
            // rows; TAIL_EXIT = false (tuning variant) instead runs the tail as a
            // whole group, computing the surplus rows on clamped data and dropping
            // them at the buffer store
            const int nrow = i1 - i0;
            const int ngrp = TAIL_EXIT ? nrow / 5 : (nrow + 4) / 5;
            int i = UPW ? i1 - 1 : i0;
            for (int g = 0; g < ngrp; ++g, i += UPW ? -5 : 5) {
                step(I0{}, i);
                step(I1{}, i);
                step(I2{}, i);
                step(I3{}, i);
                step(I4{}, i);
            }
            const int rem = TAIL_EXIT ? nrow - ngrp * 5 : 0;
            if (rem > 0) {
                step(I0{}, i);
                if (rem > 1) {
                    step(I1{}, i);
                    if (rem > 2) {
                        step(I2{}, i);
                        if (rem > 3) step(I3{}, i);
                    }
                }
            }
        };
        if (ALT && (rb & 1))  // wave-uniform
            walk(std::true_type{});
        else
            walk(std::false_type{});
        if constexpr (PEER) {
            if (edge) {
                // the write-through edge-row stores are acknowledged at system scope
                // before the count goes up: no L2 write-back fence needed
                __builtin_amdgcn_s_waitcnt(0);
                if (lane == 0) {
                    const int n_edge = nrb > 1 ? 2 * strips : strips;
                    const uint32_t c = __hip_atomic_fetch_add(pr.sync + kSyncCtr, 1u, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT);
                    if (c + 1 == (uint32_t)n_edge) {  // last edge wave of this sweep
                        __hip_atomic_store(pr.sync + kSyncCtr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        // release at system scope: every edge wave's write-through row
                        // stores were acknowledged (waitcnt above, then the counter)
                        peer::publish(pr.sync + kSyncIter, it + 1);
                    }
                }
            }
        }
    }
    if (resid) {  // block-uniform; no wave returned early, so the barrier is safe
        // one agent-scope load + atomic per workgroup, not per wave: the load
        // misses every XCD's L2 (~1-2 us), and per wave those tails cost the
        // residual sweep ~60 us at 16384^2
        using B = typename JVec<T>::bits;
        __shared__ T s_m[WPB];
        const T m = wave_max_dpp(rmax);
        if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            T mm = s_m[0];
#pragma unroll
            for (int q = 1; q < WPB; ++q) mm = s_m[q] > mm ? s_m[q] : mm;
            if (mm > (T)0) residual_max(reinterpret_cast<B *>(resid), __builtin_bit_cast(B, mm));
        }
    }
}

}  // namespace
}  // namespace mpx
