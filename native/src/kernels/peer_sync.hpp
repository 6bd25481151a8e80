// Device-side primitives of the one-sided (IPC-mapped, xGMI) transports:
// bounded waits on a neighbour's counter, counter publication with release
// semantics, and system-scope loads / stores of the rows a neighbour shares.
// Used by the Jacobi peer sweep (jacobi.hip), the streaming conv halo fetch
// and the start-up kernel-path probes (peer.hip). The reference has no
// multi-GPU code: this is the north-star halo tier.
//
// Memory-model contract (gfx950, HIP scopes):
//  * a producer makes rows visible to another device by storing them with the
//    system-scope cache policy (SC0|SC1: written through the L2) or by a
//    kernel boundary (agent-scope release writes the multi-XCD L2s back), then
//    publishes its counter with a system-scope RELEASE store (waits for every
//    earlier store of the wave to be acknowledged first);
//  * a consumer polls the counter with system-scope loads and reads the shared
//    rows with system-scope loads (SC0|SC1: never served from a stale L2
//    line), so no cache-invalidate fence is needed after the wait;
//  * every wait is bounded: a wave that gives up sets an error word and
//    returns, the host raises (no hang on a stalled or dead neighbour).
#pragma once

#include "internal.hpp"

namespace mpx {
namespace peer {

constexpr int kCpolSystem = 1 | 16;              // gfx950 cache policy SC0 | SC1: system scope
constexpr uint32_t kSpinDefault = 1u << 22;     // polls (s_sleep 4 each): seconds, not minutes

// Wait until *flag >= target; false (and *err = 1) when the wait gave up.
// Once any wait of this rank has given up (*err set), later waits return
// false at once (checked on entry and every 1024 polls) instead of spinning
// their full limit each — a stalled neighbour costs one timeout, not one per
// remaining step.
__device__ __forceinline__ bool wait_at_least(const uint32_t *flag, uint32_t target, uint32_t *err, uint32_t limit) {
    uint32_t spins = 0;
    const uint32_t lim = limit ? limit : kSpinDefault;
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
        if ((spins & 1023u) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)
            return false;
        if (++spins > lim) {
            __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return false;
        }
        __builtin_amdgcn_s_sleep(4);
    }
    return true;
}

// Publish a counter value after this wave's earlier stores (release at system
// scope: the compiler waits for their acknowledgement before the store).
__device__ __forceinline__ void publish(uint32_t *flag, uint32_t v) {
    __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16-byte system-scope load / store at byte offset `off` of `base` (`bytes`
// bounds the buffer descriptor: out-of-range lanes read 0 / store nothing).
__device__ __forceinline__ u32x4 load16_sys(const void *base, uint32_t off, uint32_t bytes) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, bytes, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kCpolSystem);
}

__device__ __forceinline__ void store16_sys(void *base, uint32_t off, uint32_t bytes, u32x4 v) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, kCpolSystem);
}

// The same 16-byte load with the default cache policy (the conv kernels' load
// path for neighbour rows that do not change while mapped).
__device__ __forceinline__ u32x4 load16(const void *base, uint32_t off, uint32_t bytes) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, bytes, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
}

}  // namespace peer
}  // namespace mpx
