// ring.hpp — 3-slot LDS weight-slice ring shared by the runtime-loop kernels (fused_kernels.hpp, w3_kernel.hpp).
#pragma once
#include "siren_common.h"

namespace siren {

// ------------------------------------------------------------------------------------------------------
// Weight-slice ring: wave w copies 4 KiB (4 x 1 KiB global_load_lds_dwordx4) of every 16 KiB slice.
// ------------------------------------------------------------------------------------------------------
__device__ __forceinline__ void ring_issue(const float* __restrict__ stream, float* ring, int s, int nslices,
                                           int wave, int lane) {
    if (s < nslices) {
        const int wu = __builtin_amdgcn_readfirstlane(wave);
        const char* src = (const char*)(stream + (int64_t)s * SLICE + wu * 1024);
        const unsigned dst = lds_addr(ring + (s % NBUF) * SLICE + wu * 1024);
#pragma unroll
        for (int q = 0; q < 4; ++q) glds_x4(src + q * 1024, 16u * lane, dst + q * 1024);
    }
}

// Wait until this wave's part of slice s has landed (slice s+1 may stay in flight), then barrier so
// every wave's part has landed and every wave has finished reading the slot that is refilled next.
__device__ __forceinline__ void ring_wait(int s, int nslices) {
    if (s + 1 < nslices)
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

// Mid-slice form (slice_mma_mid): in slice s, wait until slice s+1 has landed (it is the newest load in flight; a
// pass's epilogue stores are waited for too), barrier, then refill the slot of slice s-1 with slice s+2.
__device__ __forceinline__ void ring_mid(const float* __restrict__ stream, float* ring, int s, int nslices, int wave,
                                         int lane) {
    if (s + 1 < nslices) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    ring_issue(stream, ring, s + 2, nslices, wave, lane);
}

}  // namespace siren
