// lds_ops.h — weight-operand reads of the MFMA slice loops, issued ahead of their use.
//
// A slice of the LDS weight ring holds, for every output block ob, lane l's A operands of the slice's 4 K-steps as
// the 16 B at ob * 1 KiB + 16 l (pack_kernel's layout). hipcc, left alone, reads each block's operands right before
// its MFMAs and waits lgkmcnt(0): one exposed LDS latency every 4-8 MFMAs (at one or two waves per SIMD nothing
// else covers it; DESIGN.md §3.11 measured it as the hidden-512 kernel's largest loss). These helpers issue the
// reads by inline asm one block (or block pair) ahead and tie the consumer MFMAs to a counted s_waitcnt through
// "+v" operands, so the next operands are in flight while the current ones compute.
#pragma once
#include "siren_common.h"

namespace siren {

// ds_read_b128 at a compile-time byte offset from a VGPR base (not visible to hipcc's waitcnt insertion)
template <int OFF>
__device__ __forceinline__ f32x4 lds_read4(unsigned vaddr) {
    static_assert(OFF >= 0 && OFF < 65536, "ds offset field is 16 bits");
    f32x4 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(vaddr), "i"(OFF));
    return r;
}
// two ds_read_b128 and their wait in ONE statement: the outputs are valid when the statement ends, so the compiler may
// copy them freely (the loop-carried operands at a persistent tile seam; an asm read's destination counts as written
// at its own ASMEND and was copied before the data landed, tools/check_asm_waits.py)
template <int OFF>
__device__ __forceinline__ void lds_read4x2_wait(unsigned vaddr, f32x4& a, f32x4& b) {
    static_assert(OFF >= 0 && OFF + 1024 < 65536, "ds offset field is 16 bits");
    asm volatile("ds_read_b128 %0, %2 offset:%3\n\tds_read_b128 %1, %2 offset:%4\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(a), "=&v"(b)
                 : "v"(vaddr), "i"(OFF), "i"(OFF + 1024));
}
template <int N>
__device__ __forceinline__ void lgkm_wait(f32x4& a, f32x4& b) {
    asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(N));
}
template <int N>
__device__ __forceinline__ void lgkm_wait1(f32x4& a) {
    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "i"(N));
}

// acc[ob] += W-slice(ob) x bop for the output-block pairs P .. NBLK/2 - 1 of one slice: 8 MFMAs per pair, the two
// accumulators alternating (a dependent MFMA is 64 cycles behind, past the 40-cycle latency of 16x16x4 f32); the
// next pair's operands are read before this pair's wait, which is lgkmcnt(2).
template <int P, int NBLK>
__device__ __forceinline__ void slice_pairs(unsigned vaddr, const f32x4& bop, f32x4 (&acc)[NBLK], f32x4 a0,
                                            f32x4 a1) {
    constexpr int ob = 2 * P;
    f32x4 n0, n1;
    if constexpr (P + 1 < NBLK / 2) {
        n0 = lds_read4<(ob + 2) * 1024>(vaddr);
        n1 = lds_read4<(ob + 3) * 1024>(vaddr);
        lgkm_wait<2>(a0, a1);
    } else {
        lgkm_wait<0>(a0, a1);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        acc[ob] = mfma4(a0[r], bop[r], acc[ob]);
        acc[ob + 1] = mfma4(a1[r], bop[r], acc[ob + 1]);
    }
    if constexpr (P + 1 < NBLK / 2) slice_pairs<P + 1, NBLK>(vaddr, bop, acc, n0, n1);
}

// Mid-slice ring protocol (the W1 kernel's; here for the runtime-loop kernels): the barrier sits
// after output-block pair MID of slice s instead of at the slice start. It publishes slice s+1 (its loads were
// issued one slice earlier) and frees the slot of slice s-1 for slice s+2, so the pair-ahead operand reads run on
// across the slice seam (the last pair of a slice reads the next slice's first pair) and no wave waits for the
// barrier with an empty MFMA queue. mid() = the wait + barrier + issue; NEXT = read the next slice's first pair.
template <int P, int NBLK, int MID, bool NEXT, class Mid>
__device__ __forceinline__ void slice_pairs_mid(unsigned vaddr, unsigned vnext, const f32x4& bop, f32x4 (&acc)[NBLK],
                                                f32x4 a0, f32x4 a1, f32x4& o0, f32x4& o1, Mid& mid) {
    constexpr int ob = 2 * P;
    constexpr bool last = P + 1 == NBLK / 2;
    if constexpr (P == MID) mid();
    f32x4 n0, n1;
    if constexpr (!last) {
        n0 = lds_read4<(ob + 2) * 1024>(vaddr);
        n1 = lds_read4<(ob + 3) * 1024>(vaddr);
        lgkm_wait<2>(a0, a1);
    } else if constexpr (NEXT) {
        n0 = lds_read4<0>(vnext);
        n1 = lds_read4<1024>(vnext);
        lgkm_wait<2>(a0, a1);
    } else {
        lgkm_wait<0>(a0, a1);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        acc[ob] = mfma4(a0[r], bop[r], acc[ob]);
        acc[ob + 1] = mfma4(a1[r], bop[r], acc[ob + 1]);
    }
    if constexpr (!last) {
        slice_pairs_mid<P + 1, NBLK, MID, NEXT>(vaddr, vnext, bop, acc, n0, n1, o0, o1, mid);
    } else if constexpr (NEXT) {
        o0 = n0;
        o1 = n1;
    }
}
// one slice with the mid-slice barrier: a0 / a1 = its first pair (in flight); with NEXT, o0 / o1 receive the next
// slice's first pair (in flight)
template <int NBLK, int MID, bool NEXT, class Mid>
__device__ __forceinline__ void slice_mma_mid(unsigned vaddr, unsigned vnext, const f32x4& bop, f32x4 (&acc)[NBLK],
                                              f32x4 a0, f32x4 a1, f32x4& o0, f32x4& o1, Mid&& mid) {
    slice_pairs_mid<0, NBLK, MID, NEXT>(vaddr, vnext, bop, acc, a0, a1, o0, o1, mid);
}

// one slice; vaddr = LDS byte address of the ring slot + 16 * lane
template <int NBLK>
__device__ __forceinline__ void slice_mma(unsigned vaddr, const f32x4& bop, f32x4 (&acc)[NBLK]) {
    const f32x4 a0 = lds_read4<0>(vaddr);
    const f32x4 a1 = lds_read4<1024>(vaddr);
    slice_pairs<0, NBLK>(vaddr, bop, acc, a0, a1);
}

// two column tiles sharing every A operand (W3: primal bp and tangent bt): 8 MFMAs per block read, the next block's
// operands in flight (lgkmcnt(1))
template <int OB, int NBLK>
__device__ __forceinline__ void slice_singles2(unsigned vaddr, const f32x4& bp, const f32x4& bt, f32x4 (&accp)[NBLK],
                                               f32x4 (&acct)[NBLK], f32x4 a) {
    f32x4 nx;
    if constexpr (OB + 1 < NBLK) {
        nx = lds_read4<(OB + 1) * 1024>(vaddr);
        lgkm_wait1<1>(a);
    } else {
        lgkm_wait1<0>(a);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        accp[OB] = mfma4(a[r], bp[r], accp[OB]);
        acct[OB] = mfma4(a[r], bt[r], acct[OB]);
    }
    if constexpr (OB + 1 < NBLK) slice_singles2<OB + 1, NBLK>(vaddr, bp, bt, accp, acct, nx);
}

template <int NBLK>
__device__ __forceinline__ void slice_mma2(unsigned vaddr, const f32x4& bp, const f32x4& bt, f32x4 (&accp)[NBLK],
                                           f32x4 (&acct)[NBLK]) {
    slice_singles2<0, NBLK>(vaddr, bp, bt, accp, acct, lds_read4<0>(vaddr));
}

// slice_singles2 with the mid-slice barrier (slice_pairs_mid): mid() before block MID, the last block reads the next
// slice's first block (NEXT) into o
template <int OB, int NBLK, int MID, bool NEXT, class Mid>
__device__ __forceinline__ void slice_singles2_mid(unsigned vaddr, unsigned vnext, const f32x4& bp, const f32x4& bt,
                                                   f32x4 (&accp)[NBLK], f32x4 (&acct)[NBLK], f32x4 a, f32x4& o,
                                                   Mid& mid) {
    constexpr bool last = OB + 1 == NBLK;
    if constexpr (OB == MID) mid();
    f32x4 nx;
    if constexpr (!last) {
        nx = lds_read4<(OB + 1) * 1024>(vaddr);
        lgkm_wait1<1>(a);
    } else if constexpr (NEXT) {
        nx = lds_read4<0>(vnext);
        lgkm_wait1<1>(a);
    } else {
        lgkm_wait1<0>(a);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        accp[OB] = mfma4(a[r], bp[r], accp[OB]);
        acct[OB] = mfma4(a[r], bt[r], acct[OB]);
    }
    if constexpr (!last) {
        slice_singles2_mid<OB + 1, NBLK, MID, NEXT>(vaddr, vnext, bp, bt, accp, acct, nx, o, mid);
    } else if constexpr (NEXT) {
        o = nx;
    }
}
template <int NBLK, int MID, bool NEXT, class Mid>
__device__ __forceinline__ void slice_mma2_mid(unsigned vaddr, unsigned vnext, const f32x4& bp, const f32x4& bt,
                                               f32x4 (&accp)[NBLK], f32x4 (&acct)[NBLK], f32x4 a, f32x4& o, Mid&& mid) {
    slice_singles2_mid<0, NBLK, MID, NEXT>(vaddr, vnext, bp, bt, accp, acct, a, o, mid);
}

// three column tiles sharing every A operand (hess_kernel.hpp: 8 coordinates x 6 Hessian-jet streams): 12 MFMAs per
// block read, K-step-major so a dependent MFMA is two MFMAs (64 cycles) behind; otherwise slice_singles2_mid
template <int OB, int NBLK, int MID, bool NEXT, class Mid>
__device__ __forceinline__ void slice_singles3_mid(unsigned vaddr, unsigned vnext, const f32x4& b0, const f32x4& b1,
                                                   const f32x4& b2, f32x4 (&acc)[3][NBLK], f32x4 a, f32x4& o,
                                                   Mid& mid) {
    constexpr bool last = OB + 1 == NBLK;
    if constexpr (OB == MID) mid();
    f32x4 nx;
    if constexpr (!last) {
        nx = lds_read4<(OB + 1) * 1024>(vaddr);
        lgkm_wait1<1>(a);
    } else if constexpr (NEXT) {
        nx = lds_read4<0>(vnext);
        lgkm_wait1<1>(a);
    } else {
        lgkm_wait1<0>(a);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        acc[0][OB] = mfma4(a[r], b0[r], acc[0][OB]);
        acc[1][OB] = mfma4(a[r], b1[r], acc[1][OB]);
        acc[2][OB] = mfma4(a[r], b2[r], acc[2][OB]);
    }
    if constexpr (!last) {
        slice_singles3_mid<OB + 1, NBLK, MID, NEXT>(vaddr, vnext, b0, b1, b2, acc, nx, o, mid);
    } else if constexpr (NEXT) {
        o = nx;
    }
}
template <int NBLK, int MID, bool NEXT, class Mid>
__device__ __forceinline__ void slice_mma3_mid(unsigned vaddr, unsigned vnext, const f32x4& b0, const f32x4& b1,
                                               const f32x4& b2, f32x4 (&acc)[3][NBLK], f32x4 a, f32x4& o, Mid&& mid) {
    slice_singles3_mid<0, NBLK, MID, NEXT>(vaddr, vnext, b0, b1, b2, acc, a, o, mid);
}

}  // namespace siren
