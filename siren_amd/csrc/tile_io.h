// tile_io.h — saddr-form global tile I/O and the LDS transpose that turns a C/D-layout block into one coalesced
// 1 KiB store, shared by the kernels whose epilogues run inside the MFMA stream (w1 memory modes, w3i, qfi, widei).
// Inline asm, so every op is one counted vector-memory instruction: the slice loops' exact s_waitcnt vmcnt(N)
// allowances count them.
#pragma once
#include "siren_common.h"

// the nontemporal hint of the epilogue stores (siren_common.h st_tile: SIREN_STORE_NT)
#if SIREN_STORE_NT != 0
#define SIREN_STPOL " nt"
#else
#define SIREN_STPOL ""
#endif

namespace siren {

// Every epilogue load / store is in saddr form: a wave-uniform base in SGPRs, made opaque right before its use (hipcc
// would otherwise precompute the addresses of every (buffer, layer, block) up front: 100+ SGPR pairs / 64-bit VGPR
// addresses, spilled), plus one per-lane VGPR offset shared by all of them.
__device__ __forceinline__ const char* w3_at(const char* base, int64_t off) {
    asm volatile("" : "+s"(base));
    return base + off;
}
// The s_nop after a 16-byte store: a VALU may not overwrite a store's data VGPRs in the next two wait states (the
// store reads them late; gfx940+ store-data hazard). hipcc inserts those for its own stores, not for inline asm — without
// it the coordinates of lanes 12..15 of every 16-lane row came back wrong once the allocator reused a stored register.
__device__ __forceinline__ void w3_store16(const char* base, unsigned voff, const f32x4& v) {
    asm volatile("global_store_dwordx4 %0, %1, %2" SIREN_STPOL "\n\ts_nop 1" ::"v"(voff), "v"(v), "s"(base));
}
// The same block as the four 64 B pieces at the lane's (4 g 16 + c) offset (voff = 4 (4 g 16 + c); what store_block
// writes), one counted instruction each
__device__ __forceinline__ void w3_store_tile(const char* base, unsigned voff, const f32x4& v) {
    asm volatile(
        "global_store_dword %0, %1, %5" SIREN_STPOL "\n\t"
        "global_store_dword %0, %2, %5 offset:64" SIREN_STPOL "\n\t"
        "global_store_dword %0, %3, %5 offset:128" SIREN_STPOL "\n\t"
        "global_store_dword %0, %4, %5 offset:192" SIREN_STPOL "\n\t"
        "s_nop 1" ::"v"(voff),
        "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "s"(base));
}
// A block of the wgrad tile layout (element (neuron 16 rb + 4 g + r, coordinate c) at rb 256 + neuron 16 + c, what
// store_block writes as four dword stores of 64 B pieces) goes out as ONE coalesced 1 KiB global_store_dwordx4: the
// wave transposes it through a 16 x 20-float LDS scratch (conflict-free b32 writes, 16 B-aligned b128 reads; LDS ops of
// a wave run in order, so consecutive blocks reuse it). In the slice loop the transposed registers are stored one slice
// later, after the lgkmcnt wait that retires them (w3_tile_flush); four dword stores per block cost the kernel ~25 %.
__device__ __forceinline__ void w3_stage(f32x4& out, const f32x4& v, unsigned tw, unsigned tr) {
    asm volatile(
        "ds_write_b32 %1, %2\n\t"
        "ds_write_b32 %1, %3 offset:80\n\t"
        "ds_write_b32 %1, %4 offset:160\n\t"
        "ds_write_b32 %1, %5 offset:240\n\t"
        "ds_read_b128 %0, %6"
        : "=&v"(out)
        : "v"(tw), "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(tr));
}
// the same, waited for and stored at once (the serial layer-0 epilogue after the last GEMM)
__device__ __forceinline__ void w3_stage_store(const char* base, const f32x4& v, unsigned tw, unsigned tr,
                                               unsigned voff) {
    f32x4 t;
    asm volatile(
        "ds_write_b32 %1, %2\n\t"
        "ds_write_b32 %1, %3 offset:80\n\t"
        "ds_write_b32 %1, %4 offset:160\n\t"
        "ds_write_b32 %1, %5 offset:240\n\t"
        "ds_read_b128 %0, %6\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "global_store_dwordx4 %7, %0, %8" SIREN_STPOL "\n\t"
        "s_nop 1"
        : "=&v"(t)
        : "v"(tw), "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(tr), "v"(voff), "s"(base));
}
// wave-uniform address + this lane's 16 B: one global_load_dwordx4 in saddr form
__device__ __forceinline__ void w3_load16(f32x4& r, const char* base, unsigned voff) {
    asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(r) : "v"(voff), "s"(base));
}
// the same with the nontemporal hint, for data read exactly once: the kept Hessian reverse's kept-jet reloads
// (A/B round 6: qfi_rev_kernel<3> -2.6 %; neutral on w3i / widei / the fp32 reverse, which keep w3_load16)
__device__ __forceinline__ void w3_load16_once(f32x4& r, const char* base, unsigned voff) {
    asm volatile("global_load_dwordx4 %0, %1, %2 nt" : "=v"(r) : "v"(voff), "s"(base));
}
}  // namespace siren
