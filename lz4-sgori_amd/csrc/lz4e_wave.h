// lz4e_wave.h -- the wave64 primitives the gfx950 LZ4E kernels are written
// against: lane identity, ballots, cross-lane reads, byte alignment, the
// shader clock and the global-memory pointer types.  Kernel code uses only
// these (never the amdgcn builtins directly).
//
// The host-side lane emulator (tools/emu/, test tooling) compiles this same
// header: it supplies the amdgcn builtins themselves (each lane a thread,
// tools/emu/include/hip/hip_runtime.h, with the hardware's semantics: DPP row
// shifts and broadcasts, ds_(b)permute, v_perm, ...), so every helper below
// -- match_any6, the DPP scans, the byte-table gathers -- runs the same code
// there.  Only what a host thread cannot express differs under LZ4E_EMU:
// inline asm (register constraints, m0), the buffer-resource type, and the
// places that rely on a wave's lanes running in lockstep, which become
// barriers of the emulated wave.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define LZ4E_DEV __device__ __forceinline__

namespace lz4e {

constexpr uint32_t kWave = 64;

LZ4E_DEV uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
LZ4E_DEV uint64_t ballot(bool p) { return __ballot(p); }
// v_readfirstlane: the value of the first active lane, as a scalar.
LZ4E_DEV uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// v_readlane: lane l's value, as a scalar (l wave-uniform).
LZ4E_DEV uint32_t lane_val(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
// v with lane l (wave-uniform) set to the uniform value x.
LZ4E_DEV uint32_t set_lane(uint32_t v, uint32_t x, uint32_t l) {
    return lane_id() == l ? x : v;
}
// v_writelane: v with lane l (wave-uniform) set to the wave-uniform x.  No
// builtin exists; gfx9 takes a variable lane select from m0 only (as the
// compiler's own lowering of llvm.amdgcn.writelane does, m0 being set right
// before every use), and the s_nop covers the lane-select hazard.
#ifndef LZ4E_EMU
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
LZ4E_DEV uint32_t put_lane(uint32_t v, uint32_t x, uint32_t l) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 4\n\tv_writelane_b32 %0, %1, m0"
                 : "+v"(v)
                 : "s"(x), "s"(l)
                 : "m0");
    return v;
}
#pragma clang diagnostic pop
#else
LZ4E_DEV uint32_t put_lane(uint32_t v, uint32_t x, uint32_t l) {
    return set_lane(v, uni(x), l);
}
#endif
// Lanes whose 6-bit key equals mine (key < 64): one ballot per key bit, no
// loop over the distinct keys.
LZ4E_DEV uint64_t match_any6(uint32_t key) {
    uint64_t m = ~0ull;
#pragma unroll
    for (uint32_t b = 0; b < 6; ++b) {
        const bool bit = (key >> b) & 1;
        const uint64_t bb = ballot(bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}
// Wave issue priority from the share of its work still ahead (q: quarters
// done, 0..3): the wave furthest behind wins issue slots on its SIMD, which
// shortens the batch's longest block ("least progress first").
LZ4E_DEV void wave_prio_for(uint32_t q) {
    if (q == 0) __builtin_amdgcn_s_setprio(3);
    else if (q == 1) __builtin_amdgcn_s_setprio(2);
    else if (q == 2) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}
// ds_permute: lane l sends v to lane dst (l's own choice); a lane nobody
// sends to receives an unspecified value.
LZ4E_DEV uint32_t push_lane(uint32_t v, uint32_t dst) {
    return (uint32_t)__builtin_amdgcn_ds_permute((int)(dst << 2), (int)v);
}
// Keeps a value (e.g. a prefetch load's result) alive until here without
// using it: the wait for it is placed here, not at the load.
#ifndef LZ4E_EMU
LZ4E_DEV void consume(uint32_t v) { asm volatile("" ::"v"(v)); }
#else
LZ4E_DEV void consume(uint32_t) {}
#endif
// ds_bpermute: lane src's value (src mod 64), per lane.  (HIP's __shfl adds
// the lane id and a width mask around it: two VALU more per shuffle.)
LZ4E_DEV uint32_t shfl(uint32_t v, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((src & 63u) << 2), (int)v);
}
// ds_bpermute with the byte address given (4 x source lane, mod 256): no
// index arithmetic around it.
LZ4E_DEV uint32_t shfl_addr(uint32_t v, uint32_t addr) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)addr, (int)v);
}
// v_perm_b32: byte i of the result is byte sel_i of {hi:lo} (0-3: lo, 4-7:
// hi), 0 for a selector byte 0x0C.
LZ4E_DEV uint32_t perm_bytes(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}
LZ4E_DEV int32_t shfl_up(int32_t v, uint32_t d) { return __shfl_up(v, d); }
// Inclusive prefix sum over the 64 lanes with DPP (row_shr 1/2/4/8 inside
// each row of 16, then row_bcast:15 and row_bcast:31 across rows).
LZ4E_DEV uint32_t wave_incl_add(uint32_t v) {
    const uint32_t lane = lane_id();
    uint32_t x = v, t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
    x += (lane & 15) >= 1 ? t : 0u;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
    x += (lane & 15) >= 2 ? t : 0u;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
    x += (lane & 15) >= 4 ? t : 0u;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
    x += (lane & 15) >= 8 ? t : 0u;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
    x += (lane & 16) ? t : 0u;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
    x += (lane & 32) ? t : 0u;
    return x;
}
// Exclusive prefix min / max over the 64 lanes (lane 0 gets the identity):
// the DPP inclusive scan, then one lane shift.
template <bool kMax>
LZ4E_DEV int32_t wave_excl_minmax(int32_t v) {
    const uint32_t lane = lane_id();
    const int32_t id = kMax ? INT32_MIN : INT32_MAX;
    auto op = [](int32_t a, int32_t b) { return kMax ? (a > b ? a : b) : (a < b ? a : b); };
    int32_t x = v, t;
    t = __builtin_amdgcn_update_dpp(id, x, 0x111, 0xf, 0xf, false);
    x = (lane & 15) >= 1 ? op(x, t) : x;
    t = __builtin_amdgcn_update_dpp(id, x, 0x112, 0xf, 0xf, false);
    x = (lane & 15) >= 2 ? op(x, t) : x;
    t = __builtin_amdgcn_update_dpp(id, x, 0x114, 0xf, 0xf, false);
    x = (lane & 15) >= 4 ? op(x, t) : x;
    t = __builtin_amdgcn_update_dpp(id, x, 0x118, 0xf, 0xf, false);
    x = (lane & 15) >= 8 ? op(x, t) : x;
    t = __builtin_amdgcn_update_dpp(id, x, 0x142, 0xa, 0xf, false);
    x = (lane & 16) ? op(x, t) : x;
    t = __builtin_amdgcn_update_dpp(id, x, 0x143, 0xc, 0xf, false);
    x = (lane & 32) ? op(x, t) : x;
    const int32_t e = __shfl_up(x, 1);
    return lane == 0 ? id : e;
}
LZ4E_DEV int32_t wave_excl_min(int32_t v) { return wave_excl_minmax<false>(v); }
LZ4E_DEV int32_t wave_excl_max(int32_t v) { return wave_excl_minmax<true>(v); }
// v_alignbyte: bytes r..r+3 of the 64-bit value hi:lo.
LZ4E_DEV uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t r) {
    return __builtin_amdgcn_alignbyte(hi, lo, r);
}
// s_memtime: shader clock (diagnostic builds only).
LZ4E_DEV uint64_t clock64() { return __builtin_amdgcn_s_memtime(); }
// s_memrealtime: the constant 100 MHz clock (diagnostic builds only).
#ifndef LZ4E_EMU
LZ4E_DEV uint64_t realtime64() { return __builtin_amdgcn_s_memrealtime(); }
#else
inline uint64_t realtime64() { return 0; }
#endif
#ifndef LZ4E_EMU
// Order this wave's LDS/global accesses (memory model fence, wavefront scope).
LZ4E_DEV void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }
// wave_fence for code run by groups of `width` lanes that diverge from each
// other (the group decoder): the same fence on the GPU, a barrier of the
// group's lanes in the emulator.
LZ4E_DEV void group_fence(uint32_t) { wave_fence(); }
// The lanes of a wave execute in lockstep: a memory instruction completes
// (LDS) or is ordered (global stores to one address) for every lane before
// the wave's next one.  Marks the places that rely on it -- a whole-wave put
// followed by a read-back, a lane's store overwriting bytes another lane
// stored just before.  It emits no instruction, but it is a compiler memory
// barrier: no access moves across it, whatever the access types (the
// emulator's lockstep is a barrier of the emulated wave, so both builds
// enforce the same order at the same places).
LZ4E_DEV void lockstep() { asm volatile("" ::: "memory"); }
// Workgroup barrier.
LZ4E_DEV void block_sync() { __syncthreads(); }
// Every global store of this wave has completed (before a flag says so).
LZ4E_DEV void stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// Moves a (possibly wave-uniform) byte offset into a VGPR.  A uniform load
// from read-only memory would otherwise become s_load_*, which ignores the
// low two address bits -- wrong for unaligned reads.
LZ4E_DEV uint32_t vaddr(uint32_t q) {
    asm("" : "+v"(q));
    return q;
}
#else
// Lane emulator: each lane is a host thread, so every place that relies on
// lockstep execution is a barrier of the emulated wave; the workgroup
// barrier is the emulated workgroup's.
LZ4E_DEV void wave_fence() { emu_wave_barrier(); }
LZ4E_DEV void group_fence(uint32_t width) { emu_group_barrier(width); }
LZ4E_DEV void lockstep() { emu_wave_barrier(); }
LZ4E_DEV void block_sync() { __syncthreads(); }
LZ4E_DEV void stores_done() { __atomic_thread_fence(__ATOMIC_SEQ_CST); }
LZ4E_DEV uint32_t vaddr(uint32_t q) { return q; }
#endif

// Global-memory pointer types: pointers rebuilt from integer addresses lose
// their address space and would otherwise compile to flat_* accesses, which
// also count on lgkmcnt (coupling them to every LDS wait).
typedef __attribute__((address_space(1))) const uint32_t gcu32;

// n bytes at p as a raw buffer resource: dword loads at byte offset q return
// 0 when the dword is not entirely inside [0, n) (hardware range check).
#ifndef LZ4E_EMU
struct ByteBuf {
    __amdgpu_buffer_rsrc_t r;
};
LZ4E_DEV ByteBuf buf_make(const void* p, uint32_t n) {
    return ByteBuf{__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)n,
                                                     0x00020000)};
}
LZ4E_DEV uint32_t buf_ld32(const ByteBuf& b, uint32_t q) {
    return __builtin_amdgcn_raw_buffer_load_b32(b.r, q, 0, 0);
}
// Byte at q (0 past the range).
LZ4E_DEV uint32_t buf_ld8(const ByteBuf& b, uint32_t q) {
    return __builtin_amdgcn_raw_buffer_load_b8(b.r, q, 0, 0);
}
#else
struct ByteBuf {
    const uint8_t* p;
    uint32_t n;
};
inline ByteBuf buf_make(const void* p, uint32_t n) { return ByteBuf{(const uint8_t*)p, n}; }
inline uint32_t buf_ld32(const ByteBuf& b, uint32_t q) {
    if ((uint64_t)q + 4 > b.n) return 0;
    uint32_t v;
    __builtin_memcpy(&v, b.p + q, 4);
    return v;
}
inline uint32_t buf_ld8(const ByteBuf& b, uint32_t q) { return q < b.n ? b.p[q] : 0u; }
#endif
typedef __attribute__((address_space(1))) const uint8_t gcu8;

}  // namespace lz4e
