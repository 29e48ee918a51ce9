// lz4e_decompress.hip -- gfx950 LZ4E safe block decoders.
//
// Restates /root/reference/lz4e/lz4e_decompress.c:62-469
// (LZ4E_decompress_generic, instance endOnInputSize + decode_full_block +
// noDict).  The batch decoders share one parse (parse_batch) and differ in
// how the copies of a batch are scheduled; the group decoder runs the scalar
// loop per group of 8 lanes.  launch_impl picks one per launch ("Auto
// mode, in full"):
//
//  * Parse, in batches of up to 64 sequences: the token stream is walked
//    wave-uniformly with the reference's exact sequence of bound checks --
//    including the two-stage 16/18-byte shortcut, whose entry conditions
//    change which malformed inputs are rejected and where -- so the return
//    value, including the error code -(ip - src) - 1, is the reference's.  A
//    fast batch (no extension bytes, far from both block ends) is found by
//    pointer doubling over a 256-byte window of the token stream; anything
//    else is one sequence on the exact scalar path.  Sequence k of a batch is
//    recorded in lane k (literal source, literal length, output position,
//    offset, match length).
//  * decompress_kernel, one wave per block (small and 256 KiB blocks): the wave
//    parses a batch, then copies it -- fast batches assembled in a small LDS
//    span (literals from a 1 KiB LDS ring that mirrors the compressed
//    segments the parse loaded, match sources before the batch from HBM,
//    in-batch dependencies in rounds or by pointer jumping over the span's
//    bytes) and written with one pass of 16-byte stores; scalar-path batches
//    (long runs, block ends) copy in HBM.  LDS per block: ring 1 KiB +
//    mirror 128 B + store sink 256 B + span 2,112 B + jump table 4,224 B =
//    7,744 B.  Its LDS form (blocks of <= 4608 bytes) stages the whole input
//    and assembles the whole output in LDS.
//  * decompress_pipe_kernel, one 4-wave workgroup per block (16-128 KiB, and
//    batches of at most 1024 blocks): wave 0 parses while three copier waves
//    assemble three batches at once, cross-batch sources resolved from the
//    spans of the two previous batches (see the section below).  19 KiB of
//    LDS per block.
//  * decompress_group_kernel, one block per group of 8 lanes (>= kGroupMinBlocks
//    blocks of <= 4608 bytes), handing blocks of short sequences to
//    decompress_resume_kernel.
//  (The chunked and relay decoders of round 4, never picked by auto mode,
//  were removed in round 5, and round 4's one-block-per-lane decoder gave way
//  to the group decoder)
//
// Overlapping matches follow LZ semantics out[op + t] = out[op - off + t]
// byte by byte; offset 0 writes zeros, which is what the reference's
// LZ4_write32(op, offset) + overlap copy produce (lz4e_decompress.c:313,
// 407-415).  Same-wave stores and loads to one global address are ordered by
// the hardware (one vector L1 per CU), and wavefront-scope fences keep the
// compiler from moving a phase's loads above the previous phase's stores.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>


#include "lz4e_device.h"
#include "lz4e_gpu.h"
#include "lz4e_order.h"
#include "lz4e_results.h"

namespace lz4e {

namespace {

constexpr int32_t kLongPiece = 64;  // longer literal runs / matches go to the whole wave

// LDS per block: the input ring (+ mirror), the store sink, the span buffer.
constexpr uint32_t kRing = 1024;                    // 4 segments of 256 B
constexpr uint32_t kRingPad = 128;                  // mirror of ring bytes [0, 128)
constexpr uint32_t kSink = 4 * kWave;               // a dword per lane for unwanted stores
constexpr uint32_t kSpan = 64 * 32 + 16 + 48;       // a fast batch's output, 16-B aligned start
constexpr uint32_t kJump = 2 * kSpan;               // u16 per span byte (chain resolution)
constexpr uint16_t kFinal = 0xFFFF;                 // jump entry of a byte whose value is final
// Small blocks (decode_block's LDS form): output and input both staged in
// LDS, at most kSmallOut bytes each, kSmallBuf bytes of LDS each.
constexpr int32_t kSmallOut = 4608;  // 4 KiB blocks and their 4 KiB + 32 capacities
constexpr uint32_t kSmallBuf = kSmallOut + 64;
constexpr int32_t kSmallBatchOut = 1024;                  // fast-batch output cap there
constexpr uint32_t kSmallJump = 2 * (kSmallBatchOut + 64);  // its jump table

// LDS access types.  Every wider type may alias every other (may_alias):
// the decoders read LDS bytes through whichever width suits the step, so no
// access order may rest on type-based alias analysis.
typedef __attribute__((address_space(3))) uint8_t lu8;
typedef __attribute__((address_space(3), may_alias)) uint32_t lu32;
typedef __attribute__((address_space(3), may_alias)) uint16_t lu16;
typedef uint32_t __attribute__((aligned(1), may_alias)) u32a1;
typedef __attribute__((address_space(3))) u32a1 lu32a1;

LZ4E_DEV uint32_t ld4(const lu8* p) { return *(const lu32a1*)p; }
LZ4E_DEV void st4(lu8* p, uint32_t v) { *(lu32a1*)p = v; }

// Two 256-byte windows of the compressed block, A = segment seg and B =
// segment seg + 1, where segment s is block bytes [256 s - shift, +256)
// (shift = the block's offset inside its first aligned word), plus C =
// segment seg + 2 loaded ahead.  Word loads are clamped to the block.  With
// a ring, every segment is written to LDS slot s & 3 when it becomes B.
struct InWindow {
    gcu32* w;        // word-aligned base of the block
    int32_t shift;   // byte offset of the block inside w[0]
    int32_t last;    // last word index that belongs to the block
    uint32_t lane;
    int32_t seg;     // segment of window A
    int32_t base;    // block position of window A byte 0 (256 seg - shift)
    int32_t ring_lo; // lowest block position held by the ring
    uint32_t a, b, c;  // this lane's dword of A, B and C
    lu32* ring;      // kRing + kRingPad bytes of LDS
    // Small blocks: the whole block staged in LDS (words 0..last, 64 bytes of
    // slack after), read instead of HBM and instead of the ring; nullptr:
    // HBM + ring.
    const lu8* lb = nullptr;

    LZ4E_DEV uint32_t load(int32_t wi) const {
        wi = wi < 0 ? 0 : wi;
        wi = wi < last ? wi : last;
        return lb ? ((const lu32*)lb)[wi] : w[wi];
    }
    LZ4E_DEV void put_ring(int32_t s, uint32_t v) const {
        if (lb) return;
        const uint32_t slot = (uint32_t)s & 3;
        ring[slot * 64 + lane] = v;
        if (slot == 0 && lane < kRingPad / 4) ring[kRing / 4 + lane] = v;
    }
    LZ4E_DEV void reload(int32_t p) {
        seg = (p + shift) >> 8;
        base = seg * 256 - shift;
        a = load(seg * 64 + (int32_t)lane);
        b = load(seg * 64 + 64 + (int32_t)lane);
        c = load(seg * 64 + 128 + (int32_t)lane);
        put_ring(seg, a);
        put_ring(seg + 1, b);
        ring_lo = base;
        lockstep();  // other lanes read the ring next
    }
    LZ4E_DEV void slide() {
        a = b;
        b = c;
        seg++;
        base += 256;
        put_ring(seg + 1, b);
        c = load(seg * 64 + 128 + (int32_t)lane);
        const int32_t lo = base - 512;  // segments seg-2 .. seg+1 stay in the ring
        ring_lo = ring_lo > lo ? ring_lo : lo;
        lockstep();  // other lanes read the ring next
    }
    // Byte p of the block (reloads when p is outside [base, base + 512)).
    LZ4E_DEV uint32_t byte(int32_t p) {
        uint32_t r = (uint32_t)(p - base);
        if (r >= 512) {
            if (r < 768) slide();
            else reload(p);
            r = (uint32_t)(p - base);
        }
        const uint32_t w = r < 256 ? lane_val(a, r >> 2) : lane_val(b, (r - 256) >> 2);
        return (w >> ((r & 3) * 8)) & 0xFFu;
    }
    // Length-extension scan, 256 bytes per step: the first block position
    // q >= p0 whose byte is not 255 or that is >= plim (the reference reads
    // such runs one byte at a time, lz4e_decompress.c:201-206, 319-326; a
    // byte at a time cost one v_readlane round trip each).  Bytes past the
    // block read as the clamped last word, never past q's decision: q <= plim
    // and plim lies inside the block.
    LZ4E_DEV int32_t ext_stop(int32_t p0, int32_t plim) {
        for (int32_t p = p0;;) {
            follow(p);  // p in window A = [base, base + 256)
            const int32_t pa = base + 4 * (int32_t)lane;
            uint32_t m = 0;
#pragma unroll
            for (uint32_t t = 0; t < 4; ++t) {
                const int32_t q = pa + (int32_t)t;
                const bool stop = q >= p && (((a >> (8 * t)) & 0xFFu) != 0xFFu || q >= plim);
                m |= (stop ? 1u : 0u) << t;
            }
            const uint64_t bm = ballot(m != 0);
            if (bm) {
                const uint32_t l = ctz64(bm);
                return base + 4 * (int32_t)l + (int32_t)__builtin_ctz(lane_val(m, l));
            }
            p = base + 256;
        }
    }
    // Byte at window offset r (< 512), no range check.
    LZ4E_DEV uint32_t ubyte(uint32_t r) const {
        const uint32_t w = r < 256 ? lane_val(a, r >> 2) : lane_val(b, (r - 256) >> 2);
        return (w >> ((r & 3) * 8)) & 0xFFu;
    }
    // Little-endian 16 bits at window offset r (r + 2 <= 512), no range check.
    LZ4E_DEV uint32_t ule16(uint32_t r) const { return ubyte(r) | (ubyte(r + 1) << 8); }
    // Keep the parse position inside window A.
    LZ4E_DEV void follow(int32_t p) {
        const uint32_t r = (uint32_t)(p - base);
        if (r >= 256 && r < 512) slide();
        else if (r >= 512) reload(p);
    }
    // Little-endian 32 / 16 bits at block position p from the ring
    // (p in [ring_lo, base + 512 - 4 / 2)).
    LZ4E_DEV uint32_t rd4(int32_t p) const { return ld4(at(p)); }
    // LDS address of block byte p (held: see holds); 16 bytes readable from it.
    LZ4E_DEV const lu8* at(int32_t p) const {
        if (lb) return lb + (uint32_t)(p + shift);
        return reinterpret_cast<const lu8*>(ring) + ((uint32_t)(p + shift) & (kRing - 1));
    }
    LZ4E_DEV uint32_t rd16(int32_t p) const { return rd4(p) & 0xFFFFu; }
    // Block bytes [p, p + n) all held by the ring (at ring offsets that may
    // wrap: see wave_lit_ring).
    LZ4E_DEV bool holds(int32_t p, int32_t n) const {
        return lb || (p >= ring_lo && p + n <= base + 512);
    }
    // The ring copy of block bytes [p, p + n), or nullptr when not all held.
    LZ4E_DEV const lu8* in_ring(int32_t p, int32_t n) const {
        if (lb) return lb + (uint32_t)(p + shift);
        if (p < ring_lo || p + n > base + 512) return nullptr;
        const uint32_t i = (uint32_t)(p + shift) & (kRing - 1);
        // contiguous through the mirror, reads of up to 3 bytes past included
        if (i + (uint32_t)n + 3 > kRing + kRingPad) return nullptr;
        return reinterpret_cast<const lu8*>(ring) + i;
    }
};

// a > b for an unsigned a < 2^32 and a signed b (the reference compares
// pointers; b = end - k may lie before the buffer).
LZ4E_DEV bool ugt(uint32_t a, int32_t b) { return b < 0 || a > (uint32_t)b; }

constexpr uint32_t kSat = 0x7FFFFFFFu;  // length saturation: keeps every bound check's outcome

// ---------------------------------------------------------------- HBM copies

LZ4E_DEV uint4 ld16(const uint8_t* p) { return *reinterpret_cast<const uint4*>(p); }
// Global-address-space forms (flat accesses would also count on lgkmcnt,
// coupling them to every LDS wait).
typedef __attribute__((address_space(1))) uint8_t gu8;
typedef __attribute__((address_space(1))) uint32_t gu32w;
LZ4E_DEV uint4 ldg16(const uint8_t* p) {
    const gu32w* q = (const gu32w*)p;
    return make_uint4(q[0], q[1], q[2], q[3]);
}
LZ4E_DEV void stg16(uint8_t* p, uint4 v) {
    gu32w* q = (gu32w*)p;
    q[0] = v.x;
    q[1] = v.y;
    q[2] = v.z;
    q[3] = v.w;
}
LZ4E_DEV void st16(uint8_t* p, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }

// Exact store of n (< 16) bytes of chunk c at p: 8/4/2/1-byte pieces.
LZ4E_DEV void st_tail(uint8_t* p, uint4 c, uint32_t n) {
    uint64_t lo = ((uint64_t)c.y << 32) | c.x, hi = ((uint64_t)c.w << 32) | c.z;
    if (n & 8) {
        *reinterpret_cast<uint64_t*>(p) = lo;
        p += 8;
        lo = hi;
        hi = 0;
    }
    if (n & 4) {
        *reinterpret_cast<uint32_t*>(p) = (uint32_t)lo;
        p += 4;
        lo = (lo >> 32) | (hi << 32);
    }
    if (n & 2) {
        *reinterpret_cast<uint16_t*>(p) = (uint16_t)lo;
        p += 2;
        lo >>= 16;
    }
    if (n & 1) *p = (uint8_t)lo;
}

// Per-lane copy of len (1..64) bytes, src entirely before dst or in another
// buffer: every load is issued before the first store (one round trip).
// Loads never read at or past lim (byte path near the end of a buffer).
LZ4E_DEV void lane_copy64(uint8_t* dst, const uint8_t* src, int32_t len, const uint8_t* lim) {
    const uint32_t nch = ((uint32_t)len + 15) >> 4;
    if (src + 16 * nch > lim) {
        for (int32_t t = 0; t < len; ++t) dst[t] = src[t];
        return;
    }
    const uint4 c0 = ld16(src);
    uint4 c1 = c0, c2 = c0, c3 = c0;
    if (nch > 1) c1 = ld16(src + 16);
    if (nch > 2) c2 = ld16(src + 32);
    if (nch > 3) c3 = ld16(src + 48);
    const uint32_t full = (uint32_t)len >> 4, tail = (uint32_t)len & 15;
    if (full > 0) st16(dst, c0);
    if (full > 1) st16(dst + 16, c1);
    if (full > 2) st16(dst + 32, c2);
    if (full > 3) st16(dst + 48, c3);
    if (tail) {
        const uint4 ct = full == 0 ? c0 : full == 1 ? c1 : full == 2 ? c2 : c3;
        st_tail(dst + 16 * full, ct, tail);
    }
}

// Byte j (< 16) of a 16-byte register pattern.
LZ4E_DEV uint32_t pat_byte(uint4 p, uint32_t j) {
    const uint32_t w = j < 8 ? (j < 4 ? p.x : p.y) : (j < 12 ? p.z : p.w);
    return (w >> ((j & 3) * 8)) & 0xFFu;
}

// Per-lane match copy of len (1..64) bytes at dst with offset off; the bytes
// before dst are final.
LZ4E_DEV void lane_match(uint8_t* dst, uint32_t off, int32_t len, const uint8_t* lim) {
    if ((int32_t)off >= len) {
        lane_copy64(dst, dst - off, len, lim);  // no self-overlap
        return;
    }
    if (off >= 16) {
        // self-overlap with a period >= 16: the first period, then chunks
        // copied from the start, each at most as long as what is written
        lane_copy64(dst, dst - off, (int32_t)off, lim);
        for (int32_t t = (int32_t)off; t < len;) {
            const int32_t c = len - t < t ? len - t : t;
            lane_copy64(dst + t, dst, c, lim);
            t += c;
        }
        return;
    }
    if (off == 0) {
        for (int32_t t = 0; t < len; ++t) dst[t] = 0;
        return;
    }
    // 1 <= off < 16: repeat the final period [dst-off, dst) 4 bytes at a time
    // (the 16-byte load may cover bytes at/after dst: never used)
    if (dst - off + 16 > lim) {
        for (int32_t t = 0; t < len; ++t) dst[t] = dst[t - (int32_t)off];
        return;
    }
    const uint4 p = ld16(dst - off);
    uint32_t j = 0;
    int32_t t = 0;
    for (; t + 4 <= len; t += 4) {
        uint32_t w = 0;
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
            w |= pat_byte(p, j) << (8 * i);
            j = (j + 1 == off) ? 0 : j + 1;
        }
        *reinterpret_cast<uint32_t*>(dst + t) = w;
    }
    for (; t < len; ++t) {
        dst[t] = (uint8_t)pat_byte(p, j);
        j = (j + 1 == off) ? 0 : j + 1;
    }
}

// Whole-wave copy of len literal bytes (non-overlapping), 16 B per lane.
// With kU > 1 long runs move kU KiB per HBM round trip: a wave's loads wait
// behind its earlier stores (one in-order vmcnt), so 1 KiB steps hold an
// incompressible block's copy at one round trip per KiB.  (The pipelined
// decoder uses 4; the one-wave decoder keeps 1: 16 more VGPRs would cost it
// a wave per SIMD.)
// Progress signal of a long copy (the pipelined decoder's watchdog
// heartbeat, see wait_for); the one-wave decoder passes none.
struct NoBeat {
    LZ4E_DEV void operator()() const {}
};

template <int kU = 1, class Beat = NoBeat>
LZ4E_DEV void wave_copy(uint8_t* dst, const uint8_t* src, int32_t len, uint32_t lane,
                        Beat beat = Beat()) {
    constexpr int32_t kStep = 16 * kWave;
    int32_t k = 16 * (int32_t)lane;
    if constexpr (kU > 1) {
        for (; k + (kU - 1) * kStep + 16 <= len; k += kU * kStep) {
            uint4 v[kU];
#pragma unroll
            for (int j = 0; j < kU; ++j) v[j] = *reinterpret_cast<const uint4*>(src + k + j * kStep);
#pragma unroll
            for (int j = 0; j < kU; ++j) *reinterpret_cast<uint4*>(dst + k + j * kStep) = v[j];
            beat();
        }
    }
    for (; k + 16 <= len; k += 16 * kWave)
        *reinterpret_cast<uint4*>(dst + k) = *reinterpret_cast<const uint4*>(src + k);
    for (int32_t t = (len & ~15) + lane; t < len; t += kWave) dst[t] = src[t];
}

// Whole-wave match copy: out[op + t] = out[op - off + t mod off].
template <class Beat = NoBeat>
LZ4E_DEV void wave_match(uint8_t* out, int32_t op, uint32_t off, int32_t len, uint32_t lane,
                         Beat beat = Beat()) {
    if (off == 0) {
        for (int32_t t = lane; t < len; t += kWave) out[op + t] = 0;
        return;
    }
    const int32_t src = op - (int32_t)off;  // signed: a dictionary source lies before out
    if (off >= 16 * kWave) {
        // each 1 KiB step reads bytes written before the step
        for (int32_t k0 = 0; k0 < len; k0 += 16 * kWave) {
            const int32_t k = k0 + 16 * (int32_t)lane;
            if (k + 16 <= len) {
                *reinterpret_cast<uint4*>(out + op + k) =
                    *reinterpret_cast<const uint4*>(out + src + k);
            } else {
                for (int32_t t = k; t < len && t < k + 16; ++t) out[op + t] = out[src + t];
            }
            wave_fence();
            beat();
        }
        return;
    }
    // off < 1024: period P = off * ceil(1024 / off) >= 1024; the first P bytes
    // come from the final period [op-off, op), the rest from P bytes back.
    // (Measured against 16-byte chunks built in registers from the period
    // and against offset-doubling rounds: both slower on fio4k, 2.73 ->
    // 3.15 / 4.91 ms one-wave: the byte loop's loads all read the final
    // period and issue together.)
    const int32_t P = (int32_t)off * ((16 * kWave + off - 1) / off);
    const int32_t head = len < P ? len : P;
    for (int32_t t = lane; t < head; t += kWave) out[op + t] = out[src + (int32_t)(t % off)];
    wave_fence();
    for (int32_t k0 = P; k0 < len; k0 += 16 * kWave) {
        const int32_t k = k0 + 16 * (int32_t)lane;
        if (k + 16 <= len) {
            *reinterpret_cast<uint4*>(out + op + k) =
                *reinterpret_cast<const uint4*>(out + op + k - P);
        } else {
            for (int32_t t = k; t < len && t < k + 16; ++t) out[op + t] = out[op + t - P];
        }
        wave_fence();
        beat();
    }
}

// ---------------------------------------------------------------- LDS copies
// Unaligned dword LDS accesses (gfx950 DS unaligned mode).  Sources may be
// read up to 3 bytes past their end: the output block is followed by the
// ring, and ring reads start below kRing with the kRingPad mirror after it.

// One piece of at most 16 bytes, src + n <= dst or another buffer: four
// dword loads, then the stores, branch-free: a store whose bytes are not
// all wanted goes to the lane's own dword of the sink instead.
LZ4E_DEV void piece16(lu8* dst, const lu8* src, uint32_t n, lu8* sink) {
    const uint32_t w0 = ld4(src), w1 = ld4(src + 4), w2 = ld4(src + 8), w3 = ld4(src + 12);
    st4(n >= 4 ? dst : sink, w0);
    st4(n >= 8 ? dst + 4 : sink, w1);
    st4(n >= 12 ? dst + 8 : sink, w2);
    st4(n >= 16 ? dst + 12 : sink, w3);
    const uint32_t k = n & 12u, r = n & 3u;
    const uint32_t wt = k == 0 ? w0 : (k == 4 ? w1 : (k == 8 ? w2 : w3));
    *(r > 0 ? dst + k : sink) = (uint8_t)wt;
    *(r > 1 ? dst + k + 1 : sink) = (uint8_t)(wt >> 8);
    *(r > 2 ? dst + k + 2 : sink) = (uint8_t)(wt >> 16);
}

// The store half of piece16: n (<= 16) bytes of v at dst.
LZ4E_DEV void put16(lu8* dst, uint4 v, uint32_t n, lu8* sink) {
    st4(n >= 4 ? dst : sink, v.x);
    st4(n >= 8 ? dst + 4 : sink, v.y);
    st4(n >= 12 ? dst + 8 : sink, v.z);
    st4(n >= 16 ? dst + 12 : sink, v.w);
    const uint32_t k = n & 12u, r = n & 3u;
    const uint32_t wt = k == 0 ? v.x : (k == 4 ? v.y : (k == 8 ? v.z : v.w));
    *(r > 0 ? dst + k : sink) = (uint8_t)wt;
    *(r > 1 ? dst + k + 1 : sink) = (uint8_t)(wt >> 8);
    *(r > 2 ? dst + k + 2 : sink) = (uint8_t)(wt >> 16);
}

// len zero bytes (offset-0 matches: the reference writes zeros).
LZ4E_DEV void lane_zero(lu8* dst, int32_t len, lu8* sink) {
    for (int32_t t = 0; t < len; t += 16)
        put16(dst + t, make_uint4(0, 0, 0, 0), (uint32_t)(len - t < 16 ? len - t : 16), sink);
}

// Chains of dependent matches (a match whose source is the output of an
// earlier, still pending one) by pointer jumping over span bytes: every byte
// of a pending match points at the byte it copies (x - off), every other byte
// of [lo_i, hi_i) is final; each whole-wave round either copies a byte whose
// target is final or jumps it to its target's target, so a chain of depth d
// takes about log2(d) rounds.  Targets lie at or after lo_i (the parts before
// the batch were copied from HBM first).  Returns the number of rounds.
LZ4E_DEV uint32_t resolve_chains(lu8* span, lu16* jump, int32_t lo_i, int32_t hi_i, int32_t s0,
                                 bool mine, int32_t ms, int32_t m, int32_t off, uint32_t lane) {
    for (int32_t i = lo_i + (int32_t)lane; i < hi_i; i += kWave) jump[i] = kFinal;
    wave_fence();
    if (mine) {
        for (int32_t t = 0; t < m; ++t) {
            if (off != 0) jump[ms + t] = (uint16_t)(ms + t - off);
            else span[ms + t] = 0;  // offset 0: zeros, final
        }
    }
    wave_fence();
    uint32_t rounds = 0;
    for (;;) {
        bool more = false;
        for (int32_t i = s0 + (int32_t)lane; i < hi_i; i += kWave) {
            const uint32_t y = jump[i];
            if (y != kFinal) {
                const uint32_t z = jump[y];
                if (z == kFinal) {
                    span[i] = span[y];
                    jump[i] = kFinal;
                } else {
                    jump[i] = (uint16_t)z;
                    more = true;
                }
            }
        }
        wave_fence();
        rounds++;
        if (!ballot(more)) break;
    }
    return rounds;
}

// Per-lane copy of len bytes, non-overlapping, in 16-byte pieces.
LZ4E_DEV void lane_copy(lu8* dst, const lu8* src, int32_t len, lu8* sink) {
    for (int32_t t = 0; t < len; t += 16) {
        const int32_t c = len - t < 16 ? len - t : 16;
        piece16(dst + t, src + t, (uint32_t)c, sink);
    }
}

// Per-lane match copy of len bytes at dst with offset off >= 1 (any
// overlap), in pieces whose source is already final: piece [t, t + c) comes
// from D bytes back, D a multiple of off with c <= D <= t (first piece: D =
// off, from before dst); D doubles while 2D <= t.
LZ4E_DEV void lane_match(lu8* dst, uint32_t off, int32_t len, lu8* sink) {
    int32_t t = 0, D = (int32_t)off;
    while (t < len) {
        int32_t c = len - t < 16 ? len - t : 16;
        c = c < D ? c : D;
        piece16(dst + t, dst + t - D, (uint32_t)c, sink);
        t += c;
        if (2 * D <= t) D *= 2;
    }
}

// Per-lane copy of len (1..64) bytes from HBM into LDS (loads never read
// at or past lim).
LZ4E_DEV void lane_copy64(lu8* dst, const uint8_t* src, int32_t len, const uint8_t* lim) {
    const uint32_t nch = ((uint32_t)len + 15) >> 4;
    if (src + 16 * nch > lim) {
        for (int32_t t = 0; t < len; ++t) dst[t] = src[t];
        return;
    }
    uint4 c[4];
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) c[i] = i < nch ? ld16(src + 16 * i) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        const uint32_t w[4] = {c[i].x, c[i].y, c[i].z, c[i].w};
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t k = 16 * i + 4 * j;
            if (k + 4 <= (uint32_t)len) {
                st4(dst + k, w[j]);
            } else if (k < (uint32_t)len) {
                for (uint32_t q = 0; k + q < (uint32_t)len; ++q) dst[k + q] = (uint8_t)(w[j] >> (8 * q));
            }
        }
    }
}

// ---------------------------------------------------------------- parse helpers

// Byte x (< 256) of a 256-byte table held one dword per lane (ds_bpermute).
LZ4E_DEV uint32_t table_at(uint32_t tab, uint32_t x) {
    return (shfl_addr(tab, x & 0xFCu) >> ((x & 3) * 8)) & 0xFFu;
}

// The composed table B[A[p]] for this lane's 4 positions p: four gathers of
// the source dwords (byte address = index & ~3), the wanted bytes picked and
// packed by two v_perm_b32.
LZ4E_DEV uint32_t table_compose(uint32_t A, uint32_t B) {
    const uint32_t a = A & 0xFCFCFCFCu;
    const uint32_t g0 = shfl_addr(B, a & 0xFFu), g1 = shfl_addr(B, (a >> 8) & 0xFFu);
    const uint32_t g2 = shfl_addr(B, (a >> 16) & 0xFFu), g3 = shfl_addr(B, a >> 24);
    const uint32_t s = A & 0x03030303u;
    const uint32_t r01 = perm_bytes(g1, g0, (s & 0xFFFFu) + 0x0C0C0400u);
    const uint32_t r23 = perm_bytes(g3, g2, (s >> 16) + 0x0C0C0400u);
    return r01 | (r23 << 16);
}


// ---------------------------------------------------------------- the parse

// Parse state of one block: wave-uniform scalars plus the input window.
struct Parse {
    InWindow win;
    int32_t iend, oend, shortiend, shortoend;
    int32_t ip, op;
    int32_t D;  // dictionary bytes before the output (<= 65536; 0: noDict)
    bool done;  // the final literal run has been parsed

    // lin (small blocks, srcSize <= kSmallOut): stage the whole block into
    // these kSmallBuf bytes of LDS first, one round trip for all its loads.
    // (ip0, op0): resume at a sequence boundary (the group decoder's hand-over)
    LZ4E_DEV void init(const uint8_t* in, int32_t srcSize, int32_t outSize, lu32* ring,
                       uint32_t lane, int32_t dict = 0, lu8* lin = nullptr, int32_t ip0 = 0,
                       int32_t op0 = 0) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(in);
        win.shift = (int32_t)(a & 3);
        win.w = (gcu32*)(a - win.shift);
        win.last = (srcSize + win.shift - 1) >> 2;
        win.lane = lane;
        win.ring = ring;
        win.lb = nullptr;
        if (lin) {
            constexpr int kR = (kSmallOut + 4 + 16 * kWave - 1) / (16 * kWave);
            uint32_t v[kR][4];
#pragma unroll
            for (int r = 0; r < kR; ++r)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int32_t wi = 4 * ((int32_t)lane + r * (int32_t)kWave) + q;
                    v[r][q] = win.w[wi < win.last ? wi : win.last];
                }
#pragma unroll
            for (int r = 0; r < kR; ++r) {
                const int32_t wi = 4 * ((int32_t)lane + r * (int32_t)kWave);
                if (wi <= win.last) {
                    lu32* d = (lu32*)lin + wi;
                    d[0] = v[r][0];
                    d[1] = v[r][1];
                    d[2] = v[r][2];
                    d[3] = v[r][3];
                }
            }
            lockstep();  // every lane reads the staged words next
            win.lb = lin;
        }
        win.reload(ip0);
        iend = srcSize;
        oend = outSize;
        shortiend = iend - 14 - 2;  // :100-101
        shortoend = oend - 14 - 18; // :102-103
        ip = ip0;
        op = op0;
        D = dict;
        done = false;
    }
};

// One parsed batch: lane k < n holds sequence k (literal source, literal
// length, output position, offset, match length; the final literal run has
// match length 0).
struct Batch {
    int32_t ls = 0, L = 0, op = 0, off = 0, M = 0;
    uint32_t n = 0;
};

enum ParseResult { kParsedFast, kParsedScalar, kParseFail };

// The next batch of the token stream, with every bound check of the
// reference in its order (lz4e_decompress.c:123-446).  kParsedFast: up to 64
// sequences without extension bytes, far from both block ends (each literal
// run <= 14, match length <= 18, output <= 32 bytes per sequence); with kExt
// also sequences whose length fields carry one extension byte below
// kExtByteMax (literal run <= 46, match <= 50 bytes), further from the ends;
// kParsedScalar: one sequence of any length; kParseFail: malformed input or
// too small a capacity, the return value is -(P.ip) - 1.  A fast batch's
// output is at most cap_out (>= 32) bytes.
struct NoLap {
    LZ4E_DEV void operator()(int) const {}
};
constexpr uint32_t kExtByteMax = 32;  // fast literal runs <= 46, matches <= 50 bytes
// LZ4E_FAST_EXT=0 builds the decoders without extension sequences on the
// fast path (A/B experiments).
#ifndef LZ4E_FAST_EXT
#define LZ4E_FAST_EXT 0
#endif
constexpr bool kFastExt = LZ4E_FAST_EXT;

// Window offset (from ip) of the token after the one at offset p, for the
// fast path: token t, e1 the byte after it; 255 when the sequence cannot be
// on the fast path (without kExt: any extension byte; with kExt: a 255
// extension byte, or one of kExtByteMax and more).  A match-length
// extension byte is read from the ring (offsets past the window read stale
// ring bytes: the result then exceeds 254 and is declined by the caller).
template <bool kExt>
LZ4E_DEV uint32_t fast_next(uint32_t t, uint32_t e1, uint32_t p, const InWindow& win, int32_t ip) {
    const uint32_t Lt = t >> 4, Mt = t & 15;
    if constexpr (!kExt) {
        return (Lt != 15 && Mt != 15) ? p + Lt + 3 : 255u;
    } else {
        if (Lt == 15 && e1 >= kExtByteMax) return 255u;
        const uint32_t q = Lt == 15 ? p + 2 + 15 + e1 : p + 1 + Lt;  // the offset's position
        if (Mt != 15) return q + 2;
        if (q + 2 > 253) return 255u;
        const uint32_t e2 = win.rd4(ip + (int32_t)(q + 2)) & 0xFFu;
        return e2 < kExtByteMax ? q + 3 : 255u;
    }
}
// kVecExt: length-extension runs by 256-byte vector scans (the pipelined
// decoder; the one-wave decoder keeps the byte loop: 2 more VGPRs would cost
// it a wave per SIMD, and its <= 16 KiB blocks hold short runs).
// The one-wave decoder's choice; the CPU lane emulator's test build turns it
// on (-DLZ4E_ONEWAVE_VEC_EXT=true) so that the vector scan runs under ASan
// against the oracle (tests/test_emulator.py).
#ifndef LZ4E_ONEWAVE_VEC_EXT
#define LZ4E_ONEWAVE_VEC_EXT false
#endif
constexpr bool kOneWaveVecExt = LZ4E_ONEWAVE_VEC_EXT;
template <bool kVecExt = false, bool kExt = false, class Lap = NoLap>
LZ4E_DEV ParseResult parse_batch(Parse& P, Batch& b, uint32_t lane, int32_t cap_out = 64 * 32,
                                 Lap lap = Lap()) {
    const int32_t iend = P.iend, oend = P.oend;
    int32_t ip = P.ip, op = P.op;
    InWindow& win = P.win;

    // Fast path: a run of tokens with no length-extension bytes, far from
    // both block ends, where the reference takes its two-stage shortcut
    // (:150-191).  The token chain inside the 256-byte window at ip is found
    // by pointer doubling: jump tables J_{2^i} (window offset -> offset 2^i
    // tokens on, 255 = chain end; one byte per position, lane l holding
    // positions 4l..4l+3) are composed with ds_bpermute gathers, then lane k
    // follows the bits of k to token k.  Every field and check is then
    // evaluated per lane.
    bool fast = ip <= iend - 18 && op <= oend - 32;
    uint32_t wv = 0;
    if (fast) {
        win.follow(ip);
        wv = win.rd4(ip + 4 * (int32_t)lane);
        // A batch that starts at a token the fast path cannot take -- every
        // such token ends the fast batch before it -- is the scalar path's:
        // lane 0's token would fail `cand` below, so no tables are composed.
        const uint32_t w0 = lane_val(wv, 0);
        fast = fast_next<kExt>(w0 & 0xFFu, (w0 >> 8) & 0xFFu, 0, win, ip) <= 254;
    }
    if (fast) {
        const int32_t r0 = ip - win.base;                  // < 256
        const int32_t rin = iend - 18 - win.base;          // last token offset on the fast path
        const int32_t jlim = (rin < 494 ? rin : 494) - r0;  // (offset bytes stay in A+B)
        uint32_t J[6];
        {
            uint32_t j1 = 0;
            const uint32_t wn = kExt ? shfl(wv, lane + 1) : 0u;  // byte 0: the byte after q = 3
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
                const uint32_t t = (wv >> (8 * q)) & 0xFFu, p = 4 * lane + q;
                const uint32_t e1 = q < 3 ? (wv >> (8 * q + 8)) & 0xFFu : wn & 0xFFu;
                const uint32_t n = fast_next<kExt>(t, e1, p, win, ip);
                // an extension sequence also ends before jlim (its bytes stay
                // in the window; the end checks of the general path hold)
                const bool ext = kExt && ((t >> 4) == 15 || (t & 15) == 15);
                const bool go = (int32_t)p <= jlim && n <= 254 && (!ext || (int32_t)n <= jlim);
                j1 |= (go ? n : 255u) << (8 * q);
            }
            J[0] = j1;
        }
        lap(0);
#pragma unroll
        for (int i = 1; i < 6; ++i) J[i] = table_compose(J[i - 1], J[i - 1]);
        lap(1);
        uint32_t x = 0;  // lane k: window offset of token k (255: past the chain)
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const uint32_t y = table_at(J[i], x);
            x = (lane >> i) & 1 ? y : x;
        }
        lap(2);
        const uint32_t t = table_at(wv, x);  // token byte
        const int32_t Lt = (int32_t)(t >> 4), Mt = (int32_t)(t & 15);
        int32_t L = Lt, M = Mt + 4, lp = ip + (int32_t)x + 1;  // literal start
        bool cand, ext = false;
        int32_t off, nxt;
        if constexpr (kExt) {
            // one extension byte per field at most (fast_next's rule)
            const uint32_t e1 = table_at(wv, x + 1);  // (x <= 251 when cand)
            if (Lt == 15) {
                L = 15 + (int32_t)e1;
                lp++;
            }
            const uint32_t ow = win.rd4(lp + L);  // offset, then the match extension byte
            off = (int32_t)(ow & 0xFFFFu);
            const uint32_t e2 = (ow >> 16) & 0xFFu;
            if (Mt == 15) M = 19 + (int32_t)e2;
            nxt = lp + L + 2 + (Mt == 15 ? 1 : 0);
            ext = Lt == 15 || Mt == 15;
            cand = x != 255 && (int32_t)x <= jlim && (Lt != 15 || e1 < kExtByteMax) &&
                   (Mt != 15 || e2 < kExtByteMax) && (!ext || nxt - ip <= jlim);
            off = cand ? off : 0;
        } else {
            cand = x != 255 && Lt != 15 && Mt != 15 && (int32_t)x <= jlim;
            off = cand ? (int32_t)win.rd16(lp + L) : 0;
            nxt = lp + L + 2;
        }
        const int32_t size = cand ? L + M : 0;
        const int32_t incl = (int32_t)wave_incl_add((uint32_t)size);
        const int32_t o_k = op + incl - size;
        const int32_t m_k = o_k + L;
        // the reference's checks on this path: shortcut entry (op <= oend-32,
        // input side guaranteed by jlim), match inside the block (:299-302),
        // and for offsets < 8 the _copy_match end check (:422-431); a source
        // in the dictionary takes _copy_match: offset inside dictionary +
        // block (:299-302), then the extDict end check (:341-346).  An
        // extension sequence takes the general path (:194-336): its output
        // ending 32 bytes before oend passes every end check there.
        const bool ok = cand && o_k <= oend - 32 && incl <= cap_out &&
                        (!ext || o_k + size <= oend - 32) &&
                        (m_k >= off ? (off >= 8 || m_k + M <= oend - 5)
                                    : (m_k - off + P.D >= 0 && m_k + M <= oend - 5));
        const uint64_t okm = ballot(ok);
        const uint32_t nf = (~okm) ? ctz64(~okm) : kWave;  // first failing lane
        if (nf > 0) {
            b.ls = lp;
            b.L = L;
            b.op = o_k;
            b.off = off;
            b.M = M;
            b.n = nf;
            P.op = op + lane_val((uint32_t)incl, nf - 1);
            P.ip = lane_val((uint32_t)nxt, nf - 1);  // the token after the last one
            lap(3);
            return kParsedFast;
        }
    }

    // Exact scalar path (extension bytes, block ends, anything the fast path
    // declined): one sequence.
    win.follow(ip);  // ip now in window A: bytes up to ip + 256 are readable unchecked
    const uint32_t r0 = (uint32_t)(ip - win.base);
    const uint32_t token = win.ubyte(r0);
    ip++;
    uint32_t length = token >> 4;  // saturates at kSat
    int32_t offset = 0, lit_ip, lit_op;
    uint32_t L;

    if (length != 15 && ip < P.shortiend && op <= P.shortoend) {
        // Two-stage shortcut (:150-191): literals 0..14 fit, offset read.
        lit_ip = ip;
        lit_op = op;
        L = length;
        offset = (int32_t)win.ule16(r0 + 1 + length);
        op += (int32_t)length;
        ip += (int32_t)length + 2;
        length = token & 15;
        if (length != 15 && offset >= 8 && op >= offset) {
            // 18-byte shortcut copy: match length 4..18, no checks left
            length += 4;
            goto record;
        }
        goto copy_match_checks;
    }
    if (length == 15) {  // :194-220
        if (ip >= iend - 15) goto fail;
        if constexpr (kVecExt) {
            // bytes ip .. q: 255 each, then s; the loop goes on while the
            // next position is below iend - 15
            const int32_t q = win.ext_stop(ip, iend - 16);
            const uint64_t sum = (uint64_t)length + 255ull * (uint64_t)(q - ip) + win.byte(q);
            length = sum > kSat ? kSat : (uint32_t)sum;
            ip = q + 1;
        } else {
            uint32_t s;
            do {
                s = win.byte(ip);
                ip++;
                length = length + s > kSat ? kSat : length + s;
            } while (ip < iend - 15 && s == 255);
        }
    }
    {
        const uint32_t cpy = (uint32_t)op + length;  // :223-288
        const uint32_t iln = (uint32_t)ip + length;
        lit_ip = ip;
        lit_op = op;
        L = length;
        if (ugt(cpy, oend - 12) || ugt(iln, iend - 8)) {
            if (iln != (uint32_t)iend || ugt(cpy, oend)) goto fail;
            ip += (int32_t)length;
            op += (int32_t)length;
            length = 0;
            P.done = true;  // final literal run: no match
            goto record;
        }
        ip += (int32_t)length;
        op = (int32_t)cpy;
    }
    offset = (int32_t)(win.byte(ip) | (win.byte(ip + 1) << 8));  // :291-296
    ip += 2;
    length = token & 15;

copy_match_checks:
    // _copy_match (:298-336, :422-431); with a dictionary the source may lie
    // up to D bytes before the output (:299-302, checkOffset)
    if (op - offset + P.D < 0) goto fail;
    if (length == 15) {
        // bytes ip .. q: 255 each, then s; reading a byte at or past
        // iend - 5 fails (ip > iend - 5 after the read)
        if constexpr (kVecExt) {
            const int32_t q = win.ext_stop(ip, iend - 5);
            if (q + 1 > iend - 5) {
                ip = q + 1;
                goto fail;
            }
            const uint64_t sum = (uint64_t)length + 255ull * (uint64_t)(q - ip) + win.byte(q);
            length = sum > kSat ? kSat : (uint32_t)sum;
            ip = q + 1;
        } else {
            uint32_t s;
            do {
                s = win.byte(ip);
                ip++;
                if (ip > iend - 5) goto fail;
                length = length + s > kSat ? kSat : length + s;
            } while (s == 255);
        }
    }
    if (ugt((uint32_t)op + length + 4, oend - 5)) goto fail;
    length += 4;

record:
    {
        const bool me = lane == 0;
        b.ls = me ? lit_ip : 0;
        b.L = me ? (int32_t)L : 0;
        b.op = me ? lit_op : 0;
        b.off = me ? offset : 0;
        b.M = me ? (int32_t)length : 0;
        b.n = 1;
    }
    P.op = op + (int32_t)length;
    P.ip = ip;
    return kParsedScalar;
fail:
    P.ip = ip;
    return kParseFail;
}

// ---------------------------------------------------------------- batch copies

// Copies of a scalar-path batch (one sequence, any length) in HBM: the
// literal run, then the match; same-wave stores and loads to one global
// address are ordered by the hardware (one vector L1 per CU) and the
// wavefront fences keep the compiler from moving loads above the stores.
template <int kU = 1, class Beat = NoBeat>
LZ4E_DEV void copy_scalar_hbm(const Batch& b, const uint8_t* in, int32_t srcSize, uint8_t* gout,
                              int32_t outSize, uint32_t lane, Beat beat = Beat()) {
    const int32_t L = lane_val((uint32_t)b.L, 0), op = lane_val((uint32_t)b.op, 0);
    const int32_t ls = lane_val((uint32_t)b.ls, 0);
    const int32_t M = lane_val((uint32_t)b.M, 0), off = lane_val((uint32_t)b.off, 0);
    wave_fence();
    if (L > 0 && L <= kLongPiece) {
        if (lane == 0) lane_copy64(gout + op, in + ls, L, in + srcSize);
    } else if (L > kLongPiece) {
        wave_copy<kU>(gout + op, in + ls, L, lane, beat);
    }
    wave_fence();
    const int32_t ms = op + L;
    if (M > 0 && M <= kLongPiece) {
        if (lane == 0) lane_match(gout + ms, (uint32_t)off, M, gout + outSize);
    } else if (M > kLongPiece) {
        wave_match(gout, ms, (uint32_t)off, M, lane, beat);
    }
    wave_fence();
}

// ---------------------------------------------------------------- block-per-group decoder
// Large batches of small blocks whose sequences are long (fio-style 4 KiB
// buffers: ~14 sequences of ~300 bytes) leave the one-wave decoder parsing
// one scalar sequence at a time with the other 63 lanes idle: ~24 k issue
// cycles per block (tools/wavestamps.py).  Here a group of kGroup lanes
// decodes a block of its own (64 / kGroup blocks per wave): the reference's
// scalar loop (lz4e_decompress.c:123-446, the same checks in the same order
// as parse_batch's exact path, so values and error codes are the
// reference's), run by every lane of the group, with each literal run and
// match copied by the whole group, up to 256 bytes per round.  Round 4's
// version ran one block per lane with 16-byte copies per lane (fio4k 1.39
// ms); groups of 8 lanes take 0.88-0.89 ms (groups of 2 / 4 / 16 / 32: 1.10
// / 0.91 / 0.94 / 1.42 ms, profiles/r05/group_decoder/).

typedef __attribute__((address_space(1))) const uint8_t gcu8;
LZ4E_DEV uint32_t ldb(const uint8_t* p, int32_t i) { return ((gcu8*)p)[i]; }
// Global-address-space stores of the group decoder (flat ones would also
// count on lgkmcnt and make every wait a wait for both counters).
typedef __attribute__((address_space(1))) uint64_t gu64w;
typedef __attribute__((address_space(1))) uint16_t gu16w;
LZ4E_DEV void gst_tail(uint8_t* p, uint4 c, uint32_t n) {
    uint64_t lo = ((uint64_t)c.y << 32) | c.x, hi = ((uint64_t)c.w << 32) | c.z;
    if (n & 8) {
        *(gu32w*)p = (uint32_t)lo;
        *(gu32w*)(p + 4) = (uint32_t)(lo >> 32);
        p += 8;
        lo = hi;
        hi = 0;
    }
    if (n & 4) {
        *(gu32w*)p = (uint32_t)lo;
        p += 4;
        lo = (lo >> 32) | (hi << 32);
    }
    if (n & 2) {
        *(gu16w*)p = (uint16_t)lo;
        p += 2;
        lo >>= 16;
    }
    if (n & 1) *(gu8*)p = (uint8_t)lo;
}

// A lane's 16-byte window of its input (token, extension and offset bytes
// mostly come from one load): bytes [base, base + 16) in w.
struct LaneIn {
    const uint8_t* in;
    int32_t n, base;
    uint4 w;
    LZ4E_DEV void fill(int32_t p) {
        base = p;
        if (p + 16 <= n) {
            w = ldg16(in + p);
        } else {
            uint32_t x[4] = {0, 0, 0, 0};
#pragma unroll
            for (int32_t k = 0; k < 16; ++k)
                if (p + k < n) x[k >> 2] |= ldb(in, p + k) << (8 * (k & 3));
            w = make_uint4(x[0], x[1], x[2], x[3]);
        }
    }
    // byte p (< n)
    LZ4E_DEV uint32_t byte(int32_t p) {
        if ((uint32_t)(p - base) >= 16) fill(p);
        return pat_byte(w, (uint32_t)(p - base));
    }
};

// A group whose block turns out to hold short sequences (fewer than
// kLaneBailBytes output bytes per sequence over the last kLaneBailSeqs
// sequences: text, tables) hands the block over at a sequence boundary --
// such a block would hold its wave for milliseconds: group_decode returns
// kLaneHandOver with (*ip_out, *op_out), and the one-wave decoder resumes
// there (a group pays a few round trips per sequence, which only long
// sequences amortise).
constexpr int32_t kLaneHandOver = INT32_MIN;
#ifndef LZ4E_LANE_BAIL_SEQS
#define LZ4E_LANE_BAIL_SEQS 4
#endif
#ifndef LZ4E_LANE_FIRST_LIT
#define LZ4E_LANE_FIRST_LIT 200
#endif
constexpr int32_t kLaneBailSeqs = LZ4E_LANE_BAIL_SEQS;
constexpr int32_t kLaneBailBytes = 64;
constexpr uint32_t kLaneFirstLit = LZ4E_LANE_FIRST_LIT;  // (fio-style: 256)
// A literal run or a match piece of up to 256 bytes leaves in kPer 16-byte
// loads and stores per lane, contiguous per block.  The group's lanes run the
// same scalar parse (their input window loads are one address per group).
// s: the lane's index in its group; dst and src are the group's.

// LZ4E_GROUP: lanes per block (2 .. 16, a power of two; experiments).
#ifndef LZ4E_GROUP
#define LZ4E_GROUP 8
#endif
constexpr uint32_t kGroup = LZ4E_GROUP;
// A round moves up to 256 bytes of a block: kPer 16-byte chunks per lane,
// every load of the round issued before its first store (loads and stores
// share one in-order counter, so a load after a store waits for the store).
constexpr int32_t kRound = 256;
constexpr uint32_t kPer = kRound / (16 * kGroup);
static_assert(kGroup >= 2 && kGroup <= 16 && (kGroup & (kGroup - 1)) == 0 && kPer * 16 * kGroup == kRound,
              "lanes per block: 2 .. 16, a power of two (the emulator's group barriers exist for 2 .. 32)");

// Literal run: dst[t] = src[t] for t in [0, len), src a different buffer;
// loads never read at or past lim.
// 16 bytes at p (n of them wanted), byte by byte where a 16-byte load
// would reach lim.
LZ4E_DEV uint4 ld16_lim(const uint8_t* p, uint32_t n, const uint8_t* lim) {
    if (p + 16 <= lim) return ldg16(p);
    uint32_t x[4] = {0, 0, 0, 0};
    for (uint32_t k = 0; k < n; ++k) x[k >> 2] |= ldb(p, (int32_t)k) << (8 * (k & 3));
    return make_uint4(x[0], x[1], x[2], x[3]);
}
LZ4E_DEV void st16_n(uint8_t* p, uint4 v, uint32_t n) {
    if (n == 16) stg16(p, v);
    else gst_tail(p, v, n);
}

LZ4E_DEV void group_copy(uint8_t* dst, const uint8_t* src, int32_t len, const uint8_t* lim, uint32_t s) {
    for (int32_t t0 = 0; t0 < len; t0 += kRound) {
        uint4 v[kPer];
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
            const int32_t q = t0 + 16 * (int32_t)(s + kGroup * i);
            if (q < len) v[i] = ld16_lim(src + q, (uint32_t)(len - q < 16 ? len - q : 16), lim);
        }
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
            const int32_t q = t0 + 16 * (int32_t)(s + kGroup * i);
            if (q < len) st16_n(dst + q, v[i], (uint32_t)(len - q < 16 ? len - q : 16));
        }
    }
}

// 16 bytes of the period p (off < 16 bytes, pattern byte j = p's byte j)
// starting at phase j0.
LZ4E_DEV uint4 period16(uint4 p, uint32_t off, uint32_t j0) {
    uint32_t w[4] = {0, 0, 0, 0};
    uint32_t j = j0;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
        w[k >> 2] |= pat_byte(p, j) << (8 * (k & 3));
        j = (j + 1 == off) ? 0 : j + 1;
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Match: dst[t] = dst[t - off] for t in [0, len), any overlap (offset 0:
// zeros).  Periods below 16: every lane builds its 16-byte pieces from the
// period in registers (one pass); otherwise pieces [t, t + c) from D bytes
// back, D a multiple of off with c <= D <= t (doubling, up to 256 bytes a
// piece), so every source byte is written before its piece is read (same-wave
// stores and loads to one address are ordered; group_fence keeps the compiler
// from moving the loads up).  Loads never read at or past lim.
LZ4E_DEV void group_match(uint8_t* dst, uint32_t off, int32_t len, const uint8_t* lim, uint32_t s) {
    if (off == 0 || off < 16) {
        uint4 p = make_uint4(0, 0, 0, 0);
        if (off != 0) {
            if (dst - off + 16 <= lim) {
                p = ldg16(dst - off);
            } else {
                uint32_t x[4] = {0, 0, 0, 0};
                for (uint32_t k = 0; k < off; ++k) x[k >> 2] |= ldb(dst, (int32_t)k - (int32_t)off) << (8 * (k & 3));
                p = make_uint4(x[0], x[1], x[2], x[3]);
            }
        }
        for (int32_t t = 16 * (int32_t)s; t < len; t += 16 * (int32_t)kGroup) {
            const uint32_t n = (uint32_t)(len - t < 16 ? len - t : 16);
            const uint4 v = off == 0 ? make_uint4(0, 0, 0, 0) : period16(p, off, (uint32_t)t % off);
            st16_n(dst + t, v, n);
        }
        return;
    }
    uint32_t D = off;
    for (int32_t t = 0; t < len;) {
        int32_t c = len - t < (int32_t)D ? len - t : (int32_t)D;
        c = c < kRound ? c : kRound;
        uint4 v[kPer];
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
            const int32_t q = 16 * (int32_t)(s + kGroup * i);
            if (q < c) v[i] = ld16_lim(dst + t + q - (int32_t)D, (uint32_t)(c - q < 16 ? c - q : 16), lim);
        }
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
            const int32_t q = 16 * (int32_t)(s + kGroup * i);
            if (q < c) st16_n(dst + t + q, v[i], (uint32_t)(c - q < 16 ? c - q : 16));
        }
        group_fence(kGroup);
        t += c;
        while (2 * D <= (uint32_t)t) D *= 2;
    }
}

// One block on one group: the return value of LZ4E_decompress_safe (D
// dictionary bytes before out), or kLaneHandOver with (*ip_out, *op_out).
LZ4E_DEV int32_t group_decode(const uint8_t* in, int32_t srcSize, uint8_t* out, int32_t outSize,
                              int32_t D, bool may_bail, int32_t* ip_out, int32_t* op_out, uint32_t s) {
    const int32_t iend = srcSize, oend = outSize;
    const int32_t shortiend = iend - 14 - 2, shortoend = oend - 14 - 18;  // :100-103
    const uint8_t* ilim = in + srcSize;
    const uint8_t* olim = out + outSize;
    int32_t ip = 0, op = 0;
    LaneIn I;
    I.in = in;
    I.n = srcSize;
    I.fill(0);
    if (may_bail) {
        // a block that opens with a short literal run is most likely one of
        // short sequences: straight to the one-wave decoder (nor does one
        // whose first match is short: both must be long)
        const uint32_t t0 = I.byte(0);
        const uint32_t l0 = (t0 >> 4) == 15 && srcSize > 1 ? 15 + I.byte(1) : t0 >> 4;
        const int32_t q = 2 + (int32_t)l0 + 2;  // the first match's extension byte
        const bool long_m = l0 >= kLaneFirstLit && (t0 & 15) == 15 && q < srcSize && I.byte(q) >= 64 - 19;
        if (!long_m) {
            *ip_out = 0;
            *op_out = 0;
            return kLaneHandOver;
        }
    }
    int32_t op_chk = 0;  // output position at the last check
    for (int32_t nseq = 0;; ++nseq) {
        if (may_bail && nseq >= kLaneBailSeqs && nseq % kLaneBailSeqs == 0) {
            if (op - op_chk >= kLaneBailBytes * kLaneBailSeqs) {
                op_chk = op;
            } else {
                *ip_out = ip;
                *op_out = op;
                return kLaneHandOver;
            }
        }
        const uint32_t token = I.byte(ip);
        ip++;
        uint32_t length = token >> 4;  // saturates at kSat
        int32_t offset;
        if (length != 15 && ip < shortiend && op <= shortoend) {
            // two-stage shortcut (:150-191)
            if (length) group_copy(out + op, in + ip, (int32_t)length, ilim, s);
            op += (int32_t)length;
            ip += (int32_t)length;
            offset = (int32_t)(I.byte(ip) | (I.byte(ip + 1) << 8));
            ip += 2;
            length = token & 15;
            if (length != 15 && offset >= 8 && op >= offset) {
                group_fence(kGroup);
                group_match(out + op, (uint32_t)offset, (int32_t)length + 4, olim, s);
                group_fence(kGroup);
                op += (int32_t)length + 4;
                continue;
            }
        } else {
            if (length == 15) {  // :194-220
                if (ip >= iend - 15) break;
                uint32_t sb;
                do {
                    sb = I.byte(ip);
                    ip++;
                    length = length + sb > kSat ? kSat : length + sb;
                } while (ip < iend - 15 && sb == 255);
            }
            const uint32_t cpy = (uint32_t)op + length;  // :223-288
            const uint32_t iln = (uint32_t)ip + length;
            if (ugt(cpy, oend - 12) || ugt(iln, iend - 8)) {
                if (iln != (uint32_t)iend || ugt(cpy, oend)) break;
                group_copy(out + op, in + ip, (int32_t)length, ilim, s);  // final literal run
                return (int32_t)cpy;
            }
            if ((uint32_t)(ip + (int32_t)length - I.base) + 2 > 16) I.fill(ip + (int32_t)length);
            group_copy(out + op, in + ip, (int32_t)length, ilim, s);
            ip += (int32_t)length;
            op = (int32_t)cpy;
            offset = (int32_t)(I.byte(ip) | (I.byte(ip + 1) << 8));  // :291-296
            ip += 2;
            length = token & 15;
        }
        // _copy_match (:298-336, :422-431)
        if (op - offset + D < 0) break;
        if (length == 15) {
            uint32_t sb;
            bool bad = false;
            do {
                sb = I.byte(ip);
                ip++;
                if (ip > iend - 5) {
                    bad = true;
                    break;
                }
                length = length + sb > kSat ? kSat : length + sb;
            } while (sb == 255);
            if (bad) break;
        }
        if (ugt((uint32_t)op + length + 4, oend - 5)) break;
        group_fence(kGroup);  // the literal run's stores before the match's loads
        group_match(out + op, (uint32_t)offset, (int32_t)length + 4, olim, s);
        group_fence(kGroup);
        op += (int32_t)length + 4;
    }
    return -ip - 1;
}

// ---------------------------------------------------------------- small blocks in LDS
// A block of at most kSmallOut output bytes without a dictionary (4 KiB
// blocks, the drop-in single calls) can keep its whole output in LDS: a
// scalar-path sequence (long literal runs and matches, as in fio-style
// data) then copies LDS to LDS at LDS latency instead of a store, a load
// that waits behind it and another store in HBM per sequence, and the block
// leaves in one pass of 16-byte stores at the end.

// Whole-wave copy of n (<= 1024 per call of a round) bytes of a literal run
// from the input ring (block bytes [p, p + n) held by it): 16 bytes per lane,
// ring offsets wrap through the mirror.
LZ4E_DEV void wave_lit_ring(lu8* dst, const InWindow& w, int32_t p, int32_t n, lu8* sink,
                            uint32_t lane) {
    for (int32_t k = 16 * (int32_t)lane; k < n; k += 16 * (int32_t)kWave)
        piece16(dst + k, w.at(p + k), (uint32_t)(n - k < 16 ? n - k : 16), sink);
}

// Whole-wave copy of n (<= kSmallOut) literal bytes from HBM into LDS: every
// load before the first store (one round trip); loads never read at or past
// srcSize.
LZ4E_DEV void wave_lit_hbm(lu8* dst, const uint8_t* in, int32_t p, int32_t n, int32_t srcSize,
                           lu8* sink, uint32_t lane) {
    constexpr int kR = (kSmallOut + 16 * kWave - 1) / (16 * kWave);
    uint4 v[kR];
#pragma unroll
    for (int j = 0; j < kR; ++j) {
        const int32_t k = 16 * ((int32_t)lane + j * (int32_t)kWave);
        v[j] = (k < n && p + k + 16 <= srcSize) ? ldg16(in + p + k) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < kR; ++j) {
        const int32_t k = 16 * ((int32_t)lane + j * (int32_t)kWave);
        if (k >= n) continue;
        const int32_t c = n - k < 16 ? n - k : 16;
        if (p + k + 16 <= srcSize) put16(dst + k, v[j], (uint32_t)c, sink);
        else
            for (int32_t t = 0; t < c; ++t) dst[k + t] = in[p + k + t];
    }
}

// Whole-wave match copy inside LDS: out[op + t] = out[op + t - off] for t in
// [0, len), any overlap (offset 0: zeros).  Round r copies [t, t + c) from D
// bytes back, D a multiple of off with c <= D <= t + off, so every source
// byte is final before the round; D doubles while 2D <= t (a run of period
// 1 takes ~log2(len) rounds).  The loop is wave-uniform.
LZ4E_DEV void wave_match_lds(lu8* out, int32_t op, uint32_t off, int32_t len, lu8* sink,
                             uint32_t lane) {
    if (off == 0) {
        for (int32_t k = 16 * (int32_t)lane; k < len; k += 16 * (int32_t)kWave)
            put16(out + op + k, make_uint4(0, 0, 0, 0), (uint32_t)(len - k < 16 ? len - k : 16), sink);
        return;
    }
    if (off < 16) {
        // short periods from registers (see wave_match): one LDS read of the
        // final period, then every chunk without waiting on earlier ones
        const lu8* pp = out + op - (int32_t)off;
        const uint4 pv = make_uint4(ld4(pp), ld4(pp + 4), ld4(pp + 8), ld4(pp + 12));
        const uint32_t step = (16u * kWave) % off;
        uint32_t ph = (16u * lane) % off;
        for (int32_t k = 16 * (int32_t)lane; k < len; k += 16 * (int32_t)kWave) {
            uint32_t w[4] = {0, 0, 0, 0}, j = ph;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                w[q >> 2] |= pat_byte(pv, j) << (8 * (q & 3));
                j = j + 1 == off ? 0 : j + 1;
            }
            put16(out + op + k, make_uint4(w[0], w[1], w[2], w[3]), (uint32_t)(len - k < 16 ? len - k : 16), sink);
            ph += step;
            ph = ph >= off ? ph - off : ph;
        }
        return;
    }
    int32_t t = 0, D = (int32_t)off;
    while (t < len) {
        int32_t c = len - t < D ? len - t : D;
        c = c < 16 * (int32_t)kWave ? c : 16 * (int32_t)kWave;
        lu8* d = out + op + t;
        const int32_t k = 16 * (int32_t)lane;
        if (k < c) piece16(d + k, d + k - D, (uint32_t)(c - k < 16 ? c - k : 16), sink);
        lockstep();  // the next round reads these bytes
        t += c;
        while (2 * D <= t) D *= 2;
    }
}

// Copies of a scalar-path batch (one sequence, any length) into the LDS
// output: the literal run from the input ring when it holds it, else from
// HBM, then the match.
LZ4E_DEV void copy_scalar_lds(const Batch& b, const InWindow& win, const uint8_t* in,
                              int32_t srcSize, lu8* obuf, lu8* sink, uint32_t lane) {
    const int32_t L = lane_val((uint32_t)b.L, 0), op = lane_val((uint32_t)b.op, 0);
    const int32_t ls = lane_val((uint32_t)b.ls, 0);
    const int32_t M = lane_val((uint32_t)b.M, 0), off = lane_val((uint32_t)b.off, 0);
    if (L > 0) {
        if (win.holds(ls, L) && (win.lb || L <= 16 * (int32_t)kWave))
            wave_lit_ring(obuf + op, win, ls, L, sink, lane);
        else wave_lit_hbm(obuf + op, in, ls, L, srcSize, sink, lane);
        lockstep();
    }
    if (M > 0) wave_match_lds(obuf, op + L, (uint32_t)off, M, sink, lane);
}

// The LDS output [0, n) to HBM in 16-byte stores (the partial end chunk by
// bytes: nothing past n is written).
LZ4E_DEV void flush_lds(uint8_t* gout, const lu8* obuf, int32_t n, uint32_t lane) {
    for (int32_t c0 = 16 * (int32_t)lane; c0 < n; c0 += 16 * (int32_t)kWave) {
        const lu8* sc = obuf + c0;
        if (c0 + 16 <= n) stg16(gout + c0, make_uint4(ld4(sc), ld4(sc + 4), ld4(sc + 8), ld4(sc + 12)));
        else
            for (int32_t x = c0; x < n; ++x) *(gu8*)(gout + x) = sc[x - c0];
    }
}

struct WaveStamps {
    uint64_t t = 0, acc[4] = {0, 0, 0, 0}, batches = 0, rounds = 0;
};

// Decode one block into HBM on one wave.  LDS: the input ring, the store
// sink, the span buffer of the fast batches and its jump table.  kLdsOut:
// the whole output is assembled in obuf (kSmallBuf bytes; outSize <=
// kSmallOut, no dictionary) and stored at the end; a fast batch's span is
// then obuf itself.
template <bool kStamps, bool kLdsOut = false>
LZ4E_DEV void decode_block(const uint8_t* in, int32_t srcSize, uint8_t* gout, int32_t outSize,
                           int32_t* ret_slot, uint64_t* dbg, uint32_t lane, lu8* span_buf,
                           lu32* ring, lu16* jump, int32_t dict, lu8* sinkb, lu8* obuf = nullptr,
                           lu8* lin = nullptr, int32_t ip0 = 0, int32_t op0 = 0) {
    WaveStamps st;
    [[maybe_unused]] uint64_t t_start = 0, r_start = 0;
    if constexpr (kStamps) {
        t_start = clock64();
        r_start = realtime64();
    }
    auto lap = [&](int ph) {
        if constexpr (kStamps) {
            const uint64_t now = clock64();
            st.acc[ph] += now - st.t;
            st.t = now;
        }
    };
    if constexpr (kStamps) st.t = clock64();
    lu8* sink = sinkb + 4 * lane;
    Parse P;
    P.init(in, srcSize, outSize, ring, lane, dict, lin, ip0, op0);

    for (;;) {
        Batch b;
        const ParseResult pr =
            parse_batch<kOneWaveVecExt, kFastExt>(P, b, lane, kLdsOut ? kSmallBatchOut : 64 * 32);
        if (pr == kParseFail) {
            if (lane == 0) *ret_slot = -P.ip - 1;
            break;
        }
        lap(0);
        if constexpr (kStamps) st.batches++;
        const bool valid = lane < b.n;
        const int32_t op = P.op;  // end of the batch's output
        if (pr == kParsedFast) {
            // ---------------- span-staged copies (fast batches) -------------
            // The batch's output [lo, op) (<= 64 x 32 bytes) is assembled in
            // LDS: literals from the ring; the part of a match source that
            // lies before lo from HBM (final: written by earlier batches);
            // the rest in LDS dependency rounds.  Then one store pass.
            const int32_t lo = lane_val((uint32_t)b.op, 0);
            const int32_t a0 = lo & ~15;  // span index of position x: x - a0
            lu8* span = kLdsOut ? obuf + a0 : span_buf;
            const int32_t ms = b.op + b.L, ss = ms - b.off;
            int32_t n0 = 0;
            uint4 h0 = make_uint4(0, 0, 0, 0), h1 = h0;
            if (valid && ss < lo) {  // fast path: lo <= oend - 32, so [ss, ss + 32) is in the block
                n0 = b.M < lo - ss ? b.M : lo - ss;
                if constexpr (!kLdsOut) {
                    h0 = ldg16(gout + ss);
                    if (n0 > 16) h1 = ldg16(gout + ss + 16);
                }
            }
            if (valid && b.L > 0) {
                const lu8* rs = P.win.in_ring(b.ls, b.L);
                if (rs) lane_copy(span + (b.op - a0), rs, b.L, sink);
                else lane_copy64(span + (b.op - a0), in + b.ls, b.L, in + srcSize);
            }
            if constexpr (kLdsOut) {
                // the source bytes before lo are final in obuf (and end before ms)
                if (n0 > 0) lane_copy(span + (ms - a0), obuf + ss, n0, sink);
            } else if (n0 > 0) {
                put16(span + (ms - a0), h0, n0 < 16 ? n0 : 16, sink);
                if (n0 > 16) put16(span + (ms - a0) + 16, h1, n0 < 32 ? n0 - 16 : 16, sink);
                // extension matches (up to 50 bytes): the rest in a
                // second round trip, rare
                for (int32_t t = 32; t < n0; t += 16)
                    put16(span + (ms - a0) + t, ldg16(gout + ss + t), n0 - t < 16 ? n0 - t : 16, sink);
            }
            lap(1);
            const int32_t ms2 = ms + n0, m2 = b.M - n0, me = ms + b.M;
            const int32_t ss2 = ss + n0;
            const int32_t need = me - b.off < ms2 ? me - b.off : ms2;  // source part before own output
            uint64_t pending = ballot(valid && m2 > 0);
            while (pending) {
                // ready when [ss2, need) overlaps no earlier pending output
                const bool mine = (pending >> lane) & 1;
                const int32_t mn = wave_excl_min(mine ? ms2 : INT32_MAX);
                const int32_t mx = wave_excl_max(mine ? me : INT32_MIN);
                const bool ready = mine && (need <= mn || ss2 >= mx);
                const uint64_t rm = ballot(ready);
                const uint32_t np = popc64(pending);
                if ((rm == (pending & (0 - pending)) && np > 1) || (np >= 4 && 4 * popc64(rm) <= np)) {
                    // Dependency chains (few of the pending matches are
                    // ready): resolve every pending byte by pointer jumping.
                    const int32_t s0 = (int32_t)lane_val((uint32_t)ms2, ctz64(pending)) - a0;
                    const uint32_t nr = resolve_chains(span, jump, lo - a0, op - a0, s0, mine,
                                                       ms2 - a0, m2, b.off, lane);
                    if constexpr (kStamps) st.rounds += nr;
                    break;
                }
                if (ready) {
                    if (b.off != 0) lane_match(span + (ms2 - a0), (uint32_t)b.off, m2, sink);
                    else lane_zero(span + (ms2 - a0), m2, sink);
                }
                pending &= ~rm;
                if constexpr (kStamps) st.rounds++;
            }
            lap(2);
            lockstep();  // the last round's span bytes, read by other lanes
            // store pass: 16-byte HBM chunks of [lo, op); partial end chunks by bytes
            const int32_t nch = kLdsOut ? 0 : (op - a0 + 15) >> 4;
            for (int32_t i = (int32_t)lane; i < nch; i += kWave) {
                const int32_t c0 = a0 + 16 * i;
                const lu8* sc = span + 16 * i;
                if (c0 >= lo && c0 + 16 <= op) {
                    stg16(gout + c0, make_uint4(ld4(sc), ld4(sc + 4), ld4(sc + 8), ld4(sc + 12)));
                } else {
                    for (int32_t x = c0 > lo ? c0 : lo; x < c0 + 16 && x < op; ++x)
                        *(gu8*)(gout + x) = sc[x - c0];
                }
            }
            lap(3);
        } else {
            // ---------------- in-HBM copies (scalar-path batches) -----------
            if constexpr (kLdsOut) {
                copy_scalar_lds(b, P.win, in, srcSize, obuf, sink, lane);
                lockstep();  // later batches read these bytes
            } else {
                copy_scalar_hbm(b, in, srcSize, gout, outSize, lane);
            }
            lap(2);
        }
        if (P.done) {
            if (lane == 0) *ret_slot = P.op;
            break;
        }
    }
    // (a failed block leaves the output its completed batches wrote, as the
    // HBM form does)
    if constexpr (kLdsOut) flush_lds(gout, obuf, P.op, lane);
    if constexpr (kStamps) {
        if (lane == 0 && dbg) {
            dbg[0] = st.acc[0];
            dbg[1] = st.acc[1];
            dbg[2] = st.acc[2];
            dbg[3] = st.batches;
            dbg[4] = st.rounds;
            dbg[5] = st.acc[3];
            dbg[6] = clock64() - t_start;     // the block's shader cycles
            dbg[7] = realtime64() - r_start;  // and its 100 MHz ticks (its clock)
        }
    }
}

// Dictionary bytes of block b: the dict_len[b] bytes before its output;
// anything from 64 KiB on behaves alike (no offset reaches further, and the
// reference's checkOffset is off, :93).
LZ4E_DEV int32_t dict_of(const int32_t* dict_len, uint32_t b) {
    if (!dict_len) return 0;
    const int32_t d = dict_len[b];
    return d <= 0 ? 0 : (d > 65536 ? 65536 : d);
}

// The reference's special cases (lz4e_decompress.c:113-120); true when the
// block is fully handled.
LZ4E_DEV bool special_case(const uint8_t* in, int32_t srcSize, int32_t outSize, int32_t* ret_slot,
                           uint32_t lane) {
    if (outSize == 0) {
        if (lane == 0) *ret_slot = (srcSize == 1 && in[0] == 0) ? 0 : -1;
        return true;
    }
    if (srcSize == 0) {
        if (lane == 0) *ret_slot = -1;
        return true;
    }
    if (srcSize < 0) {  // token read, then every path fails at ip == 1
        if (lane == 0) *ret_slot = -2;
        return true;
    }
    return false;
}

// kSmall: the LDS-output form for blocks of at most kSmallOut bytes without
// a dictionary (other blocks of the launch take the HBM form).
template <bool kStamps, bool kSmall = false>
__global__ __launch_bounds__(64) void decompress_kernel(const uint8_t* __restrict__ src,
                                                        const uint64_t* __restrict__ src_off,
                                                        const int32_t* __restrict__ src_len,
                                                        uint8_t* dst,
                                                        const uint64_t* __restrict__ dst_off,
                                                        const int32_t* __restrict__ dst_cap,
                                                        int32_t* __restrict__ ret, uint32_t nblocks,
                                                        uint64_t* __restrict__ dbg,
                                                        const int32_t* __restrict__ dict_len) {
    const uint32_t b = blockIdx.x;
    if (b >= nblocks) return;
    const uint32_t lane = lane_id();
    const int32_t srcSize = src_len[b];
    const int32_t outSize = dst_cap[b];
    const uint8_t* in = src + src_off[b];
    uint8_t* out = dst + dst_off[b];
    uint64_t* d = kStamps && dbg ? dbg + 8 * (size_t)b : nullptr;
    if (special_case(in, srcSize, outSize, ret + b, lane)) return;
    // LDS: [input ring + mirror] [store sink] [span] [jump table]; small
    // blocks: [store sink] [output] [jump table] [input]
    constexpr uint32_t kWaveLds = kRing + kRingPad + kSink + kSpan + kJump;
    // (+ 256 B after the staged input: the fast path's window probe reads up
    // to ~258 bytes past ip, beyond any byte it uses; 12 032 B, still 13 per CU)
    constexpr uint32_t kSmallLds = kSink + kSmallBuf + kSmallJump + kSmallBuf + 256;
    __shared__ __attribute__((aligned(16))) uint8_t smem[kSmall && kSmallLds > kWaveLds ? kSmallLds : kWaveLds];
    const int32_t dict = dict_of(dict_len, b);
    if (kSmall && dict == 0 && outSize <= kSmallOut && srcSize <= kSmallOut) {
        lu8* obuf = (lu8*)(smem + kSink);
        decode_block<kStamps, true>(in, srcSize, out, outSize, ret + b, d, lane, obuf, nullptr,
                                    (lu16*)(obuf + kSmallBuf), 0, (lu8*)smem, obuf,
                                    obuf + kSmallBuf + kSmallJump);
    } else {
        lu8* sinkb = (lu8*)(smem + kRing + kRingPad);
        decode_block<kStamps>(in, srcSize, out, outSize, ret + b, d, lane, sinkb + kSink, (lu32*)smem,
                              (lu16*)(sinkb + kSink + kSpan), dict, sinkb);
    }
}

// The block-per-group decoder (see group_decode): block b on group
// b % (kGroupWg / kGroup) of workgroup b / (kGroupWg / kGroup).
// LZ4E_GROUP_WG: threads per workgroup (experiments: one wave per workgroup
// is fastest, fio4k 0.836 ms against 0.850 / 0.892 / 0.988 / 1.012 ms for
// 128 / 256 / 512 / 1024 threads, profiles/r05/group_decoder/wg/).
#ifndef LZ4E_GROUP_WG
#define LZ4E_GROUP_WG 64
#endif
constexpr uint32_t kGroupWg = LZ4E_GROUP_WG;
// LZ4E_GROUP_PAD: LDS the workgroup never uses (a residency cap; experiments:
// none is fastest, 4 workgroups per CU cost a third).
#ifndef LZ4E_GROUP_PAD
#define LZ4E_GROUP_PAD 0
#endif
// (6 waves per SIMD asked of the compiler: 80 VGPRs instead of 82, one wave
// more per SIMD; fio4k 0.84 -> 0.80 ms; 8 spills and is slower)
__global__ __launch_bounds__(kGroupWg, 6) void decompress_group_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const int32_t* __restrict__ src_len, uint8_t* dst, const uint64_t* __restrict__ dst_off,
    const int32_t* __restrict__ dst_cap, int32_t* __restrict__ ret, uint32_t nblocks,
    const int32_t* __restrict__ dict_len, uint32_t* __restrict__ handover) {
#if LZ4E_GROUP_PAD
    __shared__ uint8_t pad[LZ4E_GROUP_PAD];
    if (nblocks == 0xFFFFFFFFu) ((volatile uint8_t*)pad)[threadIdx.x] = 1;
#endif
    const uint32_t tid = threadIdx.x, s = tid % kGroup, lane = lane_id();
    const uint32_t b = blockIdx.x * (kGroupWg / kGroup) + tid / kGroup;
    // (no lane leaves early: the hand-over below is a whole-wave step)
    bool act = b < nblocks;
    int32_t r = 0, ip = 0, op = 0;
    if (act) {
        const int32_t srcSize = src_len[b], outSize = dst_cap[b];
        const uint8_t* in = src + src_off[b];
        if (special_case(in, srcSize, outSize, ret + b, s)) act = false;
        else r = group_decode(in, srcSize, dst + dst_off[b], outSize, dict_of(dict_len, b), handover != nullptr,
                              &ip, &op, s);
    }
    // hand-over list entries from each group's lane 0, one atomic per wave
    const bool ho = act && r == kLaneHandOver;
    const uint64_t m = ballot(ho && s == 0);
    if (m) {
        const uint32_t lead = ctz64(m);
        uint32_t base = 0;
        if (lane == lead) base = atomicAdd(handover, popc64(m));
        base = shfl(base, lead);
        if (ho && s == 0) {
            const uint32_t k = base + popc64(m & ((1ull << lane) - 1));
            handover[1 + 3 * k] = b;
            handover[2 + 3 * k] = (uint32_t)ip;
            handover[3 + 3 * k] = (uint32_t)op;
        }
    }
    if (act && !ho && s == 0) ret[b] = r;
}

// The blocks the group decoder handed over, one wave each from their
// sequence boundary on (decode_block's HBM form; the output before it is in
// HBM): workgroup i takes entry i, those past the count leave at once (as
// balanced as the one-wave kernel itself; a fixed grid striding over the
// list measured 1.31 vs 1.12 ms when every block was handed over).
template <bool kStamps>
__global__ __launch_bounds__(64) void decompress_resume_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const int32_t* __restrict__ src_len, uint8_t* dst, const uint64_t* __restrict__ dst_off,
    const int32_t* __restrict__ dst_cap, int32_t* __restrict__ ret, const uint32_t* __restrict__ handover,
    uint64_t* __restrict__ dbg, const int32_t* __restrict__ dict_len) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kRing + kRingPad + kSink + kSpan + kJump];
    const uint32_t lane = lane_id();
    const uint32_t cnt = handover[0];
    for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {  // (one pass: grid = every block)
        const uint32_t b = handover[1 + 3 * i];
        const int32_t ip0 = (int32_t)handover[2 + 3 * i], op0 = (int32_t)handover[3 + 3 * i];
        uint64_t* d = kStamps && dbg ? dbg + 8 * (size_t)b : nullptr;
        lu8* sinkb = (lu8*)(smem + kRing + kRingPad);
        decode_block<kStamps>(src + src_off[b], src_len[b], dst + dst_off[b], dst_cap[b], ret + b, d, lane,
                              sinkb + kSink, (lu32*)smem, (lu16*)(sinkb + kSink + kSpan), dict_of(dict_len, b),
                              sinkb, nullptr, nullptr, ip0, op0);
        lockstep();  // the next block reuses the LDS
    }
}

// ============================================================================
// Pipelined decoder: one block per 4-wave workgroup
// ============================================================================
//
// The one-wave decoder above runs the parse and the copies of each batch one
// after the other, and a block's time is the sum of both over its ~150
// batches; with ~3 blocks per SIMD the kernel time is the slowest block's
// chain.  Here the parse and the copies of different batches overlap:
//
//  * wave 0 parses (parse_batch: the reference's exact checks, so the return
//    value is decided here) and publishes each batch -- per-lane sequence
//    records plus its output range [lo, hi) -- in a ring of record slots;
//  * waves 1..3 (copier c = wave - 1) copy batches j = c, c+3, c+6, ... so
//    three batches are in flight at once.  A fast batch (at most kPipeOut
//    output bytes) is assembled in an LDS span; every output byte is a
//    literal (from the compressed input in HBM), a match byte whose source
//    lies before the far line F (final in HBM: loaded), one whose source lies
//    in the batch itself (internal pointer) or one whose source lies in the
//    spans of batches j-1 / j-2, still in LDS (cross pointer).  Match byte t
//    of a sequence copies output byte x - off, also inside a self-overlapping
//    match, so the pointers are linear in t.  Internal pointers resolve by
//    pointer jumping (a chain of depth d in log2 d rounds) in parallel with
//    the other copiers; only the gather of the cross bytes waits for batches
//    j-1 and j-2, and that is one LDS round trip, so the batches' serial
//    chain is short.  The span then leaves in 16-byte stores.  A scalar-path
//    batch (long runs, block ends) copies in HBM once every earlier batch is
//    stored.
//
// Progress flags (LDS, workgroup-scope acquire/release): `resolved` counts
// the batches whose bytes are final (in order), `stored` is the output
// prefix known to be in HBM (each batch's stores waited for with
// s_waitcnt vmcnt(0) before it moves, in order).  Far loads wait for
// stored >= F.  Measured against per-copier flags (batches finishing out of
// order, "all batches <= k" read off three flags): the in-order counters
// poll one word instead of three and were 10 % faster on silesia64k.  Every
// wait is bounded (watchdog).
// LZ4E_PIPE_WAVES: workgroup size of the pipelined decoder (parser + copiers;
// experiments only -- 2, 3 and 5 waves measured slower than 4).
#ifndef LZ4E_PIPE_WAVES
#define LZ4E_PIPE_WAVES 4
#endif
constexpr uint32_t kPipeWaves = LZ4E_PIPE_WAVES;
constexpr uint32_t kCopiers = kPipeWaves - 1;
// LZ4E_PIPE_RECS: record slots between the parser and the copiers (how far
// the parser may run ahead of the slowest copier; experiments: 6, 8 and 12
// measured 0.874 / 0.882 / 0.902 ms against 0.878-0.883 ms for 4 on
// silesia64k, profiles/r05/pipe_recs/).
#ifndef LZ4E_PIPE_RECS
#define LZ4E_PIPE_RECS 4
#endif
constexpr uint32_t kPipeRecs = LZ4E_PIPE_RECS;
constexpr uint32_t kPipeSpans = kCopiers + 2;  // see copy_fast's slot safety
constexpr int32_t kPipeOut = 1024;                   // output bytes per fast batch
constexpr uint32_t kPipeSpan = kPipeOut + 16 + 48;   // its span (16-B aligned start)
constexpr uint16_t kCross = 0x8000;  // jump entry: 0x8000 | (source - F)
enum : int32_t { kKindFast = 0, kKindHbm = 1 };
// record header: sequences, kind, output range, far line F, the starts of
// batches j-1 and j-2
enum { kHdrN, kHdrKind, kHdrLo, kHdrHi, kHdrF, kHdrLo1, kHdrLo2, kHdrWords = 8 };

struct PipeLds {
    uint32_t ring[(kRing + kRingPad) / 4];     // parser input ring
    int32_t rec[kPipeRecs][5][kWave];          // ls, L, op, off, M per sequence
    int32_t hdr[kPipeRecs][kHdrWords];
    uint8_t span[kPipeSpans][kPipeSpan];
    uint16_t jump[kCopiers][kPipeSpan];
    uint8_t sink[kCopiers][kSink];
    int32_t pub[kPipeRecs], con[kPipeRecs];    // record slot published / consumed (batch index)
    int32_t resolved;                          // batches whose bytes are final, in order
    int32_t stored;                            // output prefix known to be in HBM
    int32_t nb_total;                          // batches, once the parser is done
    int32_t abort;                             // a wait timed out (watchdog): every wave leaves
    int32_t beat;                              // heartbeat of a long in-HBM copy (watchdog)
    int32_t result;                            // the parse's return value (decided by wave 0)
    uint32_t spin_max;                         // the watchdog's limit for this block (see below)
};

// Watchdog of the waits: a wait that sees the counters it watches stand
// still for S.spin_max sleeps in a row means a broken invariant; the block
// then fails (ret = kPipeAbort = LZ4E_DECODE_ABORTED, include/lz4e.h: the
// host entry points report it through lz4e_last_error) instead of hanging.
// The bound, from the frame's own worst case ("Watchdog"):
// between two moves of a watched counter a valid frame's decode does one
// of (a) a batch's parse and copies (<= 64 sequences, <= 1 KiB of output:
// tens of k cycles), (b) a scalar sequence's copy in HBM, which bumps
// `beat` every round trip, or (c) the parser's vector scan of one length-
// extension run, 256 bytes per ~1-2 k-cycle step and no counter moved:
// at most srcSize / 256 steps.  A sleep is >= 128 cycles (s_sleep 2), so
// spin_max = kSpinMax (2^23 sleeps, ~0.6 s at 2.4 GHz, for (a) and
// anything the hardware adds) + srcSize >> kSpinBytesShift sleeps (64 per
// 256 bytes: 4-8x the scan's worst case) can only fire on a broken
// invariant.  Progress resets the count.  LZ4E_SPIN_MAX / _BYTES_SHIFT
// override the terms (the emulator's watchdog test builds a limit of one
// sleep and no per-byte term).
#ifndef LZ4E_SPIN_MAX
#define LZ4E_SPIN_MAX (1u << 23)
#endif
#ifndef LZ4E_SPIN_BYTES_SHIFT
#define LZ4E_SPIN_BYTES_SHIFT 2
#endif
constexpr uint32_t kSpinMax = LZ4E_SPIN_MAX;
constexpr uint32_t kSpinBytesShift = LZ4E_SPIN_BYTES_SHIFT;
constexpr int32_t kPipeAbort = kDecodeAborted;  // lz4e_results.h

LZ4E_DEV int32_t lds_acquire(int32_t* p) {
    return (int32_t)uni((uint32_t)__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
// Called by every lane of the wave: the wave's earlier LDS / global
// accesses have all been issued before it (lockstep).
LZ4E_DEV void lds_release(int32_t* p, int32_t v) {
    lockstep();
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// u16 x 4 at a jump-table index (unaligned forms for the pointer runs).
typedef uint64_t __attribute__((aligned(2), may_alias)) u64a2;
typedef __attribute__((address_space(3))) u64a2 lu64a2;
typedef __attribute__((address_space(3), may_alias)) uint64_t lu64;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3), may_alias)) u32x4 lu128;
LZ4E_DEV int32_t wave_min_i32(int32_t v) {
    const int32_t e = wave_excl_min(v);
    const int32_t m = e < v ? e : v;
    return (int32_t)lane_val((uint32_t)m, kWave - 1);
}


// Cycle counters of the stamped build, per block (u64 x 20): parser parse,
// parser waits, copier other work, copier waits for records, for far loads,
// for batch j-1 (resolved), for the in-order store flag, batches; copier
// phases: loads + span setup, internal rounds, cross gather, store pass,
// store completion; internal rounds, batches with internal pointers; copier
// pointer entries; parser phases: window, table composition, follow, fields;
// the block's shader cycles and 100 MHz ticks (wave 0, start to end).
enum { kStParse, kStPWait, kStWork, kStRec, kStFar, kStPrev, kStStore, kStBatches, kStLoads,
       kStRounds, kStGather, kStSpass, kStVm, kStNRounds, kStNInt, kStPtrs,
       kStPWin, kStPComp, kStPFollow, kStPFields, kStT, kStR, kStSlots };
// The accumulators live in LDS (a row per wave), so that the stamped build
// has the register allocation of the real one.
struct PipeStamps {
    uint64_t* acc = nullptr;  // LDS row of this wave (stamped build)
    uint64_t t = 0;
    LZ4E_DEV void lap(bool on, int k) {
        if (!on) return;
        const uint64_t now = clock64();
        if (lane_id() == 0) acc[k] += now - t;
        t = now;
    }
    LZ4E_DEV void bump(bool on, int k) {
        if (on && lane_id() == 0) acc[k]++;
    }
};

// Waits until ready(); false when the watchdog fired (here or in another
// wave).  watch() is the LDS counter the wait depends on: the watchdog
// counts sleeps since it last moved.
template <class SL, class F, class W>
LZ4E_DEV bool wait_for(SL& S, F ready, W watch) {
    int32_t last = watch();
    for (uint32_t k = 0; !ready(); ++k) {
        const int32_t now = watch();
        if (now != last) {
            last = now;
            k = 0;
        }
        if (k >= S.spin_max || lds_acquire(&S.abort)) {
            lds_release(&S.abort, 1);
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    return true;
}

template <bool kStamps, class F, class W>
LZ4E_DEV bool spin(PipeLds& S, F ready, W watch, PipeStamps& st, int k) {
    st.lap(kStamps, kStWork);
    const bool ok = wait_for(S, ready, watch);
    st.lap(kStamps, k);
    return ok;
}

// A fast batch j (see above).  Slot safety with K copiers in round robin
// and K + 2 spans: span slot j % (K+2) last held batch j-K-2, read by
// batches j-K-1 and j-K (cross gathers) and by its own store pass; j-K was
// this wave's previous batch, j-K-1's gather happened before `resolved`
// reached j-K (this wave waited for that), and j-K-2 was stored before this
// wave's batch j-K could be.
template <bool kStamps>
LZ4E_DEV bool copy_fast(PipeLds& S, uint32_t c, int32_t j, const Batch& b, const int32_t* hdr,
                        const uint8_t* in, int32_t srcSize, uint8_t* gout, uint32_t lane,
                        PipeStamps& st) {
    const int32_t lo = hdr[kHdrLo], hi = hdr[kHdrHi], F = hdr[kHdrF];
    const int32_t a0 = lo & ~15;
    const int32_t s0 = lo - a0, s1 = hi - a0;  // span indices of [lo, hi)
    lu8* span = (lu8*)S.span[(uint32_t)j % kPipeSpans];
    lu16* jt = (lu16*)S.jump[c];
    lu8* sink = (lu8*)S.sink[c] + 4 * lane;
    const bool valid = lane < b.n;
    const int32_t ms = b.op + b.L, ss = ms - b.off;
    // Match byte t of a sequence copies output byte ss + t; bytes [0, nf)
    // come from before F (HBM).
    int32_t nf = 0;
    if (valid && b.off != 0 && ss < F) nf = b.M < F - ss ? b.M : F - ss;
    if (ballot(nf > 0) &&
        !spin<kStamps>(S, [&] { return lds_acquire(&S.stored) >= F; },
                       [&] { return lds_acquire(&S.stored) + lds_acquire(&S.beat); }, st, kStFar))
        return false;
    // loads first (far source bytes, the literal run), consumed below
    uint4 h0 = make_uint4(0, 0, 0, 0), h1 = h0, lv = h0;
    if (nf > 0) {
        h0 = ldg16(gout + ss);
        if (nf > 16) h1 = ldg16(gout + ss + 16);
    }
    const bool lfast = valid && b.L > 0 && b.ls + 16 <= srcSize;
    if (lfast) lv = ldg16(in + b.ls);
    // every byte of [lo, hi) final until shown otherwise: 4 entries per
    // 8-byte store (the row is 16-byte aligned; entries outside [lo, hi) are
    // never read as pointers -- `entry` masks them)
    for (int32_t g = (s0 & ~3) + 4 * (int32_t)lane; g < s1; g += 4 * (int32_t)kWave)
        *(lu64*)(jt + g) = ~0ull;
    wave_fence();
    // match bytes [nf, M): a cross pointer below lo, else an internal one
    const bool ptrs = valid && b.off != 0 && nf < b.M;
    if (ptrs) {
        lu16* e = jt + (ms - a0);
#pragma clang loop unroll(disable) vectorize(disable)
        for (int32_t t = nf; t < b.M; ++t) {
            const int32_t y = ss + t;
            e[t] = (uint16_t)(y < lo ? (int32_t)kCross + (y - F) : y - a0);
        }
    }
    const bool has_cross = ptrs && ss + nf < lo;
    const bool has_int = ptrs && ss + b.M > lo;
    // rounds and gather start at the first pointer byte
    const int32_t i0 = (int32_t)uni((uint32_t)wave_min_i32(ptrs ? ms + nf - a0 : s1));
    st.lap(kStamps, kStPtrs);
    // the loaded bytes into the span
    if (valid && b.L > 0) {
        if (lfast) {
            put16(span + (b.op - a0), lv, b.L < 16 ? (uint32_t)b.L : 16u, sink);
            // extension literal runs (up to 46 bytes, rare): the
            // rest in a second round trip; ls + L <= srcSize - 18 on the
            // fast path
#pragma clang loop unroll(disable) vectorize(disable)
            for (int32_t t = 16; t < b.L; t += 16)
                put16(span + (b.op - a0) + t, ldg16(in + b.ls + t), (uint32_t)(b.L - t < 16 ? b.L - t : 16),
                      sink);
        } else {
#pragma clang loop unroll(disable) vectorize(disable)
            for (int32_t t = 0; t < b.L; ++t) span[b.op - a0 + t] = in[b.ls + t];
        }
    }
    if (nf > 0) {
        put16(span + (ms - a0), h0, nf < 16 ? nf : 16, sink);
        if (nf > 16) put16(span + (ms - a0) + 16, h1, nf < 32 ? nf - 16 : 16, sink);
#pragma clang loop unroll(disable) vectorize(disable)
        for (int32_t t = 32; t < nf; t += 16)  // extension matches: a second round trip
            put16(span + (ms - a0) + t, ldg16(gout + ss + t), (uint32_t)(nf - t < 16 ? nf - t : 16), sink);
    }
    if (valid && b.off == 0)  // offset 0 writes zeros (:313, 407-415)
#pragma clang loop unroll(disable) vectorize(disable)
        for (int32_t t = 0; t < b.M; ++t) span[ms - a0 + t] = 0;
    wave_fence();
    st.lap(kStamps, kStLoads);
    // internal pointers: pointer jumping until each byte is final or cross.
    // Lane l owns the 8 span bytes / jump entries at g = b0 + 8l (+ 512k):
    // one 16-byte entry read and one 8-byte span read per group, the 8
    // dependent entry reads and byte reads independent of each other, and
    // one write back of each (positions outside [i0, s1) keep their values).
    const int32_t b0 = i0 & ~7;
    auto entry = [&](const u32x4& jv, int q, int32_t g) -> uint32_t {
        const uint32_t e = (jv[q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
        return (g + q >= i0 && g + q < s1) ? e : kFinal;
    };
    if (ballot(has_int)) {
        st.bump(kStamps, kStNInt);
        for (;;) {
            st.bump(kStamps, kStNRounds);
            bool more = false;
            for (int32_t g = b0 + 8 * (int32_t)lane; g < s1; g += 8 * (int32_t)kWave) {
                u32x4 jv = *(const lu128*)(jt + g);
                uint64_t sp = *(const lu64*)(span + g);
                uint32_t v[8], w[8], sb[8];
                bool anyp = false;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    v[q] = entry(jv, q, g);
                    anyp |= v[q] < kCross;
                }
                if (!anyp) continue;  // (exec mask: only lanes with pointers read)
                // unconditional reads (index 0 when unused): no branches
                // between them, so all eight are in flight together
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const uint32_t x = jt[v[q] < kCross ? v[q] : 0u];
                    w[q] = v[q] < kCross ? x : kFinal;
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) sb[q] = span[v[q] < kCross ? v[q] : 0u];
                bool any = false;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const bool ptr = v[q] < kCross, fin = w[q] == kFinal;
                    any |= ptr;
                    more |= ptr && w[q] < kCross;
                    const uint32_t sh = 16 * (q & 1);
                    const uint32_t cur = (jv[q >> 1] >> sh) & 0xFFFFu;
                    const uint32_t ne = ptr ? w[q] : cur;
                    jv[q >> 1] = (jv[q >> 1] & ~(0xFFFFu << sh)) | (ne << sh);
                    const uint64_t bm = 0xFFull << (8 * q);
                    sp = (ptr && fin) ? ((sp & ~bm) | ((uint64_t)(sb[q] & 0xFFu) << (8 * q))) : sp;
                }
                if (any) {
                    *(lu64*)(span + g) = sp;
                    *(lu128*)(jt + g) = jv;
                }
            }
            wave_fence();
            if (!ballot(more)) break;
        }
    }
    st.lap(kStamps, kStRounds);
    // cross bytes: batches j-1 and j-2 are final once `resolved` reaches j
    if (!spin<kStamps>(S, [&] { return lds_acquire(&S.resolved) >= j; },
                       [&] { return lds_acquire(&S.resolved) + lds_acquire(&S.beat); }, st, kStPrev))
        return false;
    if (ballot(has_cross)) {
        const int32_t lo1 = hdr[kHdrLo1], lo2 = hdr[kHdrLo2];
        const lu8* p1 = (const lu8*)S.span[(uint32_t)(j + kPipeSpans - 1) % kPipeSpans] - (lo1 & ~15);
        const lu8* p2 = (const lu8*)S.span[(uint32_t)(j + kPipeSpans - 2) % kPipeSpans] - (lo2 & ~15);
        for (int32_t g = b0 + 8 * (int32_t)lane; g < s1; g += 8 * (int32_t)kWave) {
            const u32x4 jv = *(const lu128*)(jt + g);
            uint64_t sp = *(const lu64*)(span + g);
            uint32_t x[8];
            bool any = false;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint32_t v = entry(jv, q, g);
                any |= v != kFinal && v >= kCross;
            }
            if (!any) continue;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint32_t v = entry(jv, q, g);
                const bool cr = v != kFinal && v >= kCross;
                const int32_t y = cr ? F + (int32_t)(v - kCross) : lo1;
                x[q] = y >= lo1 ? p1[y] : p2[y];  // unconditional (p1[lo1] when unused)
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint32_t v = entry(jv, q, g);
                const bool cr = v != kFinal && v >= kCross;
                any |= cr;
                const uint64_t bm = 0xFFull << (8 * q);
                sp = cr ? ((sp & ~bm) | ((uint64_t)(x[q] & 0xFFu) << (8 * q))) : sp;
            }
            if (any) *(lu64*)(span + g) = sp;
        }
        wave_fence();
    }
    lds_release(&S.resolved, j + 1);
    st.lap(kStamps, kStGather);
    // store pass: 16-byte HBM chunks of [lo, hi); partial end chunks by bytes
    const int32_t nch = (hi - a0 + 15) >> 4;
    for (int32_t i = (int32_t)lane; i < nch; i += kWave) {
        const int32_t c0 = a0 + 16 * i;
        const lu8* sc = span + 16 * i;
        if (c0 >= lo && c0 + 16 <= hi) {
            const u32x4 v = *(const lu128*)sc;
            stg16(gout + c0, make_uint4(v.x, v.y, v.z, v.w));
        } else {
#pragma clang loop unroll(disable) vectorize(disable)
            for (int32_t x = c0 > lo ? c0 : lo; x < c0 + 16 && x < hi; ++x)
                *(gu8*)(gout + x) = sc[x - c0];
        }
    }
    st.lap(kStamps, kStSpass);
    if (!spin<kStamps>(S, [&] { return lds_acquire(&S.stored) >= lo; },
                       [&] { return lds_acquire(&S.stored) + lds_acquire(&S.beat); }, st, kStStore))
        return false;
    stores_done();
    lds_release(&S.stored, hi);
    st.lap(kStamps, kStVm);
    return true;
}

// 6 workgroups (24 waves) per CU: 76 VGPRs and 19 KiB of LDS each.
// (LZ4E_PIPE_MINWG: the occupancy asked of the compiler, experiments.)
#ifndef LZ4E_PIPE_MINWG
#define LZ4E_PIPE_MINWG 6
#endif
template <bool kStamps>
__global__ __launch_bounds__(kPipeWaves * kWave, LZ4E_PIPE_MINWG) void decompress_pipe_kernel(
    const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
    const int32_t* __restrict__ src_len, uint8_t* dst, const uint64_t* __restrict__ dst_off,
    const int32_t* __restrict__ dst_cap, int32_t* __restrict__ ret, uint32_t nblocks,
    uint64_t* __restrict__ dbg, const int32_t* __restrict__ dict_len,
    const uint32_t* __restrict__ order) {
    __shared__ __attribute__((aligned(16))) PipeLds S;
    if (blockIdx.x >= nblocks) return;
    const uint32_t b = order ? order[blockIdx.x] : blockIdx.x;
    const uint32_t tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
    const int32_t srcSize = src_len[b];
    const int32_t outSize = dst_cap[b];
    const uint8_t* in = src + src_off[b];
    uint8_t* gout = dst + dst_off[b];
    if (special_case(in, srcSize, outSize, ret + b, tid)) return;
    if (tid < kPipeRecs) {
        S.pub[tid] = -1;
        S.con[tid] = (int32_t)tid - (int32_t)kPipeRecs;
    }
    if (tid == 0) {
        S.nb_total = INT32_MAX;
        S.resolved = 0;
        S.stored = 0;
        S.abort = 0;
        S.beat = 0;
        S.result = kPipeAbort;
        S.spin_max = kSpinMax + (kSpinBytesShift < 31 ? (uint32_t)srcSize >> kSpinBytesShift : 0u);
    }
    __syncthreads();
    PipeStamps st;
    __shared__ uint64_t st_rows[kStamps ? kPipeWaves * kStSlots : 1];
    [[maybe_unused]] uint64_t t_start = 0, r_start = 0;
    if (kStamps) {
        st.acc = st_rows + wave * kStSlots;
        if (lane < kStSlots) st.acc[lane] = 0;
        st.t = clock64();
        t_start = st.t;
        r_start = realtime64();
    }

    if (wave == 0) {
        // ---------------- parser ----------------
        // (the critical path of the block: first in issue arbitration)
        __builtin_amdgcn_s_setprio(3);
        Parse P;
        P.init(in, srcSize, outSize, (lu32*)S.ring, lane, dict_of(dict_len, b));
        int32_t j = 0, lo1 = 0, lo2 = 0, hi1 = 0, hi2 = 0;
        bool hbm1 = false, hbm2 = false;
        for (;;) {
            Batch bt;
            const int32_t lo = P.op;
            const ParseResult pr = parse_batch<true, kFastExt>(P, bt, lane, kPipeOut, [&](int k) {
                if (kStamps) st.lap(true, kStPWin + k);
            });
            st.lap(kStamps, kStParse);
            if (pr == kParseFail) {
                if (lane == 0) S.result = -P.ip - 1;
                break;
            }
            // far line: sources before it are read from HBM (see copy_fast)
            int32_t F = j >= 2 ? lo2 : 0;
            if (j >= 2 && hbm2) F = F > hi2 ? F : hi2;
            if (j >= 1 && hbm1) F = F > hi1 ? F : hi1;
            const uint32_t slot = (uint32_t)j % kPipeRecs;
            if (!wait_for(S, [&] { return lds_acquire(&S.con[slot]) == j - (int32_t)kPipeRecs; },
                          [&] { return lds_acquire(&S.beat) + lds_acquire(&S.con[slot]); })) {
                lds_release(&S.abort, 1);
                break;
            }
            st.lap(kStamps, kStPWait);
            S.rec[slot][0][lane] = bt.ls;
            S.rec[slot][1][lane] = bt.L;
            S.rec[slot][2][lane] = bt.op;
            S.rec[slot][3][lane] = bt.off;
            S.rec[slot][4][lane] = bt.M;
            if (lane < kHdrWords) {
                const int32_t h[kHdrWords] = {(int32_t)bt.n, pr == kParsedScalar ? kKindHbm : kKindFast,
                                              lo, P.op, F, lo1, lo2, 0};
                int32_t v = 0;
#pragma unroll
                for (uint32_t q = 0; q < kHdrWords; ++q) v = lane == q ? h[q] : v;
                S.hdr[slot][lane] = v;
            }
            lds_release(&S.pub[slot], j);
            lo2 = lo1;
            hi2 = hi1;
            hbm2 = hbm1;
            lo1 = lo;
            hi1 = P.op;
            hbm1 = pr == kParsedScalar;
            j++;
            if (P.done) {
                if (lane == 0) S.result = P.op;
                break;
            }
        }
        lds_release(&S.nb_total, j);
        st.lap(kStamps, kStParse);
    } else {
        // ---------------- copiers ----------------
        const uint32_t c = wave - 1;
        for (int32_t j = (int32_t)c;; j += kCopiers) {
            const uint32_t slot = (uint32_t)j % kPipeRecs;
            st.lap(kStamps, kStWork);
            const bool ok = wait_for(
                S, [&] { return lds_acquire(&S.pub[slot]) == j || lds_acquire(&S.nb_total) <= j; },
                [&] { return lds_acquire(&S.beat) + lds_acquire(&S.pub[slot]); });
            st.lap(kStamps, kStRec);
            if (!ok) {
                lds_release(&S.abort, 1);
                break;
            }
            if (lds_acquire(&S.pub[slot]) != j) break;  // the parser ended before batch j
            Batch bt;
            bt.ls = S.rec[slot][0][lane];
            bt.L = S.rec[slot][1][lane];
            bt.op = S.rec[slot][2][lane];
            bt.off = S.rec[slot][3][lane];
            bt.M = S.rec[slot][4][lane];
            int32_t hdr[kHdrWords];
#pragma unroll
            for (uint32_t q = 0; q < kHdrWords; ++q) hdr[q] = (int32_t)uni((uint32_t)S.hdr[slot][q]);
            bt.n = (uint32_t)hdr[kHdrN];
            lds_release(&S.con[slot], j);
            st.bump(kStamps, kStBatches);
            if (hdr[kHdrKind] == kKindHbm) {
                // every earlier batch in HBM, then in place
                if (!spin<kStamps>(S, [&] { return lds_acquire(&S.stored) >= hdr[kHdrLo]; },
                                   [&] { return lds_acquire(&S.stored) + lds_acquire(&S.beat); }, st, kStStore)) {
                    lds_release(&S.abort, 1);
                    break;
                }
                copy_scalar_hbm<4>(bt, in, srcSize, gout, outSize, lane, [&] {
                    // (called in lane-divergent loops: lane 0 alone, no ordering)
                    if (lane == 0)
                        __hip_atomic_fetch_add(&S.beat, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                });
                stores_done();
                lds_release(&S.resolved, j + 1);
                lds_release(&S.stored, hdr[kHdrHi]);
                st.lap(kStamps, kStVm);
            } else if (!copy_fast<kStamps>(S, c, j, bt, hdr, in, srcSize, gout, lane, st)) {
                lds_release(&S.abort, 1);
                break;
            }
        }
    }
    // Every wave has left its loop (each wait is bounded by the watchdog):
    // the block's value is the parse's unless a wave gave up, which fails
    // the whole block -- the parser may finish its parse without ever
    // waiting, so only here are all waves' outcomes known.
    __syncthreads();
    if (tid == 0) ret[b] = __hip_atomic_load(&S.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                               ? kPipeAbort
                               : S.result;
    if constexpr (kStamps) {
        if (lane == 0 && wave == 0) {
            st.acc[kStT] = clock64() - t_start;     // the block's shader cycles
            st.acc[kStR] = realtime64() - r_start;  // and its 100 MHz ticks (its clock)
        }
        if (lane == 0 && dbg) {
            uint64_t* d = dbg + kStSlots * (size_t)b;
            for (int k = 0; k < kStSlots; ++k)
                if (st.acc[k]) atomicAdd((unsigned long long*)(d + k), (unsigned long long)st.acc[k]);
        }
    }
}

// Blocks whose capacity lies in [kPipeMinCap, kPipeMaxCap) take the
// pipelined decoder.  Small blocks parse in a few batches, and one wave each
// keeps more of them resident.  Large blocks (256 KiB: ~560 batches each)
// decode faster one wave per block as well: 20 resident blocks per CU
// against 6 four-wave ones, so a 3 815-block batch runs in one round of
// workgroups instead of 2.5 (text256k decompress-only 4.33 -> 3.04 ms,
// profiles/r04/decmodes.txt); at 64 KiB the pipelined decoder's per-block
// speed wins (silesia64k 0.85 vs 1.20 ms).
constexpr uint32_t kPipeMinCap = 16384;
// Batches of at least this many blocks of <= kSmallOut bytes take the group
// decoder (blocks that open with a short sequence go straight on to the
// one-wave decoder).  Fio-style blocks (tools/decmodes.py, group vs one-wave
// vs LDS form): 4 096 blocks 0.080 / 0.055 / 0.067 ms, 16 384 0.093 / 0.170 /
// 0.189, 65 536 0.279 / 0.717 / 0.693, 262 144 0.89 / 2.76 / 2.69; 4 KiB
// Silesia-proxy blocks, all handed over: 65 536 1.215 / 1.131 / 1.316
// (profiles/r05/group_decoder/).
constexpr uint32_t kGroupMinBlocks = 16384;
// Batches of small blocks that fit one round of the LDS form's workgroups
// (11.8 KiB of LDS: 13 per CU) take that form: no HBM round trip inside a
// block's decode (drop-in single call, 4 KiB text: 89 -> 79 us p50); with
// more rounds the one-wave form's 20 workgroups per CU win (65 536 4 KiB
// Silesia-proxy blocks: 1.13 vs 1.30 ms).
constexpr uint32_t kSmallMaxBlocks = 256 * 13;
// Batches that leave most of the pipelined decoder's round of workgroups
// (1 536) unused are latency-bound whatever the block size: the pipelined
// decoder overlaps a block's parse with its copies (drop-in single call,
// 4 KiB text: 71 us p50 against 82 us for the LDS form and 92 us one-wave,
// tools/single_call_trace.py; 1 024 4 KiB Silesia-proxy blocks 0.085 ms
// against 0.101 / 0.102, fio 0.036 / 0.034 / 0.035; at 3 072 blocks the LDS
// form wins, 0.115 against 0.162 ms; tools/decmodes.py).
constexpr uint32_t kLatencyMaxBlocks = 1024;
constexpr uint32_t kPipeMaxCap = 131072;

// Launch order of the pipelined decoder when the batch takes more than one
// round of workgroups (lz4e_order.h): a block's decode time grows with its
// sequence count, estimated by its compressed size; frames within 1/16 of
// their capacity (stored / incompressible data: a few long literal runs) are
// the lightest.
constexpr uint32_t kOrderMin = 256 * (24 / kPipeWaves);  // one round of pipelined workgroups
struct DecodeWeight {
    const int32_t* src_len;
    const int32_t* dst_cap;
    LZ4E_DEV uint32_t operator()(uint32_t b) const {
        const int64_t c = src_len[b], cap = dst_cap[b];
        if (cap <= 0 || c >= cap - cap / 16) return kOrderBuckets - 1;
        const int64_t q = c <= 0 ? 0 : c * (kOrderBuckets - 1) / cap;  // < 63
        return (uint32_t)(kOrderBuckets - 2 - (q < kOrderBuckets - 2 ? q : kOrderBuckets - 2));
    }
};

template <bool kStamps>
hipError_t launch_impl(const DecompressBatch& a, hipStream_t stream, uint64_t* dbg) {
    if (a.nblocks == 0) return hipSuccess;
    // LZ4E_DECOMPRESS_MODE=w|p|s|g (one-wave, pipelined, LDS form, group)
    // overrides the choice for A/B experiments; any other value is auto.
    // Auto, in order: capacity 16-128 KiB (or unknown) -> pipelined; blocks
    // of <= kSmallOut bytes in batches of >= kGroupMinBlocks -> group; batches
    // of <= kLatencyMaxBlocks blocks of any size -> pipelined; blocks of
    // <= kSmallOut bytes in batches of <= kSmallMaxBlocks -> LDS form;
    // everything else -> one wave per block.
    static const char* env = getenv("LZ4E_DECOMPRESS_MODE");
    uint32_t mode = a.mode;
    if (mode == kDecAuto && env)
        mode = env[0] == 'w'   ? kDecWave
               : env[0] == 'p' ? kDecPipe
               : env[0] == 's' ? kDecSmall
               : env[0] == 'g' ? kDecGroup
                               : kDecAuto;
    if (mode == kDecAuto)
        mode = (a.max_cap == 0 || (a.max_cap >= kPipeMinCap && a.max_cap < kPipeMaxCap))
                   ? kDecPipe
                   : (a.max_cap <= (uint32_t)kSmallOut && a.nblocks >= kGroupMinBlocks
                          ? kDecGroup
                          : (a.nblocks <= kLatencyMaxBlocks
                                 ? kDecPipe
                                 : (a.max_cap <= (uint32_t)kSmallOut && a.nblocks <= kSmallMaxBlocks ? kDecSmall
                                                                                                     : kDecWave)));
    if (mode == kDecPipe) {
        const int om = launch_order_mode(false);
        uint32_t* order = nullptr;
        if ((om == kOrderAlways || (om == kOrderAuto && a.nblocks > kOrderMin)) &&
            hipMallocAsync((void**)&order, sizeof(uint32_t) * a.nblocks, stream) == hipSuccess) {
            hipLaunchKernelGGL((order_kernel<DecodeWeight>), dim3(1), dim3(kOrderThreads), 0, stream,
                               DecodeWeight{a.src_len, a.dst_cap}, a.nblocks, order);
        } else {
            (void)hipGetLastError();  // a failed pool allocation only costs the ordering
            order = nullptr;
        }
        hipLaunchKernelGGL((decompress_pipe_kernel<kStamps>), dim3(a.nblocks), dim3(kPipeWaves * kWave),
                           0, stream, a.src, a.src_off, a.src_len, a.dst, a.dst_off, a.dst_cap, a.ret,
                           a.nblocks, dbg, a.dict_len, (const uint32_t*)order);
        const hipError_t err = hipGetLastError();
        if (order) (void)hipFreeAsync(order, stream);
        return err;
    }
    if (mode == kDecGroup || mode == kDecGroupNoBail) {
        // hand-over list (count + 3 words per block); without it (or in the
        // no-hand-over test mode) every group decodes its block to the end
        uint32_t* ho = nullptr;
        if (mode == kDecGroup && (hipMallocAsync((void**)&ho, 4 + 12 * (size_t)a.nblocks, stream) != hipSuccess ||
                                  hipMemsetAsync(ho, 0, 4, stream) != hipSuccess)) {
            (void)hipGetLastError();
            if (ho) (void)hipFreeAsync(ho, stream);
            ho = nullptr;
        }
        hipLaunchKernelGGL(decompress_group_kernel, dim3((a.nblocks + kGroupWg / kGroup - 1) / (kGroupWg / kGroup)),
                           dim3(kGroupWg), 0, stream, a.src, a.src_off, a.src_len, a.dst, a.dst_off, a.dst_cap,
                           a.ret, a.nblocks, a.dict_len, ho);
        hipError_t err = hipGetLastError();
        if (ho) {
            if (err == hipSuccess) {
                hipLaunchKernelGGL((decompress_resume_kernel<kStamps>), dim3(a.nblocks), dim3(kWave), 0, stream, a.src,
                                   a.src_off, a.src_len, a.dst, a.dst_off, a.dst_cap, a.ret, ho, dbg,
                                   a.dict_len);
                err = hipGetLastError();
            }
            (void)hipFreeAsync(ho, stream);
        }
        return err;
    }
    if (mode == kDecSmall)
        hipLaunchKernelGGL((decompress_kernel<kStamps, true>), dim3(a.nblocks), dim3(kWave), 0, stream,
                           a.src, a.src_off, a.src_len, a.dst, a.dst_off, a.dst_cap, a.ret, a.nblocks,
                           dbg, a.dict_len);
    else
        hipLaunchKernelGGL((decompress_kernel<kStamps>), dim3(a.nblocks), dim3(kWave), 0, stream,
                           a.src, a.src_off, a.src_len, a.dst, a.dst_off, a.dst_cap, a.ret, a.nblocks,
                           dbg, a.dict_len);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_decompress(const DecompressBatch& a, hipStream_t stream) {
    return launch_impl<false>(a, stream, nullptr);
}

hipError_t launch_decompress_stamped(const DecompressBatch& a, hipStream_t stream, uint64_t* dbg) {
    return launch_impl<true>(a, stream, dbg);
}

}  // namespace lz4e
