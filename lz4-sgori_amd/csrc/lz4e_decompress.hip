// lz4e_decompress.hip -- gfx950 LZ4E safe block decoder.
//
// Restates /root/reference/lz4e/lz4e_decompress.c:62-469
// (LZ4E_decompress_generic, instance endOnInputSize + decode_full_block +
// noDict) on one wave64 per block, in batches of up to 64 sequences:
//
//  1. Parse: the token stream is walked wave-uniformly (scalar registers)
//     with the reference's exact sequence of bound checks -- including the
//     two-stage 16/18-byte shortcut, whose entry conditions change which
//     malformed inputs are rejected and where -- so the return value,
//     including the error code -(ip - src) - 1, is the reference's.  The
//     compressed bytes come from two 256-byte register windows read with
//     v_readlane (a third is prefetched one segment ahead).  Sequence k of
//     the batch is recorded in lane k (literal source, literal length,
//     output position, offset, match length).  Errors depend only on the
//     token stream, so a failing block stops here.
//  2. Literals: every lane copies its own run; runs longer than kLong are
//     copied by the whole wave.
//  3. Matches, in dependency rounds: a match is ready once the part of its
//     source before its own output overlaps no earlier match of the batch
//     that is still pending (checked exactly against each pending interval).
//     Ready short matches are copied per lane, every load before any store;
//     long ones by the whole wave in lane order.  Overlapping matches follow LZ semantics
//     out[op + t] = out[op - off + t mod off]; offset 0 writes zeros, which
//     is what the reference's LZ4_write32(op, offset) + overlap copy produce
//     (lz4e_decompress.c:313, 407-415).
//
// Output placement: every block decodes in place in its HBM destination.
// A fast batch (no extension bytes, far from both block ends) is first
// assembled in a small LDS span -- literals from a 1 KiB LDS ring that
// mirrors the compressed segments the parse loaded, the part of each match
// source before the batch from HBM in one round trip, the rest in LDS
// dependency rounds or, for chains of dependent matches, by pointer jumping
// over the span's bytes -- and written to HBM with one pass of 16-byte
// stores.  Scalar-path batches (long runs, block ends) copy in HBM directly;
// same-wave stores and loads to one global address are ordered by the
// hardware (one vector L1 per CU), and wavefront-scope fences keep the
// compiler from moving a phase's loads above the previous phase's stores.
// LDS per block: ring 1 KiB + mirror 128 B + store sink 256 B + span 2,112 B
// + jump table 4,224 B = 7,744 B.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>


#include "lz4e_device.h"
#include "lz4e_gpu.h"

namespace lz4e {

namespace {

constexpr int32_t kLong = 64;  // longer literal runs / matches go to the whole wave

// LDS per block: the input ring (+ mirror), the store sink, the span buffer.
constexpr uint32_t kRing = 1024;                    // 4 segments of 256 B
constexpr uint32_t kRingPad = 128;                  // mirror of ring bytes [0, 128)
constexpr uint32_t kSink = 4 * kWave;               // a dword per lane for unwanted stores
constexpr uint32_t kSpan = 64 * 32 + 16 + 48;       // a fast batch's output, 16-B aligned start
constexpr uint32_t kJump = 2 * kSpan;               // u16 per span byte (chain resolution)
constexpr uint16_t kFinal = 0xFFFF;                 // jump entry of a byte whose value is final

typedef __attribute__((address_space(3))) uint8_t lu8;
typedef __attribute__((address_space(3))) uint32_t lu32;
typedef __attribute__((address_space(3))) uint16_t lu16;
typedef uint32_t __attribute__((aligned(1))) u32a1;
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

    LZ4E_DEV uint32_t load(int32_t wi) const {
        wi = wi < 0 ? 0 : wi;
        return w[wi < last ? wi : last];
    }
    LZ4E_DEV void put_ring(int32_t s, uint32_t v) const {
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
    LZ4E_DEV uint32_t rd4(int32_t p) const {
        return ld4(reinterpret_cast<const lu8*>(ring) + ((uint32_t)(p + shift) & (kRing - 1)));
    }
    LZ4E_DEV uint32_t rd16(int32_t p) const { return rd4(p) & 0xFFFFu; }
    // The ring copy of block bytes [p, p + n), or nullptr when not all held.
    LZ4E_DEV const lu8* in_ring(int32_t p, int32_t n) const {
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
LZ4E_DEV void wave_copy(uint8_t* dst, const uint8_t* src, int32_t len, uint32_t lane) {
    int32_t k = 16 * (int32_t)lane;
    for (; k + 16 <= len; k += 16 * kWave)
        *reinterpret_cast<uint4*>(dst + k) = *reinterpret_cast<const uint4*>(src + k);
    for (int32_t t = (len & ~15) + lane; t < len; t += kWave) dst[t] = src[t];
}

// Whole-wave match copy: out[op + t] = out[op - off + t mod off].
LZ4E_DEV void wave_match(uint8_t* out, int32_t op, uint32_t off, int32_t len, uint32_t lane) {
    if (off == 0) {
        for (int32_t t = lane; t < len; t += kWave) out[op + t] = 0;
        return;
    }
    if (off >= 16 * kWave) {
        // each 1 KiB step reads bytes written before the step
        for (int32_t k0 = 0; k0 < len; k0 += 16 * kWave) {
            const int32_t k = k0 + 16 * (int32_t)lane;
            if (k + 16 <= len) {
                *reinterpret_cast<uint4*>(out + op + k) =
                    *reinterpret_cast<const uint4*>(out + op - off + k);
            } else {
                for (int32_t t = k; t < len && t < k + 16; ++t) out[op + t] = out[op - off + t];
            }
            wave_fence();
        }
        return;
    }
    // off < 1024: period P = off * ceil(1024 / off) >= 1024; the first P bytes
    // come from the final period [op-off, op), the rest from P bytes back.
    const int32_t P = (int32_t)off * ((16 * kWave + off - 1) / off);
    const int32_t head = len < P ? len : P;
    for (int32_t t = lane; t < head; t += kWave) out[op + t] = out[op - off + (t % off)];
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
    return (shfl(tab, x >> 2) >> ((x & 3) * 8)) & 0xFFu;
}

// The composed table B[A[p]] for this lane's 4 positions p.
LZ4E_DEV uint32_t table_compose(uint32_t A, uint32_t B) {
    uint32_t r = 0;
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) r |= table_at(B, (A >> (8 * q)) & 0xFFu) << (8 * q);
    return r;
}

struct Stamps {
    uint64_t t = 0, acc[4] = {0, 0, 0, 0}, batches = 0, rounds = 0;
};

// Decode one block into HBM.  LDS: the input ring, the store sink and the
// span buffer of the fast batches.
template <bool kStamps>
LZ4E_DEV void decode_block(const uint8_t* in, int32_t srcSize, uint8_t* gout, int32_t outSize,
                           int32_t* ret_slot, uint64_t* dbg, uint32_t lane, lu8* span,
                           lu32* ring, lu16* jump) {
    Stamps st;
    auto lap = [&](int ph) {
        if constexpr (kStamps) {
            const uint64_t now = clock64();
            st.acc[ph] += now - st.t;
            st.t = now;
        }
    };
    if constexpr (kStamps) st.t = clock64();
    lu8* sink = (lu8*)ring + kRing + kRingPad + 4 * lane;  // (span follows the sink)

    InWindow win;
    {
        const uintptr_t a = reinterpret_cast<uintptr_t>(in);
        win.shift = (int32_t)(a & 3);
        win.w = (gcu32*)(a - win.shift);
        win.last = (srcSize + win.shift - 1) >> 2;
        win.lane = lane;
        win.ring = ring;
        win.reload(0);
    }

    const int32_t iend = srcSize, oend = outSize;
    const int32_t shortiend = iend - 14 - 2;  // :100-101
    const int32_t shortoend = oend - 14 - 18; // :102-103
    int32_t ip = 0, op = 0;
    bool done = false;

    while (!done) {
        // ------------------------------------------------ 1. parse a batch
        int32_t r_ls = 0, r_L = 0, r_op = 0, r_off = 0, r_M = 0;  // lane k: sequence k
        uint32_t nseq = 0;
        bool fastb = false;  // the batch came from the fast path (span-staged copies)

        // 1a. Fast path: a run of tokens with no length-extension bytes, far
        // from both block ends, where the reference takes its two-stage
        // shortcut (:150-191).  The token chain inside the 256-byte window at
        // ip is found by pointer doubling: jump tables J_{2^i} (window offset
        // -> offset 2^i tokens on, 255 = chain end; one byte per position,
        // lane l holding positions 4l..4l+3) are composed with ds_bpermute
        // gathers, then lane k follows the bits of k to token k.  Every field
        // and check is then evaluated per lane.
        if (ip <= iend - 18 && op <= oend - 32) {
            win.follow(ip);
            const int32_t r0 = ip - win.base;                  // < 256
            const int32_t rin = iend - 18 - win.base;          // last token offset on the fast path
            const int32_t jlim = (rin < 494 ? rin : 494) - r0;  // (offset bytes stay in A+B)
            const uint32_t wv = win.rd4(ip + 4 * (int32_t)lane);
            uint32_t J[6];
            {
                uint32_t j1 = 0;
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    const uint32_t t = (wv >> (8 * q)) & 0xFFu, p = 4 * lane + q;
                    const uint32_t n = p + (t >> 4) + 3;
                    const bool go = (t >> 4) != 15 && (t & 15) != 15 && (int32_t)p <= jlim && n <= 254;
                    j1 |= (go ? n : 255u) << (8 * q);
                }
                J[0] = j1;
            }
#pragma unroll
            for (int i = 1; i < 6; ++i) J[i] = table_compose(J[i - 1], J[i - 1]);
            uint32_t x = 0;  // lane k: window offset of token k (255: past the chain)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const uint32_t y = table_at(J[i], x);
                x = (lane >> i) & 1 ? y : x;
            }
            const uint32_t t = table_at(wv, x);  // token byte
            const int32_t L = (int32_t)(t >> 4), Mt = (int32_t)(t & 15);
            const bool cand = x != 255 && L != 15 && Mt != 15 && (int32_t)x <= jlim;
            const int32_t lp = ip + (int32_t)x + 1;  // literal start
            const int32_t off = cand ? (int32_t)win.rd16(lp + L) : 0;
            const int32_t size = cand ? L + Mt + 4 : 0;
            const int32_t incl = (int32_t)wave_incl_add((uint32_t)size);
            const int32_t o_k = op + incl - size;
            const int32_t m_k = o_k + L;
            // the reference's checks on this path: shortcut entry (op <= oend-32,
            // input side guaranteed by jlim), match inside the block (:299-302),
            // and for offsets < 8 the _copy_match end check (:422-431)
            const bool ok = cand && o_k <= oend - 32 && m_k >= off &&
                            (off >= 8 || m_k + Mt + 4 <= oend - 5);
            const uint64_t okm = ballot(ok);
            const uint32_t nf = (~okm) ? ctz64(~okm) : kWave;  // first failing lane
            if (nf > 0) {
                fastb = true;
                r_ls = lp;
                r_L = L;
                r_op = o_k;
                r_off = off;
                r_M = Mt + 4;
                nseq = nf;
                op += lane_val((uint32_t)incl, nf - 1);
                ip = lane_val((uint32_t)(lp + L + 2), nf - 1);  // the token after the last one
            }
        }

        // 1b. Exact scalar path (extension bytes, block ends, anything the
        // fast path declined): until the fast path applies again.
        while (nseq == 0) {
            win.follow(ip);  // ip now in window A: bytes up to ip + 256 are readable unchecked
            const uint32_t r0 = (uint32_t)(ip - win.base);
            const uint32_t token = win.ubyte(r0);
            ip++;
            uint32_t length = token >> 4;  // saturates at kSat
            int32_t offset = 0, lit_ip, lit_op;
            uint32_t L;

            if (length != 15 && ip < shortiend && op <= shortoend) {
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
                uint32_t s;
                do {
                    s = win.byte(ip);
                    ip++;
                    length = length + s > kSat ? kSat : length + s;
                } while (ip < iend - 15 && s == 255);
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
                    done = true;  // final literal run: no match
                    goto record;
                }
                ip += (int32_t)length;
                op = (int32_t)cpy;
            }
            offset = (int32_t)(win.byte(ip) | (win.byte(ip + 1) << 8));  // :291-296
            ip += 2;
            length = token & 15;

        copy_match_checks:
            // _copy_match (:298-336, :422-431)
            if (op - offset < 0) goto fail;
            if (length == 15) {
                uint32_t s;
                do {
                    s = win.byte(ip);
                    ip++;
                    if (ip > iend - 5) goto fail;
                    length = length + s > kSat ? kSat : length + s;
                } while (s == 255);
            }
            if (ugt((uint32_t)op + length + 4, oend - 5)) goto fail;
            length += 4;

        record:
            {
                const bool me = lane == nseq;  // v_cndmask into lane nseq
                r_ls = me ? lit_ip : r_ls;
                r_L = me ? (int32_t)L : r_L;
                r_op = me ? lit_op : r_op;
                r_off = me ? offset : r_off;
                r_M = me ? (int32_t)length : r_M;
            }
            op += (int32_t)length;
            nseq++;
            break;
        }
        lap(0);
        if constexpr (kStamps) st.batches++;
        const bool valid = lane < nseq;
        if (fastb) {
            // ---------------- span-staged copies (fast batches) -------------
            // The batch's output [lo, op) (<= 64 x 32 bytes) is assembled in
            // LDS: literals from the ring; the part of a match source that
            // lies before lo from HBM (final: written by earlier batches);
            // the rest in LDS dependency rounds.  Then one store pass.
            const int32_t lo = lane_val((uint32_t)r_op, 0);
            const int32_t a0 = lo & ~15;  // span index of position x: x - a0
            const int32_t ms = r_op + r_L, ss = ms - r_off;
            int32_t n0 = 0;
            uint4 h0 = make_uint4(0, 0, 0, 0), h1 = h0;
            if (valid && ss < lo) {  // fast path: lo <= oend - 32, so [ss, ss + 32) is in the block
                n0 = r_M < lo - ss ? r_M : lo - ss;
                h0 = ldg16(gout + ss);
                if (n0 > 16) h1 = ldg16(gout + ss + 16);
            }
            if (valid && r_L > 0) {
                const lu8* rs = win.in_ring(r_ls, r_L);
                if (rs) lane_copy(span + (r_op - a0), rs, r_L, sink);
                else lane_copy64(span + (r_op - a0), in + r_ls, r_L, in + srcSize);
            }
            if (n0 > 0) {
                put16(span + (ms - a0), h0, n0 < 16 ? n0 : 16, sink);
                if (n0 > 16) put16(span + (ms - a0) + 16, h1, n0 - 16, sink);
            }
            lap(1);
            const int32_t ms2 = ms + n0, m2 = r_M - n0, me = ms + r_M;
            const int32_t ss2 = ss + n0;
            const int32_t need = me - r_off < ms2 ? me - r_off : ms2;  // source part before own output
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
                                                       ms2 - a0, m2, r_off, lane);
                    if constexpr (kStamps) st.rounds += nr;
                    pending = 0;
                    break;
                }
                if (ready) {
                    if (r_off != 0) lane_match(span + (ms2 - a0), (uint32_t)r_off, m2, sink);
                    else lane_zero(span + (ms2 - a0), m2, sink);
                }
                pending &= ~rm;
                if constexpr (kStamps) st.rounds++;
            }
            lap(2);
            // store pass: 16-byte HBM chunks of [lo, op); partial end chunks by bytes
            const int32_t nch = (op - a0 + 15) >> 4;
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
            continue;
        }
        // ---------------- in-HBM copies (scalar-path batches) ---------------
        // ------------------------------------------------ 2. literals
        wave_fence();
        if (valid && r_L > 0 && r_L <= kLong) lane_copy64(gout + r_op, in + r_ls, r_L, in + srcSize);
        {
            uint64_t longs = ballot(valid && r_L > kLong);
            while (longs) {
                const uint32_t j = ctz64(longs);
                longs &= longs - 1;
                wave_copy(gout + lane_val(r_op, j), in + lane_val(r_ls, j), (int32_t)lane_val(r_L, j),
                          lane);
            }
        }
        wave_fence();
        lap(1);

        // ------------------------------------------------ 3. matches
        {
            const int32_t ms = r_op + r_L;  // match start
            const int32_t me = ms + r_M;    // match end
            const int32_t need = me - r_off < ms ? me - r_off : ms;  // source part before own output
            const int32_t ss = ms - r_off;  // source start
            const int32_t batch_lo = lane_val(r_op, 0);
            uint64_t pending = ballot(valid && r_M > 0);
            while (pending) {
                // Ready when [ss, need) is final: before this batch's output, or
                // before every pending earlier match, or after all of them.
                const bool mine = (pending >> lane) & 1;
                const bool quick = need <= batch_lo;
                bool ready = mine && quick;
                if (ballot(mine && !quick)) {
                    const int32_t mn = wave_excl_min(mine ? ms : INT32_MAX);
                    const int32_t mx = wave_excl_max(mine ? me : INT32_MIN);
                    ready = mine && (quick || need <= mn || ss >= mx);
                }
                if (ready && r_M <= kLong) lane_match(gout + ms, (uint32_t)r_off, r_M, gout + outSize);
                wave_fence();
                uint64_t longs = ballot(ready && r_M > kLong);
                while (longs) {
                    const uint32_t j = ctz64(longs);
                    longs &= longs - 1;
                    wave_match(gout, lane_val(ms, j), lane_val(r_off, j), lane_val(r_M, j), lane);
                    wave_fence();
                }
                pending &= ~ballot(ready);
                if constexpr (kStamps) st.rounds++;
            }
        }
        wave_fence();
        lap(2);
    }
    if (lane == 0) *ret_slot = op;
    goto finish;
fail:
    if (lane == 0) *ret_slot = -ip - 1;
finish:
    if constexpr (kStamps) {
        if (lane == 0 && dbg) {
            dbg[0] = st.acc[0];
            dbg[1] = st.acc[1];
            dbg[2] = st.acc[2];
            dbg[3] = st.batches;
            dbg[4] = st.rounds;
            dbg[5] = st.acc[3];
        }
    }
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

template <bool kStamps>
__global__ __launch_bounds__(64) void decompress_kernel(const uint8_t* __restrict__ src,
                                                        const uint64_t* __restrict__ src_off,
                                                        const int32_t* __restrict__ src_len,
                                                        uint8_t* dst,
                                                        const uint64_t* __restrict__ dst_off,
                                                        const int32_t* __restrict__ dst_cap,
                                                        int32_t* __restrict__ ret, uint32_t nblocks,
                                                        uint64_t* __restrict__ dbg) {
    const uint32_t b = blockIdx.x;
    if (b >= nblocks) return;
    const uint32_t lane = lane_id();
    const int32_t srcSize = src_len[b];
    const int32_t outSize = dst_cap[b];
    const uint8_t* in = src + src_off[b];
    uint8_t* out = dst + dst_off[b];
    uint64_t* d = kStamps && dbg ? dbg + 8 * (size_t)b : nullptr;
    if (special_case(in, srcSize, outSize, ret + b, lane)) return;
    // LDS: [input ring + mirror] [store sink] [span]
    __shared__ __attribute__((aligned(16))) uint8_t smem[kRing + kRingPad + kSink + kSpan + kJump];
    decode_block<kStamps>(in, srcSize, out, outSize, ret + b, d, lane,
                          (lu8*)(smem + kRing + kRingPad + kSink), (lu32*)smem,
                          (lu16*)(smem + kRing + kRingPad + kSink + kSpan));
}

// ============================================================================
// Workgroup decoder: one block per 256-thread workgroup, output image in LDS
// ============================================================================
//
// For blocks whose capacity is at most 64 KiB (the 4 KiB and 64 KiB chunk
// sizes).  The one-wave decoder above is bound by its serial chain: one
// batch of <= 64 sequences at a time, and dependent short matches (records,
// integer tables) resolved a few bytes per lane per round.  Here the four
// waves of a workgroup share the block:
//
//  1. Parse, a 1 KiB window of the token stream per batch.  Every window
//     position is parsed speculatively as if a token started there (its next
//     token position J1, extension bytes included); the true tokens are the
//     orbit of the window's first position, found by pointer doubling over
//     J (J2 = J1 o J1, ...) with the marking rule
//     mark(J_{2^k}(p)) |= mark(p): after 9 levels every chain element of
//     index < 512 (> the 342 tokens a 1 KiB window can hold) is marked.
//     A workgroup scan over the marks gives each token its rank and output
//     position.
//  2. Check, per token, every bound the reference tests on its path
//     (lz4e_decompress.c:123-446: the two-stage shortcut's entry
//     conditions, literal end margins, extension-byte limits, offset inside
//     the output, match end margin, the exact final literal run).  A block
//     with any token that fails them -- malformed input, a too-small
//     capacity -- is decoded from scratch by the one-wave exact decoder
//     above (wave 0), so return values and error codes are the reference's
//     by construction.  Blocks that pass produce the reference's bytes: its
//     copies implement plain LZ semantics (offset 0 writes zeros).
//  3. Literals: per sequence, long runs by the whole workgroup.
//  4. Matches, in output sub-spans of 2 KiB: every byte finds its sequence
//     (scatter of sequence starts + max scan), a byte whose source lies
//     before the sub-span (self-overlap folded: out[m + t] =
//     out[m - off + t mod off]) or in a literal is final at once; the rest
//     point at their source byte and resolve by pointer jumping (a chain of
//     depth d in log2 d rounds).
//  5. The finished image leaves LDS in 16-byte stores.
constexpr uint32_t kWgT = 256;                  // threads per workgroup (4 waves)
constexpr uint32_t kWgWaves = kWgT / kWave;
constexpr uint32_t kWin = 1024;                 // token-stream bytes parsed per batch
constexpr uint32_t kWinPad = 256;               // staged bytes past the window
constexpr uint32_t kMaxSeq = kWin / 3 + 2;      // a non-final sequence takes >= 3 input bytes
constexpr uint32_t kSub = 2048;                 // output bytes resolved per sub-span
constexpr uint32_t kOutMax = 65536;             // largest capacity this decoder takes
constexpr uint32_t kLevels = 9;                 // 2^9 > kMaxSeq
constexpr uint16_t kNone = 0xFFFF;              // no target / final byte
constexpr uint32_t kLongLit = 64;               // longer literal runs: whole workgroup
constexpr uint32_t kMaxLong = 32;
constexpr uint32_t kLenCap = 1u << 20;          // speculative lengths saturate here

struct WgLds {
    uint8_t out[kOutMax + 16];
    uint8_t win[kWin + kWinPad + 16];
    union {
        struct {
            uint16_t a[kWin], b[kWin];  // J_{2^k}, J_{2^{k+1}} (window offsets)
        } j;
        uint16_t ptr[kSub];  // sub-span: sequence id + 1, then source byte / kNone
    } u;
    uint8_t mark[kWin];
    uint32_t s_op[kMaxSeq], s_lit[kMaxSeq], s_len[kMaxSeq], s_off[kMaxSeq], s_m4[kMaxSeq];
    uint32_t red[4 * kWgWaves];
    uint32_t longs[kMaxLong];
    int32_t st[8];
};
static_assert(sizeof(WgLds) <= 81920, "two workgroups per CU");
static_assert(kRing + kRingPad + kSink + kSpan + kJump <= kOutMax, "fallback LDS inside the image");

typedef __attribute__((address_space(1))) const uint8_t gcu8;
typedef __attribute__((address_space(1))) const u32a1 gcu32a1;

// The staged window [ip0, ip0 + kWin + kWinPad) from LDS, anything else from
// HBM (zero past the input, like the staging).
struct WinSrc {
    const uint8_t* win;
    gcu8* in;
    int32_t n, ip0;
    LZ4E_DEV uint32_t at(int32_t q) const {
        const uint32_t r = (uint32_t)(q - ip0);
        if (r < kWin + kWinPad) return win[r];
        return q < n ? in[q] : 0u;
    }
};

// One sequence read as if a token started at t (lz4e_decompress.c:123-336
// field layout): literal start/length, offset, position after the match
// length's extension bytes (the next token), match length + MINMATCH.
struct Tok {
    uint32_t token, lit, len, off, xm, m4;
};

LZ4E_DEV Tok parse_tok(const WinSrc& S, int32_t t) {
    Tok k;
    k.token = S.at(t);
    uint32_t L = k.token >> 4, M = k.token & 15;
    int32_t x = t + 1;
    if (L == 15) {
        uint32_t s;
        do {
            s = S.at(x++);
            L += s;
        } while (s == 255 && x < S.n && L < kLenCap);
    }
    k.lit = (uint32_t)x;
    k.len = L;
    x += (int32_t)L;
    k.off = S.at(x) | (S.at(x + 1) << 8);
    x += 2;
    if (M == 15) {
        uint32_t s;
        do {
            s = S.at(x++);
            M += s;
        } while (s == 255 && x < S.n && M < kLenCap);
    }
    k.xm = (uint32_t)x;
    k.m4 = M + 4;
    return k;
}

// Next-token offset of window position r if a token started there, or kNone
// when that lies at or past the window end (only the staged bytes are read:
// anything longer leaves the window anyway).
LZ4E_DEV uint16_t jump1(const uint8_t* win, uint32_t r) {
    const uint32_t tok = win[r];
    uint32_t L = tok >> 4, x = r + 1;
    if (L == 15) {
        uint32_t s;
        do {
            s = win[x++];
            L += s;
        } while (s == 255 && x < kWin);
    }
    x += L + 2;
    if (x >= kWin) return kNone;
    if ((tok & 15) == 15) {
        uint32_t s;
        do {
            s = win[x++];
        } while (s == 255 && x < kWin);
    }
    return x < kWin ? (uint16_t)x : kNone;
}

// Exclusive workgroup prefix sums of two values; totals through t0 / t1.
LZ4E_DEV void wg_scan2(uint32_t v0, uint32_t v1, uint32_t* red, uint32_t tid, uint32_t& e0,
                       uint32_t& e1, uint32_t& t0, uint32_t& t1) {
    const uint32_t i0 = wave_incl_add(v0), i1 = wave_incl_add(v1);
    const uint32_t w = tid / kWave;
    if (tid % kWave == kWave - 1) {
        red[w] = i0;
        red[kWgWaves + w] = i1;
    }
    __syncthreads();
    uint32_t b0 = 0, b1 = 0, s0 = 0, s1 = 0;
#pragma unroll
    for (uint32_t i = 0; i < kWgWaves; ++i) {
        const uint32_t r0 = red[i], r1 = red[kWgWaves + i];
        if (i < w) b0 += r0, b1 += r1;
        s0 += r0, s1 += r1;
    }
    __syncthreads();
    e0 = b0 + i0 - v0;
    e1 = b1 + i1 - v1;
    t0 = s0;
    t1 = s1;
}

// Exclusive workgroup prefix max of values >= 0 (0 for the first thread).
LZ4E_DEV int32_t wg_excl_max(int32_t v, uint32_t* red, uint32_t tid) {
    const int32_t ex = wave_excl_max(v);  // lane 0: INT32_MIN
    const int32_t in = ex > v ? ex : v;
    const uint32_t w = tid / kWave;
    if (tid % kWave == kWave - 1) red[2 * kWgWaves + w] = (uint32_t)in;
    __syncthreads();
    int32_t b = 0;
#pragma unroll
    for (uint32_t i = 0; i < kWgWaves; ++i)
        if (i < w) b = b > (int32_t)red[2 * kWgWaves + i] ? b : (int32_t)red[2 * kWgWaves + i];
    __syncthreads();
    return b > ex ? b : ex;
}

// len literal bytes at lit into the image at o (one thread).
LZ4E_DEV void lit_copy(uint8_t* out, uint32_t o, const WinSrc& S, uint32_t lit, uint32_t len) {
    const uint32_t r = lit - (uint32_t)S.ip0;
    uint8_t* d = out + o;
    uint32_t k = 0;
    if (r + len <= kWin + kWinPad) {
        const uint8_t* s = S.win + r;
        for (; k + 4 <= len; k += 4) st4((lu8*)(d + k), ld4((const lu8*)(s + k)));
        for (; k < len; ++k) d[k] = s[k];
    } else {
        gcu8* s = S.in + lit;
        for (; k + 4 <= len; k += 4) st4((lu8*)(d + k), *(gcu32a1*)(s + k));
        for (; k < len; ++k) d[k] = s[k];
    }
}

// The one-wave exact decoder on wave 0 (reference bound checks and error
// codes), LDS carved from the image.
LZ4E_DEV void wg_fallback(WgLds& L, const uint8_t* in, int32_t srcSize, uint8_t* gout,
                          int32_t outSize, int32_t* ret_slot, uint32_t tid) {
    if (tid >= kWave) return;
    uint8_t* smem = L.out;
    decode_block<false>(in, srcSize, gout, outSize, ret_slot, nullptr, tid,
                        (lu8*)(smem + kRing + kRingPad + kSink), (lu32*)smem,
                        (lu16*)(smem + kRing + kRingPad + kSink + kSpan));
}

// Phase cycle counters of the diagnostic build (tid 0's clock; phases are
// separated by workgroup barriers): stage+J1, doubling, tokens, literals,
// matches, flush, batches, sub-span rounds.
struct WgStamps {
    uint64_t t = 0, acc[6] = {0, 0, 0, 0, 0, 0}, batches = 0, rounds = 0;
    LZ4E_DEV void lap(bool on, int ph) {
        if (!on) return;
        const uint64_t now = clock64();
        acc[ph] += now - t;
        t = now;
    }
};

template <bool kStamps>
__global__ __launch_bounds__(kWgT) void decompress_wg_kernel(const uint8_t* __restrict__ src,
                                                             const uint64_t* __restrict__ src_off,
                                                             const int32_t* __restrict__ src_len,
                                                             uint8_t* dst,
                                                             const uint64_t* __restrict__ dst_off,
                                                             const int32_t* __restrict__ dst_cap,
                                                             int32_t* __restrict__ ret,
                                                             uint32_t nblocks,
                                                             uint64_t* __restrict__ dbg) {
    __shared__ __attribute__((aligned(16))) WgLds L;
    WgStamps stp;
    const bool on = kStamps && threadIdx.x == 0;
    if (on) stp.t = clock64();
    const uint32_t b = blockIdx.x;
    if (b >= nblocks) return;
    const uint32_t tid = threadIdx.x;
    const int32_t srcSize = src_len[b];
    const int32_t outSize = dst_cap[b];
    const uint8_t* in = src + src_off[b];
    uint8_t* gout = dst + dst_off[b];
    if (special_case(in, srcSize, outSize, ret + b, tid)) return;
    if (outSize > (int32_t)kOutMax) {
        wg_fallback(L, in, srcSize, gout, outSize, ret + b, tid);
        return;
    }
    const int32_t iend = srcSize, oend = outSize;
    int32_t ip0 = 0, op = 0;
    bool fallback = false, done = false;

    while (!done) {
        // ---- stage the window, speculative next-token table --------------
        for (uint32_t i = tid; i < kWin + kWinPad; i += kWgT) {
            const int32_t q = ip0 + (int32_t)i;
            L.win[i] = q < srcSize ? in[q] : 0;
        }
        if (tid == 0) L.st[5] = 0;  // long literal runs of this batch
        __syncthreads();
        const WinSrc S{L.win, (gcu8*)in, srcSize, ip0};
#pragma unroll
        for (uint32_t k = 0; k < kWin / kWgT; ++k) {
            const uint32_t r = tid + k * kWgT;
            L.u.j.a[r] = ip0 + (int32_t)r < srcSize ? jump1(L.win, r) : kNone;
            L.mark[r] = r == 0;
        }
        __syncthreads();
        stp.lap(on, 0);
        if (on) stp.batches++;
        // ---- the true token chain: doubling + marking --------------------
        {
            uint16_t* A = L.u.j.a;
            uint16_t* B = L.u.j.b;
            for (uint32_t lev = 0; lev < kLevels; ++lev) {
                uint16_t nb[kWin / kWgT];
#pragma unroll
                for (uint32_t k = 0; k < kWin / kWgT; ++k) {
                    const uint32_t r = tid + k * kWgT;
                    const uint16_t a = A[r];
                    nb[k] = kNone;
                    if (a != kNone) {
                        if (L.mark[r]) L.mark[a] = 1;  // racy reads only add true tokens
                        nb[k] = A[a];
                    }
                }
                __syncthreads();
                if (lev + 1 < kLevels) {
#pragma unroll
                    for (uint32_t k = 0; k < kWin / kWgT; ++k) B[tid + k * kWgT] = nb[k];
                    __syncthreads();
                    uint16_t* t = A;
                    A = B;
                    B = t;
                }
            }
        }
        stp.lap(on, 1);
        // ---- tokens: rank, output position, the reference's checks --------
        const uint32_t mk = *reinterpret_cast<const uint32_t*>(&L.mark[4 * tid]);
        Tok tk[4];
        uint32_t cnt = 0, osz = 0;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            if ((mk >> (8 * q)) & 0xFF) {
                tk[q] = parse_tok(S, ip0 + (int32_t)(4 * tid + q));
                const bool fin = (int64_t)tk[q].lit + tk[q].len == iend;
                cnt++;
                osz += tk[q].len + (fin ? 0u : tk[q].m4);
                if (osz > kLenCap) osz = kLenCap;  // malformed: caught by the checks
            }
        }
        uint32_t rank, obase, nseq, osum;
        wg_scan2(cnt, osz, L.red, tid, rank, obase, nseq, osum);
        bool bad = false, fin_here = false;
        int32_t o = op + (int32_t)obase;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            if (!((mk >> (8 * q)) & 0xFF)) continue;
            const Tok& k = tk[q];
            const int32_t t = ip0 + (int32_t)(4 * tid + q);
            const uint32_t Lnib = k.token >> 4, Mnib = k.token & 15;
            const int64_t litEnd = (int64_t)k.lit + k.len;
            const bool fin = litEnd == iend;
            // the two-stage shortcut's entry (:150-155)
            const bool sc = Lnib != 15 && t + 1 < iend - 16 && o <= oend - 32;
            // literal-length varint read exactly as the reference's bounded loop (:194-220)
            const bool lext = Lnib != 15 || (int64_t)k.lit <= (int64_t)iend - 15;
            bool ok;
            if (fin) {
                // final literal run (:223-288): not on the shortcut, fits the output
                ok = !sc && lext && (int64_t)o + k.len <= oend;
                fin_here = true;
            } else {
                const int64_t mo = (int64_t)o + k.len;  // match start
                // _copy_match (:298-336, :422-431): offset inside the output,
                // extension bytes before iend - 5, match end before oend - 5
                const bool cm = (int64_t)k.off <= mo &&
                                (Mnib != 15 || (int64_t)k.xm <= (int64_t)iend - 5) &&
                                mo + k.m4 <= (int64_t)oend - 5;
                if (sc) ok = (Mnib != 15 && k.off >= 8 && (int64_t)k.off <= mo) || cm;
                else ok = lext && mo <= (int64_t)oend - 12 && litEnd <= (int64_t)iend - 8 && cm;
                ok = ok && (int64_t)k.xm < iend;  // the next token exists
            }
            bad |= !ok;
            if (rank < kMaxSeq) {
                L.s_op[rank] = (uint32_t)o;
                L.s_lit[rank] = k.lit;
                L.s_len[rank] = k.len;
                L.s_off[rank] = k.off;
                L.s_m4[rank] = fin ? 0u : k.m4;
                if (k.len > kLongLit) {
                    const uint32_t li = atomicAdd((uint32_t*)&L.st[5], 1u);
                    if (li < kMaxLong) L.longs[li] = rank;
                    else bad = true;
                }
            } else {
                bad = true;
            }
            if (rank + 1 == nseq) {  // the batch's last token: where the next batch starts
                L.st[0] = (int32_t)k.xm;
                L.st[1] = fin;
            }
            o += (int32_t)(k.len + (fin ? 0u : k.m4));
            rank++;
        }
        bad = __syncthreads_or(bad ? 1 : 0) != 0 || nseq == 0;
        const bool any_fin = __syncthreads_or(fin_here ? 1 : 0) != 0;
        if (bad || (any_fin && !L.st[1])) {
            fallback = true;
            break;
        }
        stp.lap(on, 2);
        const int32_t op_b = op, op_e = op + (int32_t)osum;
        const int32_t next_ip = L.st[0];
        const uint32_t nlong = (uint32_t)L.st[5];

        // ---- literals ------------------------------------------------------
        for (uint32_t i = tid; i < nseq; i += kWgT) {
            const uint32_t len = L.s_len[i];
            if (len > 0 && len <= kLongLit) lit_copy(L.out, L.s_op[i], S, L.s_lit[i], len);
        }
        for (uint32_t li = 0; li < nlong; ++li) {
            const uint32_t i = L.longs[li];
            const uint32_t len = L.s_len[i], o0 = L.s_op[i], lit = L.s_lit[i];
            for (uint32_t k = 4 * tid; k < len; k += 4 * kWgT) {
                const uint32_t c = len - k < 4 ? len - k : 4;
                lit_copy(L.out, o0 + k, S, lit + k, c);
            }
        }
        __syncthreads();
        stp.lap(on, 3);

        // ---- matches, 2 KiB sub-spans -----------------------------------------
        for (int32_t a = op_b; a < op_e; a += (int32_t)kSub) {
            const int32_t span = op_e - a < (int32_t)kSub ? op_e - a : (int32_t)kSub;
            for (uint32_t j = tid; j < kSub; j += kWgT) L.u.ptr[j] = 0;
            __syncthreads();
            if (tid == 0) {
                // the sequence covering a: last one starting at or before it
                uint32_t lo = 0, hi = nseq - 1;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi + 1) / 2;
                    if ((int32_t)L.s_op[mid] <= a) lo = mid;
                    else hi = mid - 1;
                }
                L.u.ptr[0] = (uint16_t)(lo + 1);
            }
            for (uint32_t i = tid; i < nseq; i += kWgT) {
                const int32_t so = (int32_t)L.s_op[i];
                if (so > a && so < a + span) L.u.ptr[so - a] = (uint16_t)(i + 1);
            }
            __syncthreads();
            // byte j = kPer tid + q of the sub-span: its sequence (max scan)
            constexpr uint32_t kPer = kSub / kWgT;
            int32_t sid[kPer];
            int32_t run = 0;
#pragma unroll
            for (uint32_t q = 0; q < kPer; ++q) {
                const int32_t v = L.u.ptr[kPer * tid + q];
                run = run > v ? run : v;
                sid[q] = run;
            }
            const int32_t pre = wg_excl_max(run, L.red, tid);
            uint16_t pv[kPer];
            uint32_t pend = 0;  // my bytes still pointing at an unresolved source
            uint32_t cs = 0xFFFFFFFFu, c_o = 0, c_len = 0, c_off = 0;
#pragma unroll
            for (uint32_t q = 0; q < kPer; ++q) {
                const int32_t s1 = sid[q] > pre ? sid[q] : pre;
                const int32_t j = (int32_t)(kPer * tid + q);
                const int32_t x = a + j;
                pv[q] = kNone;
                if (j >= span || s1 == 0) continue;
                const uint32_t s = (uint32_t)s1 - 1;
                if (s != cs) {
                    cs = s;
                    c_o = L.s_op[s];
                    c_len = L.s_len[s];
                    c_off = L.s_off[s];
                }
                const int32_t m = (int32_t)(c_o + c_len);
                if (x < m) continue;  // literal: copied above
                if (c_off == 0) {     // offset 0 writes zeros (:313, 407-415)
                    L.out[x] = 0;
                    continue;
                }
                // out[m + t] = out[m - off + t mod off]: the source is before the match
                const uint32_t t = (uint32_t)(x - m);
                const int32_t srcp = (t >= c_off) ? m - (int32_t)c_off + (int32_t)(t % c_off)
                                                  : x - (int32_t)c_off;
                if (srcp < a) {
                    L.out[x] = L.out[srcp];  // final: every byte before the sub-span is
                } else {
                    pv[q] = (uint16_t)(srcp - a);
                    pend |= 1u << q;
                }
            }
            __syncthreads();  // every sequence id read before the pointers overwrite them
#pragma unroll
            for (uint32_t q = 0; q < kPer; ++q) L.u.ptr[kPer * tid + q] = pv[q];
            // pointer jumping: a byte whose source is final copies it, the
            // others jump to their source's source
            while (__syncthreads_or(pend != 0)) {
                uint8_t val[kPer];
                uint32_t got = 0;
#pragma unroll
                for (uint32_t q = 0; q < kPer; ++q) {
                    val[q] = 0;
                    if (!((pend >> q) & 1)) continue;
                    const uint16_t py = L.u.ptr[pv[q]];
                    if (py == kNone) {
                        val[q] = L.out[a + pv[q]];
                        got |= 1u << q;
                    } else {
                        pv[q] = py;
                    }
                }
                __syncthreads();
#pragma unroll
                for (uint32_t q = 0; q < kPer; ++q) {
                    if (!((pend >> q) & 1)) continue;
                    const uint32_t j = kPer * tid + q;
                    if ((got >> q) & 1) {
                        L.out[a + j] = val[q];
                        L.u.ptr[j] = kNone;
                    } else {
                        L.u.ptr[j] = pv[q];
                    }
                }
                pend &= ~got;
                if (on) stp.rounds++;
            }
        }
        stp.lap(on, 4);
        op = op_e;
        ip0 = next_ip;
        done = any_fin;
        __syncthreads();
    }
    if (fallback) {
        __syncthreads();
        wg_fallback(L, in, srcSize, gout, outSize, ret + b, tid);
        return;
    }
    // ---- the image to HBM: 16-byte stores ---------------------------------
    typedef __attribute__((address_space(1))) uint8_t gu8b;
    const uint32_t head = (uint32_t)((16 - (reinterpret_cast<uintptr_t>(gout) & 15)) & 15);
    const uint32_t n = (uint32_t)op;
    const uint32_t h = head < n ? head : n;
    for (uint32_t i = tid; i < h; i += kWgT) ((gu8b*)gout)[i] = L.out[i];
    const uint32_t body = (n - h) & ~15u;
    for (uint32_t c = h + 16 * tid; c < h + body; c += 16 * kWgT) {
        const lu8* s = (const lu8*)(L.out + c);
        stg16(gout + c, make_uint4(ld4(s), ld4(s + 4), ld4(s + 8), ld4(s + 12)));
    }
    for (uint32_t i = h + body + tid; i < n; i += kWgT) ((gu8b*)gout)[i] = L.out[i];
    if (tid == 0) ret[b] = op;
    if (kStamps) {
        __syncthreads();
        stp.lap(on, 5);
        if (on && dbg) {
            uint64_t* d = dbg + 8 * (size_t)b;
            for (int i = 0; i < 6; ++i) d[i] = stp.acc[i];
            d[6] = stp.batches;
            d[7] = stp.rounds;
        }
    }
}

template <bool kStamps>
hipError_t launch_impl(const DecompressBatch& a, hipStream_t stream, uint64_t* dbg) {
    if (a.nblocks == 0) return hipSuccess;
    // LZ4E_DECOMPRESS_WAVE=1 keeps every block on the one-wave decoder (A/B).
    static const bool wave_only = getenv("LZ4E_DECOMPRESS_WAVE") != nullptr;
    if (!wave_only && a.max_cap > 0 && a.max_cap <= kOutMax) {
        hipLaunchKernelGGL((decompress_wg_kernel<kStamps>), dim3(a.nblocks), dim3(kWgT), 0, stream,
                           a.src, a.src_off, a.src_len, a.dst, a.dst_off, a.dst_cap, a.ret,
                           a.nblocks, dbg);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((decompress_kernel<kStamps>), dim3(a.nblocks), dim3(kWave), 0, stream,
                       a.src, a.src_off, a.src_len, a.dst, a.dst_off, a.dst_cap, a.ret, a.nblocks,
                       dbg);
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
