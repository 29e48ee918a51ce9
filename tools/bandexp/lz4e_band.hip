// lz4e_band.hip -- gfx950 band-parallel LZ4E compressor (round 5 EXPERIMENT,
// not built into the library; DESIGN.md §3 "Band compressor (experiment)").
//
// Result: bit-exact on the GPU (every compress parity test and every frame
// of the full-size configs against the oracle), but 5.6x SLOWER than the
// one-wave compressor (silesia64k compress 19.6 vs 3.5 ms): per pass every
// wave re-runs ~80 instructions per band position (candidate walks, hit
// tests, next codes, in-segment pointer doubling, scans, flags) while a pass
// commits ~480 of the 1024 positions, ~14x the one-wave kernel's
// instructions per input byte, and the kernel is issue-bound
// (profiles/r05/band_stamps.txt).  Kept as the record of the experiment:
// tools/bandexp/bandmodel.c (CPU model, pass counts), build_band.sh +
// test_emulator_band.py (sanitized lane emulator vs the oracle),
// bandstamps.py (per-phase cycles).
//
// Restates LZ4E_compress_generic (/root/reference/lz4e/lz4e_compress.c:218-534,
// noDict, acceleration 1) bit-exactly with one 256-thread workgroup per
// block and no wave-serial walk over the block's positions.
//
// The greedy parse is a pure function of the candidate every lookup sees, and
// that candidate is "the latest put of the same hash before the lookup"
// (puts: every probe :329-330, the match end - 2 :461-463, the rematch
// position :484; an empty slot reads as position 0, :548 + :150-166).  The
// workgroup works on a band of kB positions ahead of the verified frontier f,
// in passes ("Band compressor"):
//
//  1. candidates: under a guess G of the put set, a position's candidate is
//     the nearest G-marked position on its full-population same-hash chain
//     inside [f, p) (prev_kernel precomputes the chain links), else the true
//     table T (every committed put before f);
//  2. verify: each lookup the previous pass's chain made whose outcome (miss,
//     or hit and its candidate) is unchanged under the new candidates is what
//     the reference does: every lookup before the first changed one saw
//     exactly the puts its own parse made before it, so that prefix IS the
//     reference's parse;
//  3. commit the prefix: emit its sequences, write its puts to T, move f;
//  4. hits, match lengths (capped at kFCap) and catch-up lengths of the
//     positions whose candidate changed;
//  5. next(e) for every band position e: where the parse goes when a match
//     ends at e (rematch at e :467-493, else the step-1 search from e + 1,
//     :292-336, to its first hit);
//  6. the chain from the frontier's state through the band: pointer doubling
//     inside 64-position segments (one per wave slot, ds_bpermute), then a
//     stitch over the 16 segments;
//  7. the chain's own puts are the next pass's guess G.
//
// Searches past their 66th probe (skip steps >= 2) only ever start a pass
// (the entry search): its probes are evaluated in parallel over the closed-
// form schedule.  A match longer than kFCap ends a pass and is extended
// exactly by the whole workgroup.  Limited output (:358-363, :425-430,
// :505-509) is checked per sequence before its bytes are written.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "lz4e_device.h"
#include "lz4e_gpu.h"

namespace lz4e {

namespace {

#ifndef LZ4E_BAND_B
#define LZ4E_BAND_B 1024
#endif
constexpr uint32_t kB = LZ4E_BAND_B;  // band width (positions; 512 or 1024)
constexpr uint32_t kBT = 256;         // threads per workgroup (4 waves)
constexpr uint32_t kBS = kB / kBT;    // band slots per thread
constexpr uint32_t kSegs = kB / 64;   // 64-position segments (one per wave slot)
constexpr uint32_t kFCap = 32;        // match bytes compared per position (more: "long")
constexpr uint32_t kBCap = 16;        // catch-up bytes compared per position
constexpr uint32_t kFLong = 0xFFFFu;  // fwd field of a long match
constexpr uint32_t kHops = 6;         // direct chain hops before pointer jumping
constexpr uint32_t kNone = 0xFFFFu;
constexpr uint32_t kEntry = 0xFFFu;   // code value: the entry search (no node)
constexpr uint32_t kLongLits = 8;     // long literal runs copied by the workgroup per commit
constexpr uint32_t kRing = 2048;      // byte ring: the block's bytes around the band
constexpr uint32_t kRingPad = 64;     // mirror of ring bytes [0, 64): reads of <= 64 bytes never wrap

// LDS access types (unaligned dword reads of the byte ring; every width may
// alias every other)
typedef __attribute__((address_space(3))) uint8_t lu8;
typedef uint32_t __attribute__((aligned(1), may_alias)) u32a1;
typedef __attribute__((address_space(3))) u32a1 lu32a1;
typedef __attribute__((address_space(3), may_alias)) uint32_t lu32;
// waves per SIMD the register allocation must allow (LDS allows 5 workgroups
// of 4 waves per CU)
#ifndef LZ4E_BAND_WAVES
#define LZ4E_BAND_WAVES 4
#endif

// next codes (u16): kind << 12 | value (a band offset, or kEntry)
enum : uint32_t {
    kNode = 0,      // value: band offset of the next node (a match end)
    kExitRem = 1,   // value: the node; its match ends at or past the band end
    kExitSrch = 2,  // value: the node; its step-1 search runs past the band end
    kSlow = 3,      // value: the node; 66 probes, no hit: the search goes on sparse
    kEndLim = 4,    // value: the node; its search reaches mflimit: last literals
    kLong = 5,      // value: the node; its match is longer than kFCap
    kEndRem = 6,    // value: the node itself lies past mflimit: last literals
};
LZ4E_DEV uint32_t code(uint32_t kind, uint32_t v) { return kind << 12 | v; }
LZ4E_DEV uint32_t ckind(uint32_t c) { return c >> 12; }
LZ4E_DEV uint32_t cval(uint32_t c) { return c & 0xFFFu; }

// position flags (gf): what the last chain did at a position
enum : uint32_t {
    kFLook = 1,  // looked up
    kFRem = 2,   // ... as a rematch (else as a search probe)
    kFHit = 4,   // ... and found a match
    kFNode = 8,  // a match of the chain ends here (a chain node)
    kFKill = 16, // commit: a later put of the same hash exists
};

// parse states
enum : uint32_t { kStRem = 0, kStSrch = 1, kStEnd = 2 };

// uniform state slots
enum : uint32_t {
    sF = 0,                      // band start (the verified frontier)
    sEK, sEP, sEJ, sEA,          // entry state: kind, position, probe index, anchor
    sHave,                       // a chain exists for this band start
    sTK, sTP, sTJ, sTA, sTF,     // that chain's end state (+ final position of an end)
    sLQ, sLF,                    // its long match: hit position, exact length (sLQ kNone-ish: none)
    sOp,                         // output bytes emitted
    sFill,                       // the ring holds positions [.., sFill)
    sDone, sFail,
    sTerm,                       // the chain's terminal code
    sE0,                         // the chain's first code
    sNLong,                      // long literal runs of this commit
    sBadA,                       // commit: anchor offset + 1 of the first changed lookup
    sTotal,                      // commit: bytes of its sequences
    sFinal,                      // the end state's final source position
    sBFill,                      // the byte ring holds positions [.., sBFill)
    kStN
};

struct BandLds {
    // the true table at the frontier: byU16 8192 x u16, byU32 4096 x u32,
    // byU64 2048 x u32 (lz4e_compress.c:48-57)
    uint32_t T[4096];
    // per band position (ring index p & (kB - 1)):
    uint32_t ph[kB];   // prev delta (bits 0-15, 0: none), hash (16-28), G (31)
    uint32_t hi[kB];   // hit (bit 0), valid (bit 1), back (8-15), fwd (16-31, kFLong)
    uint16_t cd[kB];   // candidate delta hi[] was computed for (0: none)
    uint16_t nx[kB];   // scratch: ancestor links, segment exit codes
    uint16_t cn[kB];   // candidate delta under the current G (stable across a commit)
    uint16_t an[kB];   // the last chain's latest node at or before a position (band offset + 1; 0: none)
    uint8_t gf[kB];    // flags of the last chain (kF*)
    uint64_t hmask[kSegs];        // hit positions per segment
    uint32_t segv[kSegs];         // block scan scratch
    uint32_t hfirst[kSegs + 1];   // first hit offset at or after each segment start
    uint16_t entry[kSegs];        // chain entry lane per segment (kNone: none)
    uint32_t red[8];
    uint32_t st[kStN];
    uint32_t lng[3 * kLongLits];  // long literal runs: source, length, output position
    uint8_t by[kRing + kRingPad] __attribute__((aligned(16)));  // block byte p at p & (kRing - 1)
};

struct Img {
    ByteBuf b;
    LZ4E_DEV uint32_t rd32(uint32_t q) const { return buf_ld32(b, q); }
    LZ4E_DEV uint32_t rd8(uint32_t q) const { return buf_ld8(b, q); }
};

template <int TT>
LZ4E_DEV uint32_t hash_at(const Img& im, uint32_t p) {
    if (TT == kByU32) {
        const uint64_t v = (uint64_t)im.rd32(p) | ((uint64_t)im.rd32(p + 4) << 32);
        return hash5(v, 12);
    }
    return hash4(im.rd32(p), TT == kByU64 ? 11u : 13u);
}

// ---- wave / block helpers ---------------------------------------------------

// Inclusive scan over the 64 lanes (DPP row shifts and row broadcasts).
template <class Op>
LZ4E_DEV uint32_t wave_scan(uint32_t v, Op op, uint32_t id) {
    const uint32_t lane = lane_id();
    uint32_t x = v, t;
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x111, 0xf, 0xf, false);
    x = (lane & 15) >= 1 ? op(x, t) : x;
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x112, 0xf, 0xf, false);
    x = (lane & 15) >= 2 ? op(x, t) : x;
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x114, 0xf, 0xf, false);
    x = (lane & 15) >= 4 ? op(x, t) : x;
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x118, 0xf, 0xf, false);
    x = (lane & 15) >= 8 ? op(x, t) : x;
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x142, 0xa, 0xf, false);
    x = (lane & 16) ? op(x, t) : x;
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x143, 0xc, 0xf, false);
    x = (lane & 32) ? op(x, t) : x;
    return x;
}

struct OpMax {
    LZ4E_DEV uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; }
};
struct OpMin {
    LZ4E_DEV uint32_t operator()(uint32_t a, uint32_t b) const { return a < b ? a : b; }
};
struct OpAdd {
    LZ4E_DEV uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; }
};

// ---- per-position match data ------------------------------------------------

// Forward match length of p against c from p + 4 (lz4e_compress.c:420-423),
// bytes below matchlimit, capped: kFLong when kFCap bytes all matched and
// more remain.
LZ4E_DEV uint32_t fwd_len(const Img& im, uint32_t p, uint32_t c, uint32_t matchlimit) {
    if (p + 4 >= matchlimit) return 0;
    const uint32_t lim = matchlimit - (p + 4);
    uint32_t a[kFCap / 4], b[kFCap / 4];
#pragma unroll
    for (uint32_t i = 0; i < kFCap / 4; ++i) {
        a[i] = im.rd32(p + 4 + 4 * i);
        b[i] = im.rd32(c + 4 + 4 * i);
    }
    uint32_t n = kFCap;
#pragma unroll
    for (int i = kFCap / 4 - 1; i >= 0; --i) {
        const uint32_t x = a[i] ^ b[i];
        if (x) n = 4 * (uint32_t)i + ((uint32_t)__builtin_ctz(x) >> 3);
    }
    if (n >= lim) return lim;
    return n >= kFCap ? kFLong : n;
}

// Catch-up length of p against c (:339-349) without the anchor limit: equal
// bytes right below both while c - i > 0, capped at kBCap.
LZ4E_DEV uint32_t back_len(const Img& im, uint32_t p, uint32_t c) {
    uint32_t lim = c < kBCap ? c : kBCap;
    if (lim == 0) return 0;
    // the 4 bytes right below x - 4 i, top-aligned (below position 0: zeros,
    // never counted: lim <= c <= p)
    auto below = [&](uint32_t x, uint32_t i) -> uint32_t {
        const uint32_t q = 4 * i + 4;
        if (x >= q) return im.rd32(x - q);
        if (x > 4 * i) return im.rd32(0) << (8 * (q - x));
        return 0u;
    };
    uint32_t n = 0;
#pragma unroll
    for (uint32_t i = 0; i < kBCap / 4; ++i) {
        const uint32_t x = below(p, i) ^ below(c, i);
        if (n == 4 * i) n += x ? ((uint32_t)__builtin_clz(x) >> 3) : 4u;
    }
    return n < lim ? n : lim;
}

// The reference's catch-up loop, for a capped one that saturated.
LZ4E_DEV uint32_t back_exact(const Img& im, uint32_t p, uint32_t c, uint32_t lim) {
    uint32_t i = 0;
    while (i < lim && c - i > 0 && im.rd8(p - 1 - i) == im.rd8(c - 1 - i)) ++i;
    return i;
}

// ---- the pre-kernel: full-population same-hash links ---------------------------

// pd[p] = p - q for the latest q < p with hash(q) == hash(p) and p - q <=
// 65535, else 0, for p <= mflimit.  One wave per block walks the block in
// 64-position chunks: a lane's predecessor inside its chunk comes from one
// ballot per hash bit, otherwise from the table of latest positions (read
// before this chunk's writes; each hash written by its group's last lane).
template <int TT>
LZ4E_DEV void prev_block(const Img& im, uint32_t n, uint16_t* __restrict__ pd, uint32_t* last) {
    const uint32_t lane = lane_id();
    const uint32_t hlog = TT == kByU64 ? 11u : (TT == kByU32 ? 12u : 13u);
    // table of (latest position + 1): u16 for byU16 (positions <= 65535:
    // 65536 wraps to "none" only for the block's last hashed position, which
    // nothing follows), u32 otherwise -- 16 KiB either way
    uint16_t* last16 = (uint16_t*)last;
    for (uint32_t i = lane; i < 4096; i += 64) last[i] = 0;
    lockstep();
    const uint32_t mflimit = n - kMfLimit;
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    constexpr uint32_t kG = 8;  // chunks whose bytes are loaded together
    for (uint32_t g0 = 0; g0 <= mflimit; g0 += 64 * kG) {
        uint32_t wa[kG], wb[kG];
#pragma unroll
        for (uint32_t c = 0; c < kG; ++c) {
            const uint32_t p = g0 + 64 * c + lane;
            wa[c] = im.rd32(p);
            wb[c] = TT == kByU32 ? im.rd32(p + 4) : 0u;
        }
#pragma unroll
        for (uint32_t c = 0; c < kG; ++c) {
            const uint32_t p = g0 + 64 * c + lane;
            if (g0 + 64 * c > mflimit) break;
            const bool on = p <= mflimit;
            const uint32_t h = TT == kByU32 ? hash5((uint64_t)wa[c] | ((uint64_t)wb[c] << 32), 12)
                                            : hash4(wa[c], hlog);
            uint64_t m = ballot(on);
            for (uint32_t k = 0; k < hlog; ++k) {
                const bool bit = (h >> k) & 1;
                const uint64_t bb = ballot(bit);
                m &= bit ? bb : ~bb;
            }
            const uint64_t lower = m & below;
            // latest earlier chunk's position + 1 (read before this chunk's writes)
            const uint32_t prev_in = on ? (TT == kByU16 ? (uint32_t)last16[h] : last[h]) : 0u;
            lockstep();
            const bool group_last = ((m >> lane) >> 1) == 0;
            if (on && group_last) {
                if (TT == kByU16) last16[h] = (uint16_t)(p + 1);
                else last[h] = p + 1;
            }
            lockstep();
            uint32_t d = 0;
            if (lower) {
                d = lane - (63 - (uint32_t)__builtin_clzll(lower));
            } else if (prev_in) {
                const uint32_t q = TT == kByU16 ? prev_in - 1 : prev_in - 1;
                if (p - q <= kMaxDistance) d = p - q;
            }
            if (on) pd[p] = (uint16_t)d;
        }
    }
}

__global__ __launch_bounds__(64) void prev_kernel(const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
                                                  const uint32_t* __restrict__ src_len,
                                                  const uint8_t* __restrict__ table_type, uint16_t* __restrict__ pdbuf,
                                                  uint32_t max_len) {
    __shared__ uint32_t last[4096];
    const uint32_t b = blockIdx.x;
    const uint32_t n = src_len[b];
    if (n < kMinLength || n > max_len) return;
    const Img im{buf_make(src + src_off[b], n)};
    uint16_t* pd = pdbuf + (size_t)b * max_len;
    const int tt = table_type[b];
    if (tt == kByU32) prev_block<kByU32>(im, n, pd, last);
    else if (tt == kByU64) prev_block<kByU64>(im, n, pd, last);
    else prev_block<kByU16>(im, n, pd, last);
}

// ---- the band kernel ----------------------------------------------------------

// Stamped build (kSt): per block, thread 0's shader cycles per phase and the
// pass counts (dbg[0..7]: fill, cands, verify, commit, hits, chain, passes,
// commits), and the chain phase split (dbg[8..15]: hit masks, entry search,
// next codes, doubling, stitch, end state, node scan, flags;
// lz4e_debug_compress_band, tools/bandstamps.py).
struct BandStamps {
    uint64_t acc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t t0 = 0, t1 = 0;
    LZ4E_DEV void start() { t0 = t1 = clock64(); }
    LZ4E_DEV void lap(uint32_t k) {
        const uint64_t x = clock64();
        acc[k] += x - t0;
        t0 = x;
    }
    LZ4E_DEV void mark() { t1 = clock64(); }
    LZ4E_DEV void sub(uint32_t k) {
        const uint64_t x = clock64();
        acc[8 + k] += x - t1;
        t1 = x;
    }
};

template <int TT>
struct Band {
    BandLds& S;
    Img im;
    uint32_t n, mflimit, matchlimit, cap;
    bool limited;
    uint8_t* out;
    const uint16_t* pd;
    uint32_t t, w, lane;
    // uniform parse state: every thread keeps the same copy (values from
    // LDS read after a barrier, block reductions, or computed from them)
    uint32_t U[kStN];
    BandStamps* sp = nullptr;  // the stamped build's counters (thread 0 reads them)
    LZ4E_DEV void smark() {
        if (sp) sp->mark();
    }
    LZ4E_DEV void ssub(uint32_t k) {
        if (sp) sp->sub(k);
    }

    LZ4E_DEV static uint32_t slot(uint32_t p) { return p & (kB - 1); }
    LZ4E_DEV uint32_t F() const { return U[sF]; }
    // ring index of band offset o (hi, cd, gf persist across passes)
    LZ4E_DEV uint32_t rg(uint32_t o) const { return (U[sF] + o) & (kB - 1); }

    // block bytes p .. p + 3 from the byte ring (p in [sBFill - kRing + 64, sBFill - 4])
    LZ4E_DEV uint32_t rb32(uint32_t p) const { return *(const lu32a1*)((const lu8*)S.by + (p & (kRing - 1))); }
    LZ4E_DEV uint32_t rb8(uint32_t p) const { return ((const lu8*)S.by)[p & (kRing - 1)]; }
    LZ4E_DEV uint32_t ring_hash(uint32_t p) const {
        if (TT == kByU32) return hash5((uint64_t)rb32(p) | ((uint64_t)rb32(p + 4) << 32), 12);
        return hash4(rb32(p), TT == kByU64 ? 11u : 13u);
    }

    LZ4E_DEV uint32_t tget(uint32_t h) const {
        if (TT == kByU16) return ((const uint16_t*)S.T)[h];
        return S.T[h];
    }
    LZ4E_DEV void tput(uint32_t h, uint32_t p) const {
        if (TT == kByU16) ((uint16_t*)S.T)[h] = (uint16_t)p;
        else S.T[h] = p;
    }

    // ---- block reductions / scans ----
    template <class Op>
    LZ4E_DEV uint32_t block_reduce(uint32_t v, Op op, uint32_t id) {
        uint32_t m = wave_scan(v, op, id);
        m = lane_val(m, 63);
        if (lane == 0) S.red[w] = m;
        block_sync();
        const uint32_t r = op(op(S.red[0], S.red[1]), op(S.red[2], S.red[3]));
        block_sync();
        return r;
    }
    LZ4E_DEV uint32_t block_any(bool v) {
        const uint32_t m = ballot(v) != 0;
        if (lane == 0) S.red[w] = m;
        block_sync();
        const uint32_t r = S.red[0] | S.red[1] | S.red[2] | S.red[3];
        block_sync();
        return r;
    }
    // block minimum of two values at once (results in a, b)
    LZ4E_DEV void block_min2(uint32_t& a, uint32_t& b) {
        const uint32_t ma = lane_val(wave_scan(a, OpMin(), ~0u), 63), mb = lane_val(wave_scan(b, OpMin(), ~0u), 63);
        if (lane == 0) {
            S.red[w] = ma;
            S.red[4 + w] = mb;
        }
        block_sync();
        a = OpMin()(OpMin()(S.red[0], S.red[1]), OpMin()(S.red[2], S.red[3]));
        b = OpMin()(OpMin()(S.red[4], S.red[5]), OpMin()(S.red[6], S.red[7]));
        block_sync();
    }
    // Inclusive scan over the band in position order (slot s of thread t is
    // band offset 256 s + t: segment 4 s + wave, lane = place in it);
    // returns the total.
    template <class Op>
    LZ4E_DEV uint32_t band_scan(uint32_t (&v)[kBS], Op op, uint32_t id) {
        uint32_t x[kBS];
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            x[s] = wave_scan(v[s], op, id);
            const uint32_t tot = lane_val(x[s], 63);
            if (lane == 0) S.segv[4 * s + w] = tot;
        }
        block_sync();
        uint32_t acc = id, all = id;
        for (uint32_t k = 0; k < kSegs; ++k) {
            const uint32_t sv = S.segv[k];
#pragma unroll
            for (uint32_t s = 0; s < kBS; ++s)
                if (k == 4 * s + w) v[s] = op(acc, x[s]);
            acc = op(acc, sv);
            all = acc;
        }
        block_sync();
        return all;
    }

    // ---- ring fill: positions [max(sFill, f), f + kB) ----
    LZ4E_DEV void fill() {
        const uint32_t f = F();
        const uint32_t from = U[sFill] > f ? U[sFill] : f, to = f + kB;
        // bytes [f - 128, f + kB + 64) in the ring (aligned dwords; the bytes
        // below f serve catch-up compares and literal copies)
        {
            const uint32_t lo = f >= 128 ? f - 128 : 0u;
            const uint32_t b0 = (U[sBFill] > lo ? U[sBFill] : lo) & ~3u, b1 = (f + kB + kRingPad + 3) & ~3u;
            block_sync();
            for (uint32_t q = b0 + 4 * t; q < b1; q += 4 * kBT) {
                const uint32_t v = im.rd32(q), r = q & (kRing - 1);
                *(lu32*)((lu8*)S.by + r) = v;
                if (r < kRingPad) *(lu32*)((lu8*)S.by + kRing + r) = v;
            }
            U[sBFill] = b1;
        }
        uint32_t pdv[kBS];
#pragma unroll
        for (uint32_t k = 0; k < kBS; ++k) {
            const uint32_t p = from + t + kBT * k;
            pdv[k] = p < to && p <= mflimit ? pd[p] : 0u;
        }
        block_sync();
#pragma unroll
        for (uint32_t k = 0; k < kBS; ++k) {
            const uint32_t p = from + t + kBT * k;
            if (p >= to) continue;
            const uint32_t o = slot(p);
            if (p <= mflimit) {
                S.ph[o] = pdv[k] | (ring_hash(p) << 16) | 0x80000000u;  // G = 1: the first guess
            } else {
                S.ph[o] = 0;
            }
            S.hi[o] = 0;
            S.cd[o] = 0;
            S.gf[o] = 0;
        }
        U[sFill] = to;
        block_sync();
    }

    // ---- 1. candidates of my positions under G: delta (0: none / too far) ----
    LZ4E_DEV uint32_t from_table(uint32_t p, uint32_t e) const {
        const uint32_t q = tget((e >> 16) & 0x1FFFu);
        return p - q <= kMaxDistance ? p - q : 0u;
    }
    // Positions below `from` keep their candidate (cn): a commit changes
    // neither G nor, for the positions left in the band, what T and G give
    // together; only the positions new to the band are resolved then.
    LZ4E_DEV void cands(uint32_t (&cdl)[kBS], uint32_t from) {
        const uint32_t f = F();
        uint32_t pend = 0, mine = 0, tab = 0;
        uint32_t c[kBS], d[kBS], e[kBS];
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t o = 256 * s + t, p = f + o;
            cdl[s] = 0;
            c[s] = o;
            d[s] = 0;
            e[s] = 0;
            if (p > mflimit) continue;
            if (p < from) {
                cdl[s] = S.cn[slot(p)];
                continue;
            }
            mine |= 1u << s;
            e[s] = S.ph[slot(p)];
            d[s] = e[s] & 0xFFFFu;
        }
        // the chain walks, hop by hop for all four slots at once
        uint32_t walk = mine;
#pragma unroll
        for (uint32_t k = 0; k < kHops; ++k) {
            uint32_t ec[kBS];
#pragma unroll
            for (uint32_t s = 0; s < kBS; ++s) {
                ec[s] = 0;
                if (!((walk >> s) & 1)) continue;
                if (d[s] == 0 || d[s] > c[s]) {
                    walk &= ~(1u << s);
                    tab |= 1u << s;
                    continue;
                }
                c[s] -= d[s];
                ec[s] = S.ph[slot(f + c[s])];
            }
#pragma unroll
            for (uint32_t s = 0; s < kBS; ++s) {
                if (!((walk >> s) & 1)) continue;
                if (ec[s] >> 31) {
                    walk &= ~(1u << s);
                    cdl[s] = 256 * s + t - c[s];
                } else {
                    d[s] = ec[s] & 0xFFFFu;
                }
            }
        }
        pend = walk;
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s)
            if ((tab >> s) & 1) cdl[s] = from_table(f + 256 * s + t, e[s]);
        if (block_any(pend != 0)) resolve_pending(cdl, pend);
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s)
            if ((mine >> s) & 1) S.cn[slot(f + 256 * s + t)] = (uint16_t)cdl[s];
    }
    LZ4E_DEV void resolve_pending(uint32_t (&cdl)[kBS], uint32_t pend) {
        const uint32_t f = F();
        // pointer jumping over every band position: nx[o] = an ancestor with
        // only unmarked chain positions between (kNone: none in the band);
        // one barrier per round (the flags alternate halves of red[])
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t o = 256 * s + t, p = f + o;
            const uint32_t d = p <= mflimit ? S.ph[slot(p)] & 0xFFFFu : 0u;
            S.nx[o] = (uint16_t)((d == 0 || d > o) ? kNone : o - d);
        }
        block_sync();
        for (uint32_t r = 0;; ++r) {
            uint32_t a[kBS], m[kBS], a2[kBS];
#pragma unroll
            for (uint32_t s = 0; s < kBS; ++s) a[s] = S.nx[256 * s + t];
#pragma unroll
            for (uint32_t s = 0; s < kBS; ++s) m[s] = a[s] == kNone ? 0x80000000u : S.ph[slot(f + a[s])];
#pragma unroll
            for (uint32_t s = 0; s < kBS; ++s) a2[s] = (m[s] >> 31) ? a[s] : S.nx[a[s]];
            bool more = false;
#pragma unroll
            for (uint32_t s = 0; s < kBS; ++s) {
                if (a2[s] == a[s]) continue;
                S.nx[256 * s + t] = (uint16_t)a2[s];
                more |= a2[s] != kNone;
            }
            const uint32_t h = 4 * (r & 1);
            const uint32_t any = ballot(more) != 0;
            if (lane == 0) S.red[h + w] = any;
            block_sync();
            if (!(S.red[h] | S.red[h + 1] | S.red[h + 2] | S.red[h + 3])) break;
        }
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            if (!((pend >> s) & 1)) continue;
            const uint32_t o = 256 * s + t, p = f + o;
            const uint32_t a = S.nx[o];
            cdl[s] = a != kNone ? o - a : from_table(p, S.ph[slot(p)]);
        }
        block_sync();
    }

    LZ4E_DEV bool hit_of(uint32_t p, uint32_t d) const { return d != 0 && im.rd32(p - d) == rb32(p); }

    // probe position of index j of the entry search (state SRCH(sEP, sEJ))
    LZ4E_DEV uint32_t probe_pos(uint32_t j) const {
        return U[sEP] + (uint32_t)(probe_offset(j) - probe_offset(U[sEJ]));
    }

    // ---- 2. first lookup of the last chain whose outcome differs ----
    LZ4E_DEV uint32_t verify(const uint32_t (&cdl)[kBS]) {
        uint32_t first = ~0u;
        const uint32_t f = F();
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t o = 256 * s + t;
            const uint32_t g = S.gf[rg(o)];
            if (!(g & kFLook) || cdl[s] == S.cd[rg(o)]) continue;
            if (hit_of(f + o, cdl[s]) || (g & kFHit)) first = first < o ? first : o;
        }
        return block_reduce(first, OpMin(), ~0u);
    }

    // ---- 3. commit ----
    struct Seq {
        uint32_t lit, ll, off, ml;
    };
    // the sequence found by the lookup at band offset o, anchor a
    LZ4E_DEV Seq seq_at(uint32_t o, uint32_t a) const {
        const uint32_t x = F() + o;
        const uint32_t g = S.gf[rg(o)], h = S.hi[rg(o)], d = S.cd[rg(o)];
        uint32_t fw = h >> 16;
        if (fw == kFLong) fw = U[sLF];  // the chain's long match (sLQ == x)
        Seq q;
        q.off = d;
        if (g & kFRem) {
            q.lit = x;
            q.ll = 0;
            q.ml = 4 + fw;
        } else {
            uint32_t bk = (h >> 8) & 0xFFu;
            const uint32_t lim = x - a;
            if (bk >= kBCap && lim > kBCap) bk = back_exact(im, x, x - d, lim);
            if (bk > lim) bk = lim;
            q.lit = a;
            q.ll = x - bk - a;
            q.ml = 4 + fw + bk;
        }
        return q;
    }
    LZ4E_DEV static uint32_t seq_size(const Seq& q) {
        uint32_t sz = 1 + q.ll + 2;
        if (q.ll >= 15) sz += 1 + (q.ll - 15) / 255;
        if (q.ml - 4 >= 15) sz += 1 + (q.ml - 4 - 15) / 255;
        return sz;
    }
    // the reference's output checks of a limited call (:358-363, :425-430)
    LZ4E_DEV bool seq_fits(const Seq& q, uint32_t op) const {
        const uint64_t o1 = (uint64_t)op + 1;
        if (o1 + q.ll + 8 + q.ll / 255 > cap) return false;
        uint64_t o2 = o1 + q.ll + 2;
        if (q.ll >= 15) o2 += 1 + (q.ll - 15) / 255;
        return o2 + 6 + ((q.ml - 4) >> 8) <= cap;
    }
    LZ4E_DEV void put8(uint32_t q, uint32_t v) const { out[q] = (uint8_t)v; }
    // token and literal-length varint; returns the literals' position
    LZ4E_DEV uint32_t write_head(const Seq& q, uint32_t op) const {
        const uint32_t mc = q.ml - 4;
        const uint32_t tok = (q.ll >= 15 ? 0xF0u : q.ll << 4) + (mc >= 15 ? 15u : mc);
        put8(op++, tok);
        if (q.ll >= 15) {
            uint32_t r = q.ll - 15;
            for (; r >= 255; r -= 255) put8(op++, 255);
            put8(op++, r);
        }
        return op;
    }
    LZ4E_DEV void write_tail(const Seq& q, uint32_t op) const {
        put8(op++, q.off & 0xFFu);
        put8(op++, q.off >> 8);
        const uint32_t mc = q.ml - 4;
        if (mc >= 15) {
            uint32_t r = mc - 15;
            for (; r >= 255; r -= 255) put8(op++, 255);
            put8(op++, r);
        }
    }
    // short literal runs (<= 64 bytes, inside the byte ring) from the ring
    LZ4E_DEV void copy_lits(uint32_t dst, uint32_t src, uint32_t len) const {
        for (uint32_t i = 0; i < len; ++i) put8(dst + i, rb8(src + i));
    }
    LZ4E_DEV void copy_lits_hbm(uint32_t dst, uint32_t src, uint32_t len) const {
        for (uint32_t i = 0; i < len; ++i) put8(dst + i, im.rd8(src + i));
    }
    LZ4E_DEV void copy_lits_wg(uint32_t dst, uint32_t src, uint32_t len) const {
        for (uint32_t i = t; i < len; i += kBT) put8(dst + i, im.rd8(src + i));
    }

    // Commits the last chain's lookups before band offset `bad` (~0: all,
    // up to the chain's end state): sequences, puts to T, the new state.
    LZ4E_DEV void commit(uint32_t bad, const uint32_t (&cdl)[kBS]) {
        const uint32_t f = F();
        const uint32_t ea = U[sEA];
        // latest node at or before each position (offset + 1; 0: none), as
        // the chain that made these lookups recorded it
        uint32_t an[kBS];
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) an[s] = S.an[rg(256 * s + t)];
        // sequences of the verified finding lookups
        Seq sq[kBS];
        uint32_t sz[kBS], ex[kBS];
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t o = 256 * s + t;
            const uint32_t g = S.gf[rg(o)];
            sz[s] = 0;
            if (o < bad && (g & kFLook) && (g & kFHit)) {
                // a probe is never a node, so its latest node is before it
                const uint32_t a = an[s] ? f + an[s] - 1 : ea;
                sq[s] = seq_at(o, a);
                sz[s] = seq_size(sq[s]);
            }
            ex[s] = sz[s];
        }
        const uint32_t total = band_scan(ex, OpAdd(), 0u);
        const uint32_t op0 = U[sOp];
        bool bad_fit = false;
        if (limited) {
#pragma unroll
            for (uint32_t s = 0; s < kBS; ++s)
                if (sz[s] && !seq_fits(sq[s], op0 + ex[s] - sz[s])) bad_fit = true;
        }
        if (limited && block_any(bad_fit)) {
            U[sFail] = 1;
            U[sDone] = 1;
            return;
        }
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            if (!sz[s]) continue;
            const uint32_t lo = write_head(sq[s], op0 + ex[s] - sz[s]);
            // short runs starting inside the byte ring copy from it, the
            // others from HBM (long ones by the whole workgroup below)
            bool own = sq[s].ll <= 64 && sq[s].lit + 128 >= f;
            if (!own && sq[s].ll <= 64) {
                copy_lits_hbm(lo, sq[s].lit, sq[s].ll);
                write_tail(sq[s], lo + sq[s].ll);
                continue;
            }
            if (!own) {
                const uint32_t k = atomicAdd(&S.st[sNLong], 1u);
                if (k < kLongLits) {
                    S.lng[3 * k] = sq[s].lit;
                    S.lng[3 * k + 1] = sq[s].ll;
                    S.lng[3 * k + 2] = lo;
                } else {
                    copy_lits_hbm(lo, sq[s].lit, sq[s].ll);
                }
            }
            if (own) copy_lits(lo, sq[s].lit, sq[s].ll);
            write_tail(sq[s], lo + sq[s].ll);
        }
        block_sync();
        {
            const uint32_t nl = S.st[sNLong] < kLongLits ? S.st[sNLong] : kLongLits;
            for (uint32_t k = 0; k < nl; ++k) copy_lits_wg(S.lng[3 * k + 2], S.lng[3 * k], S.lng[3 * k + 1]);
        }
        // the new state (uniform)
        uint32_t nk, np, nj, na, nfin = 0;
        if (bad == ~0u) {
            nk = U[sTK];
            np = U[sTP];
            nj = U[sTJ];
            na = U[sTA];
            nfin = U[sTF];
        } else {
            const uint32_t x = f + bad;
            const uint32_t g = S.gf[rg(bad)];
            np = x;
            if (g & kFRem) {
                nk = kStRem;
                nj = 0;
                na = x;
            } else {
                nk = kStSrch;
                const uint32_t ba = (g & kFNode) ? 0u : S.an[rg(bad)];
                if (ba) {
                    na = f + ba - 1;
                    nj = x - (na + 1);
                } else {
                    // a probe of the entry search: its index
                    na = ea;
                    uint32_t lo = U[sEJ], hi = lo + kB;
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (probe_pos(mid) < x) lo = mid + 1;
                        else hi = mid;
                    }
                    nj = lo;
                }
            }
        }
        // T: the puts below the new frontier (kill each put's previous put of
        // its hash; the survivors are the last of theirs)
        const uint32_t nf = nk == kStEnd ? f + kB : np;
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t o = 256 * s + t, p = f + o;
            if (p >= nf || p > mflimit || !(S.ph[slot(p)] >> 31)) continue;
            const uint32_t d = cdl[s];
            if (d && d <= o) S.gf[rg(o - d)] |= kFKill;
        }
        block_sync();
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t o = 256 * s + t, p = f + o;
            if (p >= nf || p > mflimit) continue;
            const uint32_t e = S.ph[slot(p)];
            if ((e >> 31) && !(S.gf[rg(o)] & kFKill)) tput((e >> 16) & 0x1FFFu, p);
        }
        if (t == 0) {
            // a match end past the band: its put(e - 2) (:461-463)
            if (nk == kStRem && np <= mflimit && np - 2 >= f + kB) tput(hash_at<TT>(im, np - 2), np - 2);
            S.st[sNLong] = 0;  // (every thread read it before the kill barrier above)
        }
        // (the next fill's barrier publishes T before the next candidates)
        U[sOp] = op0 + total;
        U[sEK] = nk;
        U[sEP] = np;
        U[sEJ] = nj;
        U[sEA] = na;
        U[sFinal] = nfin;
        U[sHave] = 0;
        U[sLQ] = ~0u;
        if (nk == kStEnd) U[sDone] = 1;
        else U[sF] = np;
    }

    // ---- 4. hits and match lengths of the positions whose candidate changed ----
    // The candidate side's bytes come from HBM (anywhere up to 64 KiB back),
    // the position's from the byte ring; every slot's loads are issued
    // before any of them is used.
    LZ4E_DEV void hits(const uint32_t (&cdl)[kBS]) {
        const uint32_t f = F();
        uint32_t todo = 0;
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t o = 256 * s + t, p = f + o;
            if (p <= mflimit && !((S.hi[rg(o)] & 2) && S.cd[rg(o)] == cdl[s])) todo |= 1u << s;
        }
        uint32_t cw[kBS][1 + kFCap / 4 + kBCap / 4];
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t p = f + 256 * s + t, d = cdl[s];
            const uint32_t c = ((todo >> s) & 1) && d ? p - d : 0u;
            cw[s][0] = im.rd32(c);
#pragma unroll
            for (uint32_t i = 0; i < kFCap / 4; ++i) cw[s][1 + i] = im.rd32(c + 4 + 4 * i);
#pragma unroll
            for (uint32_t i = 0; i < kBCap / 4; ++i)
                cw[s][1 + kFCap / 4 + i] = c >= 4 * i + 4 ? im.rd32(c - 4 * i - 4)
                                           : (c > 4 * i ? im.rd32(0) << (8 * (4 * i + 4 - c)) : 0u);
        }
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            if (!((todo >> s) & 1)) continue;
            const uint32_t o = 256 * s + t, p = f + o, d = cdl[s];
            uint32_t h = 2;
            if (d && cw[s][0] == rb32(p)) {
                const uint32_t c = p - d;
                // forward: bytes [p + 4, matchlimit) against [c + 4, ...)
                uint32_t fw = 0;
                if (p + 4 < matchlimit) {
                    const uint32_t lim = matchlimit - (p + 4);
                    uint32_t nn = kFCap;
#pragma unroll
                    for (int i = kFCap / 4 - 1; i >= 0; --i) {
                        const uint32_t x = rb32(p + 4 + 4 * (uint32_t)i) ^ cw[s][1 + i];
                        if (x) nn = 4 * (uint32_t)i + ((uint32_t)__builtin_ctz(x) >> 3);
                    }
                    fw = nn >= lim ? lim : (nn >= kFCap ? kFLong : nn);
                }
                // backward: equal bytes right below both while c - i > 0
                const uint32_t lim = c < kBCap ? c : kBCap;
                uint32_t bk = 0;
#pragma unroll
                for (uint32_t i = 0; i < kBCap / 4; ++i) {
                    const uint32_t x = rb32(p - 4 * i - 4) ^ cw[s][1 + kFCap / 4 + i];
                    if (bk == 4 * i) bk += x ? ((uint32_t)__builtin_clz(x) >> 3) : 4u;
                }
                bk = bk < lim ? bk : lim;
                h |= 1u | (bk << 8) | (fw << 16);
            }
            S.hi[rg(o)] = h;
            S.cd[rg(o)] = (uint16_t)d;
        }
        block_sync();
    }

    // first hit at band offset >= y (kNone: none in the band)
    LZ4E_DEV uint32_t nh(uint32_t y) const {
        if (y >= kB) return kNone;
        const uint32_t k = y >> 6;
        const uint64_t m = S.hmask[k] >> (y & 63);
        return m ? y + ctz64(m) : S.hfirst[k + 1];
    }
    // last probe of the step-1 search from s (probes s, s+1, ..., each
    // passing its end check :301-302; probe 65 advances by 2); below s: none
    LZ4E_DEV uint32_t qmax_of(uint32_t s) const {
        if (s + 65 + 2 <= mflimit) return s + 65;
        const uint32_t a = s + 64, b = mflimit - 1;
        return a < b ? a : b;
    }

    // ---- 5. next code of band offset o ----
    LZ4E_DEV uint32_t next_code(uint32_t o) const {
        const uint32_t f = F(), e = f + o;
        if (e > mflimit) return code(kEndRem, o);
        uint32_t q;  // band offset of the hit
        const uint32_t h = S.hi[rg(o)];
        if (h & 1) {
            q = o;  // rematch (:484-493)
        } else {
            const uint32_t s = e + 1, qm = qmax_of(s);
            const uint32_t y = nh(o + 1);
            if (y == kNone || f + y > qm) {
                if (qm < f + kB || qm < s) return (s + 65 + 2 <= mflimit) ? code(kSlow, o) : code(kEndLim, o);
                return code(kExitSrch, o);
            }
            q = y;
        }
        const uint32_t fw = S.hi[rg(q)] >> 16;
        if (fw == kFLong) return code(kLong, o);
        const uint32_t end = q + 4 + fw;
        return end < kB ? code(kNode, end) : code(kExitRem, o);
    }

    // next codes of my four slots, each phase's LDS reads issued for all
    // slots before any is used (the same result as next_code per slot)
    LZ4E_DEV void next_codes(uint32_t (&cc)[kBS]) const {
        const uint32_t f = F();
        uint32_t h[kBS], q[kBS], hq[kBS];
        uint64_t m[kBS];
        uint32_t nf[kBS];
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) h[s] = S.hi[rg(256 * s + t)];
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t y = 256 * s + t + 1, k = y >> 6;
            m[s] = y < kB ? S.hmask[k] >> (y & 63) : 0ull;
            nf[s] = y < kB ? S.hfirst[k + 1] : kNone;
        }
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t o = 256 * s + t, y = o + 1;
            q[s] = (h[s] & 1) ? o : (m[s] ? y + ctz64(m[s]) : nf[s]);
            hq[s] = q[s] < kB ? S.hi[rg(q[s])] : 0u;
        }
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t o = 256 * s + t, e = f + o;
            uint32_t c;
            if (e > mflimit) {
                c = code(kEndRem, o);
            } else {
                bool srch_end = false;
                if (!(h[s] & 1)) {
                    const uint32_t s0 = e + 1, qm = qmax_of(s0);
                    if (q[s] == kNone || f + q[s] > qm) {
                        srch_end = true;
                        c = (qm < f + kB || qm < s0) ? ((s0 + 65 + 2 <= mflimit) ? code(kSlow, o) : code(kEndLim, o))
                                                     : code(kExitSrch, o);
                    }
                }
                if (!srch_end) {
                    const uint32_t fw = hq[s] >> 16;
                    if (fw == kFLong) c = code(kLong, o);
                    else {
                        const uint32_t end = q[s] + 4 + fw;
                        c = end < kB ? code(kNode, end) : code(kExitRem, o);
                    }
                }
            }
            cc[s] = c;
        }
    }

    // Exact match length from q + 4 against q - d + 4 (the whole workgroup).
    LZ4E_DEV uint32_t fwd_exact(uint32_t q, uint32_t d) {
        const uint32_t c = q - d, lim = q + 4 < matchlimit ? matchlimit - (q + 4) : 0u;
        for (uint32_t i = 0; i < lim; i += 4 * kBT) {
            const uint32_t k = i + 4 * t;
            uint32_t m = ~0u;
            if (k < lim) {
                uint32_t x = im.rd32(q + 4 + k) ^ im.rd32(c + 4 + k);
                if (lim - k < 4) x &= (1u << (8 * (lim - k))) - 1u;
                if (x) m = k + ((uint32_t)__builtin_ctz(x) >> 3);
            }
            const uint32_t r = block_reduce(m, OpMin(), ~0u);
            if (r != ~0u) return r;
        }
        return lim;
    }

    // ---- 6-7. the chain from the entry state; flags and the next guess ----
    LZ4E_DEV void chain() {
        smark();
        const uint32_t f = F();
        // hit masks per segment
        uint32_t hb[kBS];
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t o = 256 * s + t;
            hb[s] = (f + o <= mflimit) && (S.hi[rg(o)] & 1);
            const uint64_t m = ballot(hb[s] != 0);
            if (lane == 0) S.hmask[4 * s + w] = m;
        }
        block_sync();
        ssub(0);
        // first hit at or after each segment start: every wave writes the
        // whole (identical) table itself, so it reads only its own writes
        {
            uint32_t nxt = kNone;
            for (int k = kSegs - 1; k >= 0; --k) {
                const uint64_t m = S.hmask[k];
                if (m && (uint32_t)k >= lane) nxt = 64 * (uint32_t)k + ctz64(m);
            }
            if (lane <= kSegs) S.hfirst[lane] = lane < kSegs ? nxt : kNone;
            lockstep();
        }
        // the entry state's first event (uniform)
        const uint32_t ek = U[sEK];
        uint32_t e0;
        uint32_t jE = ~0u, jX = ~0u, qE = 0;  // entry search: first event / exit probe index
        bool eEnd = false;
        if (ek == kStRem) {
            e0 = code(kNode, 0);
        } else {
            const uint32_t j0 = U[sEJ];
            uint32_t ev = ~0u, exi = ~0u;
            for (uint32_t r = 0; r < kBS; ++r) {
                const uint32_t j = j0 + t + kBT * r, x = probe_pos(j);
                if (x >= f + kB) {
                    exi = exi < j ? exi : j;
                    continue;
                }
                if (x + probe_step(j) > mflimit || (S.hi[rg(x - f)] & 1)) ev = ev < j ? ev : j;
            }
            block_min2(ev, exi);
            jE = ev;
            jX = exi;
            if (jE < jX) {
                const uint32_t x = probe_pos(jE);
                if (x + probe_step(jE) > mflimit) {
                    eEnd = true;
                    e0 = code(kEndLim, kEntry);
                } else {
                    qE = x - f;
                    const uint32_t fw = S.hi[rg(qE)] >> 16;
                    if (fw == kFLong) e0 = code(kLong, kEntry);
                    else {
                        const uint32_t end = qE + 4 + fw;
                        e0 = end < kB ? code(kNode, end) : code(kExitRem, kEntry);
                    }
                }
            } else {
                e0 = code(kExitSrch, kEntry);
            }
        }
        ssub(1);
        // in-segment pointer doubling: J (next lane, 64: left the segment),
        // M (lanes visited), X (the exit code)
        uint32_t Mlo[kBS], Mhi[kBS], J[kBS], X[kBS];
        next_codes(X);
        ssub(2);
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t o = 256 * s + t, c = X[s];
            J[s] = (ckind(c) == kNode && (cval(c) >> 6) == (o >> 6)) ? cval(c) & 63u : 64u;
            Mlo[s] = lane < 32 ? 1u << lane : 0u;
            Mhi[s] = lane >= 32 ? 1u << (lane - 32) : 0u;
        }
        // (rounds outer, slots inner: four independent permute chains)
#pragma unroll
        for (uint32_t r = 0; r < 6; ++r) {
#pragma unroll
            for (uint32_t s = 0; s < kBS; ++s) {
                const uint32_t src = J[s] < 64 ? J[s] : lane;
                const uint32_t Jn = shfl(J[s], src), Xn = shfl(X[s], src);
                const uint32_t Ln = shfl(Mlo[s], src), Hn = shfl(Mhi[s], src);
                if (J[s] < 64) {
                    J[s] = Jn;
                    X[s] = Xn;
                    Mlo[s] |= Ln;
                    Mhi[s] |= Hn;
                }
            }
        }
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) S.nx[256 * s + t] = (uint16_t)X[s];
        block_sync();
        ssub(3);
        // the stitch (wave 0): segment k's entry lane is where the chain
        // enters it, the next entry is that lane's exit code; segments are
        // entered in increasing order, so one unrolled pass over k
        if (w == 0) {
            uint32_t X[kSegs];
#pragma unroll
            for (uint32_t k = 0; k < kSegs; ++k) X[k] = S.nx[64 * k + lane];
            uint32_t cur = e0, ent = kNone;
#pragma unroll
            for (uint32_t k = 0; k < kSegs; ++k) {
                if (ckind(cur) == kNode && (cval(cur) >> 6) == k) {
                    const uint32_t l = cval(cur) & 63u;
                    ent = lane == k ? l : ent;
                    cur = lane_val(X[k], l);
                }
            }
            if (lane < kSegs) S.entry[lane] = (uint16_t)ent;
            if (lane == 0) S.st[sTerm] = cur;
        }
        block_sync();
        const uint32_t term = S.st[sTerm];
        ssub(4);
        // node flags of my positions
        uint32_t node[kBS];
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t k = 4 * s + w, en = S.entry[k];
            uint32_t bit = 0;
            if (en != kNone) {
                const uint32_t ml = lane_val(Mlo[s], en), mh = lane_val(Mhi[s], en);
                bit = lane < 32 ? (ml >> lane) & 1u : (mh >> (lane - 32)) & 1u;
            }
            node[s] = bit;
        }
        // the terminal: the end state (uniform)
        const uint32_t tk = ckind(term), tv = cval(term);
        uint32_t TK = kStEnd, TP = 0, TJ = 0, TA = 0, TF = 0, LQ = ~0u, LF = 0;
        {
            // the hit of the terminal's node (or of the entry search)
            uint32_t q = kNone;
            if (tv == kEntry) q = qE;
            else if (tk == kExitRem || tk == kLong) q = (S.hi[rg(tv)] & 1) ? tv : nh(tv + 1);
            if (tk == kEndRem) {
                TK = kStEnd;
                TF = f + tv;
                TA = f + tv;
            } else if (tk == kEndLim) {
                TK = kStEnd;
                if (tv == kEntry) {
                    TF = jE == 0 ? f : probe_pos(jE) - probe_step(jE - 1);
                    TA = U[sEA];
                } else {
                    const uint32_t s0 = f + tv + 1, qm = qmax_of(s0);
                    TF = qm >= s0 ? qm : s0;
                    TA = f + tv;
                }
            } else if (tk == kExitSrch) {
                TK = kStSrch;
                if (tv == kEntry) {
                    TP = probe_pos(jX);
                    TJ = jX;
                    TA = U[sEA];
                } else {
                    TP = f + kB;
                    TJ = f + kB - (f + tv + 1);
                    TA = f + tv;
                }
            } else if (tk == kSlow) {
                TK = kStSrch;
                TP = f + tv + 68;
                TJ = 66;
                TA = f + tv;
            } else {  // kExitRem, kLong
                uint32_t fw = S.hi[rg(q)] >> 16;
                if (tk == kLong) {
                    fw = fwd_exact(f + q, S.cd[rg(q)]);
                    LQ = f + q;
                    LF = fw;
                }
                const uint32_t end = f + q + 4 + fw;
                TK = kStRem;
                TP = end;
                TA = end;
                if (end > mflimit) {
                    TK = kStEnd;
                    TF = end;
                }
            }
        }
        ssub(5);
        // the end state's position: flags below it, G kept at and above it
        const uint32_t tpo = TK == kStEnd ? kB : (TP - f < kB ? TP - f : kB);
        // node flags to LDS (puts at e - 2 read the neighbours')
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t o = 256 * s + t;
            S.gf[rg(o)] = node[s] ? (uint8_t)kFNode : (uint8_t)0;
        }
        // probes of the nodes' searches: latest node at or before each position
        uint32_t an[kBS];
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) an[s] = node[s] ? 256 * s + t + 1 : 0u;
        band_scan(an, OpMax(), 0u);  // (barriers: gf node flags published)
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) S.an[rg(256 * s + t)] = (uint16_t)an[s];
        uint32_t jlo = 0, jhi = 0;  // entry search probes [jlo, jhi] looked up
        bool ehit = false;
        if (ek == kStSrch) {
            jlo = U[sEJ];
            const uint32_t jl = jE < jX ? jE : jX;
            jhi = jl;  // exclusive unless the event is a hit
            ehit = jE < jX && !eEnd;
            if (ehit) jhi = jE + 1;
        }
        ssub(6);
        // (every slot's LDS reads first, then the flags)
        uint32_t h[kBS], hv[kBS], g2[kBS], eph[kBS], nfv[kBS];
        uint64_t mv[kBS];
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t o = 256 * s + t, p = f + o;
            const uint32_t v = an[s] ? an[s] - 1 : 0u, y = v + 1, k = y >> 6;
            h[s] = S.hi[rg(o)];
            hv[s] = S.hi[rg(v)];
            g2[s] = o + 2 < kB ? S.gf[rg(o + 2)] : 0u;
            eph[s] = S.ph[slot(p)];
            mv[s] = y < kB ? S.hmask[k] >> (y & 63) : 0ull;
            nfv[s] = y < kB ? S.hfirst[k + 1] : kNone;
        }
#pragma unroll
        for (uint32_t s = 0; s < kBS; ++s) {
            const uint32_t o = 256 * s + t, p = f + o;
            uint32_t g = 0;
            bool put = false;
            if (o < tpo && p <= mflimit) {
                if (node[s]) {
                    g = kFNode | kFLook | kFRem | ((h[s] & 1) ? kFHit : 0u);
                    put = true;
                } else if (an[s]) {
                    const uint32_t v = an[s] - 1;  // the latest node, before o
                    if (f + v <= mflimit && !(hv[s] & 1)) {
                        const uint32_t s0 = f + v + 1, qm = qmax_of(s0);
                        const uint32_t y = mv[s] ? v + 1 + ctz64(mv[s]) : nfv[s];
                        const uint32_t lim = (y != kNone && f + y <= qm) ? f + y : qm;
                        if (p <= lim && qm >= s0) {
                            g = kFLook | ((h[s] & 1) ? kFHit : 0u);
                            put = true;
                        }
                    }
                }
                if ((g2[s] & kFNode) && p + 2 <= mflimit) put = true;
                if (TK == kStRem && p + 2 == TP) put = true;
            }
            if (node[s]) g |= kFNode;  // (also a node past mflimit or at the end state)
            if (o < tpo) S.ph[slot(p)] = (eph[s] & 0x7FFFFFFFu) | (put ? 0x80000000u : 0u);
            S.gf[rg(o)] = (uint8_t)g;
        }
        block_sync();
        // the entry search's probes (band offsets from the schedule)
        if (ek == kStSrch) {
            for (uint32_t r = 0; r < kBS; ++r) {
                const uint32_t j = jlo + t + kBT * r;
                if (j >= jhi) continue;
                const uint32_t x = probe_pos(j);
                if (x >= f + kB) continue;
                const uint32_t o = x - f;
                S.gf[rg(o)] = (uint8_t)(kFLook | ((S.hi[rg(o)] & 1) ? kFHit : 0u));
                S.ph[slot(x)] |= 0x80000000u;
            }
        }
        ssub(7);
        U[sTK] = TK;
        U[sTP] = TP;
        U[sTJ] = TJ;
        U[sTA] = TA;
        U[sTF] = TF;
        U[sLQ] = LQ;
        U[sLF] = LF;
        U[sHave] = 1;
        // (the entry probes' flags and every G bit reach the next pass's
        // readers through its fill barrier)
    }
};

template <int TT, bool kSt>
LZ4E_DEV void band_block(BandLds& S, const Img& im, uint32_t n, uint8_t* out, uint32_t cap, const uint16_t* pd,
                         int32_t* ret, uint32_t* aux, uint64_t* dbg) {
    BandStamps st;
    if (kSt) st.start();
    const uint32_t t = threadIdx.x;
    Band<TT> B{S, im, n, n >= kMinLength ? n - kMfLimit : 0u, n >= kMinLength ? n - kLastLiterals : 0u, cap,
               cap < (uint32_t)(n + n / 255 + 16), out, pd, t, t >> 6, t & 63};
    for (uint32_t i = t; i < 4096; i += kBT) S.T[i] = 0;  // :548 (an empty slot reads as position 0)
    if (t == 0) S.st[sNLong] = 0;
    if (kSt) B.sp = &st;
    {
        for (uint32_t i = 0; i < kStN; ++i) B.U[i] = 0;
        B.U[sF] = 1;
        B.U[sEK] = kStSrch;  // :280-282: put(0) (== the empty slot), search from 1
        B.U[sEP] = 1;
        B.U[sEJ] = 0;
        B.U[sEA] = 0;
        B.U[sFill] = 1;
        B.U[sBFill] = 0;
        B.U[sLQ] = ~0u;
    }
    block_sync();
    if (n >= kMinLength) {
        // every commit moves the frontier by at least one position, so a
        // block takes at most 2 n passes; more is a broken invariant, and the
        // block fails (ret 0) instead of spinning
        uint32_t from = 0;  // positions whose candidate is to be resolved: >= from
        for (uint32_t pass = 0;; ++pass) {
            if (pass > 2 * n + 64) {
                B.U[sFail] = 1;
                break;
            }
            B.fill();
            if (kSt) st.lap(0);
            uint32_t cdl[kBS];
            const bool have = B.U[sHave] != 0;
            B.cands(cdl, have ? 0u : from);
            if (kSt) st.lap(1);
            if (have) {
                const uint32_t bad = B.verify(cdl), f0 = B.F();
                if (kSt) st.lap(2);
                B.commit(bad, cdl);
                if (kSt) {
                    st.lap(3);
                    st.acc[7]++;
                }
                if (B.U[sDone]) break;
                from = f0 + kB;  // the positions new to the band
                continue;
            }
            B.hits(cdl);
            if (kSt) st.lap(4);
            B.chain();
            if (kSt) {
                st.lap(5);
                st.acc[6]++;
            }
        }
    }
    // last literals (:500-530)
    if (B.U[sFail]) {
        if (t == 0) ret[0] = 0;
        return;
    }
    const uint32_t anchor = n >= kMinLength ? B.U[sEA] : 0u;
    const uint32_t R = n - anchor, op = B.U[sOp];
    if (B.limited && (uint64_t)op + R + 1 + (R + 240) / 255 > cap) {
        if (t == 0) ret[0] = 0;
        return;
    }
    uint32_t lo = op + 1;
    if (R >= 15) lo += 1 + (R - 15) / 255;
    if (t == 0) {
        uint32_t q = op;
        if (R >= 15) {
            uint32_t r = R - 15;
            B.put8(q++, 0xF0);
            for (; r >= 255; r -= 255) B.put8(q++, 255);
            B.put8(q++, r);
        } else {
            B.put8(q++, R << 4);
        }
    }
    B.copy_lits_wg(lo, anchor, R);
    if (kSt && t == 0 && dbg)
        for (uint32_t k = 0; k < 16; ++k) dbg[k] = st.acc[k];
    if (t == 0) {
        ret[0] = (int32_t)(lo + R);
        if (aux) {
            aux[0] = n >= kMinLength ? B.U[sFinal] : 0u;
            aux[1] = R;
        }
    }
}

template <bool kSt>
__global__ __launch_bounds__(kBT, LZ4E_BAND_WAVES) void band_kernel(const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_off,
                                                   const uint32_t* __restrict__ src_len,
                                                   const uint8_t* __restrict__ table_type, uint8_t* __restrict__ dst,
                                                   const uint64_t* __restrict__ dst_off,
                                                   const uint32_t* __restrict__ dst_cap, int32_t* __restrict__ ret,
                                                   uint32_t* __restrict__ aux, uint32_t max_len,
                                                   const uint16_t* __restrict__ pdbuf,
                                                   const uint32_t* __restrict__ order, uint64_t* dbg) {
    __shared__ BandLds S;
    const uint32_t b = order ? order[blockIdx.x] : blockIdx.x;
    const uint32_t n = src_len[b];
    if (n > max_len) {
        if (threadIdx.x == 0) ret[b] = 0;
        return;
    }
    const Img im{buf_make(src + src_off[b], n)};
    uint8_t* out = dst + dst_off[b];
    const uint16_t* pd = pdbuf + (size_t)b * max_len;
    uint32_t* ax = aux ? aux + 2 * (size_t)b : nullptr;
    const int tt = table_type[b];
    uint64_t* d = kSt && dbg ? dbg + 16 * (size_t)b : nullptr;
#ifdef LZ4E_BAND_ONLY_U16
    (void)tt;
    band_block<kByU16, kSt>(S, im, n, out, dst_cap[b], pd, ret + b, ax, d);
#else
    if (tt == kByU32) band_block<kByU32, kSt>(S, im, n, out, dst_cap[b], pd, ret + b, ax, d);
    else if (tt == kByU64) band_block<kByU64, kSt>(S, im, n, out, dst_cap[b], pd, ret + b, ax, d);
    else band_block<kByU16, kSt>(S, im, n, out, dst_cap[b], pd, ret + b, ax, d);
#endif
}

}  // namespace

// The band compressor for a batch (no dictionary): prev_kernel, then
// band_kernel in `order` (nullable).  pd scratch: 2 * max_len bytes per block.
hipError_t launch_compress_band(const CompressBatch& a, hipStream_t stream, const uint32_t* order, uint64_t* dbg) {
    if (a.nblocks == 0) return hipSuccess;
    uint16_t* pd = nullptr;
    const size_t bytes = 2 * (size_t)a.max_len * a.nblocks + 64;
    hipError_t err = hipMallocAsync((void**)&pd, bytes, stream);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(prev_kernel, dim3(a.nblocks), dim3(64), 0, stream, a.src, a.src_off, a.src_len, a.table_type, pd,
                       a.max_len);
    err = hipGetLastError();
    if (err == hipSuccess) {
        if (dbg)
            hipLaunchKernelGGL(band_kernel<true>, dim3(a.nblocks), dim3(kBT), 0, stream, a.src, a.src_off, a.src_len,
                               a.table_type, a.dst, a.dst_off, a.dst_cap, a.ret, a.aux, a.max_len, pd, order, dbg);
        else
            hipLaunchKernelGGL(band_kernel<false>, dim3(a.nblocks), dim3(kBT), 0, stream, a.src, a.src_off,
                               a.src_len, a.table_type, a.dst, a.dst_off, a.dst_cap, a.ret, a.aux, a.max_len, pd,
                               order, nullptr);
        err = hipGetLastError();
    }
    (void)hipFreeAsync(pd, stream);
    return err;
}

}  // namespace lz4e
