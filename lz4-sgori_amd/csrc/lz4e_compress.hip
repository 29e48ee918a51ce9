// lz4e_compress.hip -- gfx950 LZ4E block compressor.
//
// Bit-exact restatement of the reference greedy parse
// (/root/reference/lz4e/lz4e_compress.c:218-534, LZ4E_compress_generic with
// noDict, acceleration 1), one wave64 per block, all control flow
// wave-uniform (the parse state lives in SGPRs).  The parse is a serial
// chain of dependent round trips, so the kernel is built for the fewest
// instructions and round trips per sequence:
//
//  * The hash table (8192 x u16 for byU16, 4096 x u32 for byU32, 2048 x u32
//    for byU64) lives in LDS (16 KiB per block).  The input block is read
//    straight from HBM with unaligned dword loads (L1/L2 absorb the reuse),
//    or from an LDS copy for small blocks.
//  * Data moves in "stripes": one dword per lane, lane k holding the 4 bytes
//    at X - 4 + 4k for a base position X.  A match step loads the stripe at
//    the current position and at its candidate together; lane 0 serves the
//    backward catch-up (lz4e_compress.c:339-349), XOR + ballot counts up to
//    252 bytes per round trip (LZ4E_count, lz4e_defs.h:587-636) and, on the
//    post-match rematch (lz4e_compress.c:461-493), the same count is the
//    4-byte verify.  Literal runs are stored as one dword per lane straight
//    from the stripe; the post-match hashes are read out of the stripe with
//    v_readlane.  Token, offset and a one-byte match-length extension leave
//    as one dword store.
//  * Match search (lz4e_compress.c:292-336) is speculative over a window of
//    probes, one per lane: probe positions are a closed-form function of the
//    search start (skip step +1 every 64 probes), hashes are pure functions
//    of the data, and the candidate a probe sees is "the latest earlier probe
//    of the window with an equal hash, else the table entry from before the
//    window".  Every probe writes its position and reads it back: a lane that
//    does not see its own position shares its hash with another lane, and
//    those lane groups are resolved with one ballot per group.  The first
//    verifying lane is the reference's match; the table is then fixed up to
//    hold exactly the puts of the probes up to it.
//
// Stores may write up to 3 bytes past the bytes they own when a later store
// of the same wave (program order) rewrites those bytes, and never past the
// end of the frame: every match is followed by at least the last-literals
// token and 5 literals.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include "lz4e_device.h"
#include "lz4e_gpu.h"
#include "lz4e_order.h"

namespace lz4e {

namespace {

constexpr uint32_t kTableBytes = 16384;  // 1 << LZ4E_MEMORY_USAGE
constexpr uint32_t kStripe = 256;        // bytes covered by one stripe (lane k: X-4+4k)

typedef __attribute__((address_space(1))) uint8_t gu8;
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) const uint64_t gcu64;

// byU16 class: u16 positions (block <= 64 KiB); byU32/byU64: u32 positions.
template <int TT>
struct Table {
    uint32_t* lds;
    LZ4E_DEV uint32_t get(uint32_t h) const {
        if constexpr (TT == kByU16) return reinterpret_cast<uint16_t*>(lds)[h];
        else return lds[h];
    }
    LZ4E_DEV void put(uint32_t h, uint32_t v) const {
        if constexpr (TT == kByU16) reinterpret_cast<uint16_t*>(lds)[h] = (uint16_t)v;
        else lds[h] = v;
    }
    // Read back after a put of the whole wave: which lane's write landed is
    // only known to the LDS, so the compiler must not forward the put.
    LZ4E_DEV uint32_t reread(uint32_t h) const {
        typedef __attribute__((address_space(3))) volatile uint16_t lvu16;
        typedef __attribute__((address_space(3))) volatile uint32_t lvu32;
        if constexpr (TT == kByU16) return ((lvu16*)lds)[h];
        else return ((lvu32*)lds)[h];
    }
};

// A block in HBM, read with unaligned vector loads (gfx950 global loads need
// no alignment).  n >= kMinLength whenever the parse runs.
// Every access is a buffer load through one resource (4 SGPRs for the whole
// image: no separate base pointer or length held across the parse, which is
// at the SGPR limit), its offset forced into a VGPR (a uniform offset would
// otherwise become s_buffer_load, which ignores the low two address bits).
struct HbmImage {
    ByteBuf buf;  // the block (and its dictionary) as a buffer resource
    LZ4E_DEV uint32_t rd8(uint32_t q) const { return buf_ld8(buf, vaddr(q)); }
    // Window loads: dword at q, 0 when any of its bytes lies outside the
    // block (callers never use such a dword: every compared byte is in one
    // fully inside); buffer loads take the constant part of the offset in
    // the instruction and merge into dwordx4.
    LZ4E_DEV uint32_t wld(uint32_t q) const { return buf_ld32(buf, q); }
    // o[0] = the dword at q - 4, o[1 + i] = the dword at q + 4 i (i < 8)
    LZ4E_DEV void wld9(uint32_t q, uint32_t* o) const {
        o[0] = wld(q - 4);
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) o[1 + i] = wld(q + 4 * i);
    }
    static constexpr bool kInLds = false;
    LZ4E_DEV uint32_t ld32(uint32_t q) const { return buf_ld32(buf, vaddr(q)); }
    LZ4E_DEV uint64_t ld64(uint32_t q) const {
        const uint32_t v = vaddr(q);
        return ((uint64_t)buf_ld32(buf, v + 4) << 32) | buf_ld32(buf, v);
    }
    // Lanes past the block (or before it, X < 4) read 0 (range check) or a
    // meaningless dword; every consumer masks those bytes.
    LZ4E_DEV uint32_t stripe(uint32_t X, uint32_t lane) const { return ld32(X - 4 + 4 * lane); }
};

// A block staged in LDS as words (the last partial word zero-padded).
struct LdsImage {
    const uint32_t* w;
    uint32_t last;  // last word index
    LZ4E_DEV uint32_t word(uint32_t i) const { return w[i < last ? i : last]; }
    LZ4E_DEV uint32_t rd8(uint32_t q) const { return (word(q >> 2) >> ((q & 3) * 8)) & 0xFFu; }
    LZ4E_DEV uint32_t ld32(uint32_t q) const {
        const uint32_t i = q >> 2;
        return alignbyte(word(i + 1), word(i), q & 3);
    }
    LZ4E_DEV uint64_t ld64(uint32_t q) const {
        const uint32_t i = q >> 2, r = q & 3;
        const uint32_t w0 = word(i), w1 = word(i + 1), w2 = word(i + 2);
        return ((uint64_t)alignbyte(w2, w1, r) << 32) |
               alignbyte(w1, w0, r);
    }
    LZ4E_DEV uint32_t stripe(uint32_t X, uint32_t lane) const { return ld32(X - 4 + 4 * lane); }
    LZ4E_DEV uint32_t wld(uint32_t q) const { return ld32(q); }
    // HbmImage::wld9 from 10 shared word reads (the overlapping dwords of
    // a 36-byte run need 10 words, not 18)
    LZ4E_DEV void wld9(uint32_t q, uint32_t* o) const {
        const uint32_t i0 = (q >> 2) - 1, r = q & 3;  // (q < 4: the clamp, as in ld32)
        uint32_t w[10];
#pragma unroll
        for (uint32_t k = 0; k < 10; ++k) w[k] = word(i0 + k);
#pragma unroll
        for (uint32_t k = 0; k < 9; ++k) o[k] = alignbyte(w[k + 1], w[k], r);
    }
    static constexpr bool kInLds = true;
};

// Phase cycle counters of the diagnostic build (launch_compress_stamped).
struct Stamps {
    uint64_t t, acc[6], t0, r0;
    uint32_t cnt[4];
    LZ4E_DEV void start() {
        t = clock64();
        t0 = t;
        r0 = realtime64();
        for (int i = 0; i < 6; ++i) acc[i] = 0;
        for (int i = 0; i < 4; ++i) cnt[i] = 0;
    }
    LZ4E_DEV void lap(int phase) {
        const uint64_t now = clock64();
        acc[phase] += now - t;
        t = now;
    }
};
enum { kPhSearch, kPhStripe, kPhLit, kPhCount, kPhRematch, kPhTail };

// Event trace of the stamped build when compiled with -DLZ4E_TRACE (debug
// only): (kind << 56 | a, b) pairs after the 8 stamp words of the block.
#ifdef LZ4E_TRACE
#define LZ4E_TR(k, a, b)                                                              \
    do {                                                                              \
        if (kStamps && dbg && lane == 0 && trn < (1u << 16)) {                        \
            dbg[8 + 2 * trn] = ((uint64_t)(k) << 56) | (uint64_t)(a);                 \
            dbg[9 + 2 * trn] = (uint64_t)(b);                                         \
        }                                                                             \
        trn++;                                                                        \
    } while (0)
#else
#define LZ4E_TR(k, a, b) \
    do {                 \
    } while (0)
#endif

// hash of the position whose bytes are v (hash5 for byU32, hash4 otherwise;
// hashLog 13 / 12 / 11 for byU16 / byU32 / byU64, lz4e_compress.c:48-96)
template <int TT>
LZ4E_DEV uint32_t hash_val(uint64_t v) {
    if constexpr (TT == kByU32) return hash5(v, 12);
    else return hash4((uint32_t)v, TT == kByU16 ? 13 : 11);
}

// First byte index u >= u0 where the two stripes differ (x = si ^ sb), or
// where the comparison limit e is reached; kStripe if neither happens.
LZ4E_DEV uint32_t stripe_mismatch(uint32_t x, uint32_t u0, uint32_t e, uint32_t lane) {
    const uint32_t b = 4 * lane;
    if (b + 4 <= u0) x = 0;
    else if (b < u0) x &= ~0u << (8 * (u0 - b));
    if (b >= e) x |= 1u;
    else if (b + 4 > e) x |= 1u << (8 * (e - b));
    const uint64_t mm = ballot(x != 0);
    if (mm == 0) return kStripe;
    const uint32_t f = ctz64(mm);
    return 4 * f + (uint32_t)__builtin_ctz(lane_val(x, f)) / 8;
}

// ---- output -------------------------------------------------------------

LZ4E_DEV void st32(gu8* out, uint32_t at, uint32_t v) { *(gu32*)(out + at) = v; }

LZ4E_DEV uint32_t out_ext(gu8* out, uint32_t at, uint32_t rest, uint32_t lane) {
    // (rest)/255 bytes of 0xFF then rest % 255 (lz4e_compress.c:365-377, :432-447)
    const uint32_t nff = rest / 255;
    for (uint32_t k = lane; k < nff; k += kWave) out[at + k] = 0xFF;
    if (lane == 0) out[at + nff] = (uint8_t)(rest - nff * 255);
    return nff + 1;
}

// Literal copy of len bytes from the image, whole dwords (may write 3 bytes
// past len; from + len + 3 must stay inside the block).
template <class IMG>
LZ4E_DEV void out_copy(gu8* out, uint32_t at, const IMG& img, uint32_t from, uint32_t len,
                       uint32_t lane) {
    constexpr uint32_t kChunk = 4 * 4 * kWave;
    // Long runs (incompressible data, last literals): 2 KiB per round trip.
    // A wave's loads wait behind its earlier stores (one in-order vmcnt), so
    // the copy costs one HBM round trip per chunk; 1 KiB chunks held
    // incompressible 64 KiB blocks at ~0.5 byte per cycle.
    constexpr uint32_t kBig = 2 * kChunk;
    uint32_t base = 0;
    for (; base + kBig <= len; base += kBig) {
        uint32_t w[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = img.ld32(from + base + 4 * (j * kWave + lane));
#pragma unroll
        for (int j = 0; j < 8; ++j) st32(out, at + base + 4 * (j * kWave + lane), w[j]);
    }
    for (; base < len; base += kChunk) {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t k = base + 4 * (j * kWave + lane);
            w[j] = k < len ? img.ld32(from + k) : 0;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t k = base + 4 * (j * kWave + lane);
            if (k < len) st32(out, at + k, w[j]);
        }
    }
}

// Exact copy of the last literals (nothing may be written past the frame).
template <class IMG>
LZ4E_DEV void out_copy_exact(gu8* out, uint32_t at, const IMG& img, uint32_t from, uint32_t len,
                             uint32_t lane) {
    const uint32_t whole = len & ~3u;
    out_copy(out, at, img, from, whole, lane);
    if (lane < len - whole) out[at + whole + lane] = (uint8_t)img.rd8(from + whole + lane);
}

// Matched bytes from p against c (c < p), counting on from t bytes known
// equal, at most matchlimit - p (LZ4E_count, lz4e_defs.h:587-636); with
// t = 0 a result below 4 means the 4-byte verify failed.
template <class IMG>
LZ4E_DEV uint32_t count_from(const IMG& img, uint32_t p, uint32_t c, uint32_t t,
                             uint32_t matchlimit, uint32_t lane) {
    const uint32_t lim = matchlimit - p;
    while (t < lim) {
        const uint32_t si = img.stripe(p + t, lane);
        const uint32_t sb = img.stripe(c + t, lane);
        const uint32_t u = stripe_mismatch(si ^ sb, 4, 4 + lim - t, lane);
        t += u - 4;
        if (u < kStripe) break;
    }
    return t < lim ? t : lim;
}

// Bytes equal going backwards from p-1 / c-1, at most room (the catch-up of
// lz4e_compress.c:339-349): lane l compares byte l back, 64 bytes per round
// trip.
template <class IMG>
LZ4E_DEV uint32_t back_from(const IMG& img, uint32_t p, uint32_t c, uint32_t room) {
    const uint32_t lane = lane_id();
    for (uint32_t b = 0; b < room; b += kWave) {
        const uint32_t l = b + lane;
        const bool eq = l < room && img.rd8(p - 1 - (l < room ? l : 0)) == img.rd8(c - 1 - (l < room ? l : 0));
        const uint64_t mm = ballot(!eq);
        if (mm) return b + ctz64(mm);
    }
    return room;
}

constexpr uint32_t kFwdW = 8;            // dwords of forward bytes held per position
constexpr uint32_t kFwd = 4 * kFwdW;      // 32 bytes: matches shorter than this stay in registers
constexpr uint32_t kLong = 1u << 31;  // ml flag: kFwd bytes equal, the count goes on
constexpr uint32_t kNoBk = 0xFF;   // bk: backward bytes not available in registers

// Forward match of the kFwd bytes a[] against b[], lane-wise: 0 if the first
// 4 bytes differ, the matched length capped at lim, or kFwd | kLong.
LZ4E_DEV uint32_t fwd_match(const uint32_t* a, const uint32_t* b, uint32_t lim) {
    // first mismatching dword among 1..3, then (only if those are all equal)
    // among 4..7 -- most matches end in the first 16 bytes
    uint32_t m = 16;
#pragma unroll
    for (int i = 3; i >= 1; --i) {
        const uint32_t x = a[i] ^ b[i];
        if (x) m = 4 * (uint32_t)i + ((uint32_t)__builtin_ctz(x) >> 3);
    }
    if (m == 16) {
        m = kFwd;
#pragma unroll
        for (int i = (int)kFwdW - 1; i >= 4; --i) {
            const uint32_t x = a[i] ^ b[i];
            if (x) m = 4 * (uint32_t)i + ((uint32_t)__builtin_ctz(x) >> 3);
        }
    }
    if (a[0] != b[0]) return 0;
    if (m >= lim) return lim;
    return m == kFwd ? (kFwd | kLong) : m;
}

// fwd_match of my kFwd bytes against those of window lane cl (every lane
// calls it; `active` lanes use the result).  Lane cl's dwords 4..7 are only
// fetched (ds_bpermute) when some active lane's first 16 bytes all match:
// most matches end earlier.
LZ4E_DEV uint32_t fwd_match_lane(const uint32_t* dv, uint32_t cl, uint32_t lim, bool active) {
    uint32_t g[4];
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) g[i] = shfl(dv[i], cl);
    uint32_t m = 16;
#pragma unroll
    for (int i = 3; i >= 1; --i) {
        const uint32_t x = dv[i] ^ g[i];
        if (x) m = 4 * (uint32_t)i + ((uint32_t)__builtin_ctz(x) >> 3);
    }
    const bool eq0 = dv[0] == g[0];
    if (ballot(active && eq0 && m == 16)) {
        uint32_t h[kFwdW - 4];
#pragma unroll
        for (uint32_t i = 0; i < kFwdW - 4; ++i) h[i] = shfl(dv[4 + i], cl);
        if (m == 16) {
            m = kFwd;
#pragma unroll
            for (int i = (int)kFwdW - 1; i >= 4; --i) {
                const uint32_t x = dv[i] ^ h[i - 4];
                if (x) m = 4 * (uint32_t)i + ((uint32_t)__builtin_ctz(x) >> 3);
            }
        }
    }
    if (!eq0) return 0;
    if (m >= lim) return lim;
    return m == kFwd ? (kFwd | kLong) : m;
}

// Equal bytes at the top of two dwords (backward catch-up, up to 4).
LZ4E_DEV uint32_t back4(uint32_t a, uint32_t b) {
    const uint32_t x = a ^ b;
    return x ? (uint32_t)__builtin_clz(x) >> 3 : 4;
}

LZ4E_DEV uint64_t lane_val64(uint64_t v, uint32_t k) {
    return ((uint64_t)lane_val((uint32_t)(v >> 32), k) << 32) | lane_val((uint32_t)v, k);
}

// Lanes a..b (inclusive), a <= b <= 63.
LZ4E_DEV uint64_t lane_range(uint32_t a, uint32_t b) {
    return (b >= 63 ? ~0ull : ((2ull << b) - 1)) & ~((1ull << a) - 1);
}

// The greedy parse in windows of 64 positions, lane k <-> position B + k.
//
// Window setup (all lanes at once): the 20 bytes around each position, its
// hash, the table entry before the window (c0, the "snapshot"), the forward
// match against c0 (ml, up to kFwd = 32 bytes) and the bytes equal before both
// (bk).  Positions sharing a hash inside the window form clash groups
// (speculative put + read-back); their candidates depend on the walk's own
// puts (fixpoint chain / exact walk below).
//
// Walk (wave-uniform, mostly SALU): the reference parse over the window,
// reading the precomputed lanes with v_readlane.  The candidate of a
// position is the latest put of its hash made in the window before it, else
// the snapshot -- exactly what the reference's table holds at that point
// because the window's puts only touch the hashes of window positions.
//  * rematch at a match end e (lz4e_compress.c:461-493): puts e-2 and e,
//    candidate of e, a match iff ml != 0;
//  * search (lz4e_compress.c:292-336): probes P <= 64 advance by one byte,
//    so a search over the window is "first probe lane with a hit", every
//    probe before it put; probes with larger steps go to the generic search.
// The window's puts are written to the table once, when the walk leaves it.
// The block's results: the frame size (0: output full) and the iterator
// post-state words (final source position, last literal run).  Returned, not
// stored here: the kernel stores them through pointers it reloads after the
// parse, so that no output pointer occupies SGPRs across it.
struct CResult {
    int32_t ret = 0;
    uint32_t a0 = 0, a1 = 0;
};
// Probes done (of a search that missed through its window) from which the
// generic search takes over (LZ4E_GENERIC_FROM, experiments; 64: only for
// skip steps > 1).
#ifndef LZ4E_GENERIC_FROM
#define LZ4E_GENERIC_FROM 48
#endif
constexpr uint32_t kGenericFrom = LZ4E_GENERIC_FROM;

template <int TT, bool kStamps, class IMG>
LZ4E_DEV CResult compress_block(const IMG& img, uint32_t* smem, uint32_t n, gu8* out, uint32_t cap,
                                uint64_t* dbg, uint32_t lane, uint32_t D = 0, bool progress_prio = true) {
    CResult res;
    // Dictionary mode (D > 0): the image is [D dictionary bytes | the n-byte
    // block], the parse starts at D and the table was preloaded from the
    // dictionary; positions are image positions throughout.
    const Table<TT> T{smem};
    const uint64_t bound = (uint64_t)n + n / 255 + 16;
    // limited output (lz4e_compress.c:553-560): the output checks compare
    // against capl, which is the capacity when limited and never reached
    // otherwise (one SGPR instead of a flag and the capacity)
    const uint32_t capl = cap < bound ? cap : 0xFFFFFFFFu;
    uint32_t op = 0, anchor = D, ip = D;
    [[maybe_unused]] uint32_t trn = 0;
    Stamps st;
    if (kStamps) st.start();

    if (n >= kMinLength) {
        const uint32_t mflimit = D + n - kMfLimit;
        const uint32_t matchlimit = D + n - kLastLiterals;
        const uint64_t lanes_below = (1ull << lane) - 1;
        // First byte (lz4e_compress.c:280-282): put(D); in noDict mode that is
        // position 0 into a zeroed table, a no-op.
        if (D != 0) {
            if (lane == 0) T.put(hash_val<TT>(img.ld64(D)), D);
            lockstep();
        }

        // ---- sequence output -------------------------------------------
        // offset, match-length code and token of a sequence whose token slot
        // is tok (lz4e_compress.c:384-453); false when the output is full.
        auto emit_match = [&](uint32_t tok, uint32_t tokhi, uint32_t off, uint32_t mc) -> bool {
            const uint32_t op_off = op;
            op += 2;
            if ((uint64_t)op + 6 + (mc >> 8) > capl) return false;
            const uint32_t tokb = tokhi | (mc < 15 ? mc : 15);
            const uint32_t e1 = mc - 15;
            const uint32_t e1w = (mc >= 15 && e1 < 255) ? e1 : 0;
            if (lane == 0) {
                if (op_off == tok + 1) {
                    st32(out, tok, tokb | (off << 8) | (e1w << 24));
                } else {
                    out[tok] = (uint8_t)tokb;
                    st32(out, op_off, off | (e1w << 16));
                }
            }
            if (mc >= 15) {
                if (e1 < 255) {
                    op += 1;
                } else {
                    lockstep();  // overwrites the dword's spare byte
                    op += out_ext(out, op, e1, lane);
                }
            }
            return true;
        };

        bool rmode = false;  // e is a match end (rematch) / the next probe of a search
        uint32_t e = D + 1;  // next position of the walk
        uint32_t s = D + 1;  // start of the current search
        uint32_t jb = 0;     // probes of the current search done so far
        uint32_t pf = 0;     // prefetch of the next window's bytes (warms L1/L2)
        // Large blocks only: a batch's kernel time is its slowest block, and
        // raising the priority of the waves furthest behind shortens it
        // (silesia64k compress -9 %); 4 KiB blocks finish in a few windows.
        // q = floor(4 (e - D) / n) moves only at the quarter marks, so the
        // window loop compares e against the next mark (a division per
        // window costs ~25 instructions and two VALU -> SALU hops).
        // (q only grows: each crossing of a mark is a new quarter)
        uint32_t prio_next = (n > 16384 && progress_prio) ? D : ~0u;  // e at which q changes next
        // Put pattern the clash fixpoint starts from for the lanes ahead of a
        // chain: every lane, or (periodic data: ints, records) the previous
        // window's final puts, whichever predicted the last window better.
        uint64_t guess = ~0ull, pprev = ~0ull;
        // The next window's bytes, loaded as soon as the walk knows where it
        // starts (nB) so that the loads overlap the emit and the commit.
        uint32_t nB = ~0u, ndm1 = 0, ndv[kFwdW];
        auto preload = [&](uint32_t Bn) {
            if (Bn == nB) return;
            nB = Bn;
            uint32_t o[9];
            img.wld9(Bn + lane, o);
            ndm1 = o[0];
#pragma unroll
            for (uint32_t i = 0; i < kFwdW; ++i) ndv[i] = o[1 + i];
        };
        for (;;) {
            // ================= window setup =================================
            if (e >= prio_next) {
                const uint32_t q = (uint32_t)(((uint64_t)(e - D) * 4) / n);
                prio_next = q >= 4 ? ~0u : D + (uint32_t)(((uint64_t)(q + 1) * n + 3) / 4);
                wave_prio_for(q);
            }
            consume(pf);
            const uint32_t B = rmode ? e - 2 : e;
            const uint32_t p = B + lane;
            const bool valid = p <= mflimit;  // every put / lookup is at <= mflimit
            uint32_t dm1, dv[kFwdW];  // bytes p - 4 .. p - 1, p .. p + kFwd - 1
            if (B == nB) {
                dm1 = ndm1;
#pragma unroll
                for (uint32_t i = 0; i < kFwdW; ++i) dv[i] = ndv[i];
            } else {
                uint32_t o[9];
                img.wld9(p, o);
                dm1 = o[0];
#pragma unroll
                for (uint32_t i = 0; i < kFwdW; ++i) dv[i] = o[1 + i];
            }
            const uint32_t d0 = dv[0];
            const uint32_t h = hash_val<TT>(((uint64_t)dv[1] << 32) | d0);
            uint32_t c0 = 0, rb = p;
            lockstep();  // the previous window's commit is in the table
            if (valid) c0 = T.get(h);  // snapshot
            // the snapshot candidate's bytes: issued now, used after the clash
            // groups (a block staged in LDS: only the first dword, the rest
            // when some lane's first 4 bytes match -- windows of
            // incompressible data need none of them)
            uint32_t em1 = 0, ev[kFwdW];
            if constexpr (!IMG::kInLds) {
                uint32_t o[9];
                img.wld9(c0, o);
                em1 = o[0];
#pragma unroll
                for (uint32_t i = 0; i < kFwdW; ++i) ev[i] = o[1 + i];
            } else {
                ev[0] = img.wld(c0);
            }
            lockstep();
            if (valid) T.put(h, p);  // speculative put of every position
            lockstep();
            if (valid) rb = T.reread(h);
            const uint64_t cm = ballot(rb != p);
            uint64_t same = 0;  // valid lanes sharing my hash (clash groups only)
            if (cm) {
                // A valid lane reads back the position of its group's winning
                // put, so rb - B names the group (invalid lanes: none; their
                // `same` only steers the walk between two exact table builds).
                const uint64_t vmask = ballot(valid);
                const uint64_t m = match_any6(rb - B) & vmask;
                if (valid && (m & (m - 1))) same = m;
            }
            const uint64_t clash = ballot(same != 0);
            const uint32_t lim = matchlimit - p;
            uint32_t ml = 0, bk = kNoBk;
            {
                const bool dist_ok = (TT == kByU16) || (c0 + kMaxDistance >= p);
                // (LDS image: no lane's first dword verifying leaves ml = 0
                // everywhere -- fwd_match's result -- and bk unused)
                bool full = true;
                if constexpr (IMG::kInLds) {
                    full = ballot(valid && dist_ok && ev[0] == d0) != 0;
                    if (full) {
                        uint32_t o[9];
                        img.wld9(c0, o);
                        em1 = o[0];
#pragma unroll
                        for (uint32_t i = 1; i < kFwdW; ++i) ev[i] = o[1 + i];
                    }
                }
                if (full) {
                    if (valid && dist_ok) ml = fwd_match(dv, ev, lim);
                    if (p >= 4 && c0 >= 4) bk = back4(dm1, em1);
                }
            }
            const uint64_t hitm = ballot(ml != 0);
            uint64_t put = 0;
            bool generic = false;
            // Match of window position B + k against the earlier window position
            // B + cl, from the registers of both lanes (v_readlane): forward as
            // fwd_match (0, length < kFwd, or kFwd | kLong) and backward up to 4 bytes.
            auto lanes_match = [&](uint32_t k, uint32_t cl, uint32_t& m, uint32_t& bb) {
                const uint32_t lk = matchlimit - (B + k);
                uint32_t ak[kFwdW], ac[kFwdW];
#pragma unroll
                for (uint32_t i = 0; i < kFwdW; ++i) {
                    ak[i] = lane_val(dv[i], k);
                    ac[i] = lane_val(dv[i], cl);
                }
                m = fwd_match(ak, ac, lk);
                bb = (B + k >= 4 && B + cl >= 4) ? back4(lane_val(dm1, k), lane_val(dm1, cl)) : kNoBk;
            };

            // ---- fast chain tables, per lane k as "rmode at B + k" ---------
            // The common case of the walk below, for every lane at once given
            // each lane's candidate (vc, match vm, back bytes vb): a rematch
            // at k that hits (sequence with no literals, next rmode at
            // k + vm), or one that misses followed by a search whose first
            // probe hit j is in this window (literals [k, j - cu), next rmode
            // at j + vm(j)).  Anything else -- matches of 16+ bytes, catch-up
            // beyond the 4 bytes in registers, a search leaving the window,
            // limited output -- stops the chain and the exact walk takes over.
            // fc: next rmode lane (bits 0-6) or kStop; fe: the sequence as
            // offset | literal length << 16 | match length << 24; jv: the
            // last probe of its search (probes (k, jv]), else k.
            constexpr uint32_t kStop = 0x80;
            const int32_t lvs0 = (int32_t)mflimit - 1 - (int32_t)B;
            const uint64_t inlim0 =
                lvs0 < 0 ? 0 : (lvs0 >= 63 ? ~0ull : ((2ull << (uint32_t)lvs0) - 1));
            const uint64_t srch0 = (lane >= 63 ? 0 : (~0ull << (lane + 1))) & inlim0;
            auto chain_tables = [&](uint32_t vc, uint32_t vm, uint32_t vb, uint32_t& fc,
                                    uint32_t& fe, uint32_t& jv) {
                fc = kStop;
                fe = 0;
                jv = lane;
                const uint64_t ah = ballot(vm != 0) & srch0;
                const uint32_t j = ah ? ctz64(ah) : 64;
                const uint32_t jj = j < 64 ? j : lane;
                const uint32_t mlj = shfl(vm, jj), cj = shfl(vc, jj), bkj = shfl(vb, jj);
                if (valid) {
                    if (vm != 0) {
                        if (!(vm & kLong)) {
                            fc = lane + vm;
                            fe = (p - vc) | (vm << 24);
                        }
                    } else if (j < 64 && !(mlj & kLong) && bkj != kNoBk) {
                        const uint32_t room = j - lane < cj ? j - lane : cj;
                        const uint32_t cu = bkj < room ? bkj : room;
                        if (!(cu == 4 && room > 4)) {
                            fc = j + mlj;
                            fe = (B + j - cj) | ((j - cu - lane) << 16) | ((mlj + cu) << 24);
                            jv = j;
                        }
                    }
                }
            };
            // Tables for the snapshot candidates: exact wherever no clash lane
            // is involved; recomputed per chain otherwise (see the walk).
            uint32_t fc0 = kStop, fe0 = 0, jv0 = lane;
            bool have0 = false;  // snapshot tables built (on first use)
            // the next window starts at or a little after B + 64: touch
            // [B + 64, B + 320) now, one dword per lane, so that its loads hit
            // cache (the value is only kept alive, never used)
            if constexpr (!IMG::kInLds) pf = img.wld(B + 64 + 4 * lane);
            if (kStamps) { st.cnt[0]++; st.lap(kPhSearch); }

            // ================= walk =========================================
            for (;;) {
                // (LDS-staged blocks: a window where no lane's candidate
                // verifies and no hash is shared has no chain -- every fc is
                // kStop -- so the rematch and search below take it without the
                // tables: fio4k -2.8 %; the HBM form measured slower with it)
                if (rmode && capl == 0xFFFFFFFFu && (!IMG::kInLds || (hitm | clash) != 0)) {
                    // ---- fast chain: follow fc from the current rmode lane ----
                    // With clash lanes ahead, a candidate is "the latest put of
                    // its group before it", and the puts are the chain's own:
                    // guess them (every lane from here on), build the tables
                    // from the guess, follow the chain, and repeat with the
                    // chain's puts until they reproduce the guess below the
                    // chain's end -- that fixpoint is the reference's parse (a
                    // candidate only depends on puts before it).
                    if (kStamps) st.lap(kPhStripe);
                    const uint32_t ks = e - B;
                    uint32_t k = ks, nev = 0, ev = 0;
                    uint64_t evm = 0, pch = 0;
                    uint32_t fc = kStop, fe = 0, jv = lane;
                    if (ks < 64) {
                        const bool dyn = (clash >> ks) != 0;
                        if (!dyn) {
                            if (!have0) {
                                chain_tables(c0, ml, bk, fc0, fe0, jv0);
                                have0 = true;
                            }
                            fc = fc0;
                            fe = fe0;
                            jv = jv0;
                        }
                        uint64_t Pg = put | (1ull << (ks - 2)) | (1ull << ks) |
                                      (guess & lane_range(ks, 63));
                        constexpr uint32_t kMaxPass = 6;
                        for (uint32_t pass = 0;; ++pass) {
                            if (kStamps) st.cnt[2]++;
                            if (dyn) {
                                const uint64_t pm =
                                    ((clash >> lane) & 1) ? (same & Pg & lanes_below) : 0;
                                const uint32_t cl = pm ? 63 - (uint32_t)__builtin_clzll(pm) : lane;
                                const uint32_t gm1 = shfl(dm1, cl);
                                const uint32_t fm = fwd_match_lane(dv, cl, lim, pm && valid);
                                uint32_t vc = c0, vm = ml, vb = bk;
                                if (pm) {
                                    vc = B + cl;
                                    vm = valid ? fm : 0;
                                    vb = (p >= 4 && B + cl >= 4) ? back4(dm1, gm1) : kNoBk;
                                }
                                chain_tables(vc, vm, vb, fc, fe, jv);
                            }
                            if (kStamps) st.lap(kPhCount);
                            // The serial part: the chain from ks.  fc^2, fc^3
                            // and fc^4 (a lane past the window or stopped stays
                            // put) let one step read four links with independent
                            // readlanes instead of one dependent readlane each.
                            // (every lane takes part in each shuffle)
                            const uint32_t g1 = shfl(fc, fc & 63);
                            const uint32_t J2 = fc < 64 ? g1 : fc;
                            const uint32_t g2 = shfl(fc, J2 & 63), g3 = shfl(J2, J2 & 63);
                            const uint32_t J3 = J2 < 64 ? g2 : J2;
                            const uint32_t J4 = J2 < 64 ? g3 : J2;
                            k = ks;
                            evm = 0;
                            while (k < 64) {
                                const uint32_t x1 = lane_val(fc, k), x2 = lane_val(J2, k);
                                const uint32_t x3 = lane_val(J3, k), x4 = lane_val(J4, k);
                                if (x1 & kStop) break;
                                evm |= 1ull << k;
                                if (x1 >= 64) { k = x1; break; }
                                if (x2 & kStop) { k = x1; break; }
                                evm |= 1ull << x1;
                                if (x2 >= 64) { k = x2; break; }
                                if (x3 & kStop) { k = x2; break; }
                                evm |= 1ull << x2;
                                if (x3 >= 64) { k = x3; break; }
                                if (x4 & kStop) { k = x3; break; }
                                evm |= 1ull << x3;
                                k = x4;
                            }
                            nev = popc64(evm);
                            // the chain's puts (e-2 and e of every event, the probes
                            // (l, jv(l)] of its searches), all lanes at once
                            {
                                const uint64_t eb = evm & lanes_below;
                                const uint32_t lb = eb ? 63 - (uint32_t)__builtin_clzll(eb) : lane;
                                const uint32_t jl = shfl(jv, lb);
                                pch = ballot(eb != 0 && lane <= jl) | evm | (evm >> 2);
                            }
                            if (!dyn) break;
                            // Exact once every lane the chain used (rematch lanes and
                            // search probes: its puts minus the e-2 ones) sees the
                            // same candidate under the chain's own puts as under the
                            // guess.
                            const uint64_t Pn = put | pch;
                            const uint64_t U = pch & ~(evm >> 2);
                            const uint64_t mem = same & lanes_below;
                            const uint64_t cg = mem & Pg, cn = mem & Pn;
                            const bool bad = ((U >> lane) & 1) && cg != cn &&
                                             (cg == 0 || cn == 0 ||
                                              __builtin_clzll(cg) != __builtin_clzll(cn));
                            if (!ballot(bad)) break;  // fixpoint
                            if (pass + 1 == kMaxPass) {          // give up: exact walk
                                nev = 0;
                                k = ks;
                                pch = 0;
                                break;
                            }
                            Pg = Pn | (k >= 64 ? 0 : lane_range(k, 63));
                        }
                        put |= pch;
                        // ev: lane q < nev holds the lane of event q
                        const bool isev = (evm >> lane) & 1;
                        ev = push_lane(lane, isev ? popc64(evm & lanes_below) : 63);
                    }
                    if (kStamps) st.lap(kPhLit);
                    if (nev) {
                        // emit the nev sequences at once (lz4e_compress.c:352-453):
                        // lane q writes sequence q's token, extension bytes and
                        // offset; window lane x writes literal byte B + x.
                        const uint32_t f = shfl(fe, lane < nev ? ev : 0);
                        const uint32_t L = (f >> 16) & 0xFF, mc = (f >> 24) - 4;
                        const uint32_t hdr = L >= 15 ? 2 : 1;
                        const uint32_t size = lane < nev ? hdr + L + 2 + (mc >= 15 ? 1 : 0) : 0;
                        const uint32_t o = op + wave_incl_add(size) - size;
                        if (lane < nev) {
                            out[o] = (uint8_t)(((L < 15 ? L : 15) << 4) | (mc < 15 ? mc : 15));
                            if (L >= 15) out[o + 1] = (uint8_t)(L - 15);
                            out[o + hdr + L] = (uint8_t)f;
                            out[o + hdr + L + 1] = (uint8_t)(f >> 8);
                            if (mc >= 15) out[o + hdr + L + 2] = (uint8_t)(mc - 15);
                        }
                        // literal byte of lane x: run of the last event lane s <= x
                        const uint64_t le = evm & (lane >= 63 ? ~0ull : ((2ull << lane) - 1));
                        const uint32_t s = le ? 63 - (uint32_t)__builtin_clzll(le) : 0;
                        const uint32_t qi = popc64(evm & ((1ull << s) - 1));
                        const uint32_t Lq = shfl(L, qi), dq = shfl(o + hdr, qi);
                        if (le && lane - s < Lq) out[dq + lane - s] = (uint8_t)d0;
                        op = lane_val(o + size, nev - 1);
                        e = B + k;
                        anchor = e;
                        if (kStamps) { st.cnt[1] += nev; st.cnt[3] += nev << 16; st.lap(kPhTail); }
                        if (e > mflimit) {  // :456-457
                            ip = e;
                            goto last_literals;
                        }
                    }
                }
                if (kStamps && rmode && capl == 0xFFFFFFFFu) { st.cnt[3]++; st.lap(kPhLit); }
                if (rmode) {
                    // ---- fill table at e-2, test e (lz4e_compress.c:461-493) ----
                    const uint32_t k = e - B;
                    if (k > 63) break;
                    const uint64_t prior = put | (1ull << (k - 2));
                    uint32_t c, m;
                    if ((clash >> k) & 1) {
                        const uint64_t pm = lane_val64(same, k) & prior & ((1ull << k) - 1);
                        if (pm == 0) {
                            c = lane_val(c0, k);
                            m = lane_val(ml, k);
                        } else {
                            const uint32_t cl = 63 - (uint32_t)__builtin_clzll(pm);
                            c = B + cl;
                            uint32_t bb;
                            lanes_match(k, cl, m, bb);
                        }
                    } else {
                        c = lane_val(c0, k);
                        m = lane_val(ml, k);
                    }
                    put = prior | (1ull << k);
                    if (kStamps) st.lap(kPhCount);
                    if (m == 0) {
                        // no match at e: search from e + 1 (:496-497)
                        rmode = false;
                        s = e = e + 1;
                        jb = 0;
                        continue;
                    }
                    uint32_t t = m & ~kLong;
                    if (m & kLong) t = count_from(img, e, c, kFwd, matchlimit, lane);
                    LZ4E_TR(2, e, ((uint64_t)c << 32) | t);
                    const uint32_t tok = op++;
                    if (!emit_match(tok, 0, e - c, t - 4)) goto fail;
                    if (kStamps) st.cnt[1]++;
                    e += t;
                    anchor = e;
                    if (e > mflimit) {  // :456-457
                        ip = e;
                        goto last_literals;
                    }
                    continue;
                }

                // ---- search: probes P = jb + (k - k0) at lanes k >= k0 ----
                const uint32_t k0 = e - B;
                if (k0 > 63) break;
                const uint32_t kmax = k0 + 64 - jb < 63 ? k0 + 64 - jb : 63;  // P <= 64: step 1
                // probe q runs iff q + 1 <= mflimit (:301-302)
                const int32_t lvs = (int32_t)mflimit - 1 - (int32_t)B;
                if (lvs < (int32_t)k0) {
                    ip = jb ? e - 1 : s;  // the last probe that ran
                    goto last_literals;
                }
                const uint32_t lastv = (uint32_t)lvs < kmax ? (uint32_t)lvs : kmax;
                const uint64_t rng = lane_range(k0, lastv);
                const uint64_t A = hitm & ~clash & rng;
                uint64_t CL = clash & rng;
                if (A) CL &= (1ull << ctz64(A)) - 1;
                uint32_t hk = 64, c = 0, m = 0, b = kNoBk;
                // Every probe lane at once: a clash lane's candidate is the
                // latest member of its group put before it (the window's puts
                // so far plus this search's earlier probes), else c0; it is
                // matched against that member's registers (ds_bpermute).
                uint32_t vc = c0, vm = ml, vb = bk;
                if (CL) {
                    const bool isc = (CL >> lane) & 1;
                    const uint64_t prior_l = put | (lane > k0 ? lane_range(k0, lane - 1) : 0);
                    const uint64_t pm = isc ? (same & prior_l & lanes_below) : 0;
                    const uint32_t cl = pm ? 63 - (uint32_t)__builtin_clzll(pm) : lane;
                    const uint32_t gm1 = shfl(dm1, cl);
                    const uint32_t fm = fwd_match_lane(dv, cl, lim, pm != 0);
                    if (pm) {
                        vc = B + cl;
                        vm = fm;
                        vb = (p >= 4 && B + cl >= 4) ? back4(dm1, gm1) : kNoBk;
                    }
                }
                const uint64_t H = ballot((((CL | A) >> lane) & 1) && vm != 0);
                if (H) {
                    hk = ctz64(H);
                    c = lane_val(vc, hk);
                    m = lane_val(vm, hk);
                    b = lane_val(vb, hk);
                }
                if (hk == 64) {
                    // no hit among this window's probes: all of them put
                    put |= rng;
                    jb += lastv - k0 + 1;
                    e = B + lastv + 1;
                    if (lastv < kmax) {  // the next probe would pass mflimit
                        ip = B + lastv;
                        goto last_literals;
                    }
                    // Skip steps > 1 from probe 65 on, and then the generic
                    // search.  It also takes the search over once fewer than
                    // 64 - kGenericFrom step-1 probes are left: a window for
                    // those few lanes costs a whole setup and commit (fio's
                    // incompressible runs: the search misses through the
                    // first window, then three or four probes in a second).
                    if (jb > kGenericFrom) {
                        generic = true;
                        break;
                    }
                    continue;  // next window
                }
                put |= lane_range(k0, hk);
                if (kStamps) st.lap(kPhStripe);
                const uint32_t q = B + hk;
                // catch up (lz4e_compress.c:339-349)
                const uint32_t room = q - anchor < c ? q - anchor : c;
                uint32_t cu;
                if (b == kNoBk) {
                    cu = back_from(img, q, c, room);
                } else {
                    cu = b < room ? b : room;
                    if (cu == 4 && room > 4) cu += back_from(img, q - 4, c - 4, room - 4);
                }
                const uint32_t ipm = q - cu, cand = c - cu;
                uint32_t t = m & ~kLong;
                if (m & kLong) t = count_from(img, q, c, kFwd, matchlimit, lane);
                t += cu;
                LZ4E_TR(2, ipm, ((uint64_t)cand << 32) | t);
                // literals [anchor, ipm) (lz4e_compress.c:352-382)
                const uint32_t L = ipm - anchor;
                const uint32_t tok = op++;
                if ((uint64_t)op + L + 8 + L / 255 > capl) goto fail;
                uint32_t tokhi;
                if (L >= 15) {
                    tokhi = 0xF0;
                    op += out_ext(out, op, L - 15, lane);
                } else {
                    tokhi = L << 4;
                }
                if (anchor >= B) {
                    // the run lies in the window: lane a0 + 4i stores bytes 4i..4i+3
                    const uint32_t r = lane - (anchor - B);
                    if ((r & 3) == 0 && r < L) st32(out, op + r, d0);
                } else {
                    out_copy(out, op, img, anchor, L, lane);
                }
                op += L;
                lockstep();  // the offset overwrites the copy's spare bytes
                if (!emit_match(tok, tokhi, ipm - cand, t - 4)) goto fail;
                if (kStamps) { st.cnt[1]++; st.lap(kPhTail); }
                e = ipm + t;
                anchor = e;
                rmode = true;
                if (e > mflimit) {
                    ip = e;
                    goto last_literals;
                }
            }
            if (kStamps) st.lap(kPhStripe);

            // ================= commit the window's puts =====================
            if (!generic) preload(rmode ? e - 2 : e);
            if (valid) {
                const uint64_t pg = same & put;
                bool writer;
                uint32_t v;
                if (same == 0) {
                    writer = true;
                    v = (put >> lane) & 1 ? p : c0;
                } else if (pg) {
                    writer = lane == 63 - (uint32_t)__builtin_clzll(pg);
                    v = p;
                } else {
                    writer = lane == ctz64(same);
                    v = c0;
                }
                if (writer) T.put(h, v);
            }
            {
                const uint64_t R = ~7ull;
                const uint32_t mp = popc64((put ^ pprev) & R), mo = popc64(~put & R);
                guess = mp < mo ? put : ~0ull;
                pprev = put;
            }
            if (kStamps) st.lap(kPhRematch);
            if (!generic) continue;

            // ================= generic search (probes P >= 65) ==============
            // Skip steps > 1 (lz4e_compress.c:292-336) over windows of 64
            // probes: the candidate a probe sees is the latest earlier probe
            // of the window with an equal hash, else the table entry.
            {
                uint32_t pbase = jb, qh, ch;
                for (;;) {
                    const uint32_t P = pbase + lane;
                    const uint32_t qq = s + (uint32_t)probe_offset(P);
                    const bool pv = (uint64_t)qq + probe_step(P) <= mflimit;
                    const uint64_t vmask = ballot(pv);
                    if (vmask == 0) {
                        ip = s + (uint32_t)probe_offset(pbase - 1);
                        goto last_literals;
                    }
                    const uint32_t q = pv ? qq : s;
                    uint64_t v;
                    if constexpr (TT == kByU32) v = img.ld64(q);
                    else v = img.ld32(q);
                    const uint32_t vq = (uint32_t)v;
                    const uint32_t hq = hash_val<TT>(v);
                    uint32_t g0 = 0, grb = q;
                    lockstep();
                    if (pv) g0 = T.get(hq);
                    lockstep();
                    if (pv) T.put(hq, q);
                    lockstep();
                    if (pv) grb = T.reread(hq);
                    const uint64_t gcm = ballot(grb != q);
                    uint64_t gsame = 0;
                    uint32_t gc = g0;
                    if (gcm) {
                        uint64_t todo = gcm;
                        do {
                            const uint32_t hg = lane_val(hq, ctz64(todo));
                            const uint64_t mm = ballot(pv && hq == hg);
                            if (hq == hg) gsame = mm;
                            todo &= ~mm;
                        } while (todo);
                        const uint64_t below = gsame & lanes_below;
                        const uint32_t qp =
                            shfl(q, below ? 63 - (uint32_t)__builtin_clzll(below) : lane);
                        if (below) gc = qp;
                    }
                    bool hit = false;
                    if (pv) {
                        const bool dist_ok = (TT == kByU16) || (gc + kMaxDistance >= q);
                        hit = dist_ok && img.ld32(gc) == vq;
                    }
                    const uint64_t hm = ballot(hit);
                    const uint32_t klast = hm ? ctz64(hm) : popc64(vmask) - 1;
                    if (pv) {
                        if (gcm == 0) {
                            if (lane > klast) T.put(hq, g0);
                        } else {
                            const uint64_t upto = klast >= 63 ? ~0ull : ((2ull << klast) - 1);
                            if (lane <= klast) {
                                if ((gsame & upto & ~((2ull << lane) - 1)) == 0) T.put(hq, q);
                            } else if ((gsame & upto) == 0) {
                                T.put(hq, g0);
                            }
                        }
                    }
                    if (hm) {
                        qh = lane_val(q, klast);
                        ch = lane_val(gc, klast);
                        break;
                    }
                    if (vmask != ~0ull) {
                        ip = lane_val(q, klast);  // the last probe that ran
                        goto last_literals;
                    }
                    pbase += kWave;
                }
                const uint32_t room = qh - anchor < ch ? qh - anchor : ch;
                const uint32_t cu = back_from(img, qh, ch, room);
                const uint32_t ipm = qh - cu, cand = ch - cu;
                const uint32_t t = count_from(img, qh, ch, 4, matchlimit, lane) + cu;
                LZ4E_TR(2, ipm, ((uint64_t)cand << 32) | t);
                const uint32_t L = ipm - anchor;
                const uint32_t tok = op++;
                if ((uint64_t)op + L + 8 + L / 255 > capl) goto fail;
                uint32_t tokhi;
                if (L >= 15) {
                    tokhi = 0xF0;
                    op += out_ext(out, op, L - 15, lane);
                } else {
                    tokhi = L << 4;
                }
                out_copy(out, op, img, anchor, L, lane);
                op += L;
                lockstep();
                if (!emit_match(tok, tokhi, ipm - cand, t - 4)) goto fail;
                if (kStamps) { st.cnt[1]++; st.lap(kPhLit); }
                e = ipm + t;
                anchor = e;
                rmode = true;
                if (e > mflimit) {
                    ip = e;
                    goto last_literals;
                }
            }
        }
    }

last_literals: {
        // lz4e_compress.c:500-530
        const uint32_t R = D + n - anchor;
        if ((uint64_t)op + R + 1 + (R + 240) / 255 > capl) goto fail;
        if (R >= 15) {
            if (lane == 0) out[op] = 0xF0;
            op += 1;
            op += out_ext(out, op, R - 15, lane);
        } else {
            if (lane == 0) out[op] = (uint8_t)(R << 4);
            op += 1;
        }
        out_copy_exact(out, op, img, anchor, R, lane);
        res.ret = (int32_t)(op + R);
        res.a0 = ip - D;
        res.a1 = R;
        if (kStamps) {
            st.lap(kPhTail);
            if (lane == 0 && dbg) {
                for (int i = 0; i < 6; ++i) dbg[i] = st.acc[i];
                dbg[6] = ((uint64_t)st.cnt[1] << 32) | st.cnt[0];
                dbg[7] = ((uint64_t)st.cnt[3] << 32) | st.cnt[2];
                // the parse's shader cycles and 100 MHz ticks (its clock)
                dbg[8] = clock64() - st.t0;
                dbg[9] = realtime64() - st.r0;
            }
        }
        return res;
    }
fail:
    return res;  // 0, 0, 0
}

// Stage a block into LDS as a word image, the bytes of the last partial word
// zeroed (16-B loads when the block is 16-B aligned in HBM).  Reads past the
// image are clamped to its last word (LdsImage), so no pad is needed.
LZ4E_DEV void stage_block(uint32_t* dstw, const uint8_t* src, uint32_t n, uint32_t lane) {
    const uint32_t padded = (n + 3) & ~3u;
    uint8_t* d8 = reinterpret_cast<uint8_t*>(dstw);
    if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
        const uint4* g = reinterpret_cast<const uint4*>(src);
        uint4* l = reinterpret_cast<uint4*>(dstw);
        const uint32_t nv = n / 16;
        constexpr uint32_t U = 8;  // 8 x 16 B in flight per lane
        const uint32_t nfull = nv / (U * kWave) * (U * kWave);
        for (uint32_t base = 0; base < nfull; base += U * kWave) {
            uint4 v0 = g[base + 0 * kWave + lane], v1 = g[base + 1 * kWave + lane];
            uint4 v2 = g[base + 2 * kWave + lane], v3 = g[base + 3 * kWave + lane];
            uint4 v4 = g[base + 4 * kWave + lane], v5 = g[base + 5 * kWave + lane];
            uint4 v6 = g[base + 6 * kWave + lane], v7 = g[base + 7 * kWave + lane];
            l[base + 0 * kWave + lane] = v0; l[base + 1 * kWave + lane] = v1;
            l[base + 2 * kWave + lane] = v2; l[base + 3 * kWave + lane] = v3;
            l[base + 4 * kWave + lane] = v4; l[base + 5 * kWave + lane] = v5;
            l[base + 6 * kWave + lane] = v6; l[base + 7 * kWave + lane] = v7;
        }
        for (uint32_t i = nfull + lane; i < nv; i += kWave) l[i] = g[i];
        for (uint32_t i = nv * 16 + lane; i < padded; i += kWave) d8[i] = i < n ? src[i] : 0;
    } else {
        for (uint32_t i = lane; i < padded; i += kWave) d8[i] = i < n ? src[i] : 0;
    }
}

template <bool kStamps, class IMG>
LZ4E_DEV CResult dispatch_class(const IMG& img, uint32_t* smem, uint32_t n, int tt, gu8* out,
                                uint32_t cap, uint64_t* dbg, uint32_t lane, uint32_t D = 0,
                                bool pp = true) {
    if (tt == kByU32) return compress_block<kByU32, kStamps>(img, smem, n, out, cap, dbg, lane, D, pp);
    if (tt == kByU16) return compress_block<kByU16, kStamps>(img, smem, n, out, cap, dbg, lane, 0, pp);
    return compress_block<kByU64, kStamps>(img, smem, n, out, cap, dbg, lane, 0, pp);
}

// The kernel's explicit arguments as laid out in the kernarg segment
// (natural alignment, in order).  After the parse the kernel reloads its
// result pointers from there through a laundered pointer -- a fresh scalar
// load -- instead of keeping them live in SGPRs across the whole parse
// (which is at the SGPR limit: every pointer held there is one more spill
// reloaded inside the window loops).
struct CompressArgs {
    const uint8_t* src;
    const uint64_t* src_off;
    const uint32_t* src_len;
    const uint8_t* table_type;
    uint8_t* dst;
    const uint64_t* dst_off;
    const uint32_t* dst_cap;
    int32_t* ret;
    uint32_t* aux;
    uint32_t nblocks;
    uint32_t max_len;
    uint64_t* dbg;
    const uint32_t* dict_len;
    const uint32_t* order;
};
static_assert(offsetof(CompressArgs, ret) == 56 && offsetof(CompressArgs, order) == 96, "kernarg layout");

template <bool kLdsInput, bool kStamps>
__global__ __launch_bounds__(64) void compress_kernel(const uint8_t* __restrict__ src,
                                                      const uint64_t* __restrict__ src_off,
                                                      const uint32_t* __restrict__ src_len,
                                                      const uint8_t* __restrict__ table_type,
                                                      uint8_t* __restrict__ dst,
                                                      const uint64_t* __restrict__ dst_off,
                                                      const uint32_t* __restrict__ dst_cap,
                                                      int32_t* __restrict__ ret,
                                                      uint32_t* __restrict__ aux, uint32_t nblocks,
                                                      uint32_t max_len, uint64_t* __restrict__ dbg,
                                                      const uint32_t* __restrict__ dict_len,
                                                      const uint32_t* __restrict__ order) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    if (blockIdx.x >= nblocks) return;
    const uint32_t b = order ? order[blockIdx.x] : blockIdx.x;
    const uint32_t lane = lane_id();
    const uint32_t n = src_len[b];
    const int tt = table_type[b];
    const uint32_t cap = dst_cap[b];
    gu8* out = (gu8*)(dst + dst_off[b]);
    const uint8_t* in = src + src_off[b];
    uint64_t* dbg_slot = dbg ? dbg + kCompressStampWords * (size_t)b : nullptr;

    // Dictionary mode: the dict_len[b] (<= 64 KiB) bytes before the block
    // are its dictionary; under 8 bytes it is ignored (LZ4_loadDict:
    // dictSize < HASH_UNIT).  byU32 only, HBM image only.
    const uint32_t D = dict_len && dict_len[b] >= 8 ? dict_len[b] : 0;
    const bool tt_ok = (tt == kByU16 && n <= 65536) || tt == kByU32 || tt == kByU64;
    const bool dict_ok = D == 0 || (tt == kByU32 && D <= 65536 && !kLdsInput);
    // the launch sized LDS (staging mode) for blocks of at most max_len bytes
    const bool fits = !kLdsInput || n <= max_len;
    if (n > kMaxInput || (n >= kMinLength && !tt_ok) || !fits || !dict_ok) {
        // Input too large (lz4e_compress.c:245-248) returns 0; a malformed
        // descriptor (class/length the SG rules cannot produce, or a block
        // longer than the batch's max_len) returns -1.
        if (lane == 0) ret[b] = n > kMaxInput ? 0 : -1;
        return;
    }

    CResult res;
    if (n >= kMinLength) {
        // memset of the state (lz4e_compress.c:548): 16 KiB of table.
        uint4* t4 = reinterpret_cast<uint4*>(smem);
        for (uint32_t i = lane; i < kTableBytes / 16; i += kWave) t4[i] = make_uint4(0, 0, 0, 0);
    }

    if constexpr (kLdsInput) {
        uint32_t* inw = smem + kTableBytes / 4;
        stage_block(inw, in, n, lane);
        block_sync();
        const LdsImage img{inw, n == 0 ? 0 : (n - 1) >> 2};
        res = dispatch_class<kStamps>(img, smem, n, tt, out, cap, dbg_slot, lane);
    } else {
        block_sync();
        const uint8_t* base = in - D;
        const HbmImage img{buf_make(base, D + n)};
        if (D != 0 && n >= kMinLength) {
            // LZ4_loadDict: every third dictionary position p with p + 8 <= D
            // (HASH_UNIT), in order -- the last put of a hash wins, so the
            // largest p of each hash (LDS atomic max)
            for (uint32_t p = 3 * lane; p + 8 <= D; p += 3 * kWave)
                atomicMax(&smem[hash_val<kByU32>(img.ld64(p))], p);
            block_sync();
        }
        // Issue priority: the waves furthest behind first (progress
        // priority, 3 -> 0 by quarter of the block), except in a batch that
        // mixes heavy and light blocks (launch order with order[nblocks]
        // heavy ones, kHeavyBucket, and at least 1/16 light): there the heavy
        // blocks keep 3 for their whole parse and the light ones 0
        // (silesia64k -4 %; text256k, all heavy, is 4 % faster with progress).
        bool pp = true;
        if (order) {
            const uint32_t nh = order[nblocks];
            if (nh < nblocks - nblocks / 16) {
                pp = false;
                if (blockIdx.x < nh) __builtin_amdgcn_s_setprio(3);
            }
        }
        res = dispatch_class<kStamps>(img, smem, n, tt, out, cap, dbg_slot, lane, D, pp);
    }
    // results, through pointers reloaded now (see CompressArgs)
#ifndef LZ4E_EMU
    const __attribute__((address_space(4))) CompressArgs* ka =
        (const __attribute__((address_space(4))) CompressArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    int32_t* const retp = ka->ret;
    uint32_t* const auxp = ka->aux;
    const uint32_t* const ordp = ka->order;
#else
    int32_t* const retp = ret;
    uint32_t* const auxp = aux;
    const uint32_t* const ordp = order;
#endif
    const uint32_t b2 = ordp ? ordp[blockIdx.x] : blockIdx.x;
    if (lane == 0) {
        retp[b2] = res.ret;
        if (auxp) {
            auxp[2 * (size_t)b2] = res.a0;
            auxp[2 * (size_t)b2 + 1] = res.a1;
        }
    }
}

// ---- launch order (lz4e_order.h) -------------------------------------------
// The parse time of a block is the number of 64-position windows its walk
// visits (plus a cost per sequence): high for data full of short matches
// (text, tables, records), low for incompressible data (the search skips
// ahead) and for long runs (matches of hundreds of bytes).  A sample of 16
// chunks of 256 bytes per block estimates it: the byte entropy H, the
// fraction R of positions inside a run (5 equal bytes) and the fraction S of
// positions whose 4 bytes occurred earlier in their chunk; the weight is
// (1 - R) (0.2 + S), or 0 when H > 7.5 bits (no matches to find).  On the
// silesia proxy its rank correlation with the measured parse cycles is
// 0.85 (tools/comp_order.py measures the orders).
constexpr uint32_t kWeightChunks = 16, kWeightChunk = 256, kWeightThreads = 256;
constexpr uint32_t kOrderMinBlocks = 1024;   // fewer: about one block per CU, nothing to spread
constexpr uint32_t kOrderMinLen = 16384;     // small blocks finish in a few windows

__global__ __launch_bounds__(kWeightThreads) void weight_kernel(const uint8_t* __restrict__ src,
                                                                const uint64_t* __restrict__ src_off,
                                                                const uint32_t* __restrict__ src_len,
                                                                uint32_t nblocks,
                                                                uint32_t* __restrict__ weight) {
    // thread t: the 16 sample positions r0 .. r0 + 15 of chunk c; the
    // chunks' first-occurrence tables (position per 8-bit hash) side by side
    constexpr uint32_t kPer = kWeightChunks * kWeightChunk / kWeightThreads;  // 16
    constexpr uint32_t kTab = 256;
    __shared__ __attribute__((aligned(16))) uint8_t smp[kWeightChunks * kWeightChunk + 16];
    __shared__ uint32_t hist[256], cnt[2], tbl[kWeightChunks * kTab];
    __shared__ float esum;
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    if (b >= nblocks) return;
    const uint32_t n = src_len[b];
    if (n < kWeightChunk * 2) {
        if (t == 0) weight[b] = 0;
        return;
    }
    const uint8_t* in = src + src_off[b];
    const uint32_t c = t / (kWeightChunk / kPer), r0 = (t % (kWeightChunk / kPer)) * kPer;
    const uint32_t base = (uint32_t)((uint64_t)(n - kWeightChunk) * c / (kWeightChunks - 1));
    hist[t] = 0;
    if (t < 2) cnt[t] = 0;
    if (t == 0) esum = 0.f;
    for (uint32_t i = t; i < kWeightChunks * kTab; i += kWeightThreads) tbl[i] = ~0u;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) smp[c * kWeightChunk + r0 + k] = in[base + r0 + k];
    if (t < 16) smp[kWeightChunks * kWeightChunk + t] = 0;
    __syncthreads();
    const uint8_t* ch = smp + c * kWeightChunk;
    const uint32_t* chw = (const uint32_t*)ch;  // 4-byte aligned (chunks of 256)
    uint32_t* tb = tbl + c * kTab;
    // my 16 positions' bytes (+ the 4 after) in registers: word k = bytes
    // r0 + k .. r0 + k + 3
    uint32_t d[kPer / 4 + 1];
#pragma unroll
    for (uint32_t i = 0; i <= kPer / 4; ++i) d[i] = chw[r0 / 4 + i];
    const uint32_t prev = r0 ? ch[r0 - 1] : 0x100u;  // byte before my first position
    auto word_at = [&](uint32_t r) -> uint32_t {  // any chunk offset (2 aligned reads)
        return alignbyte(chw[r / 4 + 1], chw[r / 4], r & 3);
    };
    // No atomics on the sample's own values (runs and tables would put every
    // lane of an instruction on one LDS address): every position writes its
    // table slot and reads back the winner -- a word seen m times counts
    // m - 1 positions, as "occurred earlier" would; the byte histogram takes
    // every 4th byte.
    uint32_t w[kPer];
    uint32_t runs = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
        const uint32_t r = r0 + k;
        w[k] = alignbyte(d[k / 4 + 1], d[k / 4], k & 3);
        if (k % 4 == 0) atomicAdd(&hist[w[k] & 0xFFu], 1u);
        const uint32_t pb = k == 0 ? prev : (d[(k - 1) / 4] >> (8 * ((k - 1) & 3))) & 0xFFu;
        if (r + 4 <= kWeightChunk) {
            tb[(w[k] * 2654435761u) >> 24] = r;
            runs += w[k] == pb * 0x01010101u;  // 5 equal bytes
        }
    }
    __syncthreads();
    uint32_t seen = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
        const uint32_t r = r0 + k;
        if (r + 4 <= kWeightChunk) {
            const uint32_t f = tb[(w[k] * 2654435761u) >> 24];
            seen += f != r && word_at(f) == w[k];
        }
    }
    {
        const uint32_t rs = wave_incl_add(runs), ss = wave_incl_add(seen);
        if ((t & 63) == 63) {
            atomicAdd(&cnt[0], rs);
            atomicAdd(&cnt[1], ss);
        }
    }
    const float p = (float)hist[t] / (float)(kWeightChunks * kWeightChunk / 4);
    if (p > 0.f) atomicAdd(&esum, -p * log2f(p));
    __syncthreads();
    if (t == 0) {
        const float npos = (float)(kWeightChunks * (kWeightChunk - 3));
        const float R = (float)cnt[0] / npos, S = (float)cnt[1] / npos;
        weight[b] = esum > 7.5f ? 0u : (uint32_t)(1000.f * (1.f - R) * (0.2f + S));
    }
}

struct CompressWeight {
    const uint32_t* weight;  // 0 .. 1200
    LZ4E_DEV uint32_t operator()(uint32_t b) const {
        const uint32_t q = weight[b] * (kOrderBuckets - 1) / 1200;
        return (kOrderBuckets - 1) - (q < kOrderBuckets - 1 ? q : kOrderBuckets - 1);
    }
};
// Heavy blocks: weight >= 1200 * 7 / 63 ~ 133 (text ~290, tables and records
// 400-470; long runs ~20, incompressible 0), i.e. bucket <= 56.
constexpr uint32_t kHeavyBucket = kOrderBuckets - 1 - 7;

uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* e = getenv(name);
    return e ? (uint32_t)strtoul(e, nullptr, 10) : dflt;
}

template <bool kStamps>
hipError_t launch_compress_impl(const CompressBatch& a, hipStream_t stream, uint64_t* dbg) {
    if (a.nblocks == 0) return hipSuccess;
    // LZ4E_COMPRESS_LDS_MAX (bytes) overrides the LDS staging limit (experiments).
    static const uint32_t lds_max = env_u32("LZ4E_COMPRESS_LDS_MAX", kMaxLdsInput);
    const bool lds_input = a.max_len <= lds_max && a.dict_len == nullptr;
    const dim3 grid(a.nblocks), block(kWave);
    const uint32_t lds = compress_lds_bytes(a.max_len, lds_input);
    if (lds_input) {
        hipLaunchKernelGGL((compress_kernel<true, kStamps>), grid, block, lds, stream, a.src,
                           a.src_off, a.src_len, a.table_type, a.dst, a.dst_off, a.dst_cap, a.ret,
                           a.aux, a.nblocks, a.max_len, dbg, a.dict_len, nullptr);
        return hipGetLastError();
    }
    // heavy blocks first (see weight_kernel)
    const int om = launch_order_mode(true);
    const bool use_order = om == kOrderAlways ||
                           (om == kOrderAuto && a.nblocks >= kOrderMinBlocks && a.max_len >= kOrderMinLen);
    uint32_t* scratch = nullptr;
    if (use_order &&
        hipMallocAsync((void**)&scratch, sizeof(uint32_t) * (2 * (size_t)a.nblocks + 1), stream) == hipSuccess) {
        hipLaunchKernelGGL(weight_kernel, dim3(a.nblocks), dim3(kWeightThreads), 0, stream, a.src,
                           a.src_off, a.src_len, a.nblocks, scratch);
        hipLaunchKernelGGL((order_kernel<CompressWeight>), dim3(1), dim3(kOrderThreads), 0, stream,
                           CompressWeight{scratch}, a.nblocks, scratch + a.nblocks, kHeavyBucket,
                           scratch + 2 * (size_t)a.nblocks);
    } else {
        (void)hipGetLastError();  // a failed pool allocation only costs the ordering
        scratch = nullptr;
    }
    hipLaunchKernelGGL((compress_kernel<false, kStamps>), grid, block, lds, stream, a.src,
                       a.src_off, a.src_len, a.table_type, a.dst, a.dst_off, a.dst_cap, a.ret,
                       a.aux, a.nblocks, a.max_len, dbg, a.dict_len,
                       scratch ? (const uint32_t*)(scratch + a.nblocks) : nullptr);
    const hipError_t err = hipGetLastError();
    if (scratch) (void)hipFreeAsync(scratch, stream);
    return err;
}

}  // namespace

uint32_t compress_lds_bytes(uint32_t max_len, bool lds_input) {
    uint32_t bytes = kTableBytes;
    if (lds_input) bytes += (max_len + 15) & ~15u;
    return bytes;
}

hipError_t launch_compress(const CompressBatch& a, hipStream_t stream) {
    return launch_compress_impl<false>(a, stream, nullptr);
}

hipError_t launch_compress_stamped(const CompressBatch& a, hipStream_t stream, uint64_t* dbg) {
    return launch_compress_impl<true>(a, stream, dbg);
}

}  // namespace lz4e
