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
#include <stdint.h>
#include <stdlib.h>

#include "lz4e_device.h"
#include "lz4e_gpu.h"

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

// Moves a (possibly wave-uniform) byte offset into a VGPR.  A uniform load
// from read-only memory would otherwise become s_load_*, which ignores the
// low two address bits -- wrong for the unaligned reads below.
LZ4E_DEV uint32_t vaddr(uint32_t q) {
    asm("" : "+v"(q));
    return q;
}

// A block in HBM, read with unaligned vector loads (gfx950 global loads need
// no alignment).  n >= kMinLength whenever the parse runs.
struct HbmImage {
    gcu8* p;
    uint32_t n;
    LZ4E_DEV uint32_t rd8(uint32_t q) const { return p[q]; }
    LZ4E_DEV uint32_t ld32(uint32_t q) const { return *(gcu32*)(p + vaddr(q)); }
    LZ4E_DEV uint64_t ld64(uint32_t q) const { return *(gcu64*)(p + vaddr(q)); }
    // Lanes past the block (or before it, X < 4) read a clamped, meaningless
    // dword; every consumer masks those bytes.
    LZ4E_DEV uint32_t stripe(uint32_t X, uint32_t lane) const {
        const uint32_t q = X - 4 + 4 * lane;
        return ld32(q < n - 4 ? q : n - 4);
    }
};

// A block staged in LDS as words (the last partial word zero-padded).
struct LdsImage {
    const uint32_t* w;
    uint32_t last;  // last word index
    LZ4E_DEV uint32_t word(uint32_t i) const { return w[i < last ? i : last]; }
    LZ4E_DEV uint32_t rd8(uint32_t q) const { return (word(q >> 2) >> ((q & 3) * 8)) & 0xFFu; }
    LZ4E_DEV uint32_t ld32(uint32_t q) const {
        const uint32_t i = q >> 2;
        return __builtin_amdgcn_alignbyte(word(i + 1), word(i), q & 3);
    }
    LZ4E_DEV uint64_t ld64(uint32_t q) const {
        const uint32_t i = q >> 2, r = q & 3;
        const uint32_t w0 = word(i), w1 = word(i + 1), w2 = word(i + 2);
        return ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, r) << 32) |
               __builtin_amdgcn_alignbyte(w1, w0, r);
    }
    LZ4E_DEV uint32_t stripe(uint32_t X, uint32_t lane) const { return ld32(X - 4 + 4 * lane); }
};

// Phase cycle counters of the diagnostic build (launch_compress_stamped).
struct Stamps {
    uint64_t t, acc[6];
    uint32_t cnt[4];
    LZ4E_DEV void start() {
        t = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < 6; ++i) acc[i] = 0;
        for (int i = 0; i < 4; ++i) cnt[i] = 0;
    }
    LZ4E_DEV void lap(int phase) {
        const uint64_t now = __builtin_amdgcn_s_memtime();
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
    for (uint32_t base = 0; base < len; base += kChunk) {
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

template <int TT, bool kStamps, class IMG>
LZ4E_DEV void compress_block(const IMG& img, uint32_t* smem, uint32_t n, gu8* out, uint32_t cap,
                             int32_t* ret_slot, uint32_t* aux_slot, uint64_t* dbg, uint32_t lane) {
    const Table<TT> T{smem};
    const uint64_t bound = (uint64_t)n + n / 255 + 16;
    const bool limited = cap < bound;  // lz4e_compress.c:553-560
    uint32_t op = 0, anchor = 0, ip = 0;
    [[maybe_unused]] uint32_t trn = 0;
    Stamps st;
    if (kStamps) st.start();

    if (n >= kMinLength) {
        const uint32_t mflimit = n - kMfLimit;
        const uint32_t matchlimit = n - kLastLiterals;
        const uint64_t lanes_below = (1ull << lane) - 1;
        // Front stripe: based at the anchor A of the coming search (A is
        // always the anchor).  put(0) of the first byte stores position 0 ==
        // an empty slot, so nothing to do.
        uint32_t A = 0;
        uint32_t sa = img.stripe(A, lane);
        uint32_t s = 1;  // search start
        for (;;) {
            uint32_t cand;
            // ================= match search (lz4e_compress.c:292-336) ======
            {
                uint32_t pbase = 0;
                for (;;) {
                    const uint32_t P = pbase + lane;
                    const uint32_t qq = s + (uint32_t)probe_offset(P);
                    const bool valid = (uint64_t)qq + probe_step(P) <= mflimit;
                    const uint64_t vmask = ballot(valid);
                    if (vmask == 0) {
                        ip = pbase != 0 ? s + (uint32_t)probe_offset(pbase - 1) : s;
                        if (kStamps) st.lap(kPhSearch);
                        goto last_literals;
                    }
                    const uint32_t q = valid ? qq : s;
                    uint64_t v;
                    if (s + (uint32_t)probe_offset(pbase + kWave - 1) + 8 <= A - 4 + kStripe) {
                        // probe bytes from the front stripe (ds_bpermute, no memory)
                        const uint32_t t = q - (A - 4);
                        const uint32_t j = t >> 2, r = t & 3;
                        const uint32_t w0 = __shfl(sa, j), w1 = __shfl(sa, j + 1);
                        // hash5 reads 5 bytes: byte t+4 is byte r of w1 (the
                        // bytes above it do not enter the hash)
                        uint32_t hi = 0;
                        if constexpr (TT == kByU32) hi = __builtin_amdgcn_alignbyte(w1, w1, r);
                        v = ((uint64_t)hi << 32) | __builtin_amdgcn_alignbyte(w1, w0, r);
                    } else if constexpr (TT == kByU32) {
                        v = img.ld64(q);
                    } else {
                        v = img.ld32(q);
                    }
                    const uint32_t vq = (uint32_t)v;
                    const uint32_t h = hash_val<TT>(v);
                    uint32_t c0 = 0, rb = q;
                    if (valid) {
                        c0 = T.get(h);  // table entry from before this window
                        T.put(h, q);    // speculative put of every probe
                        rb = T.reread(h);
                    }
                    const uint64_t cm = ballot(rb != q);
                    uint64_t same = 0;  // valid lanes sharing my hash (clash groups only)
                    uint32_t c = c0;
                    if (cm) {
                        uint64_t todo = cm;
                        do {
                            const uint32_t hg = lane_val(h, ctz64(todo));
                            const uint64_t m = ballot(valid && h == hg);
                            if (h == hg) same = m;
                            todo &= ~m;
                        } while (todo);
                        const uint64_t below = same & lanes_below;
                        const uint32_t qp = __shfl(q, below ? 63 - (uint32_t)__builtin_clzll(below) : lane);
                        if (below) c = qp;  // latest earlier probe, same hash
                    }
                    bool hit = false;
                    if (valid) {
                        const bool dist_ok = (TT == kByU16) || (c + kMaxDistance >= q);
                        hit = dist_ok && img.ld32(c) == vq;
                    }
                    const uint64_t hm = ballot(hit);
                    const uint32_t klast = hm ? ctz64(hm) : popc64(vmask) - 1;
                    // Make the table hold exactly the puts of probes 0..klast.
                    if (valid) {
                        if (cm == 0) {
                            if (lane > klast) T.put(h, c0);
                        } else {
                            const uint64_t upto = klast >= 63 ? ~0ull : ((2ull << klast) - 1);
                            if (lane <= klast) {
                                if ((same & upto & ~((2ull << lane) - 1)) == 0) T.put(h, q);
                            } else if ((same & upto) == 0) {
                                T.put(h, c0);
                            }
                        }
                    }
                    if (hm) {
                        ip = lane_val(q, klast);
                        cand = lane_val(c, klast);
                        LZ4E_TR(1, ip, ((uint64_t)pbase << 32) | cand);
                        if (kStamps) { st.cnt[0]++; st.lap(kPhSearch); }
                        break;
                    }
                    if (vmask != ~0ull) {
                        ip = lane_val(q, klast);  // last probe that ran
                        if (kStamps) st.lap(kPhSearch);
                        goto last_literals;
                    }
                    pbase += kWave;
                }
            }

            // ================= stripes at (ip, cand), catch-up ==============
            uint32_t X = ip;  // base of si; sb is based at cand + (X - ip)
            uint32_t si = img.stripe(ip, lane);
            uint32_t sb = img.stripe(cand, lane);
            {
                uint32_t room = ip - anchor < cand ? ip - anchor : cand;
                if (room) {
                    uint32_t c = 0;
                    if (cand >= 4) {
                        // lane 0 holds the 4 bytes before ip / before cand
                        const uint32_t x = lane_val(si, 0) ^ lane_val(sb, 0);
                        c = x ? (uint32_t)__builtin_clz(x) / 8 : 4;
                        if (c > room) c = room;
                    }
                    ip -= c;
                    cand -= c;
                    room -= c;
                    if (room && (c == 4 || cand + c < 4)) {
                        // long catch-up or a candidate near the block start
                        // (rare): byte steps, then fresh stripes
                        while (room && img.rd8(ip - 1) == img.rd8(cand - 1)) {
                            ip--;
                            cand--;
                            room--;
                        }
                        X = ip;
                        si = img.stripe(ip, lane);
                        sb = img.stripe(cand, lane);
                    }
                }
            }
            if (kStamps) st.lap(kPhStripe);

            uint32_t tok, token;
            // ================= literals (lz4e_compress.c:352-382) ===========
            {
                const uint32_t L = ip - anchor;
                tok = op++;
                if (limited && (uint64_t)op + L + 8 + L / 255 > cap) goto fail;
                if (L >= 15) {
                    token = 0xF0;
                    op += out_ext(out, op, L - 15, lane);
                } else {
                    token = L << 4;
                }
                if (L <= kStripe - 4) {
                    // bytes [A, A+252) sit in lanes 1.. of the front stripe
                    if (lane >= 1 && 4 * (lane - 1) < L) st32(out, op + 4 * (lane - 1), sa);
                } else {
                    out_copy(out, op, img, anchor, L, lane);
                }
                op += L;
            }
            if (kStamps) st.lap(kPhLit);

            // ================= match chain ===================================
            // Each pass counts the match at ip against cand from the stripes
            // si (base X) / sb, then tries the rematch.  A sequence's stores
            // are issued after the loads of the next step: on gfx9 vmcnt also
            // counts stores, so stores issued earlier would delay every
            // following load wait by their write acknowledgement.
            for (;;) {
                // LZ4E_count from ip (lz4e_compress.c:420-423, the first 4
                // bytes are known equal): matched bytes t, mc = t - 4.
                const uint32_t u_ip = ip + 4 - X;  // ip's byte index in the stripes
                const uint32_t lim = matchlimit - ip;
                uint32_t u;
                if (u_ip + lim >= kStripe) {
                    uint32_t x = si ^ sb;
                    if (lane == 0) x = u_ip >= 4 ? 0u : x & (~0u << (8 * u_ip));
                    const uint64_t mm = ballot(x != 0);
                    u = mm ? 4 * ctz64(mm) + (uint32_t)__builtin_ctz(lane_val(x, ctz64(mm))) / 8
                           : kStripe;
                } else {
                    u = stripe_mismatch(si ^ sb, u_ip, u_ip + lim, lane);
                }
                uint32_t t = u - u_ip;
                if (u == kStripe) {
                    // long match: fresh stripe pairs, 252 bytes per round trip
                    for (;;) {
                        X = ip + t;
                        si = img.stripe(ip + t, lane);
                        sb = img.stripe(cand + t, lane);
                        u = stripe_mismatch(si ^ sb, 4, 4 + lim - t, lane);
                        t += u - 4;
                        if (u < kStripe) break;
                    }
                }
                LZ4E_TR(2, ip, ((uint64_t)cand << 32) | t);
                if (t < 4) {
                    op = tok;  // rematch verify failed (lz4e_compress.c:486-493)
                    break;
                }
                // sequence record: token (at tok), [lit ext + literals],
                // offset (at op_off), match-length extension
                const uint32_t mc = t - 4;
                const uint32_t off = ip - cand;
                const uint32_t op_off = op;
                op += 2;
                if (limited && (uint64_t)op + 6 + (mc >> 8) > cap) goto fail;
                const uint32_t tokb = token | (mc < 15 ? mc : 15);
                const uint32_t e1 = mc - 15;  // extension bytes when mc >= 15
                if (mc >= 15) op += e1 / 255 + 1;
                const uint32_t tok_at = tok;
                auto emit = [&]() {
                    const uint32_t e1w = (mc >= 15 && e1 < 255) ? e1 : 0;
                    if (lane == 0) {
                        if (op_off == tok_at + 1) {
                            st32(out, tok_at, tokb | (off << 8) | (e1w << 24));
                        } else {
                            out[tok_at] = (uint8_t)tokb;
                            st32(out, op_off, off | (e1w << 16));
                        }
                    }
                    if (mc >= 15 && e1 >= 255) out_ext(out, op_off + 2, e1, lane);
                };
#ifndef LZ4E_EMIT_LATE
                emit();
#endif
                ip += t;
                anchor = ip;
                if (kStamps) { st.cnt[1]++; st.lap(kPhCount); }
                if (ip > mflimit) {  // :456-457
#ifdef LZ4E_EMIT_LATE
                    emit();
#endif
                    goto last_literals;
                }

                // ---- fill table at ip-2, test ip (lz4e_compress.c:461-493) ----
                const uint32_t sn = img.stripe(ip, lane);
                // hash inputs ip-2 .. ip+4 read out of the current stripe, or
                // (match ending at its top) out of the new one, which is then
                // waited for: two branches, so the common path never waits.
                uint32_t uu = ip - 2 - (X - 4), w0, w1, w2;
                if (uu <= 4 * 61 + 3) {
                    const uint32_t k = uu >> 2;
                    w0 = lane_val(si, k);
                    w1 = lane_val(si, k + 1);
                    w2 = lane_val(si, k + 2);
                } else {
                    asm volatile("" ::: "memory");
                    uu = 2;  // ip-2 is byte 2 of the new stripe
                    w0 = lane_val(sn, 0);
                    w1 = lane_val(sn, 1);
                    w2 = lane_val(sn, 2);
                }
                uint64_t v1, v2;
                {
                    const uint32_t r = uu & 3;
                    const uint64_t lo = ((uint64_t)w1 << 32) | w0, hi = ((uint64_t)w2 << 32) | w1;
                    v1 = lo >> (8 * r);
                    v2 = r < 2 ? lo >> (8 * (r + 2)) : hi >> (8 * (r - 2));
                }
                const uint32_t h1 = hash_val<TT>(v1);
                const uint32_t h2 = hash_val<TT>(v2);
                T.put(h1, ip - 2);
                const uint32_t c2 = uni(T.get(h2));
                T.put(h2, ip);
                LZ4E_TR(3, ip, ((uint64_t)h2 << 32) | c2);
                LZ4E_TR(4, ip - 2, h1);
                X = ip;
                si = sn;
                const bool near = c2 + kMaxDistance >= ip;
                if (near) sb = img.stripe(c2, lane);
#ifdef LZ4E_EMIT_LATE
                emit();
#endif
                if (!near) break;
                cand = c2;
                tok = op++;
                token = 0;
                if (kStamps) { st.cnt[2]++; st.lap(kPhRematch); }
            }
            // no match at ip: the next search starts at ip + 1 (:496-497) and
            // the stripe at ip becomes the front stripe
            if (kStamps) st.lap(kPhRematch);
            A = ip;
            sa = si;
            s = ip + 1;
        }
    }

last_literals: {
        // lz4e_compress.c:500-530
        const uint32_t R = n - anchor;
        if (limited && (uint64_t)op + R + 1 + (R + 240) / 255 > cap) goto fail;
        if (R >= 15) {
            if (lane == 0) out[op] = 0xF0;
            op += 1;
            op += out_ext(out, op, R - 15, lane);
        } else {
            if (lane == 0) out[op] = (uint8_t)(R << 4);
            op += 1;
        }
        out_copy_exact(out, op, img, anchor, R, lane);
        if (lane == 0) {
            *ret_slot = (int32_t)(op + R);
            if (aux_slot) {
                aux_slot[0] = ip;
                aux_slot[1] = R;
            }
        }
        if (kStamps) {
            st.lap(kPhTail);
            if (lane == 0 && dbg) {
                for (int i = 0; i < 6; ++i) dbg[i] = st.acc[i];
                dbg[6] = ((uint64_t)st.cnt[1] << 32) | st.cnt[0];
                dbg[7] = st.cnt[2];
            }
        }
        return;
    }
fail:
    if (lane == 0) {
        *ret_slot = 0;
        if (aux_slot) {
            aux_slot[0] = 0;
            aux_slot[1] = 0;
        }
    }
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
LZ4E_DEV void dispatch_class(const IMG& img, uint32_t* smem, uint32_t n, int tt, gu8* out,
                             uint32_t cap, int32_t* ret_slot, uint32_t* aux_slot, uint64_t* dbg,
                             uint32_t lane) {
    if (tt == kByU32)
        compress_block<kByU32, kStamps>(img, smem, n, out, cap, ret_slot, aux_slot, dbg, lane);
    else if (tt == kByU16)
        compress_block<kByU16, kStamps>(img, smem, n, out, cap, ret_slot, aux_slot, dbg, lane);
    else
        compress_block<kByU64, kStamps>(img, smem, n, out, cap, ret_slot, aux_slot, dbg, lane);
}

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
                                                      uint64_t* __restrict__ dbg) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t b = blockIdx.x;
    if (b >= nblocks) return;
    const uint32_t lane = lane_id();
    const uint32_t n = src_len[b];
    const int tt = table_type[b];
    const uint32_t cap = dst_cap[b];
    gu8* out = (gu8*)(dst + dst_off[b]);
    const uint8_t* in = src + src_off[b];
    uint32_t* aux_slot = aux ? aux + 2 * (size_t)b : nullptr;
    uint64_t* dbg_slot = dbg ? dbg + 8 * (size_t)b : nullptr;

    const bool tt_ok = (tt == kByU16 && n <= 65536) || tt == kByU32 || tt == kByU64;
    if (n > kMaxInput || (n >= kMinLength && !tt_ok)) {
        // Input too large (lz4e_compress.c:245-248) returns 0; a malformed
        // descriptor (class/length the SG rules cannot produce) returns -1.
        if (lane == 0) ret[b] = n > kMaxInput ? 0 : -1;
        return;
    }

    if (n >= kMinLength) {
        // memset of the state (lz4e_compress.c:548): 16 KiB of table.
        uint4* t4 = reinterpret_cast<uint4*>(smem);
        for (uint32_t i = lane; i < kTableBytes / 16; i += kWave) t4[i] = make_uint4(0, 0, 0, 0);
    }

    if constexpr (kLdsInput) {
        uint32_t* inw = smem + kTableBytes / 4;
        stage_block(inw, in, n, lane);
        __syncthreads();
        const LdsImage img{inw, n == 0 ? 0 : (n - 1) >> 2};
        dispatch_class<kStamps>(img, smem, n, tt, out, cap, ret + b, aux_slot, dbg_slot, lane);
    } else {
        __syncthreads();
        const HbmImage img{(gcu8*)in, n};
        dispatch_class<kStamps>(img, smem, n, tt, out, cap, ret + b, aux_slot, dbg_slot, lane);
    }
}

uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* e = getenv(name);
    return e ? (uint32_t)strtoul(e, nullptr, 10) : dflt;
}

template <bool kStamps>
hipError_t launch_compress_impl(const CompressBatch& a, hipStream_t stream, uint64_t* dbg) {
    if (a.nblocks == 0) return hipSuccess;
    // LZ4E_COMPRESS_LDS_MAX (bytes) overrides the LDS staging limit (experiments).
    static const uint32_t lds_max = env_u32("LZ4E_COMPRESS_LDS_MAX", kMaxLdsInput);
    const bool lds_input = a.max_len <= lds_max;
    const dim3 grid(a.nblocks), block(kWave);
    const uint32_t lds = compress_lds_bytes(a.max_len, lds_input);
    if (lds_input) {
        hipLaunchKernelGGL((compress_kernel<true, kStamps>), grid, block, lds, stream, a.src,
                           a.src_off, a.src_len, a.table_type, a.dst, a.dst_off, a.dst_cap, a.ret,
                           a.aux, a.nblocks, dbg);
    } else {
        hipLaunchKernelGGL((compress_kernel<false, kStamps>), grid, block, lds, stream, a.src,
                           a.src_off, a.src_len, a.table_type, a.dst, a.dst_off, a.dst_cap, a.ret,
                           a.aux, a.nblocks, dbg);
    }
    return hipGetLastError();
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
