// lz4e_compress.hip -- gfx950 LZ4E block compressor.
//
// Bit-exact restatement of the reference greedy parse
// (/root/reference/lz4e/lz4e_compress.c:218-534, LZ4E_compress_generic with
// noDict, acceleration 1), one wave64 per block, all control flow
// wave-uniform (the parse state lives in SGPRs):
//
//  * The hash table (8192 x u16 for byU16, 4096 x u32 for byU32, 2048 x u32
//    for byU64) lives in LDS.  The input block is read either from an LDS
//    copy (small blocks) or straight from HBM through L1/L2 (the 16 KiB of
//    LDS per block then allows 10 blocks per CU).
//  * Data moves in "stripes": one dword per lane, lane k holding the 4 bytes
//    at X - 4 + 4k for a base position X.  A step loads the stripe at the
//    current position and the stripe at its match candidate together; lane 0
//    serves the backward catch-up (lz4e_compress.c:339-349), lane 1 the
//    4-byte verify, lanes 2.. LZ4E_count (lz4e_defs.h:587-636) by XOR +
//    ballot, 248 bytes per round trip.  Literal runs are stored straight from
//    the stripe lanes; the post-match hashes (lz4e_compress.c:461-470) are
//    read out of the stripe with v_readlane.
//  * The dominant path on compressible data is "match, then the next
//    position matches again" (lz4e_compress.c:486-493): one LDS round trip
//    for the table, one data round trip for the candidate stripe.
//  * Match search (lz4e_compress.c:292-336) is speculative over a window of
//    probes, one per lane: probe positions are a closed-form function of the
//    search start (skip step +1 every 64 probes), hashes are pure functions
//    of the data, and the candidate a probe sees is "the latest earlier probe
//    of the window with an equal hash, else the table entry from before the
//    window".  Every probe writes its position and reads it back: a lane that
//    does not see its own position shares its hash with another lane (those
//    sets are then resolved exactly, one ballot per hash bit).  The first
//    verifying lane is the reference's match; the table is then fixed up to
//    hold exactly the puts of the probes up to it.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "lz4e_device.h"
#include "lz4e_gpu.h"

namespace lz4e {

namespace {

constexpr uint32_t kTableBytes = 16384;  // 1 << LZ4E_MEMORY_USAGE
constexpr uint32_t kStripe = 256;        // bytes covered by one stripe (lane k: X-4+4k)

// byU16 class: u16 positions (block <= 64 KiB); byU32/byU64: u32 positions.
// The table lives in LDS (kG = false) or in a per-block HBM scratch slot
// (kG = true), which frees LDS for more resident blocks per CU.
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) uint16_t gu16;

template <int TT, bool kG>
struct Table {
    uint32_t* lds;
    gu32* glob;
    LZ4E_DEV uint32_t get(uint32_t h) const {
        if constexpr (kG) {
            if constexpr (TT == kByU16) return ((gu16*)glob)[h];
            else return glob[h];
        } else {
            if constexpr (TT == kByU16) return reinterpret_cast<uint16_t*>(lds)[h];
            else return lds[h];
        }
    }
    LZ4E_DEV void put(uint32_t h, uint32_t v) const {
        if constexpr (kG) {
            if constexpr (TT == kByU16) ((gu16*)glob)[h] = (uint16_t)v;
            else glob[h] = v;
        } else {
            if constexpr (TT == kByU16) reinterpret_cast<uint16_t*>(lds)[h] = (uint16_t)v;
            else lds[h] = v;
        }
    }
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

// ---- stripe helpers ---------------------------------------------------------

// 4 bytes at byte index u of a stripe (u + 4 <= 256), wave-uniform result.
LZ4E_DEV uint32_t stripe_u32(uint32_t sv, uint32_t u) {
    const uint32_t k = u >> 2, r = u & 3;
    const uint32_t lo = lane_val(sv, k);
    if (r == 0) return lo;
    const uint32_t hi = lane_val(sv, k + 1);
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * r));
}

// 8 bytes at byte index u (u + 8 <= 256); only the low 40 bits matter to hash5.
LZ4E_DEV uint64_t stripe_u64(uint32_t sv, uint32_t u) {
    const uint32_t lo = stripe_u32(sv, u), hi = stripe_u32(sv, u + 4);
    return ((uint64_t)hi << 32) | lo;
}

template <class IMG>
LZ4E_DEV uint32_t stripe_load(const IMG& img, uint32_t X, uint32_t lane) {
    // Lane 0 of a stripe based below position 4 reaches before the block:
    // those byte slots read as zero (the catch-up never looks at them).
    const int32_t p = (int32_t)(X + 4 * lane) - 4;
    const uint32_t v = img.rd32(p < 0 ? 0u : (uint32_t)p);
    return p < 0 ? (p <= -4 ? 0u : v << (8 * (uint32_t)(-p))) : v;
}

// First byte index u >= u0 where the two stripes differ, or where the
// comparison limit u0 + lim is reached; kStripe if neither happens.
LZ4E_DEV uint32_t stripe_mismatch(uint32_t x, uint32_t u0, uint32_t lim, uint32_t lane) {
    const uint32_t b = 4 * lane;
    const uint64_t e64 = (uint64_t)u0 + lim;
    const uint32_t e = e64 > kStripe ? kStripe + 4 : (uint32_t)e64;
    if (b + 4 <= u0) x = 0;
    else if (b < u0) x &= ~0u << (8 * (u0 - b));
    if (b >= e) x |= 1u;
    else if (b + 4 > e) x |= 1u << (8 * (e - b));
    const uint64_t mm = ballot(x != 0);
    if (mm == 0) return kStripe;
    const uint32_t f = ctz64(mm);
    return 4 * f + (uint32_t)__builtin_ctz(lane_val(x, f)) / 8;
}

// hash of the position whose bytes are v (hash5 for byU32, hash4 otherwise;
// hashLog 13 / 12 / 11 for byU16 / byU32 / byU64, lz4e_compress.c:48-96)
template <int TT>
LZ4E_DEV uint32_t hash_val(uint64_t v) {
    if constexpr (TT == kByU32) return hash5(v, 12);
    else return hash4((uint32_t)v, TT == kByU16 ? 13 : 11);
}

// ---- output -------------------------------------------------------------

LZ4E_DEV uint32_t out_ext(uint8_t* out, uint32_t at, uint32_t rest, uint32_t lane) {
    // (rest)/255 bytes of 0xFF then rest % 255 (lz4e_compress.c:365-377, :432-447)
    const uint32_t nff = rest / 255;
    for (uint32_t k = lane; k < nff; k += kWave) out[at + k] = 0xFF;
    if (lane == 0) out[at + nff] = (uint8_t)(rest - nff * 255);
    return nff + 1;
}

// Literal copy from the image: 4 bytes per lane, 4 words in flight per lane.
template <class IMG>
LZ4E_DEV void out_copy(uint8_t* out, uint32_t at, const IMG& img, uint32_t from, uint32_t len,
                       uint32_t lane) {
    constexpr uint32_t kChunk = 4 * 4 * kWave;
    for (uint32_t base = 0; base < len; base += kChunk) {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = img.rd32(from + base + 4 * (j * kWave + lane));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t k = base + 4 * (j * kWave + lane);
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (k + b < len) out[at + k + b] = (uint8_t)(w[j] >> (8 * b));
        }
    }
}

// Literal bytes [from, from+len) taken from the stripe based at X (they must
// lie inside it): every lane stores its own bytes, 4 masked byte stores.
LZ4E_DEV void out_copy_stripe(uint8_t* out, uint32_t at, uint32_t sv, uint32_t X, uint32_t from,
                              uint32_t len, uint32_t lane) {
    const int32_t rel = (int32_t)(X - 4 + 4 * lane) - (int32_t)from;  // offset of this lane's byte 0
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int32_t t = rel + b;
        if (t >= 0 && t < (int32_t)len) out[at + t] = (uint8_t)(sv >> (8 * b));
    }
}

template <int TT, bool kStamps, bool kG, class IMG>
LZ4E_DEV void compress_block(const IMG& img, uint32_t* smem, gu32* gtab, uint32_t n, uint8_t* out,
                             uint32_t cap, int32_t* ret_slot, uint32_t* aux_slot, uint64_t* dbg,
                             uint32_t lane) {
    constexpr uint32_t hlog = TT == kByU64 ? 11 : (TT == kByU32 ? 12 : 13);
    const Table<TT, kG> T{smem, gtab};
    const uint64_t bound = (uint64_t)n + n / 255 + 16;
    const bool limited = cap < bound;  // lz4e_compress.c:553-560
    uint32_t op = 0, anchor = 0, ip = 0;
    Stamps st;
    if (kStamps) st.start();

    if (n >= kMinLength) {
        const uint32_t mflimit = n - kMfLimit;
        const uint32_t matchlimit = n - kLastLiterals;
        // Front stripe: based at the anchor of the coming search.  put(0) of
        // the first byte stores position 0 == an empty slot, so nothing to do.
        uint32_t A = 0;
        uint32_t sa = stripe_load(img, A, lane);
        uint32_t s = 1;  // search start
        for (;;) {
            uint32_t cand;
            // ================= match search (lz4e_compress.c:292-336) ======
            {
                uint32_t pbase = 0;
                for (;;) {
                    const uint32_t P = pbase + lane;
                    const uint64_t q64 = (uint64_t)s + probe_offset(P);
                    const bool valid = q64 + probe_step(P) <= mflimit;
                    const uint64_t vmask = ballot(valid);
                    if (vmask == 0) {
                        if (pbase != 0) ip = s + (uint32_t)probe_offset(pbase - 1);
                        else ip = s;
                        if (kStamps) st.lap(kPhSearch);
                        goto last_literals;
                    }
                    const uint32_t q = valid ? (uint32_t)q64 : s;
                    uint64_t v;
                    if (pbase == 0 && s + 64 + 8 <= A - 4 + kStripe) {
                        // probe bytes from the front stripe (ds_bpermute, no memory)
                        const uint32_t t = q - (A - 4);
                        const uint32_t j = t >> 2, r = t & 3;
                        const uint32_t w0 = __shfl(sa, j), w1 = __shfl(sa, j + 1),
                                       w2 = __shfl(sa, j + 2);
                        v = ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, r) << 32) |
                            __builtin_amdgcn_alignbyte(w1, w0, r);
                    } else {
                        v = img.rd64(q);
                    }
                    const uint32_t vq = (uint32_t)v;
                    const uint32_t h = valid ? hash_val<TT>(v) : 0;
                    uint32_t c0 = 0;
                    if (valid) {
                        c0 = T.get(h);  // table entry from before this window
                        T.put(h, q);    // speculative put of every probe
                    }
                    const uint64_t cm = ballot(valid && T.get(h) != q);
                    uint64_t same = 1ull << lane;
                    uint32_t c = c0;
                    if (cm) {
                        // Exact equal-hash lane sets, one ballot per hash bit.
                        same = vmask;
                        for (uint32_t bit = 0; bit < hlog; ++bit) {
                            const bool hb = (h >> bit) & 1;
                            const uint64_t m = ballot(valid && hb);
                            same &= hb ? m : ~m;
                        }
                        const uint64_t below = same & ((1ull << lane) - 1);
                        const uint32_t pl = below ? 63 - (uint32_t)__builtin_clzll(below) : lane;
                        const uint32_t qp = __shfl(q, pl);
                        if (below) c = qp;  // latest earlier probe, same hash
                    }
                    bool hit = false;
                    if (valid) {
                        const bool dist_ok = (TT == kByU16) || (c + kMaxDistance >= q);
                        hit = dist_ok && img.rd32(c) == vq;
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
            uint32_t X = ip, Y = cand;  // stripe bases
            uint32_t si = stripe_load(img, X, lane);
            uint32_t sb = stripe_load(img, Y, lane);
            {
                uint32_t room = ip - anchor < cand ? ip - anchor : cand;
                if (room) {
                    // lane 0 holds the 4 bytes before ip / before cand
                    const uint32_t x = lane_val(si, 0) ^ lane_val(sb, 0);
                    uint32_t c = x ? (uint32_t)__builtin_clz(x) / 8 : 4;
                    if (c > room) c = room;
                    ip -= c;
                    cand -= c;
                    room -= c;
                    if (c == 4 && room) {
                        // long catch-up (rare): byte steps from memory
                        while (room && img.rd8(ip - 1) == img.rd8(cand - 1)) {
                            ip--;
                            cand--;
                            room--;
                        }
                        X = ip;
                        Y = cand;
                        si = stripe_load(img, X, lane);
                        sb = stripe_load(img, Y, lane);
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
                if (anchor >= A - 4 && ip <= A - 4 + kStripe)
                    out_copy_stripe(out, op, sa, A, anchor, L, lane);
                else
                    out_copy(out, op, img, anchor, L, lane);
                op += L;
            }
            if (kStamps) st.lap(kPhLit);

            // ================= match chain ===================================
            for (;;) {
                // offset (lz4e_compress.c:386-387)
                const uint32_t off = ip - cand;
                if (lane == 0) {
                    out[op] = (uint8_t)off;
                    out[op + 1] = (uint8_t)(off >> 8);
                }
                op += 2;
                // LZ4E_count from ip+4 / cand+4 (lz4e_compress.c:420-423)
                uint32_t mc = 0;
                {
                    const uint32_t lim = matchlimit - (ip + 4);
                    uint32_t u0 = ip + 4 - (X - 4);  // same offset in both stripes
                    for (;;) {
                        const uint32_t u = stripe_mismatch(si ^ sb, u0, lim - mc, lane);
                        if (u < kStripe) {
                            mc += u - u0;
                            break;
                        }
                        mc += kStripe - u0;
                        X = ip + 4 + mc;
                        Y = cand + 4 + mc;
                        si = stripe_load(img, X, lane);
                        sb = stripe_load(img, Y, lane);
                        u0 = 4;
                    }
                }
                ip += 4 + mc;
                if (limited && (uint64_t)op + 6 + (mc >> 8) > cap) goto fail;
                if (mc >= 15) {
                    token += 15;
                    op += out_ext(out, op, mc - 15, lane);
                } else {
                    token += mc;
                }
                if (lane == 0) out[tok] = (uint8_t)token;
                anchor = ip;
                if (kStamps) { st.cnt[1]++; st.lap(kPhCount); }
                if (ip > mflimit) goto last_literals;  // :456-457

                // ---- fill table at ip-2, test ip (lz4e_compress.c:461-493) ----
                uint64_t v1, v2;
                if (ip + 8 <= X - 4 + kStripe) {
                    v1 = stripe_u64(si, ip - 2 - (X - 4));
                    v2 = stripe_u64(si, ip - (X - 4));
                } else {
                    v1 = img.rd64(ip - 2);
                    v2 = img.rd64(ip);
                }
                const uint32_t sn = stripe_load(img, ip, lane);  // overlaps the table access
                const uint32_t h1 = hash_val<TT>(v1);
                const uint32_t h2 = hash_val<TT>(v2);
                T.put(h1, ip - 2);
                const uint32_t c2 = uni(T.get(h2));
                T.put(h2, ip);
                X = ip;
                si = sn;
                if (c2 + kMaxDistance >= ip) {
                    Y = c2;
                    sb = stripe_load(img, Y, lane);
                    if (lane_val(sb, 1) == lane_val(si, 1)) {
                        cand = c2;
                        tok = op++;
                        token = 0;
                        if (kStamps) { st.cnt[2]++; st.lap(kPhRematch); }
                        continue;
                    }
                }
                if (kStamps) st.lap(kPhRematch);
                break;
            }
            // no match at ip: the next search starts at ip + 1 (:496-497) and
            // the stripe at ip becomes the front stripe
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
        out_copy(out, op, img, anchor, R, lane);
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
// image are clamped to its last word (ClampedWords), so no pad is needed and
// a 64 KiB block + its 16 KiB table fill exactly half of a CU's LDS.
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

template <bool kStamps, bool kG, class IMG>
LZ4E_DEV void dispatch_class(const IMG& img, uint32_t* smem, gu32* gtab, uint32_t n, int tt,
                             uint8_t* out, uint32_t cap, int32_t* ret_slot, uint32_t* aux_slot,
                             uint64_t* dbg, uint32_t lane) {
    if (tt == kByU32)
        compress_block<kByU32, kStamps, kG>(img, smem, gtab, n, out, cap, ret_slot, aux_slot, dbg,
                                            lane);
    else if (tt == kByU16)
        compress_block<kByU16, kStamps, kG>(img, smem, gtab, n, out, cap, ret_slot, aux_slot, dbg,
                                            lane);
    else
        compress_block<kByU64, kStamps, kG>(img, smem, gtab, n, out, cap, ret_slot, aux_slot, dbg,
                                            lane);
}

template <bool kLdsInput, bool kStamps, bool kG>
__global__ __launch_bounds__(64) void compress_kernel(const uint8_t* __restrict__ src,
                                                      const uint64_t* __restrict__ src_off,
                                                      const uint32_t* __restrict__ src_len,
                                                      const uint8_t* __restrict__ table_type,
                                                      uint8_t* __restrict__ dst,
                                                      const uint64_t* __restrict__ dst_off,
                                                      const uint32_t* __restrict__ dst_cap,
                                                      int32_t* __restrict__ ret,
                                                      uint32_t* __restrict__ aux, uint32_t nblocks,
                                                      uint64_t* __restrict__ dbg,
                                                      uint32_t* __restrict__ gtab_all) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const uint32_t b = blockIdx.x;
    if (b >= nblocks) return;
    const uint32_t lane = lane_id();
    const uint32_t n = src_len[b];
    const int tt = table_type[b];
    const uint32_t cap = dst_cap[b];
    uint8_t* out = dst + dst_off[b];
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

    gu32* gtab = kG ? (gu32*)(gtab_all + (size_t)b * (kTableBytes / 4)) : nullptr;
    if (n >= kMinLength) {
        // memset of the state (lz4e_compress.c:548): 16 KiB of table.
        if constexpr (kG) {
            typedef uint32_t v4u __attribute__((ext_vector_type(4)));
            __attribute__((address_space(1))) v4u* t4 = (__attribute__((address_space(1))) v4u*)gtab;
            for (uint32_t i = lane; i < kTableBytes / 16; i += kWave) t4[i] = v4u{0, 0, 0, 0};
        } else {
            uint4* t4 = reinterpret_cast<uint4*>(smem);
            for (uint32_t i = lane; i < kTableBytes / 16; i += kWave) t4[i] = make_uint4(0, 0, 0, 0);
        }
    }

    if constexpr (kLdsInput) {
        uint32_t* inw = smem + kTableBytes / 4;
        stage_block(inw, in, n, lane);
        __syncthreads();
        ByteImage<ClampedWords> img{ClampedWords{inw, n == 0 ? 0 : (n - 1) >> 2}, 0};
        dispatch_class<kStamps, kG>(img, smem, gtab, n, tt, out, cap, ret + b, aux_slot, dbg_slot,
                                    lane);
    } else {
        __syncthreads();
        const uintptr_t a = reinterpret_cast<uintptr_t>(in);
        const uint32_t shift = (uint32_t)(a & 3);
        gcu32* w = (gcu32*)(a - shift);
        const uint32_t last = n + shift == 0 ? 0 : (n + shift - 1) >> 2;
        ByteImage<GlobalWords> img{GlobalWords{w, last}, shift};
        dispatch_class<kStamps, kG>(img, smem, gtab, n, tt, out, cap, ret + b, aux_slot, dbg_slot,
                                    lane);
    }
}

uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* e = getenv(name);
    return e ? (uint32_t)strtoul(e, nullptr, 10) : dflt;
}

// Per-block HBM table scratch for the global-table variant (grown on demand;
// experiments via LZ4E_COMPRESS_GTABLE=1).
uint32_t* gtable_scratch(uint32_t nblocks) {
    static uint32_t* p = nullptr;
    static size_t cap = 0;
    const size_t need = (size_t)nblocks * kTableBytes;
    if (need > cap) {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, need) != hipSuccess) return nullptr;
        cap = need;
    }
    return p;
}

template <bool kStamps>
hipError_t launch_compress_impl(const CompressBatch& a, hipStream_t stream, uint64_t* dbg) {
    if (a.nblocks == 0) return hipSuccess;
    // LZ4E_COMPRESS_LDS_MAX (bytes) overrides the LDS staging limit (experiments).
    static const uint32_t lds_max = env_u32("LZ4E_COMPRESS_LDS_MAX", kMaxLdsInput);
    static const uint32_t gtable = env_u32("LZ4E_COMPRESS_GTABLE", 0);
    const bool lds_input = a.max_len <= lds_max;
    const dim3 grid(a.nblocks), block(kWave);
    if (gtable && !lds_input) {
        uint32_t* gt = gtable_scratch(a.nblocks);
        if (!gt) return hipErrorOutOfMemory;
        hipLaunchKernelGGL((compress_kernel<false, kStamps, true>), grid, block, 0, stream, a.src,
                           a.src_off, a.src_len, a.table_type, a.dst, a.dst_off, a.dst_cap, a.ret,
                           a.aux, a.nblocks, dbg, gt);
        return hipGetLastError();
    }
    const uint32_t lds = compress_lds_bytes(a.max_len, lds_input);
    if (lds_input) {
        hipLaunchKernelGGL((compress_kernel<true, kStamps, false>), grid, block, lds, stream, a.src,
                           a.src_off, a.src_len, a.table_type, a.dst, a.dst_off, a.dst_cap, a.ret,
                           a.aux, a.nblocks, dbg, nullptr);
    } else {
        hipLaunchKernelGGL((compress_kernel<false, kStamps, false>), grid, block, lds, stream, a.src,
                           a.src_off, a.src_len, a.table_type, a.dst, a.dst_off, a.dst_cap, a.ret,
                           a.aux, a.nblocks, dbg, nullptr);
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
