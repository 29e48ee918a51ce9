// lz4e_compress.hip -- gfx950 LZ4E block compressor.
//
// Bit-exact restatement of the reference greedy parse
// (/root/reference/lz4e/lz4e_compress.c:218-534, LZ4E_compress_generic with
// noDict, acceleration 1) on one wave64 per block:
//
//  * The block's hash table (8192 x u16 for byU16, 4096 x u32 for byU32,
//    2048 x u32 for byU64) lives in LDS, and so does the input block when it
//    fits (the byte image is then read with word loads + v_alignbyte).
//  * Match search is speculative over 64 probes at once: the probe
//    positions of a search are a closed-form function of its start (skip
//    step +1 every 64 probes), the hashes are pure functions of the data,
//    and the candidate each probe would see is "the latest earlier probe of
//    the same window with an equal hash, else the table entry from before
//    the window".  Every probe first writes its position into the table and
//    reads it back: a lane that does not see its own position shares its
//    hash with another lane (fast path: none do); those sets are then found
//    exactly with one ballot per hash bit.  The first verifying lane
//    (ballot + ctz) is the reference's match; the table is then fixed up to
//    hold exactly the puts of the probes up to it, last writer wins.
//  * Backward catch-up and LZ4E_count are 64-lane compares resolved by
//    ballot; literal runs and length-extension runs are written by the whole
//    wave.
//  * All control flow is wave-uniform (scalar branches); the parse state
//    (ip, anchor, op, candidate, token position) lives in SGPRs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4e_device.h"
#include "lz4e_gpu.h"

namespace lz4e {

namespace {

constexpr uint32_t kTableBytes = 16384;   // 1 << LZ4E_MEMORY_USAGE

struct Table {
    uint16_t* t16;
    uint32_t* t32;
    bool narrow;  // byU16 class: u16 positions (block <= 64 KiB)
    LZ4E_DEV uint32_t get(uint32_t h) const { return narrow ? (uint32_t)t16[h] : t32[h]; }
    LZ4E_DEV void put(uint32_t h, uint32_t v) const {
        if (narrow) t16[h] = (uint16_t)v; else t32[h] = v;
    }
};

template <class IMG>
LZ4E_DEV uint32_t hash_at(const IMG& img, uint32_t p, int tt, uint32_t hlog) {
    if (tt == kByU32) return hash5(img.rd64(p), hlog);
    return hash4(img.rd32(p), hlog);
}

// Wave-wide byte fill / copy into the output block.
LZ4E_DEV void out_fill(uint8_t* out, uint32_t at, uint32_t len, uint8_t v, uint32_t lane) {
    for (uint32_t k = lane; k < len; k += kWave) out[at + k] = v;
}

template <class IMG>
LZ4E_DEV void out_copy(uint8_t* out, uint32_t at, const IMG& img, uint32_t from, uint32_t len,
                       uint32_t lane) {
    for (uint32_t k = lane; k < len; k += kWave) out[at + k] = (uint8_t)img.rd8(from + k);
}

// Length-extension bytes of a literal run or a match (lz4e_compress.c:365-377
// and :432-447): (len-15)/255 bytes of 0xFF then (len-15)%255.  Returns the
// number of bytes written.
LZ4E_DEV uint32_t out_ext(uint8_t* out, uint32_t at, uint32_t rest, uint32_t lane) {
    const uint32_t nff = rest / 255;
    out_fill(out, at, nff, 0xFF, lane);
    if (lane == 0) out[at + nff] = (uint8_t)(rest - nff * 255);
    return nff + 1;
}

// LZ4E_count (lz4e_defs.h:587-636): equal bytes at ip.. and m.., at most lim.
template <class IMG>
LZ4E_DEV uint32_t wave_count(const IMG& img, uint32_t ip, uint32_t m, uint32_t lim, uint32_t lane) {
    uint32_t mc = 0;
    for (;;) {
        const uint32_t rem = lim - mc;
        const uint32_t o = mc + 4 * lane;
        uint32_t x = 1;  // lanes past the limit mismatch at their first byte
        if (4 * lane < rem) {
            x = img.rd32(ip + o) ^ img.rd32(m + o);
            const uint32_t nb = rem - 4 * lane;
            if (nb < 4) x |= ~0u << (8 * nb);
        }
        const uint64_t mm = ballot(x != 0);
        if (mm == 0) { mc += 4 * kWave; continue; }
        const uint32_t f = ctz64(mm);
        return mc + 4 * f + (uint32_t)__builtin_ctz(lane_val(x, f)) / 8;
    }
}

template <class IMG>
LZ4E_DEV void compress_block(const IMG& img, const Table& T, uint32_t n, int tt,
                             uint8_t* out, uint32_t cap, int32_t* ret_slot, uint32_t* aux_slot,
                             uint32_t lane) {
    const uint32_t hlog = hash_log(tt);
    const uint64_t bound = (uint64_t)n + n / 255 + 16;
    const bool limited = cap < bound;  // lz4e_compress.c:553-560
    uint32_t op = 0, anchor = 0, ip = 0;

    if (n >= kMinLength) {
        const uint32_t mflimit = n - kMfLimit;
        const uint32_t matchlimit = n - kLastLiterals;
        // put(0) of the first byte stores position 0 == an empty slot.
        ip = 1;
        for (;;) {
            uint32_t cand;
            // ---------------- match search (lz4e_compress.c:292-336) --------
            {
                const uint32_t s = ip;
                uint32_t pbase = 0;
                for (;;) {
                    const uint32_t P = pbase + lane;
                    const uint64_t q64 = (uint64_t)s + probe_offset(P);
                    const bool valid = q64 + probe_step(P) <= mflimit;
                    const uint64_t vmask = ballot(valid);
                    if (vmask == 0) {
                        // first probe of this window fails the end test
                        if (pbase != 0) ip = s + (uint32_t)probe_offset(pbase - 1);
                        goto last_literals;
                    }
                    const uint32_t q = valid ? (uint32_t)q64 : 0;
                    uint32_t h = 0, vq = 0, c0 = 0;
                    if (valid) {
                        if (tt == kByU32) {
                            const uint64_t v = img.rd64(q);
                            vq = (uint32_t)v;
                            h = hash5(v, hlog);
                        } else {
                            vq = img.rd32(q);
                            h = hash4(vq, hlog);
                        }
                        c0 = T.get(h);  // table entry from before this window
                        T.put(h, q);    // speculative put of every probe
                    }
                    // Read-back: a lane that does not see its own position
                    // shares its hash with another lane of the window.
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
                        const bool dist_ok = (tt == kByU16) || (c + kMaxDistance >= q);
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
                        break;
                    }
                    if (vmask != ~0ull) {
                        ip = lane_val(q, klast);  // last probe that ran
                        goto last_literals;
                    }
                    pbase += kWave;
                }
            }

            // ---------------- catch up (lz4e_compress.c:339-349) -------------
            {
                uint32_t room = ip - anchor < cand ? ip - anchor : cand;
                while (room) {
                    const bool eq = lane < room && img.rd8(ip - 1 - lane) == img.rd8(cand - 1 - lane);
                    const uint64_t em = ballot(eq);
                    const uint32_t f = (~em) ? ctz64(~em) : kWave;
                    ip -= f;
                    cand -= f;
                    room -= f;
                    if (f < kWave) break;
                }
            }

            uint32_t tok;
            uint32_t token;
            // ---------------- literals (lz4e_compress.c:352-382) -------------
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
                out_copy(out, op, img, anchor, L, lane);
                op += L;
            }

            for (;;) {
                // ------------ offset + match length (:384-449) ---------------
                const uint32_t off = ip - cand;
                if (lane == 0) {
                    out[op] = (uint8_t)off;
                    out[op + 1] = (uint8_t)(off >> 8);
                }
                op += 2;
                ip += 4;
                cand += 4;
                const uint32_t mc = wave_count(img, ip, cand, matchlimit - ip, lane);
                ip += mc;
                if (limited && (uint64_t)op + 6 + (mc >> 8) > cap) goto fail;
                if (mc >= 15) {
                    token += 15;
                    op += out_ext(out, op, mc - 15, lane);
                } else {
                    token += mc;
                }
                if (lane == 0) out[tok] = (uint8_t)token;

                anchor = ip;
                if (ip > mflimit) goto last_literals;  // :456-457

                // ------------ fill table, test next position (:461-493) ------
                T.put(hash_at(img, ip - 2, tt, hlog), ip - 2);
                const uint32_t h = hash_at(img, ip, tt, hlog);
                cand = uni(T.get(h));
                T.put(h, ip);
                if (cand + kMaxDistance >= ip && img.rd32(cand) == img.rd32(ip)) {
                    tok = op++;
                    token = 0;
                    continue;
                }
                break;
            }
            ip += 1;  // :496-497
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

template <bool kLdsInput>
__global__ __launch_bounds__(64) void compress_kernel(const uint8_t* __restrict__ src,
                                                      const uint64_t* __restrict__ src_off,
                                                      const uint32_t* __restrict__ src_len,
                                                      const uint8_t* __restrict__ table_type,
                                                      uint8_t* __restrict__ dst,
                                                      const uint64_t* __restrict__ dst_off,
                                                      const uint32_t* __restrict__ dst_cap,
                                                      int32_t* __restrict__ ret,
                                                      uint32_t* __restrict__ aux, uint32_t nblocks) {
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

    const bool tt_ok = (tt == kByU16 && n <= 65536) || tt == kByU32 || tt == kByU64;
    if (n > kMaxInput || (n >= kMinLength && !tt_ok)) {
        // Input too large (lz4e_compress.c:245-248) returns 0; a malformed
        // descriptor (class/length the SG rules cannot produce) returns -1.
        if (lane == 0) ret[b] = n > kMaxInput ? 0 : -1;
        return;
    }

    Table T;
    T.narrow = (tt == kByU16);
    T.t16 = reinterpret_cast<uint16_t*>(smem);
    T.t32 = smem;

    if (n >= kMinLength) {
        // memset of the state (lz4e_compress.c:548): 16 KiB of table.
        uint4* t4 = reinterpret_cast<uint4*>(smem);
        for (uint32_t i = lane; i < kTableBytes / 16; i += kWave) t4[i] = make_uint4(0, 0, 0, 0);
    }

    if constexpr (kLdsInput) {
        uint32_t* inw = smem + kTableBytes / 4;
        stage_block(inw, in, n, lane);
        __syncthreads();
        ByteImage<ClampedWords> img{ClampedWords{inw, n == 0 ? 0 : (n - 1) >> 2}, 0};
        compress_block(img, T, n, tt, out, cap, ret + b, aux_slot, lane);
    } else {
        __syncthreads();
        const uintptr_t a = reinterpret_cast<uintptr_t>(in);
        const uint32_t shift = (uint32_t)(a & 3);
        const uint32_t* w = reinterpret_cast<const uint32_t*>(a - shift);
        const uint32_t last = n + shift == 0 ? 0 : (n + shift - 1) >> 2;
        ByteImage<ClampedWords> img{ClampedWords{w, last}, shift};
        compress_block(img, T, n, tt, out, cap, ret + b, aux_slot, lane);
    }
}

}  // namespace

uint32_t compress_lds_bytes(uint32_t max_len, bool lds_input) {
    uint32_t bytes = kTableBytes;
    if (lds_input) bytes += (max_len + 15) & ~15u;
    return bytes;
}

hipError_t launch_compress(const CompressBatch& a, hipStream_t stream) {
    if (a.nblocks == 0) return hipSuccess;
    const bool lds_input = a.max_len <= kMaxLdsInput;
    const uint32_t lds = compress_lds_bytes(a.max_len, lds_input);
    const dim3 grid(a.nblocks), block(kWave);
    if (lds_input) {
        hipLaunchKernelGGL(compress_kernel<true>, grid, block, lds, stream, a.src, a.src_off,
                           a.src_len, a.table_type, a.dst, a.dst_off, a.dst_cap, a.ret, a.aux,
                           a.nblocks);
    } else {
        hipLaunchKernelGGL(compress_kernel<false>, grid, block, lds, stream, a.src, a.src_off,
                           a.src_len, a.table_type, a.dst, a.dst_off, a.dst_cap, a.ret, a.aux,
                           a.nblocks);
    }
    return hipGetLastError();
}

}  // namespace lz4e
