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
//     v_readlane.  Sequence k of the batch is recorded in lane k (literal
//     source, literal length, output position, offset, match length).
//     Errors depend only on the token stream, so a failing block stops here.
//  2. Literals: every lane copies its own run (16-byte unaligned loads and
//     stores, exact tails); runs longer than kLong are copied by the whole
//     wave, 1 KiB per step.
//  3. Matches, in dependency rounds: a match is ready once the part of its
//     source before its own output overlaps no earlier match of the batch
//     that is still pending (checked exactly against each pending interval).
//     Ready short matches are copied per lane, every load before any store;
//     long ones by the whole wave in lane order.  Overlapping matches follow LZ semantics
//     out[op + t] = out[op - off + t mod off]; offset 0 writes zeros, which
//     is what the reference's LZ4_write32(op, offset) + overlap copy produce
//     (lz4e_decompress.c:313, 407-415).
//
// Same-wave stores and loads to the same global address are ordered by the
// hardware (one vector L1 per CU); wavefront-scope fences keep the compiler
// from moving a phase's loads above the previous phase's stores.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4e_device.h"
#include "lz4e_gpu.h"

namespace lz4e {

namespace {

constexpr int32_t kLong = 64;  // longer literal runs / matches go to the whole wave

// Two 256-byte windows of the compressed block: A = [base, base+256),
// B = [base+256, base+512).  Word loads are clamped to the block.
struct InWindow {
    gcu32* w;        // word-aligned base of the block
    int32_t shift;   // byte offset of the block inside w[0]
    int32_t last;    // last word index that belongs to the block
    uint32_t lane;
    int32_t base;    // block position of window A byte 0
    uint32_t a, b;   // this lane's dword of A and B

    LZ4E_DEV uint32_t load(int32_t wi) const {
        wi = wi < 0 ? 0 : wi;
        return w[wi < last ? wi : last];
    }
    LZ4E_DEV void reload(int32_t p) {
        const int32_t wi = (p + shift) >> 2;
        base = wi * 4 - shift;
        a = load(wi + (int32_t)lane);
        b = load(wi + 64 + (int32_t)lane);
    }
    LZ4E_DEV void slide() {
        a = b;
        base += 256;
        b = load(((base + shift) >> 2) + 64 + (int32_t)lane);
    }
    // Byte p of the block (reloads when p is outside [base, base + 512)).
    LZ4E_DEV uint32_t byte(int32_t p) {
        uint32_t r = (uint32_t)(p - base);
        if (r >= 512) {
            reload(p);
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
    // Keep the parse position inside window A (prefetching B).
    LZ4E_DEV void follow(int32_t p) {
        const uint32_t r = (uint32_t)(p - base);
        if (r >= 256 && r < 512) slide();
        else if (r >= 512) reload(p);
    }
};

// a > b for an unsigned a < 2^32 and a signed b (the reference compares
// pointers; b = end - k may lie before the buffer).
LZ4E_DEV bool ugt(uint32_t a, int32_t b) { return b < 0 || a > (uint32_t)b; }

constexpr uint32_t kSat = 0x7FFFFFFFu;  // length saturation: keeps every bound check's outcome


LZ4E_DEV uint4 ld16(const uint8_t* p) { return *reinterpret_cast<const uint4*>(p); }
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
        // self-overlap with a period >= 16: the first off bytes, then the
        // rest from off bytes back (written just before, same lane)
        lane_copy64(dst, dst - off, (int32_t)off, lim);
        lane_copy64(dst + off, dst, len - (int32_t)off, lim);
        return;
    }
    if (off == 0) {
        for (int32_t t = 0; t < len; ++t) dst[t] = 0;
        return;
    }
    // 1 <= off < 16: repeat the final period [dst-off, dst) 4 bytes at a time
    // (the 16-byte load may cover bytes at/after dst: never used)
    const uint4 p = dst - off + 16 <= lim ? ld16(dst - off) : make_uint4(0, 0, 0, 0);
    if (dst - off + 16 > lim) {
        for (int32_t t = 0; t < len; ++t) dst[t] = dst[t - (int32_t)off];
        return;
    }
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


// Per lane, for each of its 4 window bytes t: the distance to the next token
// if a token starts there and needs no length-extension bytes
// ((t >> 4) + 3: token, literals, 2 offset bytes), else 0.  Packed 4 x 8 bits.
LZ4E_DEV uint32_t pack_deltas(uint32_t w) {
    uint32_t d = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t t = (w >> (8 * j)) & 0xFFu;
        const uint32_t L = t >> 4;
        const bool simple = L != 15 && (t & 15) != 15;
        d |= (simple ? L + 3 : 0u) << (8 * j);
    }
    return d;
}

// Byte at per-lane window offset x (< 512) via ds_bpermute.
LZ4E_DEV uint32_t win_byte_lane(uint32_t a, uint32_t b, uint32_t x) {
    const uint32_t wi = x >> 2;
    const uint32_t va = shfl(a, (int)(wi & 63)), vb = shfl(b, (int)(wi & 63));
    return ((wi < 64 ? va : vb) >> ((x & 3) * 8)) & 0xFFu;
}

LZ4E_DEV int32_t excl_scan_add(int32_t v, uint32_t lane) {
    int32_t x = v;
#pragma unroll
    for (uint32_t d = 1; d < kWave; d <<= 1) {
        const int32_t y = shfl_up(x, d);
        if (lane >= d) x += y;
    }
    return x - v;
}

LZ4E_DEV int32_t excl_scan_min(int32_t v, uint32_t lane) {
    int32_t x = shfl_up(v, 1);
    if (lane == 0) x = INT32_MAX;
#pragma unroll
    for (uint32_t d = 1; d < kWave; d <<= 1) {
        const int32_t y = shfl_up(x, d);
        if (lane >= d) x = y < x ? y : x;
    }
    return x;
}

LZ4E_DEV int32_t excl_scan_max(int32_t v, uint32_t lane) {
    int32_t x = shfl_up(v, 1);
    if (lane == 0) x = INT32_MIN;
#pragma unroll
    for (uint32_t d = 1; d < kWave; d <<= 1) {
        const int32_t y = shfl_up(x, d);
        if (lane >= d) x = y > x ? y : x;
    }
    return x;
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
    uint64_t st_t = 0, st_acc[3] = {0, 0, 0}, st_batches = 0, st_rounds = 0;
    auto lap = [&](int ph) {
        if constexpr (kStamps) {
            const uint64_t now = clock64();
            st_acc[ph] += now - st_t;
            st_t = now;
        }
    };
    if constexpr (kStamps) st_t = clock64();
    const uint32_t b = blockIdx.x;
    if (b >= nblocks) return;
    const uint32_t lane = lane_id();
    const int32_t srcSize = src_len[b];
    const int32_t outSize = dst_cap[b];
    const uint8_t* in = src + src_off[b];
    uint8_t* out = dst + dst_off[b];

    // Special cases (lz4e_decompress.c:113-120).
    if (outSize == 0) {
        if (lane == 0) ret[b] = (srcSize == 1 && in[0] == 0) ? 0 : -1;
        return;
    }
    if (srcSize == 0) {
        if (lane == 0) ret[b] = -1;
        return;
    }
    if (srcSize < 0) {  // token read, then every path fails at ip == 1
        if (lane == 0) ret[b] = -2;
        return;
    }

    InWindow win;
    {
        const uintptr_t a = reinterpret_cast<uintptr_t>(in);
        win.shift = (int32_t)(a & 3);
        win.w = (gcu32*)(a - win.shift);
        win.last = (srcSize + win.shift - 1) >> 2;
        win.lane = lane;
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

        // 1a. Fast path: a run of tokens with no length-extension bytes, far
        // from both block ends, where the reference takes its two-stage
        // shortcut (:150-191).  The token chain is walked with one readlane
        // per token; every other field and check is evaluated per lane.
        if (ip <= iend - 18 && op <= oend - 32) {
            win.follow(ip);
            const uint32_t r0 = (uint32_t)(ip - win.base);  // < 256
            const uint32_t da = pack_deltas(win.a), db = pack_deltas(win.b);
            const int32_t rin = iend - 18 - win.base;       // last token offset on the fast path
            const uint32_t rlim = rin < 494 ? (uint32_t)rin : 494u;  // offset bytes stay inside
            uint32_t r = r0, k = 0;
            int32_t rk = 0;
            while (k < kWave && r <= rlim) {
                const uint32_t w = r < 256 ? lane_val(da, r >> 2) : lane_val(db, (r >> 2) - 64);
                const uint32_t d = (w >> ((r & 3) * 8)) & 0xFFu;
                if (d == 0) break;
                rk = lane == k ? (int32_t)r : rk;
                r += d;
                k++;
            }
            if (k > 0) {
                const bool cand = lane < k;
                const uint32_t x = cand ? (uint32_t)rk : r0;
                const uint32_t t = win_byte_lane(win.a, win.b, x);
                const int32_t L = (int32_t)(t >> 4), Mt = (int32_t)(t & 15);
                const uint32_t xo = x + 1 + (uint32_t)L;
                const int32_t off = (int32_t)(win_byte_lane(win.a, win.b, xo) |
                                              (win_byte_lane(win.a, win.b, xo + 1) << 8));
                const int32_t size = cand ? L + Mt + 4 : 0;
                const int32_t o_k = op + excl_scan_add(size, lane);
                const int32_t m_k = o_k + L;
                // the reference's checks on this path: shortcut entry (op <= oend-32,
                // input side guaranteed by rlim), match inside the block (:299-302),
                // and for offsets < 8 the _copy_match end check (:422-431)
                const bool ok = cand && o_k <= oend - 32 && m_k >= off &&
                                (off >= 8 || m_k + Mt + 4 <= oend - 5);
                const uint64_t okm = ballot(ok);
                const uint32_t nf = (~okm) ? ctz64(~okm) : kWave;  // first failing lane
                if (nf > 0) {
                    r_ls = win.base + (int32_t)x + 1;
                    r_L = L;
                    r_op = o_k;
                    r_off = off;
                    r_M = Mt + 4;
                    nseq = nf;
                    const int32_t last_end = lane_val(o_k + size, nf - 1);
                    ip = nf < k ? win.base + lane_val(rk, nf) : win.base + (int32_t)r;
                    op = last_end;
                }
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
        if constexpr (kStamps) st_batches++;
        // ------------------------------------------------ 2. literals
        const bool valid = lane < nseq;
        wave_fence();
        if (valid && r_L > 0 && r_L <= kLong) lane_copy64(out + r_op, in + r_ls, r_L, in + srcSize);
        {
            uint64_t longs = ballot(valid && r_L > kLong);
            while (longs) {
                const uint32_t j = ctz64(longs);
                longs &= longs - 1;
                wave_copy(out + lane_val(r_op, j), in + lane_val(r_ls, j),
                          (uint32_t)lane_val(r_L, j), lane);
            }
        }
        wave_fence();
        lap(1);

        // ------------------------------------------------ 3. matches
        const int32_t ms = r_op + r_L;  // match start
        const int32_t me = ms + r_M;    // match end
        const int32_t ss = ms - r_off;  // source start
        const int32_t need = me - r_off < ms ? me - r_off : ms;  // source part before own output
        const uint8_t* olim = out + outSize;
        const int32_t batch_lo = lane_val(r_op, 0);
        uint64_t pending = ballot(valid && r_M > 0);
        while (pending) {
            // Ready when [ss, need) is final: before this batch's output, or
            // before every pending earlier match, or after all of them.
            const bool mine = (pending >> lane) & 1;
            const bool quick = need <= batch_lo;
            bool ready = mine && quick;
            if (ballot(mine && !quick)) {
                const int32_t mn = excl_scan_min(mine ? ms : INT32_MAX, lane);
                const int32_t mx = excl_scan_max(mine ? me : INT32_MIN, lane);
                ready = mine && (quick || need <= mn || ss >= mx);
            }
            if (ready && r_M <= kLong) lane_match(out + ms, (uint32_t)r_off, r_M, olim);
            wave_fence();
            uint64_t longs = ballot(ready && r_M > kLong);
            while (longs) {
                const uint32_t j = ctz64(longs);
                longs &= longs - 1;
                wave_match(out, lane_val(ms, j), lane_val(r_off, j), (uint32_t)lane_val(r_M, j),
                           lane);
                wave_fence();
            }
            pending &= ~ballot(ready);
            if constexpr (kStamps) st_rounds++;
        }
        wave_fence();
        lap(2);
    }
    if (lane == 0) ret[b] = op;
    if constexpr (kStamps) {
        if (lane == 0 && dbg) {
            uint64_t* d = dbg + 8 * (size_t)b;
            d[0] = st_acc[0];
            d[1] = st_acc[1];
            d[2] = st_acc[2];
            d[3] = st_batches;
            d[4] = st_rounds;
        }
    }
    return;
fail:
    if (lane == 0) ret[b] = -ip - 1;
}

}  // namespace

hipError_t launch_decompress(const DecompressBatch& a, hipStream_t stream) {
    if (a.nblocks == 0) return hipSuccess;
    hipLaunchKernelGGL(decompress_kernel<false>, dim3(a.nblocks), dim3(kWave), 0, stream, a.src,
                       a.src_off, a.src_len, a.dst, a.dst_off, a.dst_cap, a.ret, a.nblocks, nullptr);
    return hipGetLastError();
}

hipError_t launch_decompress_stamped(const DecompressBatch& a, hipStream_t stream, uint64_t* dbg) {
    if (a.nblocks == 0) return hipSuccess;
    hipLaunchKernelGGL(decompress_kernel<true>, dim3(a.nblocks), dim3(kWave), 0, stream, a.src,
                       a.src_off, a.src_len, a.dst, a.dst_off, a.dst_cap, a.ret, a.nblocks, dbg);
    return hipGetLastError();
}

}  // namespace lz4e
