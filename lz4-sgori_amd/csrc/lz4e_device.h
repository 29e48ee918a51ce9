// lz4e_device.h -- device-side helpers shared by the gfx950 LZ4E kernels.
//
// Wave64 primitives, unaligned little-endian reads over a word-addressed
// byte image (LDS or HBM), and the LZ4E hashes of
// /root/reference/lz4e/lz4e_compress.c:48-96.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define LZ4E_DEV __device__ __forceinline__

namespace lz4e {

constexpr uint32_t kWave = 64;
constexpr uint32_t kMinLength = 13;      // LZ4E_MIN_LENGTH (lz4e_defs.h:88)
constexpr uint32_t kMfLimit = 12;        // MFLIMIT
constexpr uint32_t kLastLiterals = 5;    // LASTLITERALS
constexpr uint32_t kMaxDistance = 65535; // LZ4E_DISTANCE_MAX
constexpr uint32_t kMaxInput = 0x7E000000u;
constexpr int kByU16 = 1, kByU32 = 3, kByU64 = 7;

LZ4E_DEV uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
LZ4E_DEV uint64_t ballot(bool p) { return __ballot(p); }
LZ4E_DEV uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
LZ4E_DEV uint32_t lane_val(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
LZ4E_DEV uint32_t ctz64(uint64_t m) { return (uint32_t)__builtin_ctzll(m); }
LZ4E_DEV uint32_t popc64(uint64_t m) { return (uint32_t)__builtin_popcountll(m); }

// Global-memory pointer types: pointers rebuilt from integer addresses lose
// their address space and would otherwise compile to flat_* accesses, which
// also count on lgkmcnt (coupling them to every LDS wait).
typedef __attribute__((address_space(1))) const uint32_t gcu32;
typedef __attribute__((address_space(1))) const uint8_t gcu8;

// Bytes [4*i, 4*i+4) of a word image (an LDS copy of a block, or the block
// in HBM), little endian.  The word index is clamped so that a masked-off
// lane never reads outside the image.
template <class P>
struct ClampedWordsT {
    P w;
    uint32_t last;  // last readable word index
    LZ4E_DEV uint32_t word(uint32_t i) const { return w[i < last ? i : last]; }
};
using ClampedWords = ClampedWordsT<const uint32_t*>;  // LDS image
using GlobalWords = ClampedWordsT<gcu32*>;            // HBM image

// The byte image is addressed with a constant byte shift so that an HBM
// block need not start on a word boundary (shift is 0 for LDS).
template <class W>
struct ByteImage {
    W words;
    uint32_t shift;
    LZ4E_DEV uint32_t rd8(uint32_t p) const {
        const uint32_t a = p + shift;
        return (words.word(a >> 2) >> ((a & 3) * 8)) & 0xFFu;
    }
    LZ4E_DEV uint32_t rd32(uint32_t p) const {
        const uint32_t a = p + shift;
        const uint32_t i = a >> 2;
        return __builtin_amdgcn_alignbyte(words.word(i + 1), words.word(i), a & 3);
    }
    // Low 40 bits are exact (hash5 ignores the rest); returns lo in *lo.
    LZ4E_DEV uint64_t rd64(uint32_t p) const {
        const uint32_t a = p + shift;
        const uint32_t i = a >> 2;
        const uint32_t w0 = words.word(i), w1 = words.word(i + 1), w2 = words.word(i + 2);
        const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, a & 3);
        const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, a & 3);
        return ((uint64_t)hi << 32) | lo;
    }
};

// hashLog per table class (lz4e_compress.c:48-57).
LZ4E_DEV uint32_t hash_log(int tt) { return tt == kByU64 ? 11u : (tt == kByU32 ? 12u : 13u); }

// LZ4E_hash4 (lz4e_compress.c:59-66).
LZ4E_DEV uint32_t hash4(uint32_t v, uint32_t hlog) { return (v * 2654435761u) >> (32 - hlog); }

// LZ4E_hash5, little-endian branch (lz4e_compress.c:68-83).
LZ4E_DEV uint32_t hash5(uint64_t v, uint32_t hlog) {
    return (uint32_t)(((v << 24) * 889523592379ull) >> (64 - hlog));
}

// Sum of the match-finder skip steps before probe P (A3 of SURVEY.md):
// step_0 = 1, step_j = (63 + j) >> 6 for j >= 1 (lz4e_compress.c:295-307).
LZ4E_DEV uint64_t probe_offset(uint32_t P) {
    if (P == 0) return 0;
    const uint64_t m = P - 1, a = m >> 6, r = m & 63;
    return 1 + 32 * a * (a + 1) + r * (a + 1);
}
LZ4E_DEV uint32_t probe_step(uint32_t P) { return P == 0 ? 1u : (P + 63) >> 6; }

}  // namespace lz4e
