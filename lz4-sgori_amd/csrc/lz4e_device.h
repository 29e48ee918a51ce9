// lz4e_device.h -- device-side helpers shared by the gfx950 LZ4E kernels:
// LZ4E constants and the hashes / match-finder schedule of
// /root/reference/lz4e/lz4e_compress.c:48-96, 292-336 (wave primitives are
// in lz4e_wave.h).
#pragma once

#include "lz4e_wave.h"

namespace lz4e {

constexpr uint32_t kMinLength = 13;      // LZ4E_MIN_LENGTH (lz4e_defs.h:88)
constexpr uint32_t kMfLimit = 12;        // MFLIMIT
constexpr uint32_t kLastLiterals = 5;    // LASTLITERALS
constexpr uint32_t kMaxDistance = 65535; // LZ4E_DISTANCE_MAX
constexpr uint32_t kMaxInput = 0x7E000000u;
constexpr int kByU16 = 1, kByU32 = 3, kByU64 = 7;

LZ4E_DEV uint32_t ctz64(uint64_t m) { return (uint32_t)__builtin_ctzll(m); }
LZ4E_DEV uint32_t popc64(uint64_t m) { return (uint32_t)__builtin_popcountll(m); }

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
