// Lane emulator version of csrc/lz4e_wave.h (tools/emu only): every lane of
// the wave is a host thread; cross-lane operations meet at a barrier.  The
// kernels call these in wave-uniform control flow only, which is what makes
// the emulation exact (each lane executes the same sequence of them).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <barrier>
#include <climits>

#define LZ4E_DEV inline

namespace lz4e {

constexpr uint32_t kWave = 64;

struct EmuWave {
    std::barrier<> bar{64};
    uint64_t slot[64];
};
extern EmuWave* g_wave;
extern thread_local uint32_t g_lane;

inline uint64_t emu_gather(uint64_t v, uint32_t from) {
    g_wave->slot[g_lane] = v;
    g_wave->bar.arrive_and_wait();
    const uint64_t r = g_wave->slot[from & 63];
    g_wave->bar.arrive_and_wait();
    return r;
}

LZ4E_DEV uint32_t lane_id() { return g_lane; }
LZ4E_DEV uint64_t ballot(bool p) {
    g_wave->slot[g_lane] = p;
    g_wave->bar.arrive_and_wait();
    uint64_t m = 0;
    for (int i = 0; i < 64; ++i) m |= (g_wave->slot[i] ? 1ull : 0ull) << i;
    g_wave->bar.arrive_and_wait();
    return m;
}
LZ4E_DEV void wave_prio_for(uint32_t) {}
LZ4E_DEV uint64_t match_any6(uint32_t key) {
    uint64_t m = ~0ull;
    for (uint32_t b = 0; b < 6; ++b) {
        const bool bit = (key >> b) & 1;
        const uint64_t bb = ballot(bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}
LZ4E_DEV uint32_t uni(uint32_t v) { return (uint32_t)emu_gather(v, 0); }
LZ4E_DEV uint32_t lane_val(uint32_t v, uint32_t l) { return (uint32_t)emu_gather(v, l); }
LZ4E_DEV uint32_t set_lane(uint32_t v, uint32_t x, uint32_t l) {
    const uint32_t xx = (uint32_t)emu_gather(x, 0);  // x is wave-uniform
    return g_lane == (l & 63) ? xx : v;
}
LZ4E_DEV uint32_t put_lane(uint32_t v, uint32_t x, uint32_t l) {
    const uint32_t xx = (uint32_t)emu_gather(x, 0);  // x is wave-uniform
    return g_lane == (l & 63) ? xx : v;
}
LZ4E_DEV uint32_t push_lane(uint32_t v, uint32_t dst) {
    // every lane publishes (dst, v); lane l takes the value of a sender to it
    g_wave->slot[g_lane] = ((uint64_t)(dst & 63) << 32) | v;
    g_wave->bar.arrive_and_wait();
    uint32_t r = 0xDEADBEEFu;
    for (int i = 0; i < 64; ++i)
        if ((g_wave->slot[i] >> 32) == g_lane) r = (uint32_t)g_wave->slot[i];
    g_wave->bar.arrive_and_wait();
    return r;
}
LZ4E_DEV void consume(uint32_t) {}
LZ4E_DEV uint32_t shfl(uint32_t v, uint32_t src) { return (uint32_t)emu_gather(v, src); }
LZ4E_DEV uint32_t shfl_addr(uint32_t v, uint32_t addr) {
    return (uint32_t)emu_gather(v, (addr >> 2) & 63);
}
LZ4E_DEV uint32_t perm_bytes(uint32_t hi, uint32_t lo, uint32_t sel) {
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t s = (sel >> (8 * i)) & 0xFFu;
        const uint32_t b = s < 8 ? (uint32_t)(v >> (8 * s)) & 0xFFu : 0u;  // (0x0C: 0)
        r |= b << (8 * i);
    }
    return r;
}
LZ4E_DEV int32_t shfl_up(int32_t v, uint32_t d) {
    g_wave->slot[g_lane] = (uint32_t)v;
    g_wave->bar.arrive_and_wait();
    const int32_t r = g_lane >= d ? (int32_t)g_wave->slot[g_lane - d] : v;
    g_wave->bar.arrive_and_wait();
    return r;
}
LZ4E_DEV uint32_t wave_incl_add(uint32_t v) {
    g_wave->slot[g_lane] = v;
    g_wave->bar.arrive_and_wait();
    uint32_t r = 0;
    for (uint32_t i = 0; i <= g_lane; ++i) r += (uint32_t)g_wave->slot[i];
    g_wave->bar.arrive_and_wait();
    return r;
}
LZ4E_DEV int32_t wave_excl_min(int32_t v) {
    g_wave->slot[g_lane] = (uint32_t)v;
    g_wave->bar.arrive_and_wait();
    int32_t r = INT32_MAX;
    for (uint32_t i = 0; i < g_lane; ++i) r = std::min(r, (int32_t)(uint32_t)g_wave->slot[i]);
    g_wave->bar.arrive_and_wait();
    return r;
}
LZ4E_DEV int32_t wave_excl_max(int32_t v) {
    g_wave->slot[g_lane] = (uint32_t)v;
    g_wave->bar.arrive_and_wait();
    int32_t r = INT32_MIN;
    for (uint32_t i = 0; i < g_lane; ++i) r = std::max(r, (int32_t)(uint32_t)g_wave->slot[i]);
    g_wave->bar.arrive_and_wait();
    return r;
}
LZ4E_DEV uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t r) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (r & 3)));
}
LZ4E_DEV uint64_t clock64() { return 0; }
// The decoder orders a phase's LDS / global accesses after the previous
// phase's with wave_fence (lockstep on the GPU): a barrier here.
LZ4E_DEV void wave_fence() { g_wave->bar.arrive_and_wait(); }
LZ4E_DEV void lockstep() { g_wave->bar.arrive_and_wait(); }
LZ4E_DEV void block_sync() { g_wave->bar.arrive_and_wait(); }
LZ4E_DEV void stores_done() {}
LZ4E_DEV uint32_t vaddr(uint32_t q) { return q; }

typedef const uint32_t gcu32;
typedef const uint8_t gcu8;

struct ByteBuf {
    const uint8_t* p;
    uint32_t n;
};
inline ByteBuf buf_make(const void* p, uint32_t n) { return ByteBuf{(const uint8_t*)p, n}; }
inline uint32_t buf_ld32(const ByteBuf& b, uint32_t q) {
    if ((uint64_t)q + 4 > b.n) return 0;
    uint32_t v;
    __builtin_memcpy(&v, b.p + q, 4);
    return v;
}

}  // namespace lz4e
