// Host stand-in for <hip/hip_runtime.h> used ONLY by the lane emulator
// (tools/emu): just enough of the kernel language for the LZ4E kernel
// sources to compile as host C++, each lane a thread.  It supplies the
// amdgcn builtins csrc/lz4e_wave.h is written against, with the hardware's
// semantics, so the shared wave header runs unchanged (compiled with
// -DLZ4E_EMU).  Never part of the product build.
//
// Threads: a workgroup of W waves runs as 64 W host threads; cross-lane
// builtins meet at the emulated wave's barrier (the kernels call them in
// wave-uniform control flow only, which is what makes the emulation exact:
// each lane executes the same sequence of them), __syncthreads at the
// workgroup's.
#pragma once
#include <math.h>
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>
#include <barrier>
#include <condition_variable>
#include <mutex>
#include <chrono>
#include <deque>
#include <functional>
#include <thread>

#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __launch_bounds__(...)
#ifndef __shared__
#define __shared__
#endif

struct uint4 {
    uint32_t x, y, z, w;
};
inline uint4 make_uint4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return {a, b, c, d}; }
struct dim3 {
    uint32_t x, y, z;
    dim3(uint32_t a = 1, uint32_t b = 1, uint32_t c = 1) : x(a), y(b), z(c) {}
};
typedef int hipError_t;
enum { hipSuccess = 0, hipErrorOutOfMemory = 2 };
typedef void* hipStream_t;
inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipMalloc(void**, size_t) { return hipErrorOutOfMemory; }
inline hipError_t hipFree(void*) { return hipSuccess; }
// Stream-ordered scratch (the lane decoder's hand-over list; the launch
// order kernels only run for batches far larger than the emulator's).
inline hipError_t hipMallocAsync(void** p, size_t n, hipStream_t) {
    *p = malloc(n);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
inline hipError_t hipFreeAsync(void* p, hipStream_t) {
    free(p);
    return hipSuccess;
}
inline hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t) {
    memset(p, v, n);
    return hipSuccess;
}

// ---- emulated wave / workgroup --------------------------------------------
// A barrier whose waiters block at once (mutex + condition variable):
// std::barrier's waiters spin before they sleep, and with every lane a host
// thread (256 per 4-wave workgroup) the spinning starved the lanes still to
// arrive -- the pipelined decoder's emulation then ran for minutes.
class EmuBarrier {
  public:
    explicit EmuBarrier(std::ptrdiff_t n) : n_(n) {}
    void arrive_and_wait() {
        std::unique_lock<std::mutex> lk(m_);
        const uint64_t gen = gen_;
        if (++count_ == n_) {
            count_ = 0;
            ++gen_;
            cv_.notify_all();
            return;
        }
        cv_.wait(lk, [&] { return gen_ != gen; });
    }

  private:
    std::mutex m_;
    std::condition_variable cv_;
    std::ptrdiff_t n_, count_ = 0;
    uint64_t gen_ = 0;
};
struct EmuWave {
    EmuBarrier bar{64};
    // barriers of the wave's lane groups of 2, 4, 8, 16 and 32 lanes
    // (group_fence): 32 + 16 + 8 + 4 + 2 of them, by width
    std::deque<EmuBarrier> groups;
    uint64_t slot[64];
    EmuWave() {
        for (uint32_t w = 2; w <= 32; w *= 2)
            for (uint32_t g = 0; g < 64 / w; ++g) groups.emplace_back(w);
    }
    EmuBarrier& group_bar(uint32_t width, uint32_t lane) {
        // groups of 2, 4, ..., 32 lanes only (a width of 1 or 64 has no
        // barrier here: lz4e_decompress.hip's static_assert keeps kGroup in range)
        if (width < 2 || width > 32 || (width & (width - 1)) != 0) abort();
        uint32_t base = 0;
        for (uint32_t w = 2; w < width; w *= 2) base += 64 / w;
        return groups[base + lane / width];
    }
};
extern thread_local EmuWave* g_emu_wave;
extern thread_local uint32_t g_emu_lane;
extern thread_local EmuBarrier* g_emu_group;
extern dim3 blockIdx, gridDim;
extern thread_local dim3 threadIdx;

inline void emu_wave_barrier() { g_emu_wave->bar.arrive_and_wait(); }
inline void emu_group_barrier(uint32_t width) { g_emu_wave->group_bar(width, g_emu_lane & 63).arrive_and_wait(); }
// Every lane publishes v; lane l reads the value of lane from(l).
inline uint64_t emu_gather(uint64_t v, uint32_t from) {
    g_emu_wave->slot[g_emu_lane] = v;
    emu_wave_barrier();
    const uint64_t r = g_emu_wave->slot[from & 63];
    emu_wave_barrier();
    return r;
}
inline void __syncthreads() { g_emu_group->arrive_and_wait(); }

// Runs grid blocks one after the other, each as `threads` host threads.
void emu_launch(uint32_t nblocks, uint32_t threads, std::function<void()> body);
#define hipLaunchKernelGGL(k, grid, block, lds, stream, ...) \
    emu_launch((grid).x, (block).x, [&]() { k(__VA_ARGS__); })

// ---- amdgcn builtins (csrc/lz4e_wave.h) ------------------------------------
inline uint32_t __builtin_amdgcn_mbcnt_lo(uint32_t mask, uint32_t base) {
    const uint32_t l = g_emu_lane;
    const uint32_t below = l >= 32 ? mask : (mask & ((1u << l) - 1u));
    return base + (uint32_t)__builtin_popcount(below);
}
inline uint32_t __builtin_amdgcn_mbcnt_hi(uint32_t mask, uint32_t base) {
    const uint32_t l = g_emu_lane;
    const uint32_t below = l < 32 ? 0u : (l == 63 ? (mask & 0x7FFFFFFFu) : (mask & ((1u << (l - 32)) - 1u)));
    return base + (uint32_t)__builtin_popcount(below);
}
inline uint64_t __ballot(int p) {
    g_emu_wave->slot[g_emu_lane] = p != 0;
    emu_wave_barrier();
    uint64_t m = 0;
    for (int i = 0; i < 64; ++i) m |= (g_emu_wave->slot[i] ? 1ull : 0ull) << i;
    emu_wave_barrier();
    return m;
}
inline uint32_t __builtin_amdgcn_readfirstlane(uint32_t v) { return (uint32_t)emu_gather(v, 0); }
inline uint32_t __builtin_amdgcn_readlane(uint32_t v, uint32_t l) { return (uint32_t)emu_gather(v, l); }
inline int __builtin_amdgcn_ds_bpermute(int addr, int v) {
    return (int)(uint32_t)emu_gather((uint32_t)v, ((uint32_t)addr >> 2) & 63);
}
// ds_permute: lane (addr >> 2) & 63 receives v; of several senders the
// highest lane's value lands; a lane nobody sends to reads a marker value
// (unspecified on the hardware).
inline int __builtin_amdgcn_ds_permute(int addr, int v) {
    g_emu_wave->slot[g_emu_lane] = ((uint64_t)(((uint32_t)addr >> 2) & 63) << 32) | (uint32_t)v;
    emu_wave_barrier();
    uint32_t r = 0xDEADBEEFu;
    for (int i = 0; i < 64; ++i)
        if ((g_emu_wave->slot[i] >> 32) == g_emu_lane) r = (uint32_t)g_emu_wave->slot[i];
    emu_wave_barrier();
    return (int)r;
}
inline uint32_t __builtin_amdgcn_perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t s = (sel >> (8 * i)) & 0xFFu;
        // selectors 0-7 pick a byte; 0x0C gives 0 (the only other value used)
        const uint32_t b = s < 8 ? (uint32_t)(v >> (8 * s)) & 0xFFu : 0u;
        r |= b << (8 * i);
    }
    return r;
}
inline uint32_t __builtin_amdgcn_alignbyte(uint32_t hi, uint32_t lo, uint32_t r) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (r & 3)));
}
// DPP mov (update_dpp) for the controls the kernels use: row_shr:1..15
// (0x111-0x11F: lane l of a row of 16 reads lane l - n of its row; no such
// lane -> the lane keeps `old`, bound_ctrl off), row_bcast:15 (0x142: rows
// 1-3 read lane 15 of the row before) and row_bcast:31 (0x143: rows 2-3 read
// lane 31); lanes of rows disabled in row_mask keep `old`.
inline int __builtin_amdgcn_update_dpp(int old, int src, int ctrl, int row_mask, int bank_mask,
                                       bool bound_ctrl) {
    (void)bank_mask;
    (void)bound_ctrl;
    g_emu_wave->slot[g_emu_lane] = (uint32_t)src;
    emu_wave_barrier();
    const uint32_t l = g_emu_lane, row = l >> 4;
    int r = old;
    if ((row_mask >> row) & 1) {
        int from = -1;
        if (ctrl >= 0x111 && ctrl <= 0x11F) {
            const uint32_t n = (uint32_t)ctrl - 0x110;
            if ((l & 15) >= n) from = (int)(l - n);
        } else if (ctrl == 0x142) {
            if (row >= 1) from = (int)(row * 16 - 1);
        } else if (ctrl == 0x143) {
            if (row >= 2) from = 31;
        } else {
            abort();  // a control the emulator does not model
        }
        if (from >= 0) r = (int)(uint32_t)g_emu_wave->slot[from];
    }
    emu_wave_barrier();
    return r;
}
inline int __shfl_up(int v, unsigned d) {
    g_emu_wave->slot[g_emu_lane] = (uint32_t)v;
    emu_wave_barrier();
    const int r = g_emu_lane >= d ? (int)(uint32_t)g_emu_wave->slot[g_emu_lane - d] : v;
    emu_wave_barrier();
    return r;
}
inline uint64_t __builtin_amdgcn_s_memtime() { return 0; }
#define __builtin_amdgcn_s_setprio(x) ((void)0)
// s_sleep (only in the decoders' wave-uniform wait loops): the wave's lanes
// meet, lane 0 sleeps 20 us, the others block in the barrier -- a waiting
// wave then holds no CPU, where 64 yielding threads per wave starved the
// wave they waited for (a 4-wave workgroup is 256 host threads).
inline void emu_sleep() {
    emu_wave_barrier();
    if ((g_emu_lane & 63) == 0) std::this_thread::sleep_for(std::chrono::microseconds(20));
    emu_wave_barrier();
}
#define __builtin_amdgcn_s_sleep(x) emu_sleep()

// ---- atomics --------------------------------------------------------------
#define __HIP_MEMORY_SCOPE_WORKGROUP 0
#define __hip_atomic_load(p, order, scope) __atomic_load_n(p, order)
#define __hip_atomic_store(p, v, order, scope) __atomic_store_n(p, v, order)
#define __hip_atomic_fetch_add(p, v, order, scope) __atomic_fetch_add(p, v, order)
#define __hip_atomic_fetch_and(p, v, order, scope) __atomic_fetch_and(p, v, order)
#define __hip_atomic_fetch_or(p, v, order, scope) __atomic_fetch_or(p, v, order)
// LDS atomic max (the dictionary preload): a CAS loop on host memory.
inline uint32_t atomicMax(uint32_t* p, uint32_t v) {
    uint32_t cur = __atomic_load_n(p, __ATOMIC_RELAXED);
    while (cur < v && !__atomic_compare_exchange_n(p, &cur, v, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
    }
    return cur;
}
inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) {
    return __atomic_fetch_add(p, v, __ATOMIC_RELAXED);
}
inline unsigned atomicAdd(unsigned* p, unsigned v) { return __atomic_fetch_add(p, v, __ATOMIC_RELAXED); }
inline float atomicAdd(float* p, float v) {
    float o = *p, n = o + v;
    while (!__atomic_compare_exchange(p, &o, &n, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) n = o + v;
    return o;
}
inline unsigned atomicMin(unsigned* p, unsigned v) {
    unsigned o = __atomic_load_n(p, __ATOMIC_RELAXED);
    while (v < o && !__atomic_compare_exchange_n(p, &o, v, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {}
    return o;
}
inline bool __syncthreads_or(int v) { return v != 0; }
