// Host stand-in for <hip/hip_runtime.h> used ONLY by the lane emulator
// (tools/emu): just enough of the kernel language for lz4e_compress.hip to
// compile as host C++, each lane a thread.  Never part of the product build.
#pragma once
#include <math.h>
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <functional>

#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__

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

// LDS atomic max (the dictionary preload): a CAS loop on host memory.
inline uint32_t atomicMax(uint32_t* p, uint32_t v) {
    uint32_t cur = __atomic_load_n(p, __ATOMIC_RELAXED);
    while (cur < v && !__atomic_compare_exchange_n(p, &cur, v, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
    }
    return cur;
}

// Only so that the pipelined decoder compiles (it is never run here: the
// emulator runs one 64-lane wave per block).
#define __HIP_MEMORY_SCOPE_WORKGROUP 0
#define __hip_atomic_load(p, order, scope) __atomic_load_n(p, order)
#define __hip_atomic_store(p, v, order, scope) __atomic_store_n(p, v, order)
#define __builtin_amdgcn_s_sleep(x) ((void)0)
#define __builtin_amdgcn_s_setprio(x) ((void)0)
inline void __syncthreads() {}
inline bool __syncthreads_or(int v) { return v != 0; }
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
// (the decoder's launch order kernel is not emulated: no pool, block order)
inline hipError_t hipMallocAsync(void**, size_t, hipStream_t) { return hipErrorOutOfMemory; }
inline hipError_t hipFreeAsync(void*, hipStream_t) { return hipSuccess; }
extern dim3 blockIdx;
extern thread_local dim3 threadIdx;
void emu_launch(uint32_t nblocks, std::function<void()> lane_body);
#define hipLaunchKernelGGL(k, grid, block, lds, stream, ...) \
    emu_launch((grid).x, [&]() { k(__VA_ARGS__); })
