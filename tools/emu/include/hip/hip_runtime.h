// Host stand-in for <hip/hip_runtime.h> used ONLY by the lane emulator
// (tools/emu): just enough of the kernel language for lz4e_compress.hip to
// compile as host C++, each lane a thread.  Never part of the product build.
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <functional>

#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __launch_bounds__(x)
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

extern dim3 blockIdx;
void emu_launch(uint32_t nblocks, std::function<void()> lane_body);
#define hipLaunchKernelGGL(k, grid, block, lds, stream, ...) \
    emu_launch((grid).x, [&]() { k(__VA_ARGS__); })
