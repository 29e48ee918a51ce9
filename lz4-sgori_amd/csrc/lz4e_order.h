// lz4e_order.h -- launch order of a batch's blocks (both codec kernels).
//
// A batch's kernel time is its slowest block, and a block runs slower when
// other heavy blocks share its SIMD or when it starts late.  Workgroups are
// dispatched in blockIdx order, round robin over the 8 XCDs and their CUs,
// so a batch launched heaviest block first spreads its heavy blocks over
// the whole chip and leaves the light ones for the end (longest-processing-
// time order).  The codec kernels read their block index through `order`.
//
// order_kernel: counting sort of the block indices by a bucket key
// (0 = first), one 1024-thread workgroup, histogram and cursors in LDS; the
// order inside a bucket is arbitrary (it only decides which workgroup
// handles which block, never a result).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lz4e {

constexpr uint32_t kOrderBuckets = 64;
constexpr uint32_t kOrderThreads = 1024;

// heavy (nullable): the number of blocks whose key is at most heavy_key (the
// length of the launch order's heavy prefix).
template <class Key>
__global__ __launch_bounds__(kOrderThreads) void order_kernel(Key key, uint32_t nblocks,
                                                              uint32_t* __restrict__ order,
                                                              uint32_t heavy_key = 0,
                                                              uint32_t* __restrict__ heavy = nullptr) {
    __shared__ uint32_t hist[kOrderBuckets], cur[kOrderBuckets];
    const uint32_t t = threadIdx.x;
    if (t < kOrderBuckets) hist[t] = 0;
    __syncthreads();
    for (uint32_t b = t; b < nblocks; b += kOrderThreads) atomicAdd(&hist[key(b)], 1u);
    __syncthreads();
    if (t == 0) {
        uint32_t acc = 0;
        for (uint32_t k = 0; k < kOrderBuckets; ++k) {
            cur[k] = acc;
            acc += hist[k];
            if (heavy && k == heavy_key) *heavy = acc;
        }
    }
    __syncthreads();
    for (uint32_t b = t; b < nblocks; b += kOrderThreads) order[atomicAdd(&cur[key(b)], 1u)] = b;
}

}  // namespace lz4e
