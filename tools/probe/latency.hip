// Probe: single-wave dependent-chain latencies on gfx950 (cycles, s_memtime).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef __attribute__((address_space(1))) uint32_t gu32;
__device__ __forceinline__ uint32_t vaddr(uint32_t q) { asm("" : "+v"(q)); return q; }
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__global__ void lds_chain(uint32_t* out, int iters) {
    __shared__ uint32_t t[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) t[i] = (i * 97 + 13) & 4095;
    __syncthreads();
    uint32_t x = 5;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) x = uni(t[vaddr(x)]);
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = (uint32_t)(t1 - t0); out[1] = x; }
}
__global__ void glb_chain(const uint32_t* buf, uint32_t mask, uint32_t* out, int iters) {
    uint32_t x = 5;
    const gu32* b = (const gu32*)buf;
    for (int i = 0; i < 64; ++i) x = uni(b[vaddr(x & mask)]);  // warm
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) x = uni(b[vaddr(x & mask)]);
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = (uint32_t)(t1 - t0); out[1] = x; }
}
// store, then a dependent load of another (cached) address: vmcnt covers both
__global__ void st_ld_chain(const uint32_t* buf, uint32_t mask, uint32_t* sink, uint32_t* out, int iters, int do_store) {
    uint32_t x = 5;
    const gu32* b = (const gu32*)buf;
    gu32* s = (gu32*)sink;
    for (int i = 0; i < 64; ++i) x = uni(b[vaddr(x & mask)]);
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (do_store && threadIdx.x == 0) s[(i * 7) & 1023] = x;
        x = uni(b[vaddr(x & mask)]);
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = (uint32_t)(t1 - t0); out[1] = x; }
}
// whole-wave stripe load (64 lanes x dword, consecutive) dependent chain
__global__ void stripe_chain(const uint32_t* buf, uint32_t mask, uint32_t* out, int iters) {
    uint32_t x = 5;
    const gu32* b = (const gu32*)buf;
    const uint32_t lane = threadIdx.x;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        uint32_t v = b[((x & mask) & ~63u) + lane];
        x = __builtin_amdgcn_readlane(v, 7) + x;
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = (uint32_t)(t1 - t0); out[1] = x; }
}
__global__ void salu_chain(uint32_t* out, int iters, uint32_t seed) {
    uint32_t x = seed;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) x = uni((x * 2654435761u) >> 7) + i;
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = (uint32_t)(t1 - t0); out[1] = x; }
}
__global__ void readlane_chain(uint32_t* out, int iters) {
    uint32_t v = threadIdx.x * 3 + 1, x = 0;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) x = __builtin_amdgcn_readlane(v, x & 63) + 1;
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = (uint32_t)(t1 - t0); out[1] = x; }
}
__global__ void ballot_chain(uint32_t* out, int iters) {
    uint32_t v = threadIdx.x * 3 + 1, x = 0;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        uint64_t m = __ballot((v ^ x) > 100);
        x = (uint32_t)__builtin_ctzll(m | (1ull << 63)) + x;
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = (uint32_t)(t1 - t0); out[1] = x; }
}

int main() {
    const int iters = 4096;
    uint32_t *buf, *out, *sink;
    const size_t big = 1u << 28;  // 1 GiB of u32
    hipMalloc(&buf, big * 4); hipMalloc(&out, 64); hipMalloc(&sink, 4096 * 4);
    // random permutation-ish chain values
    uint32_t* h = (uint32_t*)malloc(big * 4);
    uint64_t s = 88172645463325252ull;
    for (size_t i = 0; i < big; ++i) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; h[i] = (uint32_t)s; }
    hipMemcpy(buf, h, big * 4, hipMemcpyHostToDevice);
    uint32_t r[2];
    auto rep = [&](const char* name) { hipDeviceSynchronize(); hipMemcpy(r, out, 8, hipMemcpyDeviceToHost); printf("%-28s %8.1f cycles/iter\n", name, (double)r[0] / iters); };
    lds_chain<<<1, 64>>>(out, iters); rep("lds uniform chain");
    uint32_t masks[] = {(1u << 12) - 1, (1u << 15) - 1, (1u << 18) - 1, (1u << 20) - 1, (1u << 28) - 1};
    const char* mn[] = {"glb 16KiB (L1)", "glb 128KiB", "glb 1MiB (L2)", "glb 4MiB", "glb 1GiB (HBM)"};
    for (int k = 0; k < 5; ++k) { glb_chain<<<1, 64>>>(buf, masks[k], out, iters); rep(mn[k]); }
    for (int k = 0; k < 3; ++k) {
        st_ld_chain<<<1, 64>>>(buf, masks[k], sink, out, iters, 0); rep("  no-store ld");
        st_ld_chain<<<1, 64>>>(buf, masks[k], sink, out, iters, 1); rep("  store+ld");
    }
    stripe_chain<<<1, 64>>>(buf, (1u << 12) - 1, out, iters); rep("stripe 16KiB");
    stripe_chain<<<1, 64>>>(buf, (1u << 16) - 1, out, iters); rep("stripe 256KiB");
    stripe_chain<<<1, 64>>>(buf, (1u << 20) - 1, out, iters); rep("stripe 4MiB");
    salu_chain<<<1, 64>>>(out, iters, 3); rep("mul+readfirstlane chain");
    readlane_chain<<<1, 64>>>(out, iters); rep("readlane chain");
    ballot_chain<<<1, 64>>>(out, iters); rep("ballot+ctz chain");
    // loaded GPU: 2560 waves running glb 1MiB chains concurrently
    return 0;
}
