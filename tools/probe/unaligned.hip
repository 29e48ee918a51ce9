// Probe: do global_load_dword / global_store_dword / dwordx4 work at unaligned addresses?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void k(const uint8_t* in, uint8_t* out, uint32_t* res) {
    const uint32_t t = threadIdx.x;
    const uint32_t* p = (const uint32_t*)(in + 1 + 5 * t);          // unaligned
    uint32_t v = *p;
    *(uint32_t*)(out + 3 + 7 * t) = v;                                // unaligned store
    const uint4* q = (const uint4*)(in + 2 + 17 * t);
    uint4 w = *q;
    *(uint4*)(out + 1000 + 5 + 17 * t) = w;
    res[t] = v;
}
int main() {
    uint8_t h[4096]; for (int i = 0; i < 4096; ++i) h[i] = (uint8_t)(i * 7 + 3);
    uint8_t *din, *dout; uint32_t* dres;
    hipMalloc(&din, 4096); hipMalloc(&dout, 4096); hipMalloc(&dres, 256);
    hipMemcpy(din, h, 4096, hipMemcpyHostToDevice); hipMemset(dout, 0, 4096);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout, dres);
    hipError_t e = hipDeviceSynchronize();
    uint8_t o[4096]; hipMemcpy(o, dout, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int t = 0; t < 64; ++t) {
        for (int b = 0; b < 4; ++b) bad += o[3 + 7 * t + b] != h[1 + 5 * t + b];
        for (int b = 0; b < 16; ++b) bad += o[1005 + 17 * t + b] != h[2 + 17 * t + b];
    }
    printf("sync=%s mismatches=%d\n", hipGetErrorString(e), bad);
    return bad != 0;
}
