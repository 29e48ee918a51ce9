// Lane emulator of the LZ4E one-wave decoder (debug/test tooling, tools/emu):
// compiles the unmodified decoder source as host C++ and runs each block as
// 64 threads (tools/emu/lz4e_wave.h), like emu.cpp does for the compressor.
// LDS arrays are function statics here: one instance shared by the lanes.
#include <stdint.h>
#include <string.h>

#include <hip/hip_runtime.h>
#undef __shared__
#define __shared__ static

#include "lz4e_decompress.hip"

thread_local dim3 threadIdx;

// Block i decodes src_len[i] bytes at src + src_off[i] into dst + dst_off[i]
// (capacity dst_cap[i]), dictionary: the dict_len[i] bytes before it
// (dict_len nullable).  One-wave decoder only.
extern "C" int emu_decompress_batch(const uint8_t* src, const uint64_t* src_off, const int32_t* src_len,
                                    uint8_t* dst, const uint64_t* dst_off, const int32_t* dst_cap,
                                    int32_t* ret, uint32_t nblocks, const int32_t* dict_len) {
    lz4e::DecompressBatch a{src, src_off, src_len, dst, dst_off, dst_cap, ret, nblocks, 0,
                            lz4e::kDecWave, dict_len};
    return lz4e::launch_decompress(a, nullptr) == hipSuccess ? 0 : -1;
}
