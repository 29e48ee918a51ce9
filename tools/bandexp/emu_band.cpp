// Lane emulator of the band compressor (debug/test tooling, tools/emu):
// compiles the unmodified csrc/lz4e_band.hip as host C++ and runs each
// block's 256-thread workgroup as host threads (LDS arrays are function
// statics: one instance shared by the block's threads; blocks run one after
// the other).
#include <stdint.h>
#include <string.h>

#include <hip/hip_runtime.h>
#undef __shared__
#define __shared__ static

#include "lz4e_band.hip"

// Block i: src_len[i] bytes at src + src_off[i] -> dst + dst_off[i]
// (capacity dst_cap[i]); aux nullable (final source position, last run).
extern "C" int emu_compress_band(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                                 const uint8_t* table_type, uint8_t* dst, const uint64_t* dst_off,
                                 const uint32_t* dst_cap, int32_t* ret, uint32_t* aux, uint32_t nblocks,
                                 uint32_t max_len) {
    lz4e::CompressBatch a{src, src_off, src_len, table_type, dst, dst_off, dst_cap, ret, aux, nblocks, max_len};
    return lz4e::launch_compress_band(a, nullptr, nullptr, nullptr) == hipSuccess ? 0 : -1;
}
