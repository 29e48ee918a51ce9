// Lane emulator of the LZ4E decoders (debug/test tooling, tools/emu):
// compiles the unmodified decoder source as host C++ and runs each block's
// workgroup as host threads -- one wave (64 threads) for the one-wave
// decoder, four waves (256 threads: parser + three copiers, their LDS
// progress counters as host atomics) for the pipelined decoder.  LDS arrays
// are function statics here: one instance shared by the threads of the
// block (blocks run one after the other).
#include <stdint.h>
#include <string.h>

#include <hip/hip_runtime.h>
#undef __shared__
#define __shared__ static

#include "lz4e_decompress.hip"
#include "lz4e_results.h"

// Block i decodes src_len[i] bytes at src + src_off[i] into dst + dst_off[i]
// (capacity dst_cap[i]), dictionary: the dict_len[i] bytes before it
// (dict_len nullable).  mode: 1 one-wave decoder, 2 pipelined decoder, 6 LDS form,
// 7 group decoder, 9 group decoder without the hand-over.
extern "C" int emu_decompress_batch_mode(const uint8_t* src, const uint64_t* src_off,
                                         const int32_t* src_len, uint8_t* dst, const uint64_t* dst_off,
                                         const int32_t* dst_cap, int32_t* ret, uint32_t nblocks,
                                         const int32_t* dict_len, uint32_t mode) {
    lz4e::DecompressBatch a{src, src_off, src_len, dst, dst_off, dst_cap, ret, nblocks, 0,
                            mode, dict_len};
    return lz4e::launch_decompress(a, nullptr) == hipSuccess ? 0 : -1;
}

extern "C" int emu_decompress_batch(const uint8_t* src, const uint64_t* src_off, const int32_t* src_len,
                                    uint8_t* dst, const uint64_t* dst_off, const int32_t* dst_cap,
                                    int32_t* ret, uint32_t nblocks, const int32_t* dict_len) {
    return emu_decompress_batch_mode(src, src_off, src_len, dst, dst_off, dst_cap, ret, nblocks,
                                     dict_len, lz4e::kDecWave);
}

// The host entry points' reading of a batch's return values
// (csrc/lz4e_results.h): number of blocks with ret >= 0, or -1 with the
// error text when the decoder's watchdog fired on a block.
extern "C" int emu_decode_results(const int32_t* ret, uint32_t n, char* err, uint32_t err_cap) {
    std::string e;
    const int r = lz4e::decode_results(ret, n, e);
    if (err && err_cap) {
        strncpy(err, e.c_str(), err_cap - 1);
        err[err_cap - 1] = 0;
    }
    return r;
}
