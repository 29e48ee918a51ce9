// Lane emulator of the LZ4E compress kernel (debug/test tooling, tools/emu):
// compiles the unmodified kernel source (copied next to the emulated
// lz4e_wave.h by build.sh) as host C++ and runs each block as 64 threads.
#include <stdint.h>
#include <string.h>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>

namespace lz4e {
namespace {
alignas(16) uint32_t smem[(16384 + 65536 + 64) / 4];
}
}  // namespace lz4e

#include "lz4e_compress.hip"

// The emulator launches in block order (no pool for the order's scratch).
namespace lz4e {
int launch_order_mode(bool) { return kOrderNever; }
}  // namespace lz4e

dim3 blockIdx;
namespace lz4e {
EmuWave* g_wave;
thread_local uint32_t g_lane;
}  // namespace lz4e

void emu_launch(uint32_t nblocks, std::function<void()> lane_body) {
    for (uint32_t b = 0; b < nblocks; ++b) {
        blockIdx = dim3(b);
        lz4e::EmuWave w;
        lz4e::g_wave = &w;
        memset(lz4e::smem, 0xA5, sizeof(lz4e::smem));  // LDS is not zeroed on the GPU
        std::vector<std::thread> th;
        for (uint32_t l = 0; l < 64; ++l)
            th.emplace_back([&, l]() {
                lz4e::g_lane = l;
                lane_body();
            });
        for (auto& t : th) t.join();
    }
}

extern "C" int emu_compress_batch(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                                  const uint8_t* table_type, uint8_t* dst, const uint64_t* dst_off,
                                  const uint32_t* dst_cap, int32_t* ret, uint32_t* aux,
                                  uint32_t nblocks, uint32_t max_len) {
    lz4e::CompressBatch a{src, src_off, src_len, table_type, dst, dst_off, dst_cap, ret, aux,
                          nblocks, max_len};
    return lz4e::launch_compress(a, nullptr) == hipSuccess ? 0 : -1;
}

// Dictionary mode: block i's dictionary is the dict_len[i] bytes before it.
extern "C" int emu_compress_batch_dict(const uint8_t* src, const uint64_t* src_off,
                                       const uint32_t* src_len, const uint8_t* table_type,
                                       uint8_t* dst, const uint64_t* dst_off, const uint32_t* dst_cap,
                                       int32_t* ret, uint32_t* aux, uint32_t nblocks, uint32_t max_len,
                                       const uint32_t* dict_len) {
    lz4e::CompressBatch a{src, src_off, src_len, table_type, dst, dst_off, dst_cap, ret, aux,
                          nblocks, max_len, dict_len};
    return lz4e::launch_compress(a, nullptr) == hipSuccess ? 0 : -1;
}
