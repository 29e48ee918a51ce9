// Lane emulator of the LZ4E compress kernel (debug/test tooling, tools/emu):
// compiles the unmodified kernel source (and csrc/lz4e_wave.h, with
// -DLZ4E_EMU) as host C++ and runs each workgroup as 64 threads per wave.
#include <stdint.h>
#include <string.h>
#include <memory>
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

thread_local EmuWave* g_emu_wave;
thread_local uint32_t g_emu_lane;
thread_local EmuBarrier* g_emu_group;
dim3 blockIdx, gridDim;
thread_local dim3 threadIdx;

void emu_launch(uint32_t nblocks, uint32_t threads, std::function<void()> body) {
    const uint32_t nw = (threads + 63) / 64;
    gridDim = dim3(nblocks);
    for (uint32_t b = 0; b < nblocks; ++b) {
        blockIdx = dim3(b);
        std::unique_ptr<EmuWave[]> waves(new EmuWave[nw]);
        EmuBarrier group((std::ptrdiff_t)(64 * nw));
        memset(lz4e::smem, 0xA5, sizeof(lz4e::smem));  // LDS is not zeroed on the GPU
        std::vector<std::thread> th;
        for (uint32_t t = 0; t < 64 * nw; ++t)
            th.emplace_back([&, t]() {
                g_emu_wave = &waves[t / 64];
                g_emu_lane = t % 64;
                g_emu_group = &group;
                threadIdx = dim3(t);
                body();
            });
        for (auto& x : th) x.join();
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
