// lz4e_gpu.h -- internal (C++) launch interface of the gfx950 LZ4E kernels.
// The public C ABI is include/lz4e.h; lz4e_host.hip maps it onto these.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lz4e {

// Largest block whose bytes the compressor stages in LDS.  The parse is
// latency-bound per block, so the 16 KiB table alone (10 blocks per CU,
// input read through L1/L2) beats staging for anything but small blocks.
constexpr uint32_t kMaxLdsInput = 4096;

struct CompressBatch {
    const uint8_t* src;
    const uint64_t* src_off;
    const uint32_t* src_len;
    const uint8_t* table_type;
    uint8_t* dst;
    const uint64_t* dst_off;
    const uint32_t* dst_cap;
    int32_t* ret;
    uint32_t* aux;  // nullable, 2 words per block
    uint32_t nblocks;
    uint32_t max_len;
    // Dictionary mode (nullable): block i's dictionary is the dict_len[i]
    // (<= 64 KiB) bytes right before src + src_off[i]; byU32 blocks only.
    const uint32_t* dict_len = nullptr;
};

struct DecompressBatch {
    const uint8_t* src;
    const uint64_t* src_off;
    const int32_t* src_len;
    uint8_t* dst;
    const uint64_t* dst_off;
    const int32_t* dst_cap;
    int32_t* ret;
    uint32_t nblocks;
    // Upper bound of dst_cap[] (0: unknown); with the batch size it selects
    // the decoder (launch_impl in lz4e_decompress.hip lists the order).
    uint32_t max_cap;
    uint32_t mode = 0;  // kDecAuto, or force kDecWave / kDecPipe / kDecSmall / kDecGroup / kDecGroupNoBail (tests, A/B)
    // Dictionary mode (nullable): block i decodes with the dict_len[i] bytes
    // right before dst + dst_off[i] as its dictionary (extDict semantics of
    // lz4e_decompress.c:299-302, 339-378; <= 64 KiB of it is ever read).
    const int32_t* dict_len = nullptr;
};

// (3 was the streaming decoder, removed in round 4; 4 and 5 the chunked and
// relay decoders, removed in round 5: none was ever picked by auto mode)
// kDecGroupNoBail: the group decoder with its hand-over to the one-wave
// decoder disabled -- every block decoded to its end by its group (tests and
// A/B only; auto mode never picks it).
enum : uint32_t { kDecAuto = 0, kDecWave = 1, kDecPipe = 2, kDecSmall = 6, kDecGroup = 7, kDecGroupNoBail = 9 };

// Launch order policy (lz4e_order.h): 0 block order, 1 heavy first when the
// batch is large enough (default), 2 heavy first always.  From
// lz4e_debug_set_launch_order, else LZ4E_COMPRESS_ORDER / LZ4E_DECOMPRESS_ORDER
// (0 disables), else 1.
enum : int { kOrderNever = 0, kOrderAuto = 1, kOrderAlways = 2 };
int launch_order_mode(bool compress);

uint32_t compress_lds_bytes(uint32_t max_len, bool lds_input);
hipError_t launch_compress(const CompressBatch& a, hipStream_t stream);
// Diagnostic build: per-block phase cycle counters into dbg, kCompressStampWords
// x u64 per block: 6 phase cycle sums, 2 packed counts, the parse's shader
// cycles and its 100 MHz (s_memrealtime) ticks.
constexpr uint32_t kCompressStampWords = 16;
hipError_t launch_compress_stamped(const CompressBatch& a, hipStream_t stream, uint64_t* dbg);
hipError_t launch_decompress(const DecompressBatch& a, hipStream_t stream);
hipError_t launch_decompress_stamped(const DecompressBatch& a, hipStream_t stream, uint64_t* dbg);

}  // namespace lz4e
