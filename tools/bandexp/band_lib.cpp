// The band compressor experiment as its own shared library (not part of
// liblz4e_amd.so): band_compress_dev runs prev_kernel + band_kernel on
// device-resident blocks, stamped when dbg is not null (16 x u64 per block).
#include "lz4e_band.hip"

extern "C" int band_compress_dev(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                                 const uint8_t* table_type, uint8_t* dst, const uint64_t* dst_off,
                                 const uint32_t* dst_cap, int32_t* ret, uint32_t nblocks, uint32_t max_len,
                                 void* stream, uint64_t* dbg) {
    lz4e::CompressBatch a{src, src_off, src_len, table_type, dst, dst_off, dst_cap, ret, nullptr, nblocks, max_len};
    return lz4e::launch_compress_band(a, static_cast<hipStream_t>(stream), nullptr, dbg) == hipSuccess ? 0 : -1;
}
