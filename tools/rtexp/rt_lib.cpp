// Round-5 experiment: compress and decode each block in one launch (the
// compress kernel's wave decodes its own frame with the one-wave decoder
// right after writing it), against the two-launch step.  Built as its own
// library (tools/rtexp/Makefile); not part of liblz4e_amd.so.
//
// Result (profiles/r05/fused_roundtrip_experiment.log, rtbench.py, 20 steps):
// bit-exact (frames, returns, outputs) on every workload but slower on every
// one: silesia64k 4.48 vs 4.32 ms, text256k 29.09 vs 28.45 ms, sg512 5.00 vs
// 4.78 ms, fio4k 14.77 vs 9.39 ms.  The decode tail of the heaviest blocks
// lengthens the launch's critical path, and one wave decoding its own frame
// is slower than the pipelined (64 KiB) and lane (4 KiB) decoders the
// two-launch step picks.  Not integrated.
#include "lz4e_compress.hip"
#include "lz4e_decompress.hip"

namespace lz4e {
namespace {

// kernarg layout of roundtrip_kernel (result and decode pointers are reloaded
// after the parse, as compress_kernel does: none of them is live across it)
struct RtArgs {
    const uint8_t* src;
    const uint64_t* src_off;
    const uint32_t* src_len;
    const uint8_t* table_type;
    uint8_t* dst;
    const uint64_t* dst_off;
    int32_t* ret;
    const uint32_t* order;
    uint8_t* out;
    const uint64_t* out_off;
    const int32_t* out_cap;
    int32_t* dret;
    uint32_t nblocks;
};

__global__ __launch_bounds__(64) void roundtrip_kernel(const uint8_t* __restrict__ src,
                                                       const uint64_t* __restrict__ src_off,
                                                       const uint32_t* __restrict__ src_len,
                                                       const uint8_t* __restrict__ table_type,
                                                       uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off,
                                                       int32_t* __restrict__ ret, const uint32_t* __restrict__ order,
                                                       uint8_t* __restrict__ out, const uint64_t* __restrict__ out_off,
                                                       const int32_t* __restrict__ out_cap, int32_t* __restrict__ dret,
                                                       uint32_t nblocks) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    if (blockIdx.x >= nblocks) return;
    const uint32_t b = order ? order[blockIdx.x] : blockIdx.x;
    const uint32_t lane = lane_id();
    const uint32_t n = src_len[b];
    const int tt = table_type[b];
    const uint32_t cap = n + n / 255 + 16;  // frame slots hold LZ4E_COMPRESSBOUND(n)
    gu8* fr = (gu8*)(dst + dst_off[b]);
    const uint8_t* in = src + src_off[b];
    const bool tt_ok = (tt == kByU16 && n <= 65536) || tt == kByU32 || tt == kByU64;
    if (n > kMaxInput || (n >= kMinLength && !tt_ok)) {
        if (lane == 0) {
            ret[b] = n > kMaxInput ? 0 : -1;
            dret[b] = -1;
        }
        return;
    }
    CResult res;
    if (n >= kMinLength) {
        uint4* t4 = reinterpret_cast<uint4*>(smem);
        for (uint32_t i = lane; i < kTableBytes / 16; i += kWave) t4[i] = make_uint4(0, 0, 0, 0);
    }
    block_sync();
    const HbmImage img{buf_make(in, n)};
    bool pp = true;
    if (order) {
        const uint32_t nh = order[nblocks];
        if (nh < nblocks - nblocks / 16) {
            pp = false;
            if (blockIdx.x < nh) __builtin_amdgcn_s_setprio(3);
        }
    }
    res = dispatch_class<false>(img, smem, n, tt, fr, cap, nullptr, lane, 0, pp);
    const __attribute__((address_space(4))) RtArgs* ka =
        (const __attribute__((address_space(4))) RtArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    const uint32_t* const ordp = ka->order;
    const uint32_t b2 = ordp ? ordp[blockIdx.x] : blockIdx.x;
    if (lane == 0) ka->ret[b2] = res.ret;
    // the frame is this wave's own stores: complete them, then decode it
    stores_done();
    wave_fence();
    const int32_t csize = (int32_t)uni((uint32_t)res.ret);
    const int32_t ocap = ka->out_cap[b2];
    const uint8_t* frp = ka->dst + ka->dst_off[b2];
    uint8_t* o = ka->out + ka->out_off[b2];
    int32_t* dr = ka->dret + b2;
    block_sync();  // (the table's LDS becomes the decoder's)
    if (special_case(frp, csize, ocap, dr, lane)) return;
    lu8* sinkb = (lu8*)((uint8_t*)smem + kRing + kRingPad);
    decode_block<false>(frp, csize, o, ocap, dr, nullptr, lane, sinkb + kSink, (lu32*)smem,
                        (lu16*)(sinkb + kSink + kSpan), 0, sinkb);
}

}  // namespace
}  // namespace lz4e

extern "C" int rt_roundtrip_dev(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                                const uint8_t* table_type, uint8_t* dst, const uint64_t* dst_off, int32_t* ret,
                                uint8_t* out, const uint64_t* out_off, const int32_t* out_cap, int32_t* dret,
                                uint32_t nblocks, void* stream_) {
    using namespace lz4e;
    const hipStream_t stream = static_cast<hipStream_t>(stream_);
    if (nblocks == 0) return 0;
    uint32_t* scratch = nullptr;
    if (nblocks >= kOrderMinBlocks &&
        hipMallocAsync((void**)&scratch, sizeof(uint32_t) * (2 * (size_t)nblocks + 1), stream) == hipSuccess) {
        hipLaunchKernelGGL(weight_kernel, dim3(nblocks), dim3(kWeightThreads), 0, stream, src, src_off, src_len,
                           nblocks, scratch);
        hipLaunchKernelGGL((order_kernel<CompressWeight>), dim3(1), dim3(kOrderThreads), 0, stream,
                           CompressWeight{scratch}, nblocks, scratch + nblocks, kHeavyBucket,
                           scratch + 2 * (size_t)nblocks);
    } else {
        (void)hipGetLastError();
        scratch = nullptr;
    }
    hipLaunchKernelGGL(roundtrip_kernel, dim3(nblocks), dim3(kWave), kTableBytes, stream, src, src_off, src_len,
                       table_type, dst, dst_off, ret, scratch ? (const uint32_t*)(scratch + nblocks) : nullptr, out,
                       out_off, out_cap, dret, nblocks);
    const hipError_t err = hipGetLastError();
    if (scratch) (void)hipFreeAsync(scratch, stream);
    return err == hipSuccess ? 0 : -1;
}

// the library's launch_order_mode (lz4e_host.hip) is not linked here
namespace lz4e {
int launch_order_mode(bool) { return kOrderAuto; }
}  // namespace lz4e
