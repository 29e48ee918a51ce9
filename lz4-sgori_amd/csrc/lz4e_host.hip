// lz4e_host.hip -- C ABI of include/lz4e.h on top of the gfx950 kernels.
//
// Single-call entry points keep the reference's synchronous, per-request
// contract (lz4e_bdev/lz4e_chunk.c:139-159 calls LZ4E_compress_default once
// per WRITE bio) and its reentrancy: each call leases its own stream and
// staging from a pool (no process-wide lock), gathers the SG segments into
// pinned staging, makes one H2D copy, launches the kernel, and brings back
// the results -- exactly the bytes produced -- through the host mapping of
// the pinned buffer, then scatters into the destination segments.  The
// batched entry points amortise that over many requests; the *_dev forms
// launch straight on device-resident buffers.
//
// There is no CPU codec here: without a usable gfx950 device every entry
// point fails (compress 0, decompress < 0) and lz4e_last_error() says why.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lz4e.h"
#include "lz4e_gpu.h"
#include "lz4e_results.h"

static_assert(lz4e::kDecodeAborted == LZ4E_DECODE_ABORTED, "watchdog return value");

namespace {

thread_local std::string g_err;

void set_err(const std::string& s) { g_err = s; }

bool hip_ok(hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    set_err(std::string(what) + ": " + hipGetErrorString(e));
    return false;
}

uint32_t bound_of(uint32_t n) { return n > LZ4E_MAX_INPUT_SIZE ? 0u : n + n / 255 + 16; }

uint64_t align16(uint64_t x) { return (x + 15) & ~uint64_t(15); }

// Growable device / pinned-host byte buffer.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool ensure(size_t n) {
        if (n <= cap) return true;
        const size_t want = std::max(n, cap * 2);
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (!hip_ok(hipMalloc(&p, want), "hipMalloc")) return false;
        cap = want;
        return true;
    }
};

struct HostBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool ensure(size_t n) {
        if (n <= cap) return true;
        const size_t want = std::max(n, cap * 2);
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        if (!hip_ok(hipHostMalloc(&p, want, hipHostMallocDefault), "hipHostMalloc")) return false;
        cap = want;
        return true;
    }
};

// Device check, once per process: the library only runs on gfx950.
struct DeviceGate {
    std::once_flag once;
    bool ok = false;
    std::string why;
    bool check() {
        std::call_once(once, [this] {
            int n = 0;
            if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
                why = "lz4e: no HIP device visible";
                return;
            }
            int dev = 0;
            (void)hipGetDevice(&dev);
            hipDeviceProp_t prop;
            if (hipGetDeviceProperties(&prop, dev) != hipSuccess ||
                std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
                why = std::string("lz4e: device is not gfx950 (") + prop.gcnArchName + ")";
                return;
            }
            ok = true;
        });
        if (!ok) set_err(why);
        return ok;
    }
};

DeviceGate& gate() {
    static DeviceGate g;
    return g;
}

// Per-call resources of the host entry points: a stream and growable pinned
// + HBM staging.  Calls lease one from a per-device pool for their duration,
// so concurrent callers (the reference is reentrant given distinct wrkmem,
// called from every submitting CPU: lz4e_bdev/lz4e_dev.c:174 ->
// lz4e_req.c:177) run side by side on their own streams; the pool only
// grows to the peak concurrency.  Contexts live until process exit.
struct CallCtx {
    int dev = 0;
    hipStream_t stream = nullptr;
    DevBuf d;      // [inputs | descriptors in | results | outputs]
    HostBuf h;     // pinned twin of d
    void* h_dev = nullptr;  // h as the device sees it (results come back by kernel)
    bool grow(size_t bytes) {
        if (!d.ensure(bytes)) return false;
        const void* old = h.p;
        if (!h.ensure(bytes)) return false;
        if (h.p != old || !h_dev)
            return hip_ok(hipHostGetDevicePointer(&h_dev, h.p, 0), "hipHostGetDevicePointer");
        return true;
    }
};

struct CtxPool {
    std::mutex mu;
    std::vector<CallCtx*> free_;
};

CtxPool& pool() {
    static CtxPool p;
    return p;
}

// RAII lease of a CallCtx on the calling thread's current device.
struct Lease {
    CallCtx* c = nullptr;
    bool acquire() {
        int dev = 0;
        (void)hipGetDevice(&dev);
        {
            std::lock_guard<std::mutex> lk(pool().mu);
            auto& fl = pool().free_;
            for (size_t i = 0; i < fl.size(); ++i)
                if (fl[i]->dev == dev) {
                    c = fl[i];
                    fl.erase(fl.begin() + (long)i);
                    return true;
                }
        }
        CallCtx* n = new CallCtx;
        n->dev = dev;
        if (!hip_ok(hipStreamCreateWithFlags(&n->stream, hipStreamNonBlocking), "hipStreamCreate")) {
            delete n;
            return false;
        }
        c = n;
        return true;
    }
    ~Lease() {
        if (!c) return;
        std::lock_guard<std::mutex> lk(pool().mu);
        pool().free_.push_back(c);
    }
};

// Copies blocks back into the host mapping of a pinned buffer: block b moves
// len[b] bytes (nothing when len[b] <= 0) from dev + off[b] to
// host + off[b], rounded up to 16 B (offsets are 16-B aligned and every slot
// has >= 16 B of slack).  Only the bytes that exist come back over PCIe --
// not the whole capacity -- and no DMA copy waits behind another stream's.
// Clock probe (diagnostic): one wave spins on a dependent VALU chain for
// `iters` steps between two pairs of time stamps, so the host can read the
// shader clock the chip holds right now as delta s_memtime (shader cycles,
// MI355X_MICROARCH.md:488) over delta s_memrealtime (100 MHz, :503).
__global__ __launch_bounds__(64) void clock_probe_kernel(uint64_t* out, uint32_t iters) {
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = threadIdx.x;
    for (uint32_t i = 0; i < iters; ++i) x = x * 1664525u + 1013904223u;
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = r1 - r0;
        out[2] = x;  // keeps the chain
    }
}

__global__ __launch_bounds__(256) void copy_blocks_kernel(const uint8_t* __restrict__ dev,
                                                          uint8_t* __restrict__ host,
                                                          const uint64_t* __restrict__ off,
                                                          const int32_t* __restrict__ len,
                                                          uint32_t n) {
    const uint32_t b = blockIdx.x;
    if (b >= n) return;
    const int32_t l = len[b];
    if (l <= 0) return;
    const uint4* s = reinterpret_cast<const uint4*>(dev + off[b]);
    uint4* d = reinterpret_cast<uint4*>(host + off[b]);
    const uint32_t n16 = ((uint32_t)l + 15) / 16;
    for (uint32_t i = threadIdx.x; i < n16; i += blockDim.x) d[i] = s[i];
}

// Raw copy of n bytes (16-B aligned offsets, n rounded up to 16 B).
__global__ __launch_bounds__(256) void copy_flat_kernel(const uint4* __restrict__ src,
                                                        uint4* __restrict__ dst, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
        dst[i] = src[i];
}

hipError_t copy_flat(void* host_dev, const void* dev, uint64_t off, uint64_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint64_t n16 = (n + 15) / 16;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(1024, (n16 + 255) / 256);
    hipLaunchKernelGGL(copy_flat_kernel, dim3(blocks), dim3(256), 0, st,
                       reinterpret_cast<const uint4*>(static_cast<const uint8_t*>(dev) + off),
                       reinterpret_cast<uint4*>(static_cast<uint8_t*>(host_dev) + off), n16);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// SG helpers (userspace model of lz4e/include/lz4e_defs.h:115-197)
// ---------------------------------------------------------------------------

inline const uint8_t* bv_data(const struct bio_vec& b) {
    return reinterpret_cast<const uint8_t*>(b.bv_page) + b.bv_offset;
}

// Copy `len` bytes starting at iterator `it` out of the SG list.
void sg_gather(const struct bio_vec* bv, const struct bvec_iter& it, uint8_t* to, uint32_t len) {
    uint32_t idx = it.bi_idx, done = it.bi_bvec_done;
    while (len) {
        uint32_t take = std::min(bv[idx].bv_len - done, len);
        std::memcpy(to, bv_data(bv[idx]) + done, take);
        to += take;
        len -= take;
        done = 0;
        idx++;
    }
}

void sg_scatter(struct bio_vec* bv, const struct bvec_iter& it, const uint8_t* from, uint32_t len) {
    uint32_t idx = it.bi_idx, done = it.bi_bvec_done;
    while (len) {
        uint32_t take = std::min(bv[idx].bv_len - done, len);
        std::memcpy(const_cast<uint8_t*>(bv_data(bv[idx])) + done, from, take);
        from += take;
        len -= take;
        done = 0;
        idx++;
    }
}

// Kernel bvec_iter_advance semantics: clamp (and warn) past the end.
void iter_advance(const struct bio_vec* bv, struct bvec_iter* it, uint32_t bytes) {
    if (bytes > it->bi_size) {
        it->bi_size = 0;
        return;
    }
    uint32_t idx = it->bi_idx;
    it->bi_size -= bytes;
    bytes += it->bi_bvec_done;
    while (bytes && bytes >= bv[idx].bv_len) {
        bytes -= bv[idx].bv_len;
        idx++;
    }
    it->bi_idx = idx;
    it->bi_bvec_done = bytes;
}

int table_type_of(const struct bio_vec* bv, const struct bvec_iter* it) {
    // lz4e/lz4e_compress.c:184-211 (LZ4E_fillBvIterSize)
    uint32_t size = it->bi_size, idx = it->bi_idx, done = it->bi_bvec_done, i = 0;
    int tt = LZ4E_TABLE_BYU16;
    while (size) {
        const uint32_t len = bv[idx].bv_len;
        if (i >= BIO_MAX_VECS) return 0;
        if (i >= 16 || len > 4096) tt |= LZ4E_TABLE_BYU32;
        if (len > (1u << 24)) tt |= LZ4E_TABLE_BYU64;
        size -= std::min(len - done, size);
        done = 0;
        idx++;
        i++;
    }
    return tt;
}

// Descriptor block of a batch of R blocks, at `base` inside a staging
// buffer: the inputs the kernels read, then the results they write.
struct MetaLayout {
    size_t src_off, src_len, ttype, dst_off, dst_cap, dict_len, ret, aux, total;
    MetaLayout(uint32_t R, size_t base) {
        size_t o = base;
        src_off = o;  o += align16(8ull * R);
        src_len = o;  o += align16(4ull * R);
        ttype = o;    o += align16(1ull * R);
        dst_off = o;  o += align16(8ull * R);
        dst_cap = o;  o += align16(4ull * R);
        dict_len = o; o += align16(4ull * R);
        ret = o;      o += align16(4ull * R);
        aux = o;      o += align16(8ull * R);
        total = o;
    }
};

}  // namespace

extern "C" {

const char* lz4e_last_error(void) { return g_err.c_str(); }

int lz4e_gpu_available(void) { return gate().check() ? 1 : 0; }

int lz4e_sg_table_type(const struct bio_vec* src, const struct bvec_iter* it) {
    return table_type_of(src, it);
}

}  // extern "C"

namespace {

// Dictionary bytes a request compresses against: the last <= 64 KiB of its
// dictionary, none under 8 bytes (LZ4_loadDict: dictSize < HASH_UNIT).
uint32_t dict_used(const char* const* dicts, const int* dict_sizes, uint32_t i) {
    if (!dicts || !dicts[i] || dict_sizes[i] < 8) return 0;
    return (uint32_t)std::min(dict_sizes[i], 65536);
}

// lz4e_compress_sg_batch, optionally in dictionary mode (dicts != nullptr:
// every request byU32, block i staged right after its dictionary bytes).
int compress_sg_batch_impl(struct lz4e_sg_request* reqs, int n, const char* const* dicts,
                           const int* dict_sizes) {
    if (n <= 0) return 0;
    g_err.clear();
    if (!gate().check()) return -1;
    for (int i = 0; i < n; ++i) reqs[i].ret = 0;

    // Live requests (the others return 0 before touching the GPU).
    std::vector<uint32_t> map;
    std::vector<uint8_t> ttype;
    for (uint32_t i = 0; i < (uint32_t)n; ++i) {
        const uint32_t len = reqs[i].srcIter->bi_size;
        int tt = LZ4E_TABLE_BYU16;
        if (len > LZ4E_MAX_INPUT_SIZE) continue;                                        // :245-248
        if (len >= 13 && (tt = table_type_of(reqs[i].src, reqs[i].srcIter)) == 0) continue;  // :274-277
        map.push_back(i);
        ttype.push_back((uint8_t)(dicts ? LZ4E_TABLE_BYU32 : tt));
    }
    const uint32_t L = (uint32_t)map.size();
    if (L == 0) return 0;

    // One staging image, host and device alike:
    //   [inputs (each after its dictionary bytes) | descriptors | ret/aux | frames]
    // one H2D copy of everything before ret, the compress kernel, and two
    // copy-back kernels: ret/aux, then exactly ret[i] bytes of each frame.
    std::vector<uint64_t> so(L), fo(L);
    std::vector<uint32_t> dl(L);
    uint64_t s = 0, f = 0;
    uint32_t max_len = 0;
    for (uint32_t j = 0; j < L; ++j) {
        const lz4e_sg_request& q = reqs[map[j]];
        const uint32_t len = q.srcIter->bi_size;
        dl[j] = dict_used(dicts, dict_sizes, map[j]);
        so[j] = align16(s + dl[j]);
        s = so[j] + align16(len);
        fo[j] = f;
        f += align16((uint64_t)std::min(q.dstIter->bi_size, bound_of(len)) + 64);
        max_len = std::max(max_len, len);
    }
    const MetaLayout m(L, s);
    const size_t fbase = m.total;
    Lease ls;
    if (!ls.acquire()) return -1;
    CallCtx& c = *ls.c;
    if (!c.grow(fbase + f)) return -1;
    uint8_t* hd = static_cast<uint8_t*>(c.h.p);
    for (uint32_t j = 0; j < L; ++j) {
        const lz4e_sg_request& q = reqs[map[j]];
        const uint32_t len = q.srcIter->bi_size;
        if (dl[j]) std::memcpy(hd + so[j] - dl[j], dicts[map[j]] + dict_sizes[map[j]] - dl[j], dl[j]);
        sg_gather(q.src, *q.srcIter, hd + so[j], len);
        reinterpret_cast<uint64_t*>(hd + m.src_off)[j] = so[j];
        reinterpret_cast<uint32_t*>(hd + m.src_len)[j] = len;
        (hd + m.ttype)[j] = ttype[j];
        reinterpret_cast<uint64_t*>(hd + m.dst_off)[j] = fbase + fo[j];
        reinterpret_cast<uint32_t*>(hd + m.dst_cap)[j] = q.dstIter->bi_size;
        reinterpret_cast<uint32_t*>(hd + m.dict_len)[j] = dl[j];
    }
    uint8_t* dd = static_cast<uint8_t*>(c.d.p);
    lz4e::CompressBatch a{dd,
                          reinterpret_cast<const uint64_t*>(dd + m.src_off),
                          reinterpret_cast<const uint32_t*>(dd + m.src_len),
                          dd + m.ttype,
                          dd,
                          reinterpret_cast<const uint64_t*>(dd + m.dst_off),
                          reinterpret_cast<const uint32_t*>(dd + m.dst_cap),
                          reinterpret_cast<int32_t*>(dd + m.ret),
                          reinterpret_cast<uint32_t*>(dd + m.aux),
                          L,
                          max_len};
    if (dicts) a.dict_len = reinterpret_cast<const uint32_t*>(dd + m.dict_len);
    if (!hip_ok(hipMemcpyAsync(dd, hd, m.ret, hipMemcpyHostToDevice, c.stream), "H2D") ||
        !hip_ok(lz4e::launch_compress(a, c.stream), "compress launch") ||
        !hip_ok(copy_flat(c.h_dev, dd, m.ret, m.total - m.ret, c.stream), "copy-back meta"))
        return -1;
    hipLaunchKernelGGL(copy_blocks_kernel, dim3(L), dim3(256), 0, c.stream, dd,
                       static_cast<uint8_t*>(c.h_dev),
                       reinterpret_cast<const uint64_t*>(dd + m.dst_off),
                       reinterpret_cast<const int32_t*>(dd + m.ret), L);
    if (!hip_ok(hipGetLastError(), "copy-back frames") ||
        !hip_ok(hipStreamSynchronize(c.stream), "compress sync"))
        return -1;
    int ok = 0;
    for (uint32_t j = 0; j < L; ++j) {
        lz4e_sg_request& q = reqs[map[j]];
        const int32_t r = reinterpret_cast<const int32_t*>(hd + m.ret)[j];
        const uint32_t* aux = reinterpret_cast<const uint32_t*>(hd + m.aux) + 2 * j;
        if (r <= 0) continue;
        sg_scatter(q.dst, *q.dstIter, hd + fbase + fo[j], (uint32_t)r);
        iter_advance(q.src, q.srcIter, aux[0]);
        iter_advance(q.dst, q.dstIter, (uint32_t)r - aux[1]);
        q.ret = r;
        ok++;
    }
    return ok;
}

// ---------------------------------------------------------------------------
// Coalescing of concurrent single calls.  The reference is called once per
// WRITE bio, synchronously, from every submitting CPU (lz4e_dev.c:174 ->
// lz4e_req.c:177 -> lz4e_chunk.c:139-159), and a lone block is one wave's
// serial parse on the GPU (~0.1-0.2 ms): calls that arrive while others are
// in flight are worth one launch together.  Leader / follower batching: a
// caller queues its request; when fewer than max_inflight() batches are in
// flight, it takes every queued request (its own included, up to kMaxBatch)
// and runs them as one batch on its own thread -- the same batch entry point
// as lz4e_compress_sg_batch / lz4e_decompress_batch, with identical bytes --
// while the others wait for their result.  A lone caller always leads its
// own one-request batch at once, so single-thread latency does not change.
// ---------------------------------------------------------------------------
template <class Req>
struct Coalescer {
    static constexpr int kMaxInflightDefault = 4;  // concurrent batches (= HW queues of the process)
    // LZ4E_COALESCE_INFLIGHT overrides it (A/B experiments)
    static int max_inflight() {
        static const int v = [] {
            const char* e = getenv("LZ4E_COALESCE_INFLIGHT");
            const int k = e ? atoi(e) : kMaxInflightDefault;
            return k >= 1 && k <= 64 ? k : kMaxInflightDefault;
        }();
        return v;
    }
    static constexpr size_t kMaxBatch = 1024;
    // A leader takes queued requests until their input reaches this (its own
    // request always goes): one caller's huge request does not make a
    // hundred small ones wait for its staging.
    static constexpr uint64_t kMaxBatchBytes = 64ull << 20;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<Req*> pending;
    int inflight = 0;

    // run(batch, n) fills every request's result; fail(req, why) marks one
    // failed.  Nothing in the leader's bookkeeping allocates, and run() is
    // fenced: an exception there (std::bad_alloc in the batch's staging)
    // fails that batch's requests -- every caller returns -- and the
    // coalescer stays usable.
    template <class Run, class Fail>
    void submit(Req* r, Run run, Fail fail) {
        std::unique_lock<std::mutex> lk(mu);
        try {
            pending.push_back(r);
        } catch (...) {
            lk.unlock();
            fail(r, "lz4e: out of host memory queueing the call");
            return;
        }
        while (!r->done) {
            if (!r->taken && inflight < max_inflight()) {
                Req* batch[kMaxBatch];
                size_t n = 0;
                uint64_t bytes = 0;
                batch[n++] = r;
                r->taken = true;
                bytes += r->bytes();
                for (Req* q : pending) {
                    if (q->taken || n == kMaxBatch) continue;
                    if (bytes + q->bytes() > kMaxBatchBytes) continue;
                    bytes += q->bytes();
                    q->taken = true;
                    batch[n++] = q;
                }
                pending.erase(std::remove_if(pending.begin(), pending.end(), [](Req* q) { return q->taken; }),
                              pending.end());
                inflight++;
                lk.unlock();
                try {
                    run(batch, n);
                } catch (const std::exception& e) {
                    for (size_t i = 0; i < n; ++i) fail(batch[i], std::string("lz4e: ") + e.what());
                } catch (...) {
                    for (size_t i = 0; i < n; ++i) fail(batch[i], "lz4e: exception in a coalesced batch");
                }
                lk.lock();
                inflight--;
                for (size_t i = 0; i < n; ++i) batch[i]->done = true;
                cv.notify_all();
            } else {
                cv.wait(lk);
            }
        }
    }
};

// decode_staging (defined with the C entry points below).
uint64_t decode_staging_bytes(int csize, int cap);

// Fault injection for the CPU test of the coalescer's unwinding
// (lz4e_debug_coalescer_fault): the next k batch runs throw.
std::atomic<int> g_coalescer_faults{0};
void maybe_inject_fault() {
    int k = g_coalescer_faults.load();
    while (k > 0 && !g_coalescer_faults.compare_exchange_weak(k, k - 1)) {
    }
    if (k > 0) throw std::runtime_error("injected fault (lz4e_debug_coalescer_fault)");
}

struct CompressCall {
    lz4e_sg_request q;
    bool taken = false, done = false;
    std::string err;
    uint64_t bytes() const { return q.srcIter->bi_size; }
};

struct DecompressCall {
    const char* src;
    char* dst;
    int csize, cap, ret = -1;
    bool taken = false, done = false;
    std::string err;
    uint64_t bytes() const { return (uint64_t)std::max(csize, 0) + decode_staging_bytes(csize, cap); }
};

// One coalescer per device: a batch runs on its leader's current device, so
// only requests from threads bound to the same device share it.
constexpr int kMaxDevices = 64;
int current_device() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) dev = 0;
    return dev;
}
Coalescer<CompressCall>& compress_calls() {
    static Coalescer<CompressCall> c[kMaxDevices];
    return c[current_device()];
}
Coalescer<DecompressCall>& decompress_calls() {
    static Coalescer<DecompressCall> c[kMaxDevices];
    return c[current_device()];
}

}  // namespace

extern "C" {

int lz4e_compress_sg_batch(struct lz4e_sg_request* reqs, int n) {
    return compress_sg_batch_impl(reqs, n, nullptr, nullptr);
}

// One coalesced batch of single compress calls.  A batch that fails as a
// whole (staging, launch) is bisected, so that one caller's failure is not
// everyone's and a single bad request costs O(log n) reruns, not n.
static void run_compress_calls(CompressCall** batch, size_t n) {
    std::vector<lz4e_sg_request> reqs(n);
    for (size_t i = 0; i < n; ++i) reqs[i] = batch[i]->q;
    const int r = compress_sg_batch_impl(reqs.data(), (int)n, nullptr, nullptr);
    if (r < 0 && n > 1) {
        run_compress_calls(batch, n / 2);
        run_compress_calls(batch + n / 2, n - n / 2);
        return;
    }
    for (size_t i = 0; i < n; ++i) {
        batch[i]->q.ret = r < 0 ? 0 : reqs[i].ret;
        batch[i]->err = g_err;
    }
}

int LZ4E_compress_default(const struct bio_vec* src, struct bio_vec* dst, struct bvec_iter* srcIter,
                          struct bvec_iter* dstIter, void* wrkmem) {
    if (wrkmem) std::memset(wrkmem, 0, LZ4E_MEM_COMPRESS);  // lz4e_compress.c:548
    if (srcIter->bi_size > LZ4E_MAX_INPUT_SIZE) return 0;
    CompressCall call;
    call.q = lz4e_sg_request{src, dst, srcIter, dstIter, 0};
    compress_calls().submit(
        &call,
        [](CompressCall** batch, size_t n) {
            maybe_inject_fault();
            run_compress_calls(batch, n);
        },
        [](CompressCall* c, const std::string& why) {
            c->q.ret = 0;
            c->err = why;
        });
    g_err = call.err;
    return call.q.ret;
}

int lz4e_compress_sg_batch_dict(struct lz4e_sg_request* reqs, int n, const char* const* dicts,
                                const int* dict_sizes) {
    return compress_sg_batch_impl(reqs, n, dicts, dict_sizes);
}

int LZ4E_compress_usingDict(const struct bio_vec* src, struct bio_vec* dst, struct bvec_iter* srcIter,
                            struct bvec_iter* dstIter, void* wrkmem, const char* dictionary,
                            int dictSize) {
    if (wrkmem) std::memset(wrkmem, 0, LZ4E_MEM_COMPRESS);
    if (srcIter->bi_size > LZ4E_MAX_INPUT_SIZE) return 0;
    lz4e_sg_request q{src, dst, srcIter, dstIter, 0};
    const int r = compress_sg_batch_impl(&q, 1, &dictionary, &dictSize);
    return r < 0 ? 0 : q.ret;
}

// Output staging a decode can need: a sequence of t input bytes writes at
// most 19 + 255 t bytes (the literal/match varints, lz4e_decompress.c:194-220,
// 316-336), so no input of csize bytes produces more than 263 * csize.  A
// caller's capacity beyond that is never touched, and the kernel still sees
// the caller's capacity (it steers the reference's bound checks).
static uint64_t decode_staging(int csize, int cap) {  // internal: not exported
    if (cap <= 0) return 0;
    const uint64_t most = 263ull * (uint64_t)std::max(csize, 0) + 64;
    return std::min<uint64_t>((uint64_t)cap, most);
}

// Test hook, armed only when LZ4E_TEST_FAULTS=1 is in the environment (a
// production caller cannot make the single calls fail through it): returns 0
// when armed, -1 when refused.
int lz4e_debug_coalescer_fault(int k) {
    const char* e = getenv("LZ4E_TEST_FAULTS");
    if (!e || strcmp(e, "1") != 0) return -1;
    g_coalescer_faults.store(k < 0 ? 0 : k);
    return 0;
}

}  // extern "C"

namespace {

uint64_t decode_staging_bytes(int csize, int cap) { return decode_staging(csize, cap); }

// lz4e_decompress_batch, optionally with dictionaries: block i's output is
// staged right after the last <= 64 KiB of its dictionary (the decoders read
// sources before the output from there), and the whole staging image goes
// H2D.
int decompress_batch_impl(const char* const* src, const int* csize, char* const* dst, const int* cap,
                          int* ret, int n, const char* const* dicts, const int* dict_sizes) {
    if (n <= 0) return 0;
    g_err.clear();
    for (int i = 0; i < n; ++i) ret[i] = -1;
    if (!gate().check()) return -1;
    const uint32_t R = (uint32_t)n;
    // [frames | descriptors | ret | outputs (each after its dictionary bytes)]
    std::vector<uint64_t> so(R), dso(R);
    std::vector<int32_t> dl(R, 0);
    uint64_t s = 0, d = 0;
    for (uint32_t i = 0; i < R; ++i) {
        so[i] = s;
        s += align16((uint64_t)std::max(csize[i], 0));
    }
    const size_t m_so = s, m_sl = m_so + align16(8ull * R), m_do = m_sl + align16(4ull * R),
                 m_dc = m_do + align16(8ull * R), m_dl = m_dc + align16(4ull * R),
                 m_rt = m_dl + align16(4ull * R), obase = m_rt + align16(4ull * R);
    for (uint32_t i = 0; i < R; ++i) {
        if (dicts && dicts[i] && dict_sizes[i] > 0) dl[i] = std::min(dict_sizes[i], 65536);
        dso[i] = obase + align16(d + (uint64_t)dl[i]);
        d = dso[i] - obase + align16(decode_staging(csize[i], cap[i]) + 64);
    }
    Lease ls;
    if (!ls.acquire()) return -1;
    CallCtx& c = *ls.c;
    if (!c.grow(obase + d)) return -1;
    uint8_t* hd = static_cast<uint8_t*>(c.h.p);
    for (uint32_t i = 0; i < R; ++i) {
        if (csize[i] > 0) std::memcpy(hd + so[i], src[i], (size_t)csize[i]);
        reinterpret_cast<uint64_t*>(hd + m_so)[i] = so[i];
        reinterpret_cast<int32_t*>(hd + m_sl)[i] = csize[i];
        reinterpret_cast<uint64_t*>(hd + m_do)[i] = dso[i];
        reinterpret_cast<int32_t*>(hd + m_dc)[i] = cap[i];
        reinterpret_cast<int32_t*>(hd + m_dl)[i] = dl[i];
        if (dl[i]) std::memcpy(hd + dso[i] - dl[i], dicts[i] + dict_sizes[i] - dl[i], (size_t)dl[i]);
    }
    uint8_t* dd = static_cast<uint8_t*>(c.d.p);
    lz4e::DecompressBatch a{dd,
                            reinterpret_cast<const uint64_t*>(dd + m_so),
                            reinterpret_cast<const int32_t*>(dd + m_sl),
                            dd,
                            reinterpret_cast<const uint64_t*>(dd + m_do),
                            reinterpret_cast<const int32_t*>(dd + m_dc),
                            reinterpret_cast<int32_t*>(dd + m_rt),
                            R,
                            (uint32_t)std::max(0, *std::max_element(cap, cap + n))};
    if (dicts) a.dict_len = reinterpret_cast<const int32_t*>(dd + m_dl);
    const uint64_t h2d = dicts ? obase + d : m_rt;  // the dictionaries live among the outputs
    bool ok = hip_ok(hipMemcpyAsync(dd, hd, h2d, hipMemcpyHostToDevice, c.stream), "H2D") &&
              hip_ok(lz4e::launch_decompress(a, c.stream), "decompress launch") &&
              hip_ok(copy_flat(c.h_dev, dd, m_rt, 4ull * R, c.stream), "copy-back ret");
    if (ok) {
        hipLaunchKernelGGL(copy_blocks_kernel, dim3(R), dim3(256), 0, c.stream, dd,
                           static_cast<uint8_t*>(c.h_dev),
                           reinterpret_cast<const uint64_t*>(dd + m_do),
                           reinterpret_cast<const int32_t*>(dd + m_rt), R);
        ok = hip_ok(hipGetLastError(), "copy-back data") &&
             hip_ok(hipStreamSynchronize(c.stream), "decompress sync");
    }
    if (!ok) return -1;
    for (uint32_t i = 0; i < R; ++i) ret[i] = reinterpret_cast<const int32_t*>(hd + m_rt)[i];
    std::string err;
    const int good = lz4e::decode_results(ret, R, err);
    if (good < 0) {
        set_err(err);
        return -1;
    }
    for (uint32_t i = 0; i < R; ++i)
        if (ret[i] > 0) std::memcpy(dst[i], hd + dso[i], (size_t)ret[i]);
    return good;
}

}  // namespace

extern "C" {

int lz4e_decompress_batch(const char* const* src, const int* csize, char* const* dst, const int* cap,
                          int* ret, int n) {
    return decompress_batch_impl(src, csize, dst, cap, ret, n, nullptr, nullptr);
}

// One coalesced batch of single decompress calls; a batch that fails as a
// whole (staging, launch, a watchdog on some block) is bisected, so that
// only the caller whose block failed sees the failure.
static void run_decompress_calls(DecompressCall** batch, size_t n) {
    std::vector<const char*> src(n);
    std::vector<char*> dst(n);
    std::vector<int> cs(n), cap(n), ret(n, -1);
    for (size_t i = 0; i < n; ++i) {
        src[i] = batch[i]->src;
        dst[i] = batch[i]->dst;
        cs[i] = batch[i]->csize;
        cap[i] = batch[i]->cap;
    }
    const int r = decompress_batch_impl(src.data(), cs.data(), dst.data(), cap.data(), ret.data(), (int)n,
                                        nullptr, nullptr);
    if (r < 0 && n > 1) {
        run_decompress_calls(batch, n / 2);
        run_decompress_calls(batch + n / 2, n - n / 2);
        return;
    }
    for (size_t i = 0; i < n; ++i) {
        // a failed call: the block's own value if it has one (the
        // watchdog's LZ4E_DECODE_ABORTED), else -1
        batch[i]->ret = r < 0 ? (ret[i] < 0 ? ret[i] : -1) : ret[i];
        batch[i]->err = g_err;
    }
}

int LZ4E_decompress_safe(const char* source, char* dest, int compressedSize, int maxDecompressedSize) {
    DecompressCall call{source, dest, compressedSize, maxDecompressedSize};
    decompress_calls().submit(
        &call,
        [](DecompressCall** batch, size_t n) {
            maybe_inject_fault();
            run_decompress_calls(batch, n);
        },
        [](DecompressCall* c, const std::string& why) {
            c->ret = -1;
            c->err = why;
        });
    g_err = call.err;
    return call.ret;
}

int lz4e_decompress_batch_dict(const char* const* src, const int* csize, char* const* dst,
                               const int* cap, const char* const* dicts, const int* dict_sizes,
                               int* ret, int n) {
    return decompress_batch_impl(src, csize, dst, cap, ret, n, dicts, dict_sizes);
}

int LZ4E_decompress_safe_usingDict(const char* source, char* dest, int compressedSize,
                                   int maxDecompressedSize, const char* dictStart, int dictSize) {
    int r = -1;
    char* d = dest;
    if (decompress_batch_impl(&source, &compressedSize, &d, &maxDecompressedSize, &r, 1, &dictStart,
                              &dictSize) < 0)
        return r < 0 ? r : -1;
    return r;
}

int lz4e_decompress_sg_batch(const char* const* src, const int* csize, struct bio_vec* const* dst,
                             struct bvec_iter* const* dstIter, int* ret, int n) {
    if (n <= 0) return 0;
    // decode into one host staging area, then scatter the successful blocks
    std::vector<uint64_t> at((size_t)n);
    uint64_t total = 0;
    std::vector<int> cap((size_t)n);
    for (int i = 0; i < n; ++i) {
        cap[i] = (int)std::min<uint32_t>(dstIter[i]->bi_size, 0x7FFFFFFFu);
        at[i] = total;
        total += decode_staging(csize[i], cap[i]) + 1;
    }
    std::unique_ptr<char[]> stage(new char[total + 1]);
    std::vector<char*> dp((size_t)n);
    for (int i = 0; i < n; ++i) dp[i] = stage.get() + at[i];
    const int good = lz4e_decompress_batch(src, csize, dp.data(), cap.data(), ret, n);
    if (good < 0) return -1;
    for (int i = 0; i < n; ++i) {
        if (ret[i] < 0) continue;
        sg_scatter(dst[i], *dstIter[i], reinterpret_cast<const uint8_t*>(dp[i]), (uint32_t)ret[i]);
        iter_advance(dst[i], dstIter[i], (uint32_t)ret[i]);
    }
    return good;
}

int lz4e_decompress_safe_sg(const char* source, struct bio_vec* dst, struct bvec_iter* dstIter,
                            int compressedSize) {
    int r = -1;
    if (lz4e_decompress_sg_batch(&source, &compressedSize, &dst, &dstIter, &r, 1) < 0)
        return r < 0 ? r : -1;
    return r;
}

int lz4e_compress_batch_dev(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                            const uint8_t* table_type, uint8_t* dst, const uint64_t* dst_off,
                            const uint32_t* dst_cap, int32_t* ret, uint32_t* aux, uint32_t nblocks,
                            uint32_t max_len, void* stream) {
    g_err.clear();
    lz4e::CompressBatch a{src, src_off, src_len, table_type, dst, dst_off, dst_cap, ret, aux,
                          nblocks, max_len};
    return hip_ok(lz4e::launch_compress(a, static_cast<hipStream_t>(stream)), "compress launch") ? 0
                                                                                                  : -1;
}

// Diagnostic (not part of include/lz4e.h): the compress kernel with per-block
// phase cycle counters, 8 x u64 per block into dbg.
int lz4e_debug_compress_stamped(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                                const uint8_t* table_type, uint8_t* dst, const uint64_t* dst_off,
                                const uint32_t* dst_cap, int32_t* ret, uint32_t nblocks,
                                uint32_t max_len, void* stream, uint64_t* dbg) {
    lz4e::CompressBatch a{src, src_off, src_len, table_type, dst, dst_off, dst_cap, ret, nullptr,
                          nblocks, max_len};
    return hip_ok(lz4e::launch_compress_stamped(a, static_cast<hipStream_t>(stream), dbg),
                  "compress launch")
               ? 0
               : -1;
}

// Diagnostic (not part of include/lz4e.h): clock_probe_kernel on `stream`
// (out: 3 x u64 in device memory: delta s_memtime, delta s_memrealtime, junk).
int lz4e_debug_clock_probe(void* stream, uint64_t* out, uint32_t iters) {
    hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), out, iters);
    return hip_ok(hipGetLastError(), "clock probe launch") ? 0 : -1;
}

// Diagnostic (not part of include/lz4e.h): the decompress kernels with a
// forced decoder (mode 0 auto, 1 one wave per block, 2 pipelined, 6 LDS form,
// 7 group, 9 group without the hand-over) and, when dbg is not null, the
// stamped build's per-block cycle counters (one-wave decoder and the blocks
// the group decoder hands over: 8 x u64 per block; pipelined: 22 x u64,
// tools/dstamps.py, tools/single_call_clock.py; dbg zeroed by the caller).
// The group decoder keeps no stamps of its own: in mode 7 a block it decodes
// to the end leaves its row zero, and mode 9 leaves every row zero.
int lz4e_debug_decompress_stamped(const uint8_t* src, const uint64_t* src_off, const int32_t* src_len,
                                  uint8_t* dst, const uint64_t* dst_off, const int32_t* dst_cap,
                                  int32_t* ret, uint32_t nblocks, void* stream, uint64_t* dbg,
                                  uint32_t max_cap, uint32_t mode) {
    if (mode != lz4e::kDecAuto && mode != lz4e::kDecWave && mode != lz4e::kDecPipe && mode != lz4e::kDecSmall &&
        mode != lz4e::kDecGroup && mode != lz4e::kDecGroupNoBail)
        return -1;
    lz4e::DecompressBatch a{src, src_off, src_len, dst, dst_off, dst_cap, ret, nblocks, max_cap, mode};
    const hipStream_t s = static_cast<hipStream_t>(stream);
    return hip_ok(dbg ? lz4e::launch_decompress_stamped(a, s, dbg) : lz4e::launch_decompress(a, s),
                  "decompress launch")
               ? 0
               : -1;
}

int lz4e_decompress_batch_dev2(const uint8_t* src, const uint64_t* src_off, const int32_t* src_len,
                               uint8_t* dst, const uint64_t* dst_off, const int32_t* dst_cap,
                               int32_t* ret, uint32_t nblocks, uint32_t max_cap, void* stream) {
    g_err.clear();
    lz4e::DecompressBatch a{src, src_off, src_len, dst, dst_off, dst_cap, ret, nblocks, max_cap};
    return hip_ok(lz4e::launch_decompress(a, static_cast<hipStream_t>(stream)), "decompress launch")
               ? 0
               : -1;
}

// The round-1 signature (no max_cap: the pipelined decoder for every block).
int lz4e_decompress_batch_dev(const uint8_t* src, const uint64_t* src_off, const int32_t* src_len,
                              uint8_t* dst, const uint64_t* dst_off, const int32_t* dst_cap,
                              int32_t* ret, uint32_t nblocks, void* stream) {
    return lz4e_decompress_batch_dev2(src, src_off, src_len, dst, dst_off, dst_cap, ret, nblocks, 0,
                                      stream);
}

int lz4e_compress_batch_dev_dict(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                                 const uint8_t* table_type, uint8_t* dst, const uint64_t* dst_off,
                                 const uint32_t* dst_cap, int32_t* ret, uint32_t* aux,
                                 uint32_t nblocks, uint32_t max_len, const uint32_t* dict_len,
                                 void* stream) {
    g_err.clear();
    lz4e::CompressBatch a{src, src_off, src_len, table_type, dst, dst_off, dst_cap, ret, aux,
                          nblocks, max_len, dict_len};
    return hip_ok(lz4e::launch_compress(a, static_cast<hipStream_t>(stream)), "compress launch") ? 0
                                                                                                  : -1;
}

// Diagnostic (not part of include/lz4e.h): lz4e_decompress_batch_dev_dict
// with a forced decoder (modes as lz4e_debug_decompress_stamped).
int lz4e_debug_decompress_dict(const uint8_t* src, const uint64_t* src_off, const int32_t* src_len,
                               uint8_t* dst, const uint64_t* dst_off, const int32_t* dst_cap, int32_t* ret,
                               uint32_t nblocks, uint32_t max_cap, const int32_t* dict_len, void* stream,
                               uint32_t mode) {
    if (mode != lz4e::kDecAuto && mode != lz4e::kDecWave && mode != lz4e::kDecPipe && mode != lz4e::kDecSmall &&
        mode != lz4e::kDecGroup && mode != lz4e::kDecGroupNoBail)
        return -1;
    g_err.clear();
    lz4e::DecompressBatch a{src, src_off, src_len, dst, dst_off, dst_cap, ret, nblocks, max_cap, mode, dict_len};
    return hip_ok(lz4e::launch_decompress(a, static_cast<hipStream_t>(stream)), "decompress launch")
               ? 0
               : -1;
}

int lz4e_decompress_batch_dev_dict(const uint8_t* src, const uint64_t* src_off, const int32_t* src_len,
                                   uint8_t* dst, const uint64_t* dst_off, const int32_t* dst_cap,
                                   int32_t* ret, uint32_t nblocks, uint32_t max_cap,
                                   const int32_t* dict_len, void* stream) {
    g_err.clear();
    lz4e::DecompressBatch a{src, src_off, src_len, dst, dst_off, dst_cap, ret, nblocks, max_cap,
                            0, dict_len};
    return hip_ok(lz4e::launch_decompress(a, static_cast<hipStream_t>(stream)), "decompress launch")
               ? 0
               : -1;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Chunk-layer write round trip (include/lz4e.h lz4e_chunk_write_batch)
// ---------------------------------------------------------------------------
namespace {

constexpr int kEIO = -5, kENOSPC = -28;

// Sub-batch size: a kSlots-th of the call, so that every sub-batch is in
// flight at once and the GPU sees the whole call as one batch launch would
// (a sub-batch's kernels take at least its slowest block's parse: 64 MiB of
// 256 KiB blocks is 256 blocks, a tenth of the chip), between these bounds
// of input bytes; at least kSubReqsMin requests.
constexpr uint64_t kSubBytesMin = 16ull << 20, kSubBytesMax = 256ull << 20;
constexpr uint32_t kSubReqsMin = 16384;
// Sub-batches in flight, each on its own stream, while the host gathers the
// next.
constexpr uint32_t kSlots = 4;

// Runs f(j) for j in [0, n) on up to 16 host threads when the bytes justify it.
// (Fresh threads per call: a persistent pool woken per job measured slower,
// fio4k end to end 16.3-17.9 vs 20.9-21.9 GiB/s, profiles/r06/chunk_pipeline/.)
template <class F>
void par_for(uint32_t n, uint64_t bytes, F f) {
    const uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
    const uint32_t T = bytes < (4ull << 20) ? 1u : std::min({16u, hw, n});
    if (T <= 1) {
        for (uint32_t j = 0; j < n; ++j) f(j);
        return;
    }
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            for (uint32_t j = t; j < n; j += T) f(j);
        });
    for (auto& x : th) x.join();
}

// Per-sub-batch metadata (device + pinned host), one entry per request.
struct ChunkMeta {
    size_t in_off, in_len, ttype, fr_off, fr_cap, out_off, out_cap, ret, dret, total;
    explicit ChunkMeta(uint32_t R) {
        size_t o = 0;
        in_off = o;  o += align16(8ull * R);
        in_len = o;  o += align16(4ull * R);
        ttype = o;   o += align16(1ull * R);
        fr_off = o;  o += align16(8ull * R);
        fr_cap = o;  o += align16(4ull * R);
        out_off = o; o += align16(8ull * R);
        out_cap = o; o += align16(4ull * R);
        ret = o;     o += align16(4ull * R);
        dret = o;    o += align16(4ull * R);
        total = o;
    }
};

struct ChunkSlot {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    HostBuf h_data, h_meta;
    DevBuf d_data, d_meta;
    void* h_dev = nullptr;  // h_data as the device sees it
    bool busy = false;
    bool want_frames = false;
    std::vector<uint32_t> req;        // request index per entry
    std::vector<uint64_t> fr, out;    // frame / output offsets in the data buffer
    uint64_t in_bytes = 0, fr_bytes = 0, out_bytes = 0;
    size_t meta_ret = 0, meta_dret = 0;
    // LZ4E_CHUNK_PROF=2: timing events (before H2D, after H2D, compress,
    // decompress, D2H) and host times of the sub-batch's phases
    hipEvent_t pev[5] = {};
    uint32_t sb = 0;
    double t_g0 = 0, t_g1 = 0, t_sub = 0;
};

struct ChunkCtx {
    std::mutex mu;
    ChunkSlot slot[kSlots];
    bool ready = false;
    bool init() {
        if (ready) return true;
        // Half of the slots on the high-priority stream pool: streams of one
        // priority share few hardware queues (two slots per queue were seen
        // serialising their kernels), the other pool brings its own.
        int lo = 0, hi = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = hi = 0;
        for (uint32_t i = 0; i < kSlots; ++i) {
            ChunkSlot& s = slot[i];
            if (!hip_ok(hipStreamCreateWithPriority(&s.stream, hipStreamNonBlocking,
                                                    (i & 1) ? hi : lo),
                        "hipStreamCreate") ||
                !hip_ok(hipEventCreateWithFlags(&s.done, hipEventDisableTiming), "hipEventCreate"))
                return false;
        }
        ready = true;
        return true;
    }
};

ChunkCtx& chunk_ctx() {
    static ChunkCtx c;
    return c;
}

// Waits for a slot's sub-batch and hands its results to the requests.
// LZ4E_CHUNK_PROF=1: per-phase host times of the pipeline on stderr.
double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}
struct ChunkProf {
    bool on = getenv("LZ4E_CHUNK_PROF") != nullptr;
    bool tl = on && getenv("LZ4E_CHUNK_PROF")[0] == '2';  // per-sub-batch timeline
    double t0 = 0;
    double wait = 0, out = 0, gather = 0, submit = 0;
};

// vec_count of the bio the reference completes for one successful WRITE
// (lz4e_bdev/lz4e_stats.c:47 adds bio->bi_vcnt): after the round trip the
// request's bio is reset and re-pointed at the chunk's contiguous src buffer
// (lz4e_req.c:191-197, lz4e_add_buf_to_bio :115-142), one bio_add_page per
// page piece.  bio_add_page merges a piece into the previous bio_vec when it
// starts where that one ends in memory (bvec_try_merge_page), which every
// piece of a contiguous buffer does -- in this userspace model
// page_address(p) == (char *)p, so contiguous virtual memory is contiguous
// pages: the pieces after the first all merge.
uint64_t bio_vcnt_of_buffer(const char* data, uint32_t len) {
    uint64_t vcnt = 0;
    const char* prev_end = nullptr;
    uint32_t off = (uint32_t)(reinterpret_cast<uintptr_t>(data) & (LZ4E_PAGE_SIZE - 1));
    uint32_t piece = std::min<uint32_t>(len, LZ4E_PAGE_SIZE - off);
    while (len) {
        if (data != prev_end) vcnt++;  // a new bio_vec unless it merges
        prev_end = data + piece;
        data += piece;
        len -= piece;
        piece = std::min<uint32_t>(len, LZ4E_PAGE_SIZE);
    }
    return vcnt;
}

// Debug hook (tests only, not part of include/lz4e.h): the pipeline fails
// after this many sub-batches have been submitted (-1: never).
std::atomic<int> g_chunk_fault_after{-1};

// Debug hook (tests only): sub-batches of this many input bytes instead of
// the call-sized ones (0: off), so that a small call cycles the slots.
std::atomic<uint64_t> g_chunk_sub_bytes{0};

// Launch order override per direction (compress, decompress): -1 default.
std::atomic<int> g_order_override[2] = {{-1}, {-1}};

// Waits for a slot's sub-batch and hands its results to the requests;
// counts into `st` (this call's stats, added to the caller's on success).
bool chunk_finish(ChunkSlot& s, struct lz4e_chunk_request* reqs, struct lz4e_chunk_stats& st,
                  int& good, ChunkProf& pr) {
    if (!s.busy) return true;
    s.busy = false;
    double t0 = pr.on ? now_ms() : 0;
    if (!hip_ok(hipEventSynchronize(s.done), "chunk sync")) return false;
    double t1 = pr.on ? now_ms() : 0;
    pr.wait += t1 - t0;
    const uint8_t* hd = static_cast<const uint8_t*>(s.h_data.p);
    const uint8_t* hm = static_cast<const uint8_t*>(s.h_meta.p);
    const int32_t* ret = reinterpret_cast<const int32_t*>(hm + s.meta_ret);
    const int32_t* dret = reinterpret_cast<const int32_t*>(hm + s.meta_dret);
    const uint32_t R = (uint32_t)s.req.size();
    {
        std::string err;
        if (lz4e::decode_results(dret, R, err) < 0) {
            set_err(err);
            return false;
        }
    }
    par_for(R, s.out_bytes, [&](uint32_t j) {
        lz4e_chunk_request& q = reqs[s.req[j]];
        const int32_t len = (int32_t)q.srcIter->bi_size;
        q.comp_size = ret[j] > 0 ? ret[j] : 0;
        if (ret[j] <= 0 || dret[j] != len) {  // lz4e_chunk.c:110-113, 127-133
            q.status = kEIO;
            return;
        }
        if (q.frame) {
            if (q.frame_cap < ret[j]) {
                q.status = kENOSPC;
                return;
            }
            std::memcpy(q.frame, hd + s.fr[j], (size_t)ret[j]);
        }
        if (len > 0) std::memcpy(q.data, hd + s.out[j], (size_t)len);
        q.status = 0;
    });
    if (pr.on) pr.out += now_ms() - t1;
    if (pr.tl && s.pev[4]) {
        float g[4] = {0, 0, 0, 0};
        for (int q = 0; q < 4; ++q) (void)hipEventElapsedTime(&g[q], s.pev[q], s.pev[q + 1]);
        fprintf(stderr, "  sb %u: %u reqs, gather %.2f-%.2f, submitted %.2f, waited %.2f-%.2f, copied out by %.2f;"
                " gpu h2d %.2f compress %.2f decompress %.2f d2h %.2f ms\n", s.sb, R, s.t_g0 - pr.t0,
                s.t_g1 - pr.t0, s.t_sub - pr.t0, t0 - pr.t0, t1 - pr.t0, now_ms() - pr.t0, g[0], g[1],
                g[2], g[3]);
    }
    // Stats as the reference keeps them: lz4e_stats_update runs only in
    // lz4e_end_io (lz4e_bdev/lz4e_req.c:231-246), i.e. for a WRITE whose
    // round trip succeeded and whose bio was submitted; a request failing in
    // lz4e_write_req_init (compress or decompress failure, -EIO) returns
    // through lz4e_dev.c:187-202 without touching any counter.  reqs_failed
    // counts completed bios the underlying device failed (lz4e_stats.c:43-45):
    // there is no underlying device here, so it stays 0.
    for (uint32_t j = 0; j < R; ++j) {
        const lz4e_chunk_request& q = reqs[s.req[j]];
        if (q.status != 0) continue;
        good++;
        st.reqs_total++;
        st.data_in_bytes += q.srcIter->bi_size;
        st.vec_count += bio_vcnt_of_buffer(q.data, q.srcIter->bi_size);
        st.frame_bytes += (uint64_t)q.comp_size;
    }
    s.req.clear();
    return true;
}

// After a failure: wait out every slot still in flight (its kernels and
// copies still target the slot's buffers) and forget its requests, so that
// nothing of this call leaks into the next one.
void chunk_drain(ChunkCtx& cc) {
    for (uint32_t t = 0; t < kSlots; ++t) {
        ChunkSlot& s = cc.slot[t];
        // (the failure may have come before `done` was recorded)
        if (s.busy) (void)hipStreamSynchronize(s.stream);
        s.busy = false;
        s.req.clear();
    }
}

}  // namespace

namespace lz4e {
int launch_order_mode(bool compress) {
    const int o = g_order_override[compress ? 0 : 1].load();
    if (o >= kOrderNever && o <= kOrderAlways) return o;
    const char* e = getenv(compress ? "LZ4E_COMPRESS_ORDER" : "LZ4E_DECOMPRESS_ORDER");
    return (e && e[0] == '0') ? kOrderNever : kOrderAuto;
}
}  // namespace lz4e

extern "C" {

void lz4e_debug_chunk_fault_after(int subbatches) { g_chunk_fault_after.store(subbatches); }
void lz4e_debug_chunk_sub_bytes(uint64_t bytes) { g_chunk_sub_bytes.store(bytes); }

// Diagnostic: launch order policy of the device batches (lz4e_order.h) for
// compress / decompress: -1 default (environment), 0 block order, 1 heavy
// first for large batches, 2 heavy first always.  Results never depend on it.
void lz4e_debug_set_launch_order(int compress_mode, int decompress_mode) {
    g_order_override[0].store(compress_mode);
    g_order_override[1].store(decompress_mode);
}

int lz4e_chunk_write_batch(struct lz4e_chunk_request* reqs, int n, struct lz4e_chunk_stats* stats) {
    if (n <= 0) return 0;
    auto fail_all = [&]() {
        for (int i = 0; i < n; ++i) {
            reqs[i].comp_size = 0;
            reqs[i].status = kEIO;
        }
        return -1;
    };
    fail_all();
    g_err.clear();
    if (!gate().check()) return -1;
    ChunkCtx& cc = chunk_ctx();
    std::lock_guard<std::mutex> lk(cc.mu);
    if (!cc.init()) return -1;
    chunk_drain(cc);  // nothing of an earlier call may still be pending

    struct lz4e_chunk_stats st = {0, 0, 0, 0, 0};
    int good = 0;
    uint32_t i = 0, k = 0;
    const uint32_t N = (uint32_t)n;
    ChunkProf pr;
    const double tstart = pr.on ? now_ms() : 0;
    pr.t0 = tstart;
    auto abort = [&]() {
        chunk_drain(cc);
        return fail_all();
    };
    uint64_t total = 0;
    for (uint32_t r = 0; r < N; ++r) total += reqs[r].srcIter->bi_size;
    const uint64_t forced = g_chunk_sub_bytes.load();
    const uint64_t sub_bytes =
        forced ? forced : std::min(kSubBytesMax, std::max(kSubBytesMin, (total + kSlots - 1) / kSlots));
    const uint32_t sub_reqs = forced ? kSubReqsMin : std::max(kSubReqsMin, (N + kSlots - 1) / kSlots);
    while (i < N) {
        ChunkSlot& s = cc.slot[k % kSlots];
        if (!chunk_finish(s, reqs, st, good, pr)) return abort();
        const int fa = g_chunk_fault_after.load();
        if (fa >= 0 && k >= (uint32_t)fa) {
            set_err("lz4e: injected pipeline fault");
            return abort();
        }
        // ---- form the sub-batch: requests [i, e) ----
        s.req.clear();
        s.fr.clear();
        s.out.clear();
        std::vector<uint64_t> in;
        std::vector<uint8_t> tt;
        uint64_t ib = 0, fb = 0, ob = 0;
        uint32_t max_len = 0;
        bool frames = false;
        for (; i < N && s.req.size() < sub_reqs && (s.req.empty() || ib < sub_bytes); ++i) {
            const lz4e_chunk_request& q = reqs[i];
            const uint32_t len = q.srcIter->bi_size;
            int t = LZ4E_TABLE_BYU16;
            // compress returns 0 -> -EIO, no stats (lz4e_dev.c:187-202)
            if (len > LZ4E_MAX_INPUT_SIZE) continue;  // lz4e_compress.c:245-248
            if (len >= 13 && (t = table_type_of(q.src, q.srcIter)) == 0) continue;  // :274-277
            s.req.push_back(i);
            in.push_back(ib);
            tt.push_back((uint8_t)t);
            ib += align16(len);
            s.fr.push_back(fb);
            fb += align16((uint64_t)bound_of(len) + 64);
            s.out.push_back(ob);
            ob += align16((uint64_t)len + 64);
            max_len = std::max(max_len, len);
            frames |= q.frame != nullptr;
        }
        const uint32_t R = (uint32_t)s.req.size();
        if (R == 0) continue;
        for (uint32_t j = 0; j < R; ++j) {  // one data buffer: [inputs | frames | outputs]
            s.fr[j] += ib;
            s.out[j] += ib + fb;
        }
        s.in_bytes = ib;
        s.fr_bytes = fb;
        s.out_bytes = ob;
        s.want_frames = frames;
        const ChunkMeta m(R);
        const uint64_t total = ib + fb + ob;
        if (!s.h_data.ensure(total) || !s.d_data.ensure(total) || !s.h_meta.ensure(m.total) ||
            !s.d_meta.ensure(m.total) ||
            !hip_ok(hipHostGetDevicePointer(&s.h_dev, s.h_data.p, 0), "hipHostGetDevicePointer"))
            return abort();
        uint8_t* hd = static_cast<uint8_t*>(s.h_data.p);
        uint8_t* hm = static_cast<uint8_t*>(s.h_meta.p);
        // ---- gather (overlaps the other slots' GPU work) ----
        const double tg = pr.on ? now_ms() : 0;
        par_for(R, ib, [&](uint32_t j) {
            const lz4e_chunk_request& q = reqs[s.req[j]];
            sg_gather(q.src, *q.srcIter, hd + in[j], q.srcIter->bi_size);
        });
        const double ts = pr.on ? now_ms() : 0;
        pr.gather += ts - tg;
        if (pr.tl) {
            for (hipEvent_t& ev : s.pev)
                if (!ev && hipEventCreate(&ev) != hipSuccess) ev = nullptr;
            s.sb = k;
            s.t_g0 = tg;
            s.t_g1 = ts;
        }
        auto mark = [&](int q) {
            if (pr.tl && s.pev[q]) (void)hipEventRecord(s.pev[q], s.stream);
        };
        for (uint32_t j = 0; j < R; ++j) {
            const uint32_t len = reqs[s.req[j]].srcIter->bi_size;
            reinterpret_cast<uint64_t*>(hm + m.in_off)[j] = in[j];
            reinterpret_cast<uint32_t*>(hm + m.in_len)[j] = len;
            (hm + m.ttype)[j] = tt[j];
            reinterpret_cast<uint64_t*>(hm + m.fr_off)[j] = s.fr[j];
            reinterpret_cast<uint32_t*>(hm + m.fr_cap)[j] = bound_of(len);  // dst_buf.buf_size
            reinterpret_cast<uint64_t*>(hm + m.out_off)[j] = s.out[j];
            reinterpret_cast<int32_t*>(hm + m.out_cap)[j] = (int32_t)len;  // src_buf.buf_size
        }
        s.meta_ret = m.ret;
        s.meta_dret = m.dret;
        uint8_t* dd = static_cast<uint8_t*>(s.d_data.p);
        uint8_t* dm = static_cast<uint8_t*>(s.d_meta.p);
        const lz4e::CompressBatch ca{dd,
                                     reinterpret_cast<const uint64_t*>(dm + m.in_off),
                                     reinterpret_cast<const uint32_t*>(dm + m.in_len),
                                     dm + m.ttype,
                                     dd,
                                     reinterpret_cast<const uint64_t*>(dm + m.fr_off),
                                     reinterpret_cast<const uint32_t*>(dm + m.fr_cap),
                                     reinterpret_cast<int32_t*>(dm + m.ret),
                                     nullptr,
                                     R,
                                     max_len};
        // the frame sizes feed the decoder straight from HBM (no host trip)
        const lz4e::DecompressBatch da{dd,
                                       reinterpret_cast<const uint64_t*>(dm + m.fr_off),
                                       reinterpret_cast<const int32_t*>(dm + m.ret),
                                       dd,
                                       reinterpret_cast<const uint64_t*>(dm + m.out_off),
                                       reinterpret_cast<const int32_t*>(dm + m.out_cap),
                                       reinterpret_cast<int32_t*>(dm + m.dret),
                                       R,
                                       max_len};
        // from here on the slot has work in flight: a failure must drain it
        s.busy = true;
        mark(0);
        if (!hip_ok(hipMemcpyAsync(dd, hd, ib, hipMemcpyHostToDevice, s.stream), "H2D data") ||
            !hip_ok(hipMemcpyAsync(dm, hm, m.ret, hipMemcpyHostToDevice, s.stream), "H2D meta"))
            return abort();
        mark(1);
        if (!hip_ok(lz4e::launch_compress(ca, s.stream), "compress launch")) return abort();
        mark(2);
        if (!hip_ok(lz4e::launch_decompress(da, s.stream), "decompress launch")) return abort();
        mark(3);
        if (!hip_ok(hipMemcpyAsync(hm + m.ret, dm + m.ret, m.total - m.ret, hipMemcpyDeviceToHost,
                                   s.stream), "D2H meta") ||
            (frames && !hip_ok(copy_flat(s.h_dev, dd, ib, fb, s.stream), "D2H frames")) ||
            !hip_ok(copy_flat(s.h_dev, dd, ib + fb, ob, s.stream), "D2H data"))
            return abort();
        mark(4);
        if (!hip_ok(hipEventRecord(s.done, s.stream), "event record")) return abort();
        s.t_sub = pr.on ? now_ms() : 0;
        k++;
        if (pr.on) pr.submit += now_ms() - ts;
    }
    for (uint32_t t = 0; t < kSlots; ++t)
        if (!chunk_finish(cc.slot[(k + t) % kSlots], reqs, st, good, pr)) return abort();
    if (pr.on)
        fprintf(stderr, "lz4e chunk: %u sub-batches, total %.2f ms: gpu wait %.2f, copy-out %.2f, "
                "gather %.2f, submit %.2f\n", k, now_ms() - tstart, pr.wait, pr.out, pr.gather,
                pr.submit);
    if (stats) {
        stats->reqs_total += st.reqs_total;
        stats->reqs_failed += st.reqs_failed;
        stats->vec_count += st.vec_count;
        stats->data_in_bytes += st.data_in_bytes;
        stats->frame_bytes += st.frame_bytes;
    }
    return good;
}

}  // extern "C"
