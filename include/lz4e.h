/*
 * lz4e.h -- C ABI of the MI355X-native LZ4E scatter-gather block codec.
 *
 * Drop-in boundary for the reference's two exported symbols:
 *   LZ4E_compress_default  <- /root/reference/lz4e/include/lz4e.h:47-48
 *                             (definition lz4e/lz4e_compress.c:563-569)
 *   LZ4E_decompress_safe   <- /root/reference/lz4e/include/lz4e.h:50-51
 *                             (definition lz4e/lz4e_decompress.c:462-470)
 * plus the sizing macros of lz4e/include/lz4e.h:9-28,53-55 and the
 * LZ4E_stream_t work-memory layout of lz4e/include/lz4e.h:33-45.
 *
 * Both single-call entry points run on the GPU (gfx950): the host shim
 * gathers the bio_vec segments into pinned staging, copies them to HBM,
 * launches the hand-written HIP kernel and scatters the frame back into the
 * destination bio_vecs.  Like the reference they are reentrant.  Concurrent
 * callers on one device are coalesced: a caller queues its request, and a
 * caller that finds fewer than 4 batches in flight runs every queued
 * request of that device (its own included) as one batch launch on its own
 * thread and leased HIP stream while the others wait for their result; a
 * lone caller runs at once.  A batch that fails as a whole is rerun call by
 * call, so one caller's failure is not another's.  There is no CPU codec
 * behind these symbols; when no GPU is usable they fail (compress returns
 * 0, decompress returns a negative value) and lz4e_last_error() says why.
 *
 * The batched lz4e_*_batch_* entry points are the throughput path: many
 * independent blocks per launch, device-resident buffers, caller's stream.
 *
 * Plain C, no torch types.  All sizes are bytes.
 */
#ifndef LZ4E_AMD_H
#define LZ4E_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* Userspace view of the kernel block-layer SG types (doc/API.md:47-82).     */
/* ------------------------------------------------------------------------ */
#ifndef LZ4E_HAVE_KERNEL_BVEC
/*
 * A page frame.  Userspace model: page_address(p) == (char *)p and a
 * multi-page bvec covers physically contiguous pages, so byte k of a bvec
 * lives at (char *)bv_page + bv_offset + k.
 */
struct page;

struct bio_vec {
	struct page *bv_page;   /* first page the segment lives on        */
	unsigned int bv_len;    /* segment length in bytes                */
	unsigned int bv_offset; /* offset of the segment inside bv_page   */
};

struct bvec_iter {
	uint64_t bi_sector;        /* unused by the codec                  */
	unsigned int bi_size;      /* residual bytes                       */
	unsigned int bi_idx;       /* current index into the bio_vec array */
	unsigned int bi_bvec_done; /* bytes done in the current bio_vec    */
};
#endif

#define LZ4E_PAGE_SIZE 4096u
#ifndef BIO_MAX_VECS
#define BIO_MAX_VECS 256
#endif

/* ------------------------------------------------------------------------ */
/* Sizing macros (values fixed by the reference: lz4e/include/lz4e.h)        */
/* ------------------------------------------------------------------------ */
#define LZ4E_NAME "lz4e"
#define LZ4E_ACCELERATION_DEFAULT 1
#define LZ4E_MEMORY_USAGE 14
#define LZ4E_HASHLOG (LZ4E_MEMORY_USAGE - 2)
#define LZ4E_HASH_SIZE_U32 (1 << LZ4E_HASHLOG)
#define LZ4E_HASH_SIZE_U64 (LZ4E_HASH_SIZE_U32 >> 1)
#define LZ4E_BV_ITER_SIZE_U64 (BIO_MAX_VECS >> 1)
#define LZ4E_STREAMSIZE_U64 (LZ4E_HASH_SIZE_U64 + LZ4E_BV_ITER_SIZE_U64 + 4)
#define LZ4E_STREAMSIZE (LZ4E_STREAMSIZE_U64 * sizeof(unsigned long long))
#define LZ4E_MEM_COMPRESS LZ4E_STREAMSIZE /* 17440 bytes */

#define LZ4E_MAX_INPUT_SIZE 0x7E000000 /* 2 113 929 216 bytes */
#define LZ4E_COMPRESSBOUND(isize)                                        \
	((unsigned int)(isize) > (unsigned int)LZ4E_MAX_INPUT_SIZE ? 0 :  \
	 (isize) + ((isize) / 255) + 16)

#ifndef LZ4E_DISTANCE_MAX
#define LZ4E_DISTANCE_MAX 65535
#endif

/* Work-memory layout (same size/shape as the reference's LZ4E_stream_t). */
typedef struct {
	uint32_t bvIterSize[BIO_MAX_VECS];
	uint32_t hashTable[LZ4E_HASH_SIZE_U32];
	uint32_t currentOffset;
	uint32_t initCheck;
	const uint8_t *dictionary;
	uint8_t *bufferStart;
	uint32_t dictSize;
} LZ4E_stream_t_internal;

typedef union {
	unsigned long long table[LZ4E_STREAMSIZE_U64];
	LZ4E_stream_t_internal internal_donotuse;
} LZ4E_stream_t;

/* Hash-table address classes chosen from the SG layout
 * (lz4e/include/lz4e_defs.h:689, rules lz4e/lz4e_compress.c:184-211). */
#define LZ4E_TABLE_BYU16 1
#define LZ4E_TABLE_BYU32 3
#define LZ4E_TABLE_BYU64 7

/* ------------------------------------------------------------------------ */
/* Reference entry points (drop-in).                                         */
/* ------------------------------------------------------------------------ */

/*
 * Compress srcIter->bi_size bytes read through the bio_vec list `src`
 * (starting at *srcIter) into one raw LZ4 block written through `dst`
 * starting at *dstIter; dstIter->bi_size is the output capacity.
 * Returns the block size, or 0 on failure (input too large, more than
 * BIO_MAX_VECS segments, output capacity too small, or no usable GPU).
 * On success *dstIter is advanced by (ret - last literal run) and *srcIter
 * to the last position the match finder visited, like the reference.
 * `wrkmem` must point to LZ4E_MEM_COMPRESS bytes; it is zeroed on entry
 * (the match finder's state itself lives in GPU LDS).
 * Replaces lz4e/lz4e_compress.c:563.
 */
int LZ4E_compress_default(const struct bio_vec *src, struct bio_vec *dst,
			  struct bvec_iter *srcIter, struct bvec_iter *dstIter,
			  void *wrkmem);

/*
 * Safe full-block decode of `compressedSize` bytes at `source` into at most
 * `maxDecompressedSize` bytes at `dest` (contiguous host buffers).
 * Returns the number of bytes written, or -(input position of the error)-1.
 * Replaces lz4e/lz4e_decompress.c:462 (and, with the same signature, the
 * kernel LZ4_decompress_safe call at lz4e_bdev/lz4e_chunk.c:125).
 */
int LZ4E_decompress_safe(const char *source, char *dest, int compressedSize,
			 int maxDecompressedSize);

/* ------------------------------------------------------------------------ */
/* Extensions                                                                */
/* ------------------------------------------------------------------------ */

/* Table class of an SG source (1/3/7), or 0 when it spans more than
 * BIO_MAX_VECS segments.  Only meaningful for bi_size >= 13 (smaller inputs
 * never consult the table).  Rules of lz4e/lz4e_compress.c:184-211. */
int lz4e_sg_table_type(const struct bio_vec *src, const struct bvec_iter *it);

/* Human-readable reason for the last failure on this thread ("" if none). */
const char *lz4e_last_error(void);

/* 1 if a gfx950 device is usable by the library, else 0. */
int lz4e_gpu_available(void);

/*
 * One SG compress request of a host batch.  Same meaning as the arguments
 * of LZ4E_compress_default; `ret` receives its return value.  The
 * iterators are updated exactly like the single-call form.
 */
struct lz4e_sg_request {
	const struct bio_vec *src;
	struct bio_vec *dst;
	struct bvec_iter *srcIter;
	struct bvec_iter *dstIter;
	int ret;
};

/* Compress `n` independent SG requests with one gather, one H2D copy, one
 * kernel launch, one D2H copy and one scatter.  Returns the number of
 * requests that succeeded (ret > 0), or -1 when no GPU is usable. */
int lz4e_compress_sg_batch(struct lz4e_sg_request *reqs, int n);

/* Decompress `n` independent contiguous host blocks (src[i], csize[i]) into
 * (dst[i], cap[i]); ret[i] receives LZ4E_decompress_safe's value.  Returns
 * the number of blocks with ret >= 0, or -1 when no GPU is usable. */
int lz4e_decompress_batch(const char *const *src, const int *csize,
			  char *const *dst, const int *cap, int *ret, int n);

/*
 * Device-resident batch compress (the throughput path).  All pointers are
 * device (HBM) pointers; `stream` is a hipStream_t (NULL = default stream).
 * Block i reads src_len[i] bytes at src + src_off[i], uses table class
 * table_type[i] (1/3/7, from lz4e_sg_table_type of its SG layout) and writes
 * at most dst_cap[i] bytes at dst + dst_off[i]; ret[i] receives the block
 * size or 0.  `aux` (nullable, 2 words per block) receives
 * {final src position, last literal run} for iterator post-state.
 * `max_len` bounds src_len[] (it selects the LDS staging mode).  Batches
 * of 1024+ blocks of 16 KiB+ are launched heaviest block first (a sampled
 * weight per block and a counting sort on `stream`, scratch from the
 * stream-ordered pool: hipMallocAsync / hipFreeAsync); the bytes written
 * never depend on it.
 * Returns 0 on a successful launch, else a negative error.
 */
int lz4e_compress_batch_dev(const uint8_t *src, const uint64_t *src_off,
			    const uint32_t *src_len, const uint8_t *table_type,
			    uint8_t *dst, const uint64_t *dst_off,
			    const uint32_t *dst_cap, int32_t *ret, uint32_t *aux,
			    uint32_t nblocks, uint32_t max_len, void *stream);

/*
 * Device-resident batch decompress.  Block i decodes src_len[i] bytes at
 * src + src_off[i] into at most dst_cap[i] bytes at dst + dst_off[i];
 * ret[i] receives LZ4E_decompress_safe's return value.  `max_cap` bounds
 * dst_cap[] (0 = unknown) and selects the decoder: 16-128 KiB (or unknown),
 * and any batch of at most 1024 blocks, the pipelined one (one parser wave
 * and three copier waves per block); <= 4608 bytes the group decoder for
 * batches of >= 16384 blocks (one block per group of 8 lanes, blocks of
 * short sequences handed to the one-wave decoder), the one-wave decoder's LDS
 * form for 1025-3328 blocks; otherwise one wave per block.  All return identical values and bytes.  Pipelined batches of more
 * than 1536 blocks are launched in decreasing compressed-size order (as for
 * compress, on `stream`).  LZ4E_DECOMPRESS_MODE=w|p|s|g (one-wave,
 * pipelined, LDS form, group) overrides the choice for experiments.
 * Returns 0 on a successful launch, else a negative error.
 *
 * ret[i] == LZ4E_DECODE_ABORTED: the pipelined decoder's watchdog fired
 * (one of its waves waited ~1 s while nothing it depends on moved: a broken
 * invariant of the decoder, never a property of the input).  The reference
 * has no such outcome (lz4e_decompress.c:449-459 returns bytes written or
 * -(ip - src) - 1); the host entry points turn it into a failed call:
 * lz4e_decompress_batch / _dict / _sg_batch return -1, LZ4E_decompress_safe
 * (and _usingDict / lz4e_decompress_safe_sg) return LZ4E_DECODE_ABORTED,
 * lz4e_chunk_write_batch returns -1, each with lz4e_last_error() saying so.
 * (A genuine -(ip - src) - 1 equals it only for ip = 2^31 - 1, an input the
 * 0x7E000000-byte block limit cannot produce.)
 *
 * lz4e_decompress_batch_dev2 is the current form; lz4e_decompress_batch_dev
 * keeps the round-1 signature (no max_cap: pipelined decoder throughout).
 */
#define LZ4E_DECODE_ABORTED (-2147483647 - 1)
int lz4e_decompress_batch_dev2(const uint8_t *src, const uint64_t *src_off,
			       const int32_t *src_len, uint8_t *dst,
			       const uint64_t *dst_off, const int32_t *dst_cap,
			       int32_t *ret, uint32_t nblocks, uint32_t max_cap,
			       void *stream);
int lz4e_decompress_batch_dev(const uint8_t *src, const uint64_t *src_off,
			      const int32_t *src_len, uint8_t *dst,
			      const uint64_t *dst_off, const int32_t *dst_cap,
			      int32_t *ret, uint32_t nblocks, void *stream);

/*
 * Dictionary mode.  The reference stubs its dictionary
 * path out (lz4e/lz4e_compress.c:250-266, 315-324, 393-419, 472-482; the
 * dictionary fields of LZ4E_stream_t, lz4e/include/lz4e.h:36-40) and its
 * exported decoder never instantiates the extDict branches
 * (lz4e/lz4e_decompress.c:299-302, 339-378, 462-469).  This is the LZ4E
 * extension built on them; no reference run pins its frames (parity
 * unpinned), the decoder restates those branches exactly.
 *
 * LZ4E_compress_usingDict: LZ4E_compress_default's contract (bio_vec source
 * and destination, iterators, wrkmem) compressing against the last <= 64 KiB
 * of `dictionary` (ignored under 8 bytes): the hash table is preloaded the
 * way LZ4_loadDict does it (every third dictionary position, in order), the
 * table class is byU32 whatever the SG layout, and matches may start in the
 * dictionary (offsets <= LZ4E_DISTANCE_MAX) and run on into the block.  The
 * >256-segment and size limits of LZ4E_compress_default still return 0.
 *
 * LZ4E_decompress_safe_usingDict: LZ4E_decompress_safe with a dictionary that
 * logically precedes `dest` (extDict): match bytes before `dest` read the
 * dictionary's end; with dictSize < 64 KiB an offset reaching before the
 * dictionary fails (-(ip - src) - 1, :299-302).  dictSize 0 is
 * LZ4E_decompress_safe.  Frames of LZ4E_compress_usingDict decode with the
 * same dictionary, so do those of any LZ4 dictionary compressor.
 */
int LZ4E_compress_usingDict(const struct bio_vec *src, struct bio_vec *dst,
			    struct bvec_iter *srcIter, struct bvec_iter *dstIter,
			    void *wrkmem, const char *dictionary, int dictSize);
int LZ4E_decompress_safe_usingDict(const char *source, char *dest,
				   int compressedSize, int maxDecompressedSize,
				   const char *dictStart, int dictSize);

/* Batch forms: request i with dictionary (dicts[i], dict_sizes[i]) (NULL or
 * size 0: none, still byU32 on the compress side); returns as the
 * dictionary-less batch calls. */
int lz4e_compress_sg_batch_dict(struct lz4e_sg_request *reqs, int n,
				const char *const *dicts, const int *dict_sizes);
int lz4e_decompress_batch_dict(const char *const *src, const int *csize,
			       char *const *dst, const int *cap,
			       const char *const *dicts, const int *dict_sizes,
			       int *ret, int n);

/* Device-resident dictionary batches: block i's dictionary is the
 * dict_len[i] bytes right before its input (compress: src + src_off[i],
 * table_type[i] must be 3 = byU32; at most 64 KiB used) or right before its
 * output (decompress: dst + dst_off[i] -- e.g. the previous block of the
 * same stream decoded in place, so a stream decodes block after block while
 * many streams decode in parallel). */
int lz4e_compress_batch_dev_dict(const uint8_t *src, const uint64_t *src_off,
				 const uint32_t *src_len, const uint8_t *table_type,
				 uint8_t *dst, const uint64_t *dst_off,
				 const uint32_t *dst_cap, int32_t *ret, uint32_t *aux,
				 uint32_t nblocks, uint32_t max_len,
				 const uint32_t *dict_len, void *stream);
int lz4e_decompress_batch_dev_dict(const uint8_t *src, const uint64_t *src_off,
				   const int32_t *src_len, uint8_t *dst,
				   const uint64_t *dst_off, const int32_t *dst_cap,
				   int32_t *ret, uint32_t nblocks, uint32_t max_cap,
				   const int32_t *dict_len, void *stream);

/*
 * LZ4E_decompress_safe into a bio_vec list (the read
 * side without a bounce buffer).  Decodes compressedSize bytes at `source`
 * into the segments of `dst` from *dstIter on, with capacity
 * dstIter->bi_size.  Returns exactly what LZ4E_decompress_safe returns for
 * that capacity (bytes written, or -(ip - src) - 1 on malformed input,
 * lz4e/lz4e_decompress.c:449-459); on success *dstIter is advanced by the
 * return value, on error nothing is written and *dstIter is untouched.
 */
int lz4e_decompress_safe_sg(const char *source, struct bio_vec *dst,
			    struct bvec_iter *dstIter, int compressedSize);

/* Batch form: request i decodes (src[i], csize[i]) into (dst[i],
 * dstIter[i]); ret[i] as above.  Returns the number of requests with
 * ret >= 0, or -1 when no GPU is usable. */
int lz4e_decompress_sg_batch(const char *const *src, const int *csize,
			     struct bio_vec *const *dst,
			     struct bvec_iter *const *dstIter, int *ret, int n);

/*
 * Chunk-layer WRITE round trip, batched and streamed.
 * Per request this is the data path of lz4e_write_req_init
 * (lz4e_bdev/lz4e_req.c:144-213): lz4e_chunk_compress_ext
 * (lz4e_bdev/lz4e_chunk.c:139-159: LZ4E_compress_default of the bio's SG
 * payload into a LZ4E_COMPRESSBOUND-sized chunk, i.e. never output-limited),
 * then lz4e_chunk_decompress (lz4e_chunk.c:119-137: LZ4_decompress_safe of
 * that frame back into the chunk's contiguous source buffer, whose size must
 * equal the bio's, lz4e_chunk.c:133).  Requests flow through four pipeline
 * slots (pinned staging + HBM buffers + a HIP stream each) in sub-batches of
 * a quarter of the call (16-256 MiB of input): the SG gather of one
 * sub-batch overlaps the H2D copies, kernels and D2H copies of the others.
 */
struct lz4e_chunk_request {
	const struct bio_vec *src;       /* original bio's bi_io_vec            */
	const struct bvec_iter *srcIter; /* original bio's bi_iter (read only:
					    the chunk layer passes a copy)      */
	char *data;        /* src_buf.data: receives srcIter->bi_size bytes    */
	char *frame;       /* nullable: receives the frame (dst_buf.data)      */
	int frame_cap;     /* bytes available at frame                         */
	int comp_size;     /* out: dst_buf.data_size (0 on compress failure)   */
	int status;        /* out: 0, -EIO (-5) like the chunk layer, or
			      -ENOSPC (-28) when frame_cap < comp_size          */
};

/* Write-side counters, the reference's struct lz4e_stats
 * (lz4e_bdev/include/lz4e_stats.h:17-22) updated as lz4e_stats_update does
 * at bio completion (lz4e_bdev/lz4e_stats.c:39-52), which only runs from
 * lz4e_end_io (lz4e_req.c:231-246): only a request whose round trip
 * completed (status 0) counts.  It adds 1 to reqs_total, the bi_vcnt of the
 * bio the reference completes (its src buffer re-added by
 * lz4e_add_buf_to_bio, lz4e_req.c:191-197: one merged bio_vec per
 * contiguous non-empty buffer) to vec_count and its size to data_in_bytes.
 * A request that fails in the write path (-EIO: compress or decompress
 * failure, more than 256 segments, oversize; -ENOSPC) returns through
 * lz4e_dev.c:187-202 in the reference and touches no counter.
 * reqs_failed counts completed bios the underlying device failed
 * (lz4e_stats.c:43-45); this library has no underlying device, so it is
 * always 0.  frame_bytes (not in the reference) = sum of comp_size of the
 * counted requests. */
struct lz4e_chunk_stats {
	uint64_t reqs_total;
	uint64_t reqs_failed;
	uint64_t vec_count;
	uint64_t data_in_bytes;
	uint64_t frame_bytes;
};

/* Returns the number of requests with status 0, or -1 on failure (no usable
 * GPU, or a HIP error part way through): every status is then -EIO, every
 * comp_size 0, `stats` is left untouched and nothing of the call is still
 * in flight.  `stats` is nullable; on success it is added to. */
int lz4e_chunk_write_batch(struct lz4e_chunk_request *reqs, int n,
			   struct lz4e_chunk_stats *stats);

#ifdef __cplusplus
}
#endif

#endif /* LZ4E_AMD_H */
