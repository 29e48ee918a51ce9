/*
 * lz4e_oracle.c -- CPU restatement of the reference LZ4E path.
 *
 * TEST INFRASTRUCTURE ONLY (see lz4e_oracle.h).  Used by tests/ as the
 * checker and by bench.py as the timed CPU baseline; never by the product.
 *
 * Reference files restated (all under /root/reference):
 *   lz4e/lz4e_compress.c      LZ4E_compress_default / _fast_extState /
 *                             _compress_generic / LZ4E_fillBvIterSize
 *   lz4e/lz4e_decompress.c    LZ4E_decompress_safe / _decompress_generic
 *   lz4e/include/lz4e_defs.h  constants, SG access helpers, LZ4E_count
 *   lz4e/include/lz4e.h       sizing macros
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "lz4e_oracle.h"

/* ---------------------------------------------------------------------- */
/* Constants and hashes (lz4e_defs.h:83-110, lz4e_compress.c:48-96)        */
/* ---------------------------------------------------------------------- */

static inline uint32_t o_bound(uint32_t n)
{
	return n > LZ4E_MAX_INPUT_SIZE ? 0 : n + n / 255 + 16;
}

/* hashLog per class: byU64 11, byU32 12, byU16 13 (lz4e_compress.c:48-57) */
static inline uint32_t o_hashlog(int tt)
{
	return tt == LZ4E_TABLE_BYU64 ? 11u : tt == LZ4E_TABLE_BYU32 ? 12u : 13u;
}

/* 4-byte multiplicative hash (lz4e_compress.c:59-66) */
static inline uint32_t o_hash4(uint32_t v, int tt)
{
	return (v * 2654435761u) >> (32 - o_hashlog(tt));
}

/* 5-byte hash of a little-endian 8-byte read (lz4e_compress.c:68-83) */
static inline uint32_t o_hash5(uint64_t v, int tt)
{
	return (uint32_t)(((v << 24) * 889523592379ull) >> (64 - o_hashlog(tt)));
}

static inline uint32_t o_ld32(const uint8_t *p)
{
	uint32_t v;

	memcpy(&v, p, 4);
	return v;
}

static inline uint64_t o_ld64(const uint8_t *p)
{
	uint64_t v;

	memcpy(&v, p, 8);
	return v;
}

/* ---------------------------------------------------------------------- */
/* Byte-access model 1: flat buffers                                       */
/* ---------------------------------------------------------------------- */

struct lin_src { const uint8_t *p; };
struct lin_dst { uint8_t *p; };

#define CORE_FN compress_core_linear
#define CORE_SRC struct lin_src
#define CORE_DST struct lin_dst
#define RD8(s, q) ((s)->p[q])
#define RD32(s, q) o_ld32((s)->p + (q))
#define RD64(s, q) o_ld64((s)->p + (q))
#define HASHAT(s, q, tt) \
	((tt) == LZ4E_TABLE_BYU32 ? o_hash5(RD64(s, q), tt) : o_hash4(RD32(s, q), tt))
#define WR8(d, q, v) ((d)->p[q] = (uint8_t)(v))
#define CPY(d, dq, s, sq, len) memcpy((d)->p + (dq), (s)->p + (sq), (len))
#include "lz4e_core.inc"
#undef CORE_FN
#undef CORE_SRC
#undef CORE_DST
#undef RD8
#undef RD32
#undef RD64
#undef HASHAT
#undef WR8
#undef CPY

/* ---------------------------------------------------------------------- */
/* Byte-access model 2: bio_vec lists, every access walks the segments     */
/* (the access pattern of lz4e_defs.h:352-585: locate the segment of a     */
/* position, then copy page-clamped pieces)                                */
/* ---------------------------------------------------------------------- */

struct sg_list {
	const struct bio_vec *bv;
	uint32_t idx0;  /* bi_idx of the start iterator      */
	uint32_t nseg;  /* segments touched                  */
	int64_t *base;  /* linear position of each bv byte 0 */
};

static uint32_t sg_count(const struct bio_vec *bv, const struct bvec_iter *it)
{
	uint32_t size = it->bi_size, idx = it->bi_idx, done = it->bi_bvec_done;
	uint32_t i = 0;

	while (size) {
		uint32_t take = bv[idx].bv_len - done;

		size -= take > size ? size : take;
		done = 0;
		idx++;
		i++;
	}
	return i;
}

/* Per-segment table, the analogue of LZ4E_fillBvIterSize's bvIterSize[]
 * (lz4e_compress.c:184-211).  Caller frees l->base. */
static void sg_build(struct sg_list *l, const struct bio_vec *bv,
		     const struct bvec_iter *it)
{
	uint32_t size = it->bi_size, idx = it->bi_idx, done = it->bi_bvec_done;
	int64_t pos = -(int64_t)done;
	uint32_t i = 0;

	l->bv = bv;
	l->idx0 = idx;
	l->nseg = sg_count(bv, it);
	l->base = malloc(sizeof(int64_t) * (l->nseg + 1));
	while (size) {
		uint32_t take = bv[idx].bv_len - done;

		l->base[i] = pos;
		pos += bv[idx].bv_len;
		size -= take > size ? size : take;
		done = 0;
		idx++;
		i++;
	}
	l->base[i] = pos;
}

/* Segment holding linear position q (binary search over base[]). */
static inline uint32_t sg_seg(const struct sg_list *l, int64_t q)
{
	uint32_t lo = 0, hi = l->nseg - 1;

	while (lo < hi) {
		uint32_t mid = (lo + hi + 1) / 2;

		if (l->base[mid] <= q)
			lo = mid;
		else
			hi = mid - 1;
	}
	return lo;
}

static inline uint8_t *sg_addr(const struct sg_list *l, uint32_t seg,
			       uint32_t off)
{
	const struct bio_vec *b = &l->bv[l->idx0 + seg];

	return (uint8_t *)b->bv_page + b->bv_offset + off;
}

static void sg_read(const struct sg_list *l, uint32_t q, uint8_t *to,
		    uint32_t len)
{
	while (len) {
		uint32_t seg = sg_seg(l, q);
		uint32_t off = (uint32_t)(q - l->base[seg]);
		const struct bio_vec *b = &l->bv[l->idx0 + seg];
		uint32_t in_seg = b->bv_len - off;
		uint32_t in_page = LZ4E_PAGE_SIZE - ((b->bv_offset + off) % LZ4E_PAGE_SIZE);
		uint32_t take = len;

		if (take > in_seg)
			take = in_seg;
		if (take > in_page)
			take = in_page;
		memcpy(to, sg_addr(l, seg, off), take);
		to += take;
		q += take;
		len -= take;
	}
}

static void sg_write(const struct sg_list *l, uint32_t q, const uint8_t *from,
		     uint32_t len)
{
	while (len) {
		uint32_t seg = sg_seg(l, q);
		uint32_t off = (uint32_t)(q - l->base[seg]);
		const struct bio_vec *b = &l->bv[l->idx0 + seg];
		uint32_t in_seg = b->bv_len - off;
		uint32_t in_page = LZ4E_PAGE_SIZE - ((b->bv_offset + off) % LZ4E_PAGE_SIZE);
		uint32_t take = len;

		if (take > in_seg)
			take = in_seg;
		if (take > in_page)
			take = in_page;
		memcpy(sg_addr(l, seg, off), from, take);
		from += take;
		q += take;
		len -= take;
	}
}

static inline uint8_t sg_rd8(const struct sg_list *l, uint32_t q)
{
	uint8_t v;

	sg_read(l, q, &v, 1);
	return v;
}

static inline uint32_t sg_rd32(const struct sg_list *l, uint32_t q)
{
	uint8_t b[4];

	sg_read(l, q, b, 4);
	return o_ld32(b);
}

static inline uint64_t sg_rd64(const struct sg_list *l, uint32_t q)
{
	uint8_t b[8];

	sg_read(l, q, b, 8);
	return o_ld64(b);
}

static void sg_copy(const struct sg_list *d, uint32_t dq,
		    const struct sg_list *s, uint32_t sq, uint32_t len)
{
	uint8_t tmp[256];

	while (len) {
		uint32_t take = len > sizeof(tmp) ? (uint32_t)sizeof(tmp) : len;

		sg_read(s, sq, tmp, take);
		sg_write(d, dq, tmp, take);
		dq += take;
		sq += take;
		len -= take;
	}
}

static inline void sg_wr8(const struct sg_list *l, uint32_t q, uint8_t v)
{
	sg_write(l, q, &v, 1);
}

#define CORE_FN compress_core_sg
#define CORE_SRC struct sg_list
#define CORE_DST struct sg_list
#define RD8(s, q) sg_rd8(s, q)
#define RD32(s, q) sg_rd32(s, q)
#define RD64(s, q) sg_rd64(s, q)
#define HASHAT(s, q, tt) \
	((tt) == LZ4E_TABLE_BYU32 ? o_hash5(RD64(s, q), tt) : o_hash4(RD32(s, q), tt))
#define WR8(d, q, v) sg_wr8(d, q, (uint8_t)(v))
#define CPY(d, dq, s, sq, len) sg_copy(d, dq, s, sq, len)
#include "lz4e_core.inc"

/* ---------------------------------------------------------------------- */
/* Public oracle entry points                                              */
/* ---------------------------------------------------------------------- */

int oracle_table_type(const struct bio_vec *src, const struct bvec_iter *it)
{
	/* lz4e_compress.c:184-211: byU16 unless >= 16 segments or a raw
	 * segment longer than 4096 (byU32), or longer than 16 MiB (byU64);
	 * more than BIO_MAX_VECS touched segments fails. */
	uint32_t size = it->bi_size, idx = it->bi_idx, done = it->bi_bvec_done;
	uint32_t i = 0;
	int tt = LZ4E_TABLE_BYU16;

	while (size) {
		uint32_t len = src[idx].bv_len;
		uint32_t take = len - done;

		if (i >= BIO_MAX_VECS)
			return 0;
		if (i >= 16 || len > 4096)
			tt |= LZ4E_TABLE_BYU32;
		if (len > (1u << 24))
			tt |= LZ4E_TABLE_BYU64;
		if (take > size)
			take = size;
		size -= take;
		done = 0;
		idx++;
		i++;
	}
	return tt;
}

int oracle_compress_linear(const uint8_t *in, uint32_t n, int table_type,
			   uint8_t *out, uint32_t cap, uint32_t *final_src,
			   uint32_t *last_run)
{
	struct lin_src s = { in };
	struct lin_dst d = { out };

	return compress_core_linear(&s, n, table_type, &d, cap, final_src,
				    last_run, 0);
}

/* Dictionary mode (the reference's stubbed dict path, lz4e_compress.c:250-266,
 * 315-324; LZ4E extension, parity unpinned): the block compressed against the
 * last <= 64 KiB of dict (ignored under 8 bytes, LZ4_loadDict), byU32. */
int oracle_compress_dict(const uint8_t *in, uint32_t n, const uint8_t *dict,
			 uint32_t dict_size, uint8_t *out, uint32_t cap)
{
	uint32_t D = dict_size > 65536 ? 65536 : dict_size;
	uint8_t *img;
	struct lin_src s;
	struct lin_dst d = { out };
	int r;

	if (D < 8)
		D = 0;
	img = malloc((size_t)D + n + 16);
	if (!img)
		return 0;
	memcpy(img, dict + dict_size - D, D);
	memcpy(img + D, in, n);
	s.p = img;
	r = compress_core_linear(&s, n, LZ4E_TABLE_BYU32,
				 &d, cap, NULL, NULL, D);
	free(img);
	return r;
}

/* Kernel bvec_iter_advance semantics (warn + clamp past the end). */
static void o_iter_advance(const struct bio_vec *bv, struct bvec_iter *it,
			   uint32_t bytes)
{
	uint32_t idx = it->bi_idx;

	if (bytes > it->bi_size) {
		it->bi_size = 0;
		return;
	}
	it->bi_size -= bytes;
	bytes += it->bi_bvec_done;
	while (bytes && bytes >= bv[idx].bv_len) {
		bytes -= bv[idx].bv_len;
		idx++;
	}
	it->bi_idx = idx;
	it->bi_bvec_done = bytes;
}

int oracle_compress_sg(const struct bio_vec *src, struct bio_vec *dst,
		       struct bvec_iter *srcIter, struct bvec_iter *dstIter,
		       void *wrkmem)
{
	struct sg_list sl, dl;
	const uint32_t n = srcIter->bi_size;
	const uint32_t cap = dstIter->bi_size;
	uint32_t final_src = 0, last_run = 0;
	int tt = LZ4E_TABLE_BYU16;
	int ret;

	memset(wrkmem, 0, LZ4E_MEM_COMPRESS); /* lz4e_compress.c:548 */
	if (n > LZ4E_MAX_INPUT_SIZE)
		return 0;
	if (n >= 13) {
		tt = oracle_table_type(src, srcIter);
		if (!tt)
			return 0;
	}
	sg_build(&sl, src, srcIter);
	sg_build(&dl, dst, dstIter);
	ret = compress_core_sg(&sl, n, tt, &dl, cap, &final_src, &last_run, 0);
	free(sl.base);
	free(dl.base);
	if (ret > 0) {
		o_iter_advance(src, srcIter, final_src);
		o_iter_advance(dst, dstIter, (uint32_t)ret - last_run);
	}
	return ret;
}

/* ---------------------------------------------------------------------- */
/* Decoder (lz4e_decompress.c:62-469, endOnInputSize, decode_full_block,   */
/* noDict).  Positions are signed integers so that the reference's pointer */
/* comparisons (e.g. ip < iend - 15 for tiny inputs) keep their meaning.   */
/* Match bytes follow LZ semantics: byte t of a match at op with offset o  */
/* is out[op - o + t] for o >= 1; offset 0 yields zeros, which is what the */
/* reference's LZ4_write32(op, offset) + overlap copy produce (:313,407).  */
/* ---------------------------------------------------------------------- */

int oracle_decompress_safe(const char *src, char *dst, int srcSize,
			   int outSize)
{
	return oracle_decompress_dict(src, dst, srcSize, outSize, NULL, 0);
}

/* Output byte at position x >= -D: the block, or before it the dictionary's
 * last bytes (extDict, lz4e_decompress.c:339-378). */
static inline uint8_t o_out(const uint8_t *d, const uint8_t *dict_end,
			    int64_t x)
{
	return x >= 0 ? d[x] : dict_end[x];
}

/* The reference decoder with a dictionary (usingExtDict, lowPrefix = dst,
 * dictStart/dictSize): checkOffset when dictSize < 64 KiB (:93), the
 * shortcut only for sources inside the block (:170-172), sources before the
 * block read from the dictionary's end (:339-378). */
int oracle_decompress_dict(const char *src, char *dst, int srcSize,
			   int outSize, const char *dict, int dictSize)
{
	const uint8_t *s = (const uint8_t *)src;
	uint8_t *d = (uint8_t *)dst;
	const uint8_t *dict_end = dict ? (const uint8_t *)dict + dictSize : NULL;
	const int64_t dsz = dict && dictSize > 0 ? dictSize : 0;
	const int64_t iend = srcSize, oend = outSize;
	const int64_t shortiend = iend - 14 - 2; /* :100-101 */
	const int64_t shortoend = oend - 14 - 18; /* :102-103 */
	int64_t ip = 0, op = 0;

	if (outSize == 0) /* :113-114 */
		return (srcSize == 1 && s[0] == 0) ? 0 : -1;
	if (srcSize == 0) /* :119-120 */
		return -1;
	if (srcSize < 0) /* token read, then every path errors at ip == 1 */
		return -2;

	for (;;) {
		const unsigned token = s[ip++];
		int64_t length = token >> 4;
		int64_t offset, match, cpy, t;

		/* Two-stage shortcut (:150-191). */
		if (length != 15 && ip < shortiend && op <= shortoend) {
			memcpy(d + op, s + ip, 16);
			op += length;
			ip += length;
			length = token & 15;
			offset = s[ip] | (s[ip + 1] << 8);
			ip += 2;
			match = op - offset;
			if (length != 15 && offset >= 8 && match >= 0) {
				for (t = 0; t < 18; t++)
					d[op + t] = d[match + t];
				op += length + 4;
				continue;
			}
			goto copy_match;
		}

		/* Literal length (:194-220). */
		if (length == 15) {
			unsigned b;

			if (ip >= iend - 15)
				goto err;
			do {
				b = s[ip++];
				length += b;
			} while (ip < iend - 15 && b == 255);
		}

		/* Literals (:223-288). */
		cpy = op + length;
		if (cpy > oend - 12 || ip + length > iend - 8) {
			if (ip + length != iend || cpy > oend)
				goto err;
			memmove(d + op, s + ip, (size_t)length);
			ip += length;
			op += length;
			break;
		}
		memcpy(d + op, s + ip, (size_t)length);
		ip += length;
		op = cpy;

		/* Offset (:291-296). */
		offset = s[ip] | (s[ip + 1] << 8);
		ip += 2;
		match = op - offset;
		length = token & 15;

copy_match:
		if (dsz < 65536 && match + dsz < 0) /* :299-302 */
			goto err;
		if (length == 15) { /* :316-334 */
			unsigned b;

			do {
				b = s[ip++];
				if (ip > iend - 5)
					goto err;
				length += b;
			} while (b == 255);
		}
		length += 4;
		cpy = op + length;
		if (cpy > oend - 5) /* :422-431 (implies cpy > oend - 12) */
			goto err;
		if (offset == 0)
			memset(d + op, 0, (size_t)length);
		else
			for (t = 0; t < length; t++)
				d[op + t] = o_out(d, dict_end, match + t);
		op = cpy;
	}
	return (int)op;
err:
	return (int)(-ip) - 1;
}

/* ---------------------------------------------------------------------- */
/* Threaded batch helpers for the CPU baseline                             */
/* ---------------------------------------------------------------------- */

struct batch_job {
	int kind; /* 0 compress, 1 decompress, 2 compress through bio_vecs */
	const uint8_t *in;
	const uint64_t *in_off;
	const void *in_len;
	const uint8_t *ttype;
	uint8_t *out;
	const uint64_t *out_off;
	const void *out_cap;
	int32_t *ret;
	uint32_t n;
	uint32_t next; /* atomic work counter */
	uint32_t seg;  /* kind 2: source segment bytes */
};

/* One block of kind 2: the source as seg-byte bio_vecs, the destination as
 * 4096-byte pages, through the faithful SG restatement (the reference's
 * per-access segment walk, lz4e_defs.h:352-585). */
static int32_t sg_block(const uint8_t *in, uint32_t n, uint32_t seg,
			uint8_t *out, uint32_t cap)
{
	uint32_t ns = n ? (n + seg - 1) / seg : 1;
	uint32_t nd = cap ? (cap + LZ4E_PAGE_SIZE - 1) / LZ4E_PAGE_SIZE : 1;
	struct bio_vec *sv = calloc(ns + nd, sizeof(*sv));
	struct bio_vec *dv = sv + ns;
	struct bvec_iter si = { 0, n, 0, 0 }, di = { 0, cap, 0, 0 };
	unsigned char wrk[LZ4E_MEM_COMPRESS];
	uint32_t k;
	int32_t r;

	for (k = 0; k < ns; k++) {
		sv[k].bv_page = (struct page *)(in + (size_t)k * seg);
		sv[k].bv_len = n - k * seg < seg ? n - k * seg : seg;
		sv[k].bv_offset = 0;
	}
	for (k = 0; k < nd; k++) {
		dv[k].bv_page = (struct page *)(out + (size_t)k * LZ4E_PAGE_SIZE);
		dv[k].bv_len = cap - k * LZ4E_PAGE_SIZE < LZ4E_PAGE_SIZE ?
			cap - k * LZ4E_PAGE_SIZE : LZ4E_PAGE_SIZE;
		dv[k].bv_offset = 0;
	}
	r = oracle_compress_sg(sv, dv, &si, &di, wrk);
	free(sv);
	return r;
}

static void *batch_worker(void *arg)
{
	struct batch_job *j = arg;

	for (;;) {
		uint32_t i = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);

		if (i >= j->n)
			break;
		if (j->kind == 2)
			j->ret[i] = sg_block(j->in + j->in_off[i],
					     ((const uint32_t *)j->in_len)[i], j->seg,
					     j->out + j->out_off[i],
					     ((const uint32_t *)j->out_cap)[i]);
		else if (j->kind == 0)
			j->ret[i] = oracle_compress_linear(
				j->in + j->in_off[i], ((const uint32_t *)j->in_len)[i],
				j->ttype[i], j->out + j->out_off[i],
				((const uint32_t *)j->out_cap)[i], NULL, NULL);
		else
			j->ret[i] = oracle_decompress_safe(
				(const char *)j->in + j->in_off[i],
				(char *)j->out + j->out_off[i],
				((const int32_t *)j->in_len)[i],
				((const int32_t *)j->out_cap)[i]);
	}
	return NULL;
}

static void run_batch(struct batch_job *j, int threads)
{
	pthread_t tid[256];
	int t;

	if (threads < 1)
		threads = 1;
	if (threads > 256)
		threads = 256;
	j->next = 0;
	for (t = 1; t < threads; t++)
		pthread_create(&tid[t], NULL, batch_worker, j);
	batch_worker(j);
	for (t = 1; t < threads; t++)
		pthread_join(tid[t], NULL);
}

void oracle_compress_linear_batch(const uint8_t *in, const uint64_t *in_off,
				  const uint32_t *in_len, const uint8_t *ttype,
				  uint8_t *out, const uint64_t *out_off,
				  const uint32_t *out_cap, int32_t *ret,
				  uint32_t n, int threads)
{
	struct batch_job j = { 0, in, in_off, in_len, ttype, out, out_off,
			       out_cap, ret, n, 0, 0 };

	run_batch(&j, threads);
}

void oracle_compress_sg_batch(const uint8_t *in, const uint64_t *in_off,
			      const uint32_t *in_len, uint32_t seg,
			      uint8_t *out, const uint64_t *out_off,
			      const uint32_t *out_cap, int32_t *ret,
			      uint32_t n, int threads)
{
	struct batch_job j = { 2, in, in_off, in_len, NULL, out, out_off,
			       out_cap, ret, n, 0, seg };

	run_batch(&j, threads);
}

void oracle_decompress_batch(const uint8_t *in, const uint64_t *in_off,
			     const int32_t *in_len, uint8_t *out,
			     const uint64_t *out_off, const int32_t *out_cap,
			     int32_t *ret, uint32_t n, int threads)
{
	struct batch_job j = { 1, in, in_off, in_len, NULL, out, out_off,
			       out_cap, ret, n, 0, 0 };

	run_batch(&j, threads);
}
