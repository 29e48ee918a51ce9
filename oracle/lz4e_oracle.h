/*
 * lz4e_oracle.h -- CPU restatement of the reference LZ4E path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (lz4-sgori_amd/, the
 * C-ABI library) may link, load or call this.  Only tests/, the smoke()
 * check in __graft_entry__.py and bench.py's cpu_baseline leg use it, and
 * only as the checker / the timed CPU baseline.
 *
 * Parity pinning: the reference is a Linux kernel module; building it needs
 * kernel headers this image does not have, so it is treated as unbuildable
 * here.  This restatement is pinned against the
 * reference outputs recorded in SURVEY.md §8c (frame sizes + SHA-256 of the
 * reference's frames for its own test_files, and the decompressor's return
 * codes), committed as tests/golden/reference_kat.json.
 */
#ifndef LZ4E_ORACLE_H
#define LZ4E_ORACLE_H

#include <stdint.h>

#include "../include/lz4e.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Table class of an SG source: 1/3/7, or 0 for > BIO_MAX_VECS segments.
 * Follows lz4e/lz4e_compress.c:184-211. */
int oracle_table_type(const struct bio_vec *src, const struct bvec_iter *it);

/* Greedy LZ4E parse + block emit over a flat buffer (lz4e_compress.c:218-534).
 * final_src / last_run (nullable) receive the iterator post-state inputs. */
int oracle_compress_linear(const uint8_t *in, uint32_t n, int table_type,
			   uint8_t *out, uint32_t cap, uint32_t *final_src,
			   uint32_t *last_run);

/* Same algorithm, every byte access walking the bio_vec lists (the access
 * pattern of lz4e/include/lz4e_defs.h:352-585).  Full API semantics of
 * LZ4E_compress_default including iterator updates. */
int oracle_compress_sg(const struct bio_vec *src, struct bio_vec *dst,
		       struct bvec_iter *srcIter, struct bvec_iter *dstIter,
		       void *wrkmem);

/* Dictionary mode (LZ4E extension of the stubbed dict path, parity
 * unpinned): compress against the last <= 64 KiB of dict, decode with a
 * dictionary (extDict branches of lz4e_decompress.c:299-302, 339-378). */
int oracle_compress_dict(const uint8_t *in, uint32_t n, const uint8_t *dict,
			 uint32_t dict_size, uint8_t *out, uint32_t cap);
int oracle_decompress_dict(const char *src, char *dst, int srcSize,
			   int outSize, const char *dict, int dictSize);

/* Safe full-block decoder (lz4e/lz4e_decompress.c:62-469). */
int oracle_decompress_safe(const char *src, char *dst, int srcSize,
			   int outSize);

/* Threaded batch helpers for the CPU baseline (one block per task). */
void oracle_compress_linear_batch(const uint8_t *in, const uint64_t *in_off,
				  const uint32_t *in_len, const uint8_t *ttype,
				  uint8_t *out, const uint64_t *out_off,
				  const uint32_t *out_cap, int32_t *ret,
				  uint32_t n, int threads);
/* The same blocks through oracle_compress_sg: source split into seg-byte
 * bio_vecs, destination 4096-byte pages (the reference's cost profile). */
void oracle_compress_sg_batch(const uint8_t *in, const uint64_t *in_off,
			      const uint32_t *in_len, uint32_t seg,
			      uint8_t *out, const uint64_t *out_off,
			      const uint32_t *out_cap, int32_t *ret,
			      uint32_t n, int threads);
void oracle_decompress_batch(const uint8_t *in, const uint64_t *in_off,
			     const int32_t *in_len, uint8_t *out,
			     const uint64_t *out_off, const int32_t *out_cap,
			     int32_t *ret, uint32_t n, int threads);

#ifdef __cplusplus
}
#endif

#endif
