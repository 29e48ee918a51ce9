/*
 * bandmodel.c -- CPU model of the band-parallel LZ4E compressor (development
 * tool; not the oracle, not the product).
 *
 * It restates, phase by phase and with plain loops where the GPU kernel runs
 * a phase across its lanes, the algorithm of csrc/lz4e_band.hip:
 *
 *   The greedy parse of lz4e/lz4e_compress.c:285-498 is a pure function of
 *   the candidate each lookup sees, and that candidate is "the latest put of
 *   the same hash before the lookup".  A pass guesses the put set G of a band
 *   of B positions ahead of the verified frontier f, resolves every
 *   position's candidate under G (nearest G-marked position on its
 *   full-population same-hash chain inside [f, p), else the true table T),
 *   builds the parse chain through the band from those candidates, and takes
 *   the chain's own puts as the next guess.  The next pass re-resolves the
 *   candidates under that guess and compares the outcome of every lookup the
 *   previous chain made (miss, or hit with its candidate): everything before
 *   the first lookup whose outcome changed is the true parse (each of its
 *   lookups saw exactly the puts the parse itself made before it), so it is
 *   committed (sequences emitted, puts written to T) and the band moves on.
 *
 * Usage: bandmodel FILE BLOCK_SIZE TABLE_CLASS [NBLOCKS] [B] [FCAP] [BCAP]
 * Compares every frame with oracle_compress_linear and prints pass counts.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/lz4e_oracle.h"

static uint32_t BW = 1024, FCAP = 32, BCAP = 8;

typedef struct {
	const uint8_t *in;
	uint32_t n, hlog, mflimit, matchlimit;
	int tt;
	uint16_t *pd;  /* prev same-hash delta (0: none within 65535) */
	uint32_t *T;   /* the true table at the frontier */
} Blk;

static inline uint32_t rd32(const Blk *b, uint32_t p) { uint32_t v; memcpy(&v, b->in + p, 4); return v; }
static inline uint64_t rd64(const Blk *b, uint32_t p) { uint64_t v; memcpy(&v, b->in + p, 8); return v; }
static inline uint32_t hashat(const Blk *b, uint32_t p)
{
	if (b->tt == LZ4E_TABLE_BYU32)
		return (uint32_t)(((rd64(b, p) << 24) * 889523592379ull) >> (64 - b->hlog));
	return (rd32(b, p) * 2654435761u) >> (32 - b->hlog);
}

/* ---- the pre-kernel: full-population same-hash predecessors ---- */
static void prev_pass(Blk *b)
{
	uint32_t *last = calloc(1u << 13, 4);
	uint8_t *seen = calloc(1u << 13, 1);
	for (uint32_t p = 0; p <= b->mflimit; p++) {
		uint32_t h = hashat(b, p), d = 0;
		if (seen[h] && p - last[h] <= 65535) d = p - last[h];
		b->pd[p] = (uint16_t)d;
		last[h] = p; seen[h] = 1;
	}
	free(last); free(seen);
}

/* advance after probe j of a search (lz4e_compress.c:306-307) */
static inline uint32_t adv(uint32_t j) { return j == 0 ? 1u : (63u + j) >> 6; }

enum { K_REM = 0, K_SRCH = 1, K_END = 2 };
typedef struct { int kind; uint32_t pos, j, a; } St;  /* REM(pos) or SRCH(pos, probe j, anchor a) */

typedef struct {             /* one lookup of a pass's chain, in order */
	uint32_t pos, cand;
	uint8_t rem, hit;
	St before;                /* parse state right before this lookup */
} Look;

typedef struct { uint32_t lit, litlen, off, mlen; } Seq;

typedef struct {
	long passes, commits, longs, slows, lookups, mism;
} Stats;

/* per-pass chain result */
typedef struct {
	Look *lk; uint32_t nlk;
	Seq *sq; uint32_t nsq;     /* sequences completed by the chain, in order */
	uint32_t *sq_lk;          /* index of the lookup that found sequence i's match */
	St term;                   /* state after the chain */
	uint8_t *put;              /* puts of the chain on the band (index p - f) */
} Chain;

static Blk B_;

/* candidate of p under guess G (band [f, f+BW), G indexed p - f) */
long g_hops[10];
long g_mk[4], g_md[8];
static uint32_t cand_of(const Blk *b, uint32_t f, const uint8_t *G, uint32_t p)
{
	uint32_t c = p, hops = 0;
	for (;;) {
		uint32_t d = b->pd[c];
		hops++;
		if (!d) break;
		c -= d;
		if (c < f) break;
		if (G[c - f]) { g_hops[hops < 9 ? hops : 9]++; return c; }
	}
	g_hops[hops < 9 ? hops : 9]++;
	return b->T[hashat(b, p)];
}

static int GUESS = 0;
/* the first guess of a position new to the band */
static uint8_t guess_new(const Blk *b, uint32_t p)
{
	if (GUESS == 0 || p < 2 || p > b->mflimit) return 1;
	/* continuation of a full-population match at p-1 and p: an interior */
	uint32_t d0 = b->pd[p], d1 = b->pd[p - 1];
	int c0 = d0 && d0 == d1 && rd32(b, p - d0) == rd32(b, p);
	int c1 = d1 && p - 1 >= d1 && rd32(b, p - 1 - d1) == rd32(b, p - 1);
	if (GUESS == 1) return !(c0 && c1);
	return !c0;
}
static int hit_of(const Blk *b, uint32_t p, uint32_t c, int rem)
{
	if ((rem || b->tt != LZ4E_TABLE_BYU16) && c + 65535 < p) return 0;
	return rd32(b, c) == rd32(b, p);
}

static uint32_t fwd_len(const Blk *b, uint32_t p, uint32_t c, uint32_t cap)
{
	uint32_t i = 0;
	while (p + 4 + i < b->matchlimit && b->in[p + 4 + i] == b->in[c + 4 + i]) {
		i++;
		if (i >= cap) return cap;
	}
	return i;
}

static uint32_t back_len(const Blk *b, uint32_t p, uint32_t c, uint32_t lim, uint32_t cap)
{
	uint32_t i = 0;
	while (i < lim && c - i > 0 && b->in[p - 1 - i] == b->in[c - 1 - i]) {
		i++;
		if (i >= cap) return cap;
	}
	return i;
}

/* Builds the chain from state s through the band [f, f+BW) with candidates
 * cand[] (index p - f).  Match lengths capped at FCAP / BCAP count as "long"
 * and are extended exactly (on the GPU: the whole workgroup, once per pass). */
static void build_chain(const Blk *b, uint32_t f, St s, const uint32_t *cand, Chain *ch, Stats *st)
{
	uint32_t end = f + BW;
	ch->nlk = 0; ch->nsq = 0;
	memset(ch->put, 0, BW);
	for (;;) {
		if (s.kind == K_END) break;
		if (s.kind == K_REM) {
			uint32_t e = s.pos;
			if (e > b->mflimit) { s.kind = K_END; break; }
			if (e >= end) {                           /* exit: REM beyond the band */
				if (e - 2 >= f && e - 2 < end) ch->put[e - 2 - f] = 1;
				break;
			}
			if (e - 2 >= f) ch->put[e - 2 - f] = 1;   /* (e-2 < f: committed with the state) */
			uint32_t c = cand[e - f];
			int h = hit_of(b, e, c, 1);
			Look *L = &ch->lk[ch->nlk++];
			L->pos = e; L->cand = c; L->rem = 1; L->hit = (uint8_t)h; L->before = s;
			ch->put[e - f] = 1;
			if (h) {
				uint32_t fl = fwd_len(b, e, c, FCAP);
				if (fl >= FCAP) { st->longs++; fl = fwd_len(b, e, c, 1u << 30); }
				Seq *q = &ch->sq[ch->nsq]; ch->sq_lk[ch->nsq++] = ch->nlk - 1;
				q->lit = e; q->litlen = 0; q->off = e - c; q->mlen = 4 + fl;
				s.kind = K_REM; s.pos = e + 4 + fl;
				if (fl >= FCAP) {                      /* a long match ends the pass */
					if (s.pos - 2 < end) ch->put[s.pos - 2 - f] = 1;
					break;
				}
				continue;
			}
			s.kind = K_SRCH; s.pos = e + 1; s.j = 0; s.a = e;
		}
		/* search from s.pos, probe index s.j, anchor s.a */
		{
			uint32_t x = s.pos, j = s.j;
			int found = 0;
			if (j > 65) st->slows++;
			for (;;) {
				uint32_t ad = adv(j);
				if (x + ad > b->mflimit) { s.kind = K_END; break; }
				if (x >= end) { s.pos = x; s.j = j; break; }  /* exit: search runs on */
				uint32_t c = cand[x - f];
				int h = hit_of(b, x, c, 0);
				Look *L = &ch->lk[ch->nlk++];
				L->pos = x; L->cand = c; L->rem = 0; L->hit = (uint8_t)h;
				L->before.kind = K_SRCH; L->before.pos = x; L->before.j = j; L->before.a = s.a;
				ch->put[x - f] = 1;
				if (h) {
					uint32_t bl = back_len(b, x, c, x - s.a, BCAP);
					if (bl >= BCAP) { st->longs++; bl = back_len(b, x, c, x - s.a, 1u << 30); }
					uint32_t fl = fwd_len(b, x, c, FCAP);
					int lng = fl >= FCAP;
					if (lng) { st->longs++; fl = fwd_len(b, x, c, 1u << 30); }
					Seq *q = &ch->sq[ch->nsq]; ch->sq_lk[ch->nsq++] = ch->nlk - 1;
					q->lit = s.a; q->litlen = x - bl - s.a; q->off = x - c; q->mlen = 4 + fl + bl;
					s.kind = K_REM; s.pos = x + 4 + fl;
					found = 1 + lng;
					break;
				}
				x += ad; j++;
			}
			if (found == 2) {
				if (s.pos - 2 < end && s.pos <= b->mflimit) ch->put[s.pos - 2 - f] = 1;
				break;
			}
			if (!found) break;
		}
	}
	ch->term = s;
}

/* encoded size of a sequence (token, literal varint, literals, offset, match varint) */
static uint32_t seq_size(const Seq *q)
{
	uint32_t sz = 1 + q->litlen + 2;
	if (q->litlen >= 15) sz += 1 + (q->litlen - 15) / 255;
	if (q->mlen - 4 >= 15) sz += 1 + (q->mlen - 4 - 15) / 255;
	return sz;
}

static uint32_t emit_seq(uint8_t *out, uint32_t op, const Blk *b, const Seq *q)
{
	uint32_t L = q->litlen, mc = q->mlen - 4, tok = op++;
	uint8_t token;
	if (L >= 15) { uint32_t r = L - 15; token = 0xF0; for (; r >= 255; r -= 255) out[op++] = 255; out[op++] = (uint8_t)r; }
	else token = (uint8_t)(L << 4);
	memcpy(out + op, b->in + q->lit, L); op += L;
	out[op++] = (uint8_t)q->off; out[op++] = (uint8_t)(q->off >> 8);
	if (mc >= 15) { uint32_t r = mc - 15; token += 15; for (; r >= 255; r -= 255) out[op++] = 255; out[op++] = (uint8_t)r; }
	else token += (uint8_t)mc;
	out[tok] = token;
	return op;
}

static int band_compress(Blk *b, uint8_t *out, Stats *st)
{
	uint32_t n = b->n, op = 0, anchor = 0;
	if (n >= 13) {
		b->mflimit = n - 12; b->matchlimit = n - 5;
		prev_pass(b);
		memset(b->T, 0, 4u << b->hlog);
		b->T[hashat(b, 0)] = 0;
		St s = {K_SRCH, 1, 0, 0};
		uint32_t f = 1;
		uint8_t *G = malloc(BW), *Gn = malloc(BW);
		uint32_t *cand = malloc(4 * BW);
		Chain ch = {malloc(sizeof(Look) * (BW + 8)), 0, malloc(sizeof(Seq) * (BW + 8)), 0,
			    malloc(4 * (BW + 8)), s, malloc(BW)};
		int have = 0;
		for (uint32_t p = f; p < f + BW; p++) G[p - f] = guess_new(b, p);
		for (;;) {
			st->passes++;
			/* 1. candidates under G */
			for (uint32_t p = f; p < f + BW && p <= b->mflimit; p++) cand[p - f] = cand_of(b, f, G, p);
			/* 2. verify the previous chain's lookups; commit the verified prefix */
			if (have) {
				uint32_t bad = ch.nlk;
				for (uint32_t i = 0; i < ch.nlk; i++) {
					const Look *L = &ch.lk[i];
					uint32_t c = cand[L->pos - f];
					int h = hit_of(b, L->pos, c, L->rem);
					if (h != L->hit || (h && c != L->cand)) {
						bad = i;
						{
							extern long g_mk[4], g_md[8];
							uint32_t hiC = c > L->cand ? c : L->cand;
							g_mk[c > L->cand ? 0 : 1]++;
							uint32_t dd = L->pos - hiC;
							g_md[dd < 16 ? 0 : dd < 64 ? 1 : dd < 256 ? 2 : dd < 1024 ? 3 : 4]++;
							g_md[5] += L->pos - f;
							g_md[6]++;
						}
						break;
					}
				}
				St ns = bad < ch.nlk ? ch.lk[bad].before : ch.term;
				if (bad < ch.nlk) st->mism++;
				/* emit the sequences whose match-finding lookup precedes `bad` */
				for (uint32_t i = 0; i < ch.nsq && ch.sq_lk[i] < bad; i++) {
					op = emit_seq(out, op, b, &ch.sq[i]);
					anchor = ch.sq[i].lit + ch.sq[i].litlen + ch.sq[i].mlen;
				}
				/* commit puts below the new frontier */
				uint32_t nf = ns.kind == K_END ? f + BW : ns.pos;
				for (uint32_t p = f; p < f + BW && p < nf; p++)
					if (ch.put[p - f]) b->T[hashat(b, p)] = p;
				if (ns.kind == K_REM && ns.pos - 2 >= f + BW && ns.pos <= b->mflimit)
					b->T[hashat(b, ns.pos - 2)] = ns.pos - 2; /* put(e-2) beyond the band */
				st->commits++;
				if (ns.kind == K_END) break;
				/* shift the band to [nf, nf + BW): keep G on the overlap */
				for (uint32_t p = nf; p < nf + BW; p++) Gn[p - nf] = guess_new(b, p);
				for (uint32_t p = nf; p < f + BW; p++) Gn[p - nf] = G[p - f];
				memcpy(G, Gn, BW);
				if (nf != f) {
					f = nf;
					for (uint32_t p = f; p < f + BW && p <= b->mflimit; p++) cand[p - f] = cand_of(b, f, G, p);
				}
				s = ns;
			}
			/* 3. the chain under the candidates */
			build_chain(b, f, s, cand, &ch, st);
			st->lookups += ch.nlk;
			have = 1;
			/* 4. next guess: the chain's puts before its end state, G beyond */
			{
				uint32_t lim = ch.term.kind == K_END ? f + BW : (ch.term.pos < f + BW ? ch.term.pos : f + BW);
				for (uint32_t p = f; p < lim; p++) G[p - f] = ch.put[p - f];
				if (ch.term.kind == K_REM && ch.term.pos - 2 >= f && ch.term.pos - 2 < f + BW)
					G[ch.term.pos - 2 - f] = 1;
			}
		}
		free(G); free(Gn); free(cand); free(ch.lk); free(ch.sq); free(ch.sq_lk); free(ch.put);
	}
	/* last literals (lz4e_compress.c:500-530) */
	{
		uint32_t R = n - anchor;
		if (R >= 15) { uint32_t r = R - 15; out[op++] = 0xF0; for (; r >= 255; r -= 255) out[op++] = 255; out[op++] = (uint8_t)r; }
		else out[op++] = (uint8_t)(R << 4);
		memcpy(out + op, b->in + anchor, R);
		op += R;
	}
	(void)seq_size;
	return (int)op;
}

int main(int argc, char **argv)
{
	if (argc < 4) { fprintf(stderr, "usage: bandmodel FILE BLOCK_SIZE TABLE_CLASS [NBLOCKS] [B] [FCAP] [BCAP]\n"); return 2; }
	FILE *fp = fopen(argv[1], "rb");
	if (!fp) return 2;
	fseek(fp, 0, SEEK_END); long sz = ftell(fp); fseek(fp, 0, SEEK_SET);
	uint8_t *all = malloc(sz + 16);
	if (fread(all, 1, sz, fp) != (size_t)sz) return 2;
	fclose(fp);
	uint32_t bs = (uint32_t)atoi(argv[2]);
	int tt = atoi(argv[3]);
	long nblk = argc > 4 ? atol(argv[4]) : 1L << 40;
	if (argc > 5) BW = (uint32_t)atoi(argv[5]);
	if (argc > 6) FCAP = (uint32_t)atoi(argv[6]);
	if (argc > 7) BCAP = (uint32_t)atoi(argv[7]);
	if (argc > 8) GUESS = atoi(argv[8]);
	Blk *b = &B_;
	b->tt = tt; b->hlog = tt == LZ4E_TABLE_BYU64 ? 11 : tt == LZ4E_TABLE_BYU32 ? 12 : 13;
	b->pd = malloc(2 * (size_t)bs + 64);
	b->T = malloc(4u << 13);
	uint8_t *o1 = malloc(bs + bs / 255 + 64), *o2 = malloc(bs + bs / 255 + 64);
	Stats st = {0};
	long nb = 0, bad = 0, maxp = 0;
	for (long off = 0; off + bs <= sz && nb < nblk; off += bs, nb++) {
		b->in = all + off; b->n = bs;
		long p0 = st.passes;
		int r1 = band_compress(b, o1, &st);
		int r2 = oracle_compress_linear(b->in, bs, tt, o2, bs + bs / 255 + 64, NULL, NULL);
		if (r1 != r2 || memcmp(o1, o2, r1)) {
			if (bad < 5) fprintf(stderr, "block %ld differs: %d vs %d\n", nb, r1, r2);
			bad++;
		}
		if (st.passes - p0 > maxp) maxp = st.passes - p0;
	}
	printf("%s bs=%u tt=%d B=%u FCAP=%u BCAP=%u blocks=%ld bad=%ld passes/blk=%.1f max=%ld longs/blk=%.1f "
	       "slow/blk=%.1f lookups/pass=%.1f mism/blk=%.1f\n",
	       argv[1], bs, tt, BW, FCAP, BCAP, nb, bad, (double)st.passes / nb, maxp, (double)st.longs / nb,
	       (double)st.slows / nb, (double)st.lookups / st.passes, (double)st.mism / nb);
	printf("mismatch: new cand later (put appeared) %ld, earlier (put vanished) %ld; lookup - changed cand: <16 %ld <64 %ld <256 %ld <1024 %ld more %ld; mean offset in band %.0f\n",
	       g_mk[0], g_mk[1], g_md[0], g_md[1], g_md[2], g_md[3], g_md[4], (double)g_md[5] / (g_md[6] ? g_md[6] : 1));
	printf("hops:"); for (int i = 1; i < 10; i++) printf(" %ld", g_hops[i]); printf("\n");
	return bad != 0;
}
