/*
 * oracle/oracle.c -- CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as a checker.
 * The product path (bowtie2-server_amd/csrc) never links or calls it.
 *
 * Plain C restatement of sfiligoi/bowtie2-server (bowtie2 2.5.4), following:
 *   SideLocus / occ counting ... bt2_idx.h:317-397, 1758-1793, 1887-2080
 *   mapLF / mapLF1 / mapBiLFEx .. bt2_idx.h:2313-2473
 *   ftab ........................ bt2_idx.h:1374-1554
 *   getOffset ................... bt2_idx.cpp:150-171
 *   exactSweep .................. aligner_seed.cpp:750-968
 *   oneMmSearch ................. aligner_seed.cpp:973-1323
 *   exact seeds (searchSeedBi) .. aligner_seed.cpp:80-122, 214-358, 498-587,
 *                                  1364-1432, 1633-1714, 1854-2033
 *   SW fills (scalar, same saturating value domains as the striped SSE code):
 *     EE u8   aligner_swsse_ee_u8.cpp:75-142, 775-1146 (gather 1176-1208)
 *     EE i16  aligner_swsse_ee_i16.cpp:75-145, 780-1200
 *     loc u8  aligner_swsse_loc_u8.cpp:75-159, 927-1336 (gather 1389-1500)
 *     loc i16 aligner_swsse_loc_i16.cpp:75-145, 938-1367 (gather 1420-1535)
 *     dispatch SwAligner::align aligner_sw.cpp:500-729; Scoring scoring.h:96-440
 *   ungapped: SwAligner::ungappedAlign aligner_sw.cpp:286-494
 *   framing: DynProgFramer dp_framer.cpp:81-129, 177-383; PairedEndPolicy::
 *     otherMate pe.cpp:161-352; Scoring::maxReadGaps/maxRefGaps scoring.cpp:42-98
 *   backtrace: SwAligner::nextAlignment aligner_sw.cpp:737-1146 with
 *     backtraceNucleotides{End2End,Local}Sse{U8,I16}
 *     (aligner_swsse_ee_u8.cpp:1283-1780, aligner_swsse_loc_u8.cpp:1588-2175,
 *      same walk in the i16 files), SSEMatrix masks aligner_swsse.h:263-494
 *
 * Pinned by tests/test_oracle_golden.py against vectors produced by the
 * reference itself (oracle/_ref/libbt2ref.so, tests/golden/make_golden.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OFF_MASK 0xffffffffu
#define MIN_I64 ((int64_t)0x8000000000000000LL)

typedef struct {
	const uint8_t*  ebwt;      /* sides, 64 B each */
	const uint32_t* fchr;      /* 5 */
	const uint32_t* ftab;
	const uint32_t* eftab;
	const uint32_t* offs;      /* may be NULL (mirror index) */
	uint32_t len;
	uint32_t zoff;
	uint32_t ftab_chars;
	uint32_t off_rate;
	int fw;                    /* 1 = forward index (Ebwt::fw()) */
} orc_ebwt;

typedef struct {
	uint32_t side_byte_off;
	uint32_t char_off;
	int by, bp;                /* bp = -1 -> invalid */
} orc_locus;

static uint8_t cnt_lut[4][4][256]; /* [bp][c][byte] as cCntLUT_4 (bp 0 = all 4) */
static int lut_ready = 0;

static void init_lut(void) {
	if(lut_ready) return;
	for(int bp = 0; bp < 4; bp++)
		for(int c = 0; c < 4; c++)
			for(int b = 0; b < 256; b++) {
				int n = 0, lim = bp == 0 ? 4 : bp;
				for(int k = 0; k < lim; k++) if(((b >> (2 * k)) & 3) == c) n++;
				cnt_lut[bp][c][b] = (uint8_t)n;
			}
	lut_ready = 1;
}

static void loc_from_row(orc_locus* l, uint32_t row) {
	uint32_t side = row / 192u;
	l->char_off = row % 192u;
	l->side_byte_off = side * 64u;
	l->by = (int)(l->char_off >> 2);
	l->bp = (int)(l->char_off & 3);
}

/* INIT_LOCS (aligner_seed.h:1847); initFromTopBot == initFromRow(bot) numerically */
static void init_locs(uint32_t top, uint32_t bot, orc_locus* t, orc_locus* b) {
	loc_from_row(t, top);
	if(bot - top == 1) b->bp = -1;
	else loc_from_row(b, bot);
}

static void zpos(const orc_ebwt* e, uint32_t* zbyte, int* zbp) {
	uint32_t side = e->zoff / 192u, co = e->zoff % 192u;
	*zbyte = side * 64u + (co >> 2);
	*zbp = (int)(co & 3);
}

static int dollar_before(const orc_ebwt* e, const orc_locus* l) {
	uint32_t zb; int zbp;
	zpos(e, &zb, &zbp);
	uint32_t p = l->side_byte_off + (uint32_t)l->by;
	if(l->side_byte_off <= zb && p >= zb) {
		if(p > zb || (p == zb && l->bp > zbp)) return 1;
	}
	return 0;
}

/* countBt2SideEx (bt2_idx.h:1887) */
static void count_side_ex(const orc_ebwt* e, const orc_locus* l, uint32_t* arrs) {
	const uint8_t* side = e->ebwt + l->side_byte_off;
	uint32_t a[4] = {0, 0, 0, 0};
	int i;
	for(i = 0; i < l->by; i++) for(int c = 0; c < 4; c++) a[c] += cnt_lut[0][c][side[i]];
	if(l->bp > 0) for(int c = 0; c < 4; c++) a[c] += cnt_lut[l->bp][c][side[i]];
	if(dollar_before(e, l)) a[0]--;
	const uint32_t* occ = (const uint32_t*)(side + 48);
	for(int c = 0; c < 4; c++) arrs[c] = a[c] + occ[c] + e->fchr[c];
}

/* countBt2Side (bt2_idx.h:1758) */
static uint32_t count_side(const orc_ebwt* e, const orc_locus* l, int c) {
	uint32_t a[4];
	count_side_ex(e, l, a);
	return a[c];
}

static int row_l(const orc_ebwt* e, const orc_locus* l) {
	return (e->ebwt[l->side_byte_off + (uint32_t)l->by] >> (2 * l->bp)) & 3;
}

/* mapLF1(row, l, c) (bt2_idx.h:2420) */
static uint32_t map_lf1c(const orc_ebwt* e, uint32_t row, const orc_locus* l, int c) {
	if(row_l(e, l) != c || row == e->zoff) return OFF_MASK;
	return count_side(e, l, c);
}

/* mapLF1(row&, l) (bt2_idx.h:2451) */
static int map_lf1(const orc_ebwt* e, uint32_t* row, const orc_locus* l) {
	if(*row == e->zoff) return -1;
	int c = row_l(e, l);
	*row = count_side(e, l, c);
	return c;
}

/* mapBiLFEx (bt2_idx.h:2372) */
static void map_bilf_ex(const orc_ebwt* e, const orc_locus* lt, const orc_locus* lb,
                        uint32_t* t, uint32_t* b, uint32_t* tp, uint32_t* bp) {
	count_side_ex(e, lt, t);
	count_side_ex(e, lb, b);
	bp[0] = tp[0] + (b[0] - t[0]);
	tp[1] = bp[0];
	bp[1] = tp[1] + (b[1] - t[1]);
	tp[2] = bp[1];
	bp[2] = tp[2] + (b[2] - t[2]);
	tp[3] = bp[2];
	bp[3] = tp[3] + (b[3] - t[3]);
}

static uint32_t ftab_hi(const orc_ebwt* e, uint32_t i) {
	uint32_t v = e->ftab[i];
	if(v <= e->len) return v;
	return e->eftab[(v ^ OFF_MASK) * 2 + 1];
}
static uint32_t ftab_lo(const orc_ebwt* e, uint32_t i) {
	uint32_t v = e->ftab[i];
	if(v <= e->len) return v;
	return e->eftab[(v ^ OFF_MASK) * 2];
}

/* ftabSeqToInt (bt2_idx.h:1374); returns OFF_MASK on N */
static uint32_t ftab_seq_to_int(const orc_ebwt* e, const uint8_t* seq, uint32_t off, int rev) {
	uint32_t fc = e->ftab_chars, lo = off, hi = off + fc, v = 0;
	for(uint32_t i = 0; i < fc; i++) {
		int fwex = e->fw;
		if(rev) fwex = !fwex;
		int c = fwex ? seq[lo + i] : seq[hi - i - 1];
		if(c > 3) return OFF_MASK;
		v = (v << 2) | (uint32_t)c;
	}
	return v;
}

void orc_ftab_lohi(const orc_ebwt* e, uint32_t i, uint32_t* top, uint32_t* bot) {
	*top = ftab_hi(e, i);
	*bot = ftab_lo(e, i + 1);
}

/* One LF/bi-LF step from [top,bot) with mirror start topp, as bt2ref_bilf. */
void orc_bilf(const orc_ebwt* e, uint32_t top, uint32_t bot, uint32_t topp,
              uint32_t* t, uint32_t* b, uint32_t* tp, uint32_t* bp) {
	init_lut();
	orc_locus lt, lb;
	init_locs(top, bot, &lt, &lb);
	for(int i = 0; i < 4; i++) { t[i] = b[i] = 0; tp[i] = topp; bp[i] = topp + (bot - top); }
	if(lb.bp >= 0) {
		map_bilf_ex(e, &lt, &lb, t, b, tp, bp);
	} else {
		uint32_t row = top;
		int c = map_lf1(e, &row, &lt);
		if(c >= 0) { t[c] = row; b[c] = row + 1; }
		for(int i = 0; i < 4; i++) { tp[i] = topp; bp[i] = topp + (i == c ? 1u : 0u); }
	}
}

/* Ebwt::getOffset (bt2_idx.cpp:150) */
uint32_t orc_get_offset(const orc_ebwt* e, uint32_t row) {
	init_lut();
	uint32_t mask = OFF_MASK << e->off_rate;
	if(row == e->zoff) return 0;
	if((row & mask) == row) return e->offs[row >> e->off_rate];
	uint32_t jumps = 0;
	orc_locus l;
	loc_from_row(&l, row);
	for(;;) {
		int c = row_l(e, &l);
		uint32_t nr = count_side(e, &l, c);
		jumps++;
		row = nr;
		if(row == e->zoff) return jumps;
		if((row & mask) == row) return jumps + e->offs[row >> e->off_rate];
		loc_from_row(&l, row);
	}
}

/* ---------------------------------------------------------------------- */
/* SwDriver::extend (aligner_sw_driver.cpp:299-483): how far a seed-hit     */
/* range extends left (forward index) and right (mirror index) without an  */
/* edit.  seq: the read's codes (patFw); fw: seed on the read (1) or on its */
/* reverse complement (0); off/len: the seed from the 5' end.               */
/* out: nlex, nrex, LF steps (PerReadMetrics::nSdFmops increments).         */
/* ---------------------------------------------------------------------- */
static uint32_t ext_walk(const orc_ebwt* e, uint32_t top, uint32_t bot, const uint8_t* seq, uint32_t rdlen, int fw,
                         uint32_t lim, int64_t i0, int dir, uint32_t* fmops) {
	uint32_t n = 0;
	orc_locus tl, bl;
	init_locs(top, bot, &tl, &bl);
	for(uint32_t ii = 0; ii < lim; ii++) {
		int64_t i = i0 + (int64_t)dir * ii;
		int rdc = fw ? seq[i] : seq[rdlen - 1 - i];
		if(!fw) rdc = rdc > 3 ? 4 : 3 - rdc;      /* patRc */
		(*fmops)++;
		if(bl.bp >= 0) {
			uint32_t t[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0}, tp[4] = {0, 0, 0, 0}, bp[4] = {0, 0, 0, 0};
			map_bilf_ex(e, &tl, &bl, t, b, tp, bp);
			int nonz = -1, abort_ = 0;
			uint32_t orig = bot - top;
			for(int j = 0; j < 4; j++) {
				if(b[j] > t[j]) {
					if(nonz >= 0) { abort_ = 1; break; }
					nonz = j;
					top = t[j];
					bot = b[j];
				}
			}
			if(abort_ || (nonz != rdc && rdc <= 3) || bot - top < orig) break;
		} else {
			int c = map_lf1(e, &top, &tl);
			if(c != rdc && rdc <= 3) break;
			bot = top + 1;
		}
		if(++n == 255u) break;
		init_locs(top, bot, &tl, &bl);
	}
	return n;
}

void orc_extend(const orc_ebwt* fwi, const orc_ebwt* bwi, const uint8_t* seq, uint32_t rdlen, int fw, uint32_t off,
                uint32_t len, uint32_t topf, uint32_t botf, uint32_t topb, uint32_t botb, uint32_t* out) {
	init_lut();
	uint32_t fmops = 0, nlex = 0, nrex = 0;
	uint32_t lim = fw ? off : rdlen - len - off;
	if(lim > 0) nlex = ext_walk(fwi, topf, botf, seq, rdlen, fw, lim, fw ? (int64_t)off - 1 : (int64_t)rdlen - off - len - 1, -1, &fmops);
	lim = fw ? rdlen - len - off : off;
	if(lim > 0 && bwi) nrex = ext_walk(bwi, topb, botb, seq, rdlen, fw, lim, fw ? (int64_t)len + off : (int64_t)rdlen - off, 1, &fmops);
	out[0] = nlex;
	out[1] = nrex;
	out[2] = fmops;
}

/* ---------------------------------------------------------------------- */
/* exactSweep (aligner_seed.cpp:750-968), one strand at a time.            */
/* ---------------------------------------------------------------------- */
static void sweep_strand(const orc_ebwt* e, const uint8_t* seq, uint32_t len, uint32_t mine_max,
                         uint32_t* mine, uint32_t* top_o, uint32_t* bot_o, uint64_t* bwops,
                         uint64_t* nelt) {
	uint32_t dep = 0, nedit = 0, top = 0, bot = 0;
	int doinit = 1, done = 0;
	orc_locus tl, bl;
	tl.bp = bl.bp = -1;
	uint32_t flen = e->ftab_chars;
	*top_o = *bot_o = 0;
	while(dep < len && !done) {
		if(doinit) {
			/* exactSweepInit */
			top = bot = 0;
			uint32_t left = len - dep;
			int doftab = flen > 1 && left >= flen;
			if(doftab) {
				uint32_t endi = len - dep - 1;
				for(uint32_t i = 0; i < flen; i++) if(seq[endi - i] > 3) { doftab = 0; break; }
			}
			if(doftab) {
				uint32_t fi = ftab_seq_to_int(e, seq, left - flen, 0);
				orc_ftab_lohi(e, fi, &top, &bot);
				dep += flen;
			} else {
				int c = seq[len - dep - 1];
				if(c < 4) { top = e->fchr[c]; bot = e->fchr[c + 1]; }
				dep++;
			}
			/* exactSweepStep */
			if(bot <= top) {
				nedit++;
				if(nedit >= mine_max) { *mine = nedit; done = 1; }
				continue;
			}
			init_locs(top, bot, &tl, &bl);
			doinit = 0;
		}
		if(dep < len) {
			/* exactSweepMapLF */
			int c = seq[len - dep - 1];
			if(c > 3) {
				top = bot = 0;
			} else if(bl.bp >= 0) {
				*bwops += 2;
				top = count_side(e, &tl, c);
				bot = count_side(e, &bl, c);
			} else {
				*bwops += 1;
				top = map_lf1c(e, top, &tl, c);
				if(top == OFF_MASK) top = bot = 0;
				else bot = top + 1;
			}
			if(bot <= top) {
				nedit++;
				if(nedit >= mine_max) { *mine = nedit; done = 1; }
				doinit = 1;
			} else {
				init_locs(top, bot, &tl, &bl);
			}
			dep++;
		}
	}
	if(!done && dep >= len) {
		*mine = nedit;
		if(nedit == 0 && bot > top) {
			*top_o = top; *bot_o = bot;
			*nelt += bot - top;
		}
	}
}

/* reads: n rows of `stride` codes (0-3, 4=N); rc computed here.
 * out per read (8 x u64): mineFw, mineRc, nelt, fwtop, fwbot, rctop, rcbot, bwops */
void orc_exact_sweep(const orc_ebwt* e, const uint8_t* reads, uint32_t stride, const uint32_t* lens,
                     uint32_t n, uint32_t mine_max, uint64_t* out) {
	init_lut();
	uint8_t* rc = (uint8_t*)malloc(stride + 1);
	for(uint32_t r = 0; r < n; r++) {
		const uint8_t* fw = reads + (size_t)r * stride;
		uint32_t len = lens[r];
		for(uint32_t i = 0; i < len; i++) { uint8_t c = fw[len - 1 - i]; rc[i] = c > 3 ? 4 : (uint8_t)(3 - c); }
		uint64_t* o = out + 8 * (size_t)r;
		uint32_t mfw = 0, mrc = 0, t1, b1, t2, b2;
		uint64_t bw = 0, nelt = 0;
		sweep_strand(e, fw, len, mine_max, &mfw, &t1, &b1, &bw, &nelt);
		sweep_strand(e, rc, len, mine_max, &mrc, &t2, &b2, &bw, &nelt);
		o[0] = mfw; o[1] = mrc; o[2] = nelt; o[3] = t1; o[4] = b1; o[5] = t2; o[6] = b2; o[7] = bw;
	}
	free(rc);
}

/* ---------------------------------------------------------------------- */
/* Exact seeds: instantiateSeeds + searchSeedBi for SEED_TYPE_EXACT         */
/* ---------------------------------------------------------------------- */
/* Search one seed string (as aligned to Watson).  Returns 1 and the 4 bounds on
 * a hit, 0 on no hit.  bwops incremented per LF step. */
int orc_search_exact_seed(const orc_ebwt* fwi, const orc_ebwt* bwi, const uint8_t* seq, uint32_t L,
                          uint32_t* out4, uint64_t* bwops) {
	init_lut();
	uint32_t topf, botf, topb, botb, step;
	uint32_t flen = fwi->ftab_chars;
	if(flen > 1 && flen <= L) {
		uint32_t off = L - flen;
		uint32_t i0f = ftab_seq_to_int(fwi, seq, off, 0);
		uint32_t i0b = ftab_seq_to_int(bwi, seq, off, 0);
		orc_ftab_lohi(fwi, i0f, &topf, &botf);
		if(botf - topf == 0) return 0;
		topb = ftab_hi(bwi, i0b);
		botb = topb + (botf - topf);
		step = flen;
	} else {
		int c = seq[L - 1];
		topf = topb = fwi->fchr[c];
		botf = botb = fwi->fchr[c + 1];
		if(botf - topf == 0) return 0;
		step = 1;
	}
	for(; step < L; step++) {
		uint32_t off = L - step - 1;
		orc_locus tl, bl;
		init_locs(topf, botf, &tl, &bl);
		uint32_t t[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
		uint32_t tp[4] = {topb, topb, topb, topb}, bp[4] = {botb, botb, botb, botb};
		(*bwops)++;
		if(bl.bp >= 0) map_bilf_ex(fwi, &tl, &bl, t, b, tp, bp);
		int c = seq[off];
		if(bl.bp < 0) {
			t[c] = map_lf1c(fwi, topf, &tl, c);
			if(t[c] == OFF_MASK) return 0;
			b[c] = t[c] + 1;
		}
		if(b[c] == t[c]) return 0;
		topf = t[c]; botf = b[c]; topb = tp[c]; botb = bp[c];
	}
	out4[0] = topf; out4[1] = botf; out4[2] = topb; out4[3] = botb;
	return 1;
}

/* One seed round: offsets off + i*interval; per read writes [2][maxseeds][4]
 * (fw then rc) bounds (zeros when no hit / filtered), nseeds, bwops. */
void orc_seed_search(const orc_ebwt* fwi, const orc_ebwt* bwi, const uint8_t* reads, uint32_t stride,
                     const uint32_t* lens, uint32_t n, uint32_t seedlen, uint32_t interval,
                     uint32_t offset, uint32_t maxseeds, uint32_t* out, int32_t* nseeds, uint64_t* bwops) {
	init_lut();
	uint8_t sq[1024];
	for(uint32_t r = 0; r < n; r++) {
		const uint8_t* rd = reads + (size_t)r * stride;
		uint32_t len = lens[r];
		uint32_t L = seedlen < len ? seedlen : len;
		uint32_t* o = out + (size_t)r * 2 * maxseeds * 4;
		memset(o, 0, sizeof(uint32_t) * 2 * maxseeds * 4);
		nseeds[r] = 0; bwops[r] = 0;
		/* bt2_search.cpp:3866-3869: round skipped if the offset drives the first seed off the end */
		if(offset > 0 && seedlen + offset > len) continue;
		int ns = 1;
		if((int)len - (int)offset > (int)seedlen) ns += ((int)len - (int)offset - (int)seedlen) / (int)interval;
		nseeds[r] = ns;
		uint64_t bw = 0;
		for(int fw = 1; fw >= 0; fw--) {
			for(int s = 0; s < ns && s < (int)maxseeds; s++) {
				uint32_t depth = (uint32_t)s * interval + offset;
				int hasn = 0;
				for(uint32_t i = 0; i < L; i++) {
					/* Read::windowGetDna: fw -> buf[depth+i]; rc -> comp(buf[depth+len-i-1]) */
					uint8_t c = fw ? rd[depth + i] : rd[depth + L - i - 1];
					if(!fw) c = c > 3 ? 4 : (uint8_t)(3 - c);
					sq[i] = c;
					if(c > 3) hasn = 1;
				}
				if(hasn) continue; /* Seed::instantiate: exact zone cannot absorb an N */
				uint32_t* q = o + ((size_t)(fw ? 0 : 1) * maxseeds + s) * 4;
				orc_search_exact_seed(fwi, bwi, sq, L, q, &bw);
			}
		}
		bwops[r] = bw;
	}
}

/* ---------------------------------------------------------------------- */
/* Scoring (scoring.h:103-131, 241-251)                                     */
/* ---------------------------------------------------------------------- */
typedef struct {
	int32_t match, mmp_max, mmp_min, npen, rdg_const, rdg_lin, rfg_const, rfg_lin, gapbar, local;
	double ncl_const, ncl_lin;
} orc_scoring;

static int mmpen_q(const orc_scoring* s, int q) {
	int ii = q < 40 ? q : 40;
	float frac = (float)ii / 40.0f;
	return s->mmp_min + (int)(frac * (s->mmp_max - s->mmp_min));
}

static int score_of(const orc_scoring* s, int rdc, int refm, int q) {
	if(rdc > 3 || refm > 15) return -s->npen;
	if((refm & (1 << rdc)) != 0) return s->match;
	return -mmpen_q(s, q);
}

/* ---------------------------------------------------------------------- */
/* oneMmSearch (aligner_seed.cpp:973-1323), rep1mm=true, repex=false        */
/* ---------------------------------------------------------------------- */
typedef struct { uint32_t top, bot; int32_t fw; int64_t score; int32_t pos, chr, qchr; } orc_mm1;

static int one_mm_read(const orc_ebwt* F, const orc_ebwt* B, const uint8_t* fwc, const uint8_t* q33,
                       uint32_t len, int64_t minsc, int local, int nofw, int norc,
                       const orc_scoring* sc, orc_mm1* hits, int cap, int* nh, uint64_t* bwops) {
	int nceil = (int)(sc->ncl_const + sc->ncl_lin * (double)len);
	if(nceil < 0) nceil = 0;
	uint32_t ns = 0;
	for(uint32_t i = 0; i < len; i++) if(fwc[i] > 3) ns++;
	*nh = 0;
	if(ns > 1) return 0;
	uint8_t patFw[1024], patRc[1024], patFwRev[1024], patRcRev[1024], qual[1024], qualRev[1024];
	for(uint32_t i = 0; i < len; i++) {
		patFw[i] = fwc[i];
		uint8_t c = fwc[len - 1 - i];
		patRc[i] = c > 3 ? 4 : (uint8_t)(3 - c);
		qual[i] = q33[i];
	}
	for(uint32_t i = 0; i < len; i++) {
		patFwRev[i] = patFw[len - 1 - i]; patRcRev[i] = patRc[len - 1 - i]; qualRev[i] = qual[len - 1 - i];
	}
	uint32_t halfFw = len >> 1, halfBw = len >> 1;
	if(len & 1) halfBw++;
	orc_locus tl, bl;
	uint32_t t[5] = {0}, b[5] = {0}, tp[5] = {0}, bp[5] = {0};
	uint32_t top = 0, bot = 0, topp = 0, botp = 0;
	int results = 0;
	int64_t matchsc = (int64_t)((float)sc->match + 0.5f);
	for(int fwi = 0; fwi < 2; fwi++) {
		int fw = fwi == 0;
		if(fw && nofw) continue;
		if(!fw && norc) continue;
		for(int ebwtfwi = 0; ebwtfwi < 2; ebwtfwi++) {
			int ebwtfw = ebwtfwi == 0;
			const orc_ebwt* ebwt = ebwtfw ? F : B;
			const orc_ebwt* ebwtp = ebwtfw ? B : F;
			const uint8_t* seq = fw ? (ebwtfw ? patFw : patFwRev) : (ebwtfw ? patRc : patRcRev);
			const uint8_t* qu = fw ? (ebwtfw ? qual : qualRev) : (ebwtfw ? qualRev : qual);
			uint32_t flen = ebwt->ftab_chars;
			uint32_t nea = ebwtfw ? halfFw : halfBw;
			int skip = 0;
			for(uint32_t dep = 0; dep < nea; dep++) if(seq[len - dep - 1] > 3) { skip = 1; break; }
			if(skip) continue;
			uint32_t dep = 0;
			if(flen > 1 && flen <= nea) {
				int rev = !ebwtfw;
				uint32_t fi = ftab_seq_to_int(ebwt, seq, len - flen, rev);
				orc_ftab_lohi(ebwt, fi, &top, &bot);
				uint32_t fip = ftab_seq_to_int(ebwtp, seq, len - flen, rev);
				orc_ftab_lohi(ebwtp, fip, &topp, &botp);
				if(bot - top == 0) continue;
				int c = seq[len - flen];
				t[c] = top; b[c] = bot; tp[c] = topp; bp[c] = botp;
				dep = flen;
			} else {
				int c = seq[len - 1];
				top = topp = tp[c] = ebwt->fchr[c];
				bot = botp = bp[c] = ebwt->fchr[c + 1];
				if(bot - top == 0) continue;
				dep = 1;
			}
			init_locs(top, bot, &tl, &bl);
			int do_continue = 0;
			for(; dep < nea; dep++) {
				int rdc = seq[len - dep - 1];
				for(int i = 0; i < 4; i++) { tp[i] = topp; bp[i] = botp; }
				if(bl.bp >= 0) {
					(*bwops)++;
					for(int i = 0; i < 4; i++) t[i] = b[i] = 0;
					map_bilf_ex(ebwt, &tl, &bl, t, b, tp, bp);
					top = t[rdc]; bot = b[rdc];
					if(bot <= top) { do_continue = 1; break; }
					topp = tp[rdc]; botp = bp[rdc];
				} else {
					(*bwops)++;
					top = map_lf1c(ebwt, top, &tl, rdc);
					if(top == OFF_MASK) { do_continue = 1; break; }
					bot = top + 1;
					t[rdc] = top; b[rdc] = bot; tp[rdc] = topp; bp[rdc] = botp;
				}
				init_locs(top, bot, &tl, &bl);
			}
			if(do_continue) continue;
			for(; dep < len; dep++) {
				int rdc = seq[len - dep - 1];
				int quc = qu[len - dep - 1];
				if(rdc > 3 && nceil == 0) break;
				for(int i = 0; i < 4; i++) { tp[i] = topp; bp[i] = botp; }
				int clo = 0, chi = 3, match = 1;
				if(bl.bp >= 0) {
					(*bwops)++;
					for(int i = 0; i < 4; i++) t[i] = b[i] = 0;
					map_bilf_ex(ebwt, &tl, &bl, t, b, tp, bp);
					match = rdc < 4;
					if(rdc < 4) { top = t[rdc]; bot = b[rdc]; topp = tp[rdc]; botp = bp[rdc]; }
				} else {
					(*bwops)++;
					clo = map_lf1(ebwt, &top, &tl);
					match = (clo == rdc);
					if(clo < 0) break;
					t[clo] = top;
					b[clo] = bot = top + 1;
					bp[clo] = botp; tp[clo] = topp;
					chi = clo;
				}
				if(ns == 0 || rdc > 3) {
					for(int j = clo; j <= chi; j++) {
						if(j == rdc || b[j] == t[j]) continue;
						uint32_t depm = dep + 1;
						uint32_t topm = t[j], botm = b[j], topmp = tp[j], botmp = bp[j];
						orc_locus tlm, blm;
						init_locs(topm, botm, &tlm, &blm);
						for(; depm < len; depm++) {
							int rdcm = seq[len - depm - 1];
							uint32_t tm[4] = {0, 0, 0, 0}, bm[4] = {0, 0, 0, 0};
							uint32_t tmp[4] = {topmp, topmp, topmp, topmp}, bmp[4] = {botmp, botmp, botmp, botmp};
							if(blm.bp >= 0) {
								(*bwops)++;
								map_bilf_ex(ebwt, &tlm, &blm, tm, bm, tmp, bmp);
								topm = tm[rdcm]; botm = bm[rdcm]; topmp = tmp[rdcm]; botmp = bmp[rdcm];
								if(botm <= topm) break;
							} else {
								(*bwops)++;
								topm = map_lf1c(ebwt, topm, &tlm, rdcm);
								if(topm == OFF_MASK) break;
								botm = topm + 1;
							}
							init_locs(topm, botm, &tlm, &blm);
						}
						if(depm == len) {
							uint32_t off5p = dep;
							if(fw == ebwtfw) off5p = len - off5p - 1;
							results = 1;
							int64_t score = (int64_t)(len - 1) * matchsc;
							int pen = score_of(sc, rdc, 1 << j, quc - 33);
							score += pen;
							int valid = 1;
							if(local) {
								int64_t lf = 0, lb = 0;
								for(uint32_t i = 0; i < len; i++) {
									if(i == dep) {
										if(lf + pen <= 0) { valid = 0; break; }
										lf += pen;
									} else lf += matchsc;
									if(len - i - 1 == dep) {
										if(lb + pen <= 0) { valid = 0; break; }
										lb += pen;
									} else lb += matchsc;
								}
							}
							if(valid) valid = score >= minsc;
							if(valid) {
								if(*nh < cap) {
									orc_mm1* h = &hits[*nh];
									h->top = ebwtfw ? topm : topmp;
									h->bot = ebwtfw ? botm : botmp;
									h->fw = fw; h->score = score; h->pos = (int32_t)off5p;
									h->chr = j; h->qchr = rdc;
								}
								(*nh)++;
							}
						}
					}
				}
				if(bot > top && match) {
					if(dep == len - 1) break;
					init_locs(top, bot, &tl, &bl);
				} else {
					break;
				}
			}
		}
	}
	return results;
}

/* out per read: cap hits x 7 int64 (top,bot,fw,score,pos,chr,qchr); counts; bwops */
void orc_one_mm(const orc_ebwt* F, const orc_ebwt* B, const uint8_t* reads, const uint8_t* quals,
                uint32_t stride, const uint32_t* lens, uint32_t n, const int64_t* minsc, int local,
                int nofw, int norc, const orc_scoring* sc, int cap, int64_t* out, int32_t* counts,
                uint64_t* bwops) {
	init_lut();
	orc_mm1* hits = (orc_mm1*)malloc(sizeof(orc_mm1) * (size_t)(cap > 0 ? cap : 1));
	for(uint32_t r = 0; r < n; r++) {
		int nh = 0;
		uint64_t bw = 0;
		one_mm_read(F, B, reads + (size_t)r * stride, quals + (size_t)r * stride, lens[r], minsc[r],
		            local, nofw, norc, sc, hits, cap, &nh, &bw);
		counts[r] = nh;
		bwops[r] = bw;
		for(int k = 0; k < nh && k < cap; k++) {
			int64_t* o = out + ((size_t)r * cap + k) * 7;
			o[0] = hits[k].top; o[1] = hits[k].bot; o[2] = hits[k].fw; o[3] = hits[k].score;
			o[4] = hits[k].pos; o[5] = hits[k].chr; o[6] = hits[k].qchr;
		}
	}
	free(hits);
}

/* ---------------------------------------------------------------------- */
/* SW fills (scalar restatement of the striped SSE2 kernels)                */
/* ---------------------------------------------------------------------- */
static inline int subs_u8(int a, int b) { int r = a - b; return r < 0 ? 0 : r; }
static inline int adds_u8(int a, int b) { int r = a + b; return r > 255 ? 255 : r; }
static inline int sat16(int x) { return x < -32768 ? -32768 : (x > 32767 ? 32767 : x); }
static inline int max2(int a, int b) { return a > b ? a : b; }
static inline int max3(int a, int b, int c) { return max2(max2(a, b), c); }

static int firsts5(int m) {
	if(m & 1) return 0;
	if(m & 2) return 1;
	if(m & 4) return 2;
	if(m & 8) return 3;
	return 4;
}

typedef struct { int64_t row, col, score; } orc_cand;

static int cand_cmp(const void* pa, const void* pb) {
	const orc_cand* a = (const orc_cand*)pa;
	const orc_cand* b = (const orc_cand*)pb;
	if(a->score != b->score) return a->score > b->score ? -1 : 1;
	if(a->row != b->row) return a->row > b->row ? -1 : 1;
	if(a->col != b->col) return a->col > b->col ? -1 : 1;
	return 0;
}

/* One DP matrix in the native value domain of `variant`:
 *   0 = EE u8, 1 = EE i16, 2 = local u8, 3 = local i16.
 * The striped SSE2 kernels compute exactly this recurrence (Farrar's lazy-F
 * loop iterates to the fixpoint), including for local mode the padding rows
 * of the last striped segment (nrow rounded up to a multiple of the lane
 * count: 16 for u8, 8 for i16; profile score 0, no gap barrier), whose H
 * values feed the per-column maximum (vcolmax) that drives lastsolcol_ and
 * the column bail.  H/E/F (real rows only) and colmax are returned. */
static void sw_fill2(int variant, const uint8_t* rd, const uint8_t* q33, int nrow, const uint8_t* rf,
                     int ncol, const orc_scoring* sc, int* H, int* E, int* F, int* colmax, int* bias_o) {
	int W = (variant == 0 || variant == 2) ? 16 : 8;
	int seglen = (nrow + W - 1) / W;
	int nrowp = (variant >= 2) ? seglen * W : nrow;
	int rdgo = sc->rdg_const + sc->rdg_lin, rdge = sc->rdg_lin;
	int rfgo = sc->rfg_const + sc->rfg_lin, rfge = sc->rfg_lin;
	int LO = (variant == 0 || variant == 2) ? 0 : -32768;
	int bias = 0;
	if(variant == 2) {
		for(int c = 0; c < 5; c++) for(int r = 0; r < nrow; r++) {
			int s = score_of(sc, rd[r], 1 << c, q33[r] - 33);
			if(s < 0 && s < bias) bias = s;
		}
		bias = -bias;
	}
	*bias_o = bias;
	int* hprev = (int*)malloc(sizeof(int) * (size_t)nrowp);
	int* ecur = (int*)malloc(sizeof(int) * (size_t)nrowp);
	for(int r = 0; r < nrowp; r++) { hprev[r] = LO; ecur[r] = LO; }
	for(int j = 0; j < ncol; j++) {
		int refc = firsts5(rf[j]);
		int cm = LO;
		int fprev = LO, hup = LO;
		int diag = (variant == 0) ? 255 : (variant == 1) ? 32767 : LO; /* row -1 of this column's diagonal */
		for(int r = 0; r < nrowp; r++) {
			int real = r < nrow;
			int s = real ? score_of(sc, rd[r], 1 << refc, q33[r] - 33) : 0;
			int bar = real && (r < sc->gapbar || nrow - r - 1 < sc->gapbar);
			int hdiag = diag;
			diag = hprev[r];
			int f, h, en;
			if(variant == 0 || variant == 2) {
				f = (r == 0) ? 0 : (bar ? 0 : max2(subs_u8(fprev, rfge), subs_u8(hup, rfgo)));
				int d = (variant == 0) ? subs_u8(hdiag, -s) : subs_u8(adds_u8(hdiag, s + bias), bias);
				h = max3(d, ecur[r], f);
				en = max2(subs_u8(ecur[r], rdge), bar ? 0 : subs_u8(h, rdgo));
			} else {
				f = (r == 0) ? -32768 : (bar ? -32768 : max2(sat16(fprev - rfge), sat16(hup - rfgo)));
				int d = sat16(hdiag + s);
				h = max3(d, ecur[r], f);
				en = max2(sat16(ecur[r] - rdge), bar ? -32768 : sat16(h - rdgo));
			}
			if(r < nrow) {
				size_t k = (size_t)r * ncol + j;
				H[k] = h; E[k] = ecur[r]; F[k] = f;
			}
			if(h > cm) cm = h;
			ecur[r] = en;
			fprev = f; hup = h;
			hprev[r] = h;
		}
		colmax[j] = cm;
	}
	free(hprev); free(ecur);
}

/* SwAligner::align for one problem.  rf: ncol+1 masks (extra column right of
 * the rectangle).  out: [0]=aligned [1]=best [2]=u8succ [3]=i16succ [4]=colstop
 * [5]=lastsolcol [6]=ncand.  cands: up to cap (row,col,score) sorted.
 * mat (optional): nrow*ncol*3 ints (H,E,F) of the successful matrix. */
int orc_sw(const uint8_t* rd, const uint8_t* q33, int nrow, const uint8_t* rf, int ncol, int64_t minsc,
           const orc_scoring* sc, int enable8, int cap, int64_t* out, int64_t* cands, int32_t* mat) {
	size_t cells = (size_t)nrow * (size_t)ncol;
	int* H = (int*)malloc(sizeof(int) * cells);
	int* E = (int*)malloc(sizeof(int) * cells);
	int* F = (int*)malloc(sizeof(int) * cells);
	int* colmax = (int*)malloc(sizeof(int) * (size_t)ncol);
	int bias = 0, flag = 0, variant = -1, u8succ = 0, i16succ = 0;
	int64_t best = MIN_I64;
	int64_t colstop = 0, lastsol = 0;
	int64_t matchsc = (int64_t)((float)sc->match + 0.5f);
	if(!sc->local) {
		variant = (enable8 && minsc >= -254) ? 0 : 1;
		sw_fill2(variant, rd, q33, nrow, rf, ncol, sc, H, E, F, colmax, &bias);
		colstop = ncol - 1; lastsol = 0;
		if(variant == 0) {
			int lrmax = 0;
			for(int j = 0; j < ncol; j++) lrmax = max2(lrmax, H[(size_t)(nrow - 1) * ncol + j]);
			int64_t score = (int64_t)lrmax - 0xff;
			if(score < minsc) { flag = -1; best = score; }
			else if(lrmax == 0) { flag = -2; best = MIN_I64; }
			else { flag = 0; best = score; }
			u8succ = flag == 0;
		} else {
			int lrmax = -32768;
			for(int j = 0; j < ncol; j++) lrmax = max2(lrmax, H[(size_t)(nrow - 1) * ncol + j]);
			int64_t score = (int64_t)lrmax - 0x7fff;
			if(score < minsc) { flag = -1; best = score; }
			else if(lrmax == -32768) { flag = -2; best = MIN_I64; }
			else { flag = 0; best = score; }
			i16succ = flag == 0;
		}
	} else {
		flag = -2;
		if(enable8) {
			variant = 2;
			sw_fill2(2, rd, q33, nrow, rf, ncol, sc, H, E, F, colmax, &bias);
			colstop = ncol; lastsol = 0;
			int vmax = 0, sat = 0;
			for(int j = 0; j < ncol; j++) {
				vmax = max2(vmax, colmax[j]);
				int s = colmax[j];
				if(s + bias >= 255) { sat = 1; break; }
				if(s < minsc) {
					int64_t ncolleft = ncol - j - 1;
					if(s + ncolleft * matchsc < minsc) { colstop = j + 1; break; }
				} else {
					lastsol = j;
				}
			}
			if(sat || vmax + bias >= 255) { flag = -2; best = MIN_I64; }
			else if(vmax == 0 || vmax < minsc) { flag = -1; best = vmax; }
			else { flag = 0; best = vmax; }
			u8succ = flag == 0;
		}
		if(flag == -2) {
			variant = 3;
			flag = 0;
			sw_fill2(3, rd, q33, nrow, rf, ncol, sc, H, E, F, colmax, &bias);
			colstop = ncol; lastsol = 0;
			int ret = -32768;
			for(int j = 0; j < ncol; j++) {
				ret = max2(ret, colmax[j]);
				int64_t s = (int64_t)colmax[j] + 0x8000;
				if(s < minsc) {
					int64_t ncolleft = ncol - j - 1;
					if(s + ncolleft * matchsc < minsc) { colstop = j + 1; break; }
				} else {
					lastsol = j;
				}
			}
			if(ret == -32768) { flag = -1; best = MIN_I64; }
			else {
				int64_t score = (int64_t)ret + 0x8000;
				if(score < minsc) { flag = -1; best = score; }
				else if(ret == 32767) { flag = -2; best = MIN_I64; }
				else { flag = 0; best = score; }
			}
			i16succ = flag == 0;
		}
	}
	int64_t ncand = 0;
	int aligned = 0;
	if(!(best == MIN_I64 || best < minsc)) {
		size_t capc = (size_t)nrow * (size_t)ncol + 1;
		orc_cand* cl = (orc_cand*)malloc(sizeof(orc_cand) * capc);
		if(!sc->local) {
			int off = (variant == 0) ? 0xff : 0x7fff;
			for(int j = 0; j < ncol; j++) {
				int64_t s = (int64_t)H[(size_t)(nrow - 1) * ncol + j] - off;
				if(s >= minsc) { cl[ncand].row = nrow - 1; cl[ncand].col = j; cl[ncand].score = s; ncand++; }
			}
		} else {
			int W = variant == 2 ? 16 : 8;
			int iter = (nrow + W - 1) / W;
			uint64_t bonus = (uint64_t)matchsc;
			uint64_t minrow = (((uint64_t)minsc + bonus - 1) / bonus) - 1;
			int64_t off = variant == 2 ? 0 : 0x8000;
			for(int64_t j = 0; j < lastsol + 1; j++) {
				if((int64_t)colmax[j] + off < minsc) continue;
				for(int i = 0; i < iter; i++) {
					for(int k = 0; k < W; k++) {
						uint64_t rdoff = (uint64_t)i + (uint64_t)k * (uint64_t)iter;
						if(rdoff >= (uint64_t)nrow) break;
						if(rdoff < minrow) continue;
						int64_t s = (int64_t)H[rdoff * ncol + j] + off;
						if(s < minsc) continue;
						int readc = rd[rdoff];
						int refc = rf[j];
						int m = (refc & (1 << readc)) != 0;
						int ms = 0;
						if(rdoff < (uint64_t)nrow - 1) {
							int readc2 = rd[rdoff + 1];
							int refc2 = rf[j + 1];
							ms = (refc2 & (1 << readc2)) != 0;
						}
						if(m && !ms) { cl[ncand].row = (int64_t)rdoff; cl[ncand].col = j; cl[ncand].score = s; ncand++; }
					}
				}
			}
		}
		qsort(cl, (size_t)ncand, sizeof(orc_cand), cand_cmp);
		for(int64_t i = 0; i < ncand && i < cap; i++) {
			cands[3 * i] = cl[i].row; cands[3 * i + 1] = cl[i].col; cands[3 * i + 2] = cl[i].score;
		}
		free(cl);
		aligned = ncand > 0;
	}
	out[0] = aligned; out[1] = best; out[2] = u8succ; out[3] = i16succ;
	out[4] = colstop; out[5] = lastsol; out[6] = ncand;
	if(mat != NULL && (u8succ || i16succ)) {
		for(size_t k = 0; k < cells; k++) { mat[3 * k] = H[k]; mat[3 * k + 1] = E[k]; mat[3 * k + 2] = F[k]; }
	}
	free(H); free(E); free(F); free(colmax);
	return 0;
}

/* ---------------------------------------------------------------------- */
/* Backtrace: the SwDriver nextAlignment loop over one filled problem.      */
/* ---------------------------------------------------------------------- */
typedef struct { int32_t pos, chr, qchr, type; } orc_edit;
typedef struct {
	size_t nedsz, celsz, row, col, gaps, rdg, rfg; int64_t score; int ns; int ct;
} orc_btframe;

enum { CT_H = 0, CT_E = 1, CT_F = 2 };
enum { BT_DIAG, BT_REF_OPEN, BT_READ_OPEN, BT_RFGAP_EXT, BT_RDGAP_EXT };

static char mask2dna_c(int m) {
	switch(m) { case 1: return 'A'; case 2: return 'C'; case 4: return 'G'; case 8: return 'T'; default: return 'N'; }
}

/* One backtrace from (row, col) (aligner_swsse_ee_u8.cpp:1283-1780 /
 * aligner_swsse_loc_u8.cpp:1588-2175).  V = H/E/F values in score units
 * (value + offsetsc); local: neighbour values must be > 0 (floorsc).  marks =
 * reportedThrough bits (aligner_swsse.h:263-278), persistent across
 * candidates.  Returns 1 on success with the alignment in *ed / aout. */
static int orc_bt_one(const int64_t* VH, const int64_t* VE, const int64_t* VF, uint8_t* marks,
                      const uint8_t* rd, const uint8_t* q33, int nrow, const uint8_t* rf, int ncol,
                      const orc_scoring* sc, int local, int triml, int corel, int corer, int nceil,
                      size_t row, size_t col, orc_edit* ed, size_t* ned_o, int64_t* aout,
                      orc_btframe* stack, size_t* cells) {
	const int rdgo = sc->rdg_const + sc->rdg_lin, rdge = sc->rdg_lin;
	const int rfgo = sc->rfg_const + sc->rfg_lin, rfge = sc->rfg_lin;
	const int64_t match30 = sc->match;
	size_t nst = 0, ncell = 0, ned = 0;
	size_t origCol = col, trimEnd = (size_t)nrow - row - 1, trimBeg = 0;
	size_t gaps = 0, readGaps = 0, refGaps = 0;
	int64_t score = 0; int ns = 0;
	int ct = CT_H;
#define V(M, r, c) (M[(size_t)(r) * ncol + (c)])
#define OK(x) (!local || (x) > 0)
	while((long)row >= 0) {
		int readc = rd[row], refm = rf[col], readq = q33[row];
		int empty = 0, canMoveThru = 1, branch = 0, cur = -1;
		if(marks[row * ncol + col]) {
			canMoveThru = 0;
		} else if(row > 0) {
			size_t rowFromEnd = (size_t)nrow - row - 1;
			int gapsAllowed = !(row < (size_t)sc->gapbar || rowFromEnd < (size_t)sc->gapbar);
			int origMask = 0;
			if(ct == CT_E) {
				int64_t cur_ = V(VE, row, col), hl = V(VH, row, col - 1), el = V(VE, row, col - 1);
				if(OK(hl) && hl - rdgo == cur_) origMask |= 1;
				if(OK(el) && el - rdge == cur_) origMask |= 2;
				/* mask == 3 picks H (the '#if 1' branch, aligner_swsse_ee_u8.cpp:1376-1392) */
				if(origMask == 3) { cur = BT_READ_OPEN; branch = 1; }
				else if(origMask == 2) cur = BT_RDGAP_EXT;
				else if(origMask == 1) cur = BT_READ_OPEN;
				else { empty = 1; canMoveThru = 1; }
			} else if(ct == CT_F) {
				int64_t cur_ = V(VF, row, col), hu = V(VH, row - 1, col), fu = V(VF, row - 1, col);
				if(OK(hu) && hu - rfgo == cur_) origMask |= 1;
				if(OK(fu) && fu - rfge == cur_) origMask |= 2;
				if(origMask == 3) { cur = BT_REF_OPEN; branch = 1; }
				else if(origMask == 2) cur = BT_RFGAP_EXT;
				else if(origMask == 1) cur = BT_REF_OPEN;
				else { empty = 1; canMoveThru = 1; }
			} else {
				int64_t cur_ = V(VH, row, col);
				int64_t fu = V(VF, row - 1, col), hu = V(VH, row - 1, col);
				int64_t hl = 0, el = 0, hul = 0; int hasl = col > 0;
				if(hasl) { hl = V(VH, row, col - 1); el = V(VE, row, col - 1); hul = V(VH, row - 1, col - 1); }
				int64_t sdiag = score_of(sc, readc, refm, readq - 33);
				if(gapsAllowed) {
					if(OK(hu) && cur_ == hu - rfgo) origMask |= 1;
					if(hasl && OK(hl) && cur_ == hl - rdgo) origMask |= 2;
					if(OK(fu) && cur_ == fu - rfge) origMask |= 4;
					if(hasl && OK(el) && cur_ == el - rdge) origMask |= 8;
				}
				if(hasl && OK(hul) && cur_ == hul + sdiag) origMask |= 16;
				/* fixed priority of the '#if 1' branch (aligner_swsse_ee_u8.cpp:1509-1520) */
				int npop = __builtin_popcount((unsigned)origMask);
				if(npop > 1) branch = 1;
				if(origMask & 16) cur = BT_DIAG;
				else if(origMask & 1) cur = BT_REF_OPEN;
				else if(origMask & 4) cur = BT_RFGAP_EXT;
				else if(origMask & 2) cur = BT_READ_OPEN;
				else if(origMask & 8) cur = BT_RDGAP_EXT;
				else { empty = 1; canMoveThru = 1; }
			}
		}
		marks[row * ncol + col] = 1;
		if(!canMoveThru) {
			if(nst > 0) {
				/* pop the last branch point (aligner_swsse_ee_u8.cpp:1560-1578) */
				orc_btframe* f = &stack[--nst];
				ncell = f->celsz; ned = f->nedsz; row = f->row; col = f->col;
				gaps = f->gaps; readGaps = f->rdg; refGaps = f->rfg; score = f->score; ns = f->ns; ct = f->ct;
				continue;
			}
			return 0;
		}
		if(empty || row == 0) {
			cells[2 * ncell] = row; cells[2 * ncell + 1] = col; ncell++;
			trimBeg = row;
			break;
		}
		if(branch) {
			orc_btframe f = { ned, ncell, row, col, gaps, readGaps, refGaps, score, ns, ct };
			stack[nst++] = f;
		}
		cells[2 * ncell] = row; cells[2 * ncell + 1] = col; ncell++;
		switch(cur) {
		case BT_DIAG: {
			int m = (refm >= 16 || readc > 3) ? -1 : (((1 << readc) & refm) ? 1 : 0);
			ct = CT_H;
			if(m != 1) {
				orc_edit e = { (int)row, mask2dna_c(refm), "ACGTN"[readc], 3 };
				ed[ned++] = e;
				score -= (readc > 3 || refm > 15) ? sc->npen : mmpen_q(sc, readq - 33);
			} else score += match30;
			if(m == -1) ns++;
			row--; col--;
			break;
		}
		case BT_REF_OPEN: case BT_RFGAP_EXT: {
			orc_edit e = { (int)row, '-', "ACGTN"[readc], 2 };
			ed[ned++] = e;
			score -= cur == BT_REF_OPEN ? rfgo : rfge;
			ct = cur == BT_REF_OPEN ? CT_H : CT_F;
			row--; gaps++; refGaps++;
			break;
		}
		default: { /* read gaps */
			orc_edit e = { (int)row + 1, mask2dna_c(rf[col]), '-', 1 };
			ed[ned++] = e;
			score -= cur == BT_READ_OPEN ? rdgo : rdge;
			ct = cur == BT_READ_OPEN ? CT_H : CT_E;
			col--; gaps++; readGaps++;
			break;
		}
		}
	}
#undef V
#undef OK
	/* must overlap a core diagonal (aligner_swsse_ee_u8.cpp:1764-1800) */
	int core = 0;
	for(size_t i = 0; i < ncell && !core; i++) {
		int64_t d = (int64_t)cells[2 * i + 1] - (int64_t)cells[2 * i] + triml;
		if(d >= 0 && d >= corel && d <= corer) core = 1;
	}
	if(!core) return 0;
	{
		int readc = rd[row], refm = rf[col];
		int m = (refm >= 16 || readc > 3) ? -1 : (((1 << readc) & refm) ? 1 : 0);
		if(m != 1) {
			orc_edit e = { (int)row, mask2dna_c(refm), "ACGTN"[readc], 3 };
			ed[ned++] = e;
			score -= (readc > 3 || refm > 15) ? sc->npen : mmpen_q(sc, q33[row] - 33);
		} else score += match30;
		if(m == -1) ns++;
	}
	if(ns > nceil) return 0;
	/* res.reverse(): edits 5'->3' of the DP read */
	for(size_t i = 0; i < ned / 2; i++) { orc_edit t = ed[i]; ed[i] = ed[ned - 1 - i]; ed[ned - 1 - i] = t; }
	/* AlnRes::setShape shifts edits by the rows trimmed at the DP top
	 * (aligner_result.cpp:101-108) */
	for(size_t i = 0; i < ned; i++) ed[i].pos -= (int32_t)trimBeg;
	size_t refns = 0;
	for(size_t i = col; i <= origCol; i++) if(rf[i] > 15) refns++;
	aout[0] = score; aout[1] = (int64_t)col; aout[2] = ns; aout[3] = (int64_t)gaps; aout[4] = (int64_t)refns;
	aout[5] = (int64_t)trimBeg; aout[6] = (int64_t)trimEnd;
	*ned_o = ned;
	return 1;
}

/* SwAligner::align + the SwDriver loop of nextAlignment calls
 * (aligner_sw_driver.cpp:1157-1180, aligner_sw.cpp:737-1146) for one problem.
 * rd/q33: the read as aligned (reverse-complemented when !fw); fw only decides
 * 5'/3' orientation of edits and trims (AlnRes::invertEdits,
 * aligner_result.h:822-828, Edit::invertPoss edit.cpp:50-78).
 * out[7] as orc_sw.  aln: per alignment 10 words {cand, score, off, refoff,
 * ns, gaps, refns, nedit, trim5p, trim3p}; edits: (pos, type, chr, qchr) x
 * maxedit per alignment; fates[i] (aligner_sw_nuc.h:83-88).  Returns the
 * number of alignments. */
int orc_sw_bt(const uint8_t* rd, const uint8_t* q33, int nrow, const uint8_t* rf, int ncol, int64_t minsc,
              const orc_scoring* sc, int enable8, int fw, int triml, int corel, int corer, int maxaln,
              int maxedit, int64_t* out, int64_t* aln, int32_t* edits, int32_t* fates, int capf) {
	size_t cells = (size_t)nrow * (size_t)ncol;
	int32_t* mat = (int32_t*)malloc(sizeof(int32_t) * 3 * cells);
	int64_t* cands = (int64_t*)malloc(sizeof(int64_t) * 3 * (cells + 1));
	orc_sw(rd, q33, nrow, rf, ncol, minsc, sc, enable8, (int)cells + 1, out, cands, mat);
	int na = 0;
	if(out[0]) {
		int local = sc->local != 0;
		int variant = local ? (out[2] ? 2 : 3) : (out[2] ? 0 : 1);
		int64_t offsc = variant == 0 ? -0xff : variant == 1 ? -0x7fff : variant == 2 ? 0 : 0x8000;
		int64_t* VH = (int64_t*)malloc(sizeof(int64_t) * cells);
		int64_t* VE = (int64_t*)malloc(sizeof(int64_t) * cells);
		int64_t* VF = (int64_t*)malloc(sizeof(int64_t) * cells);
		for(size_t k = 0; k < cells; k++) {
			VH[k] = mat[3 * k] + offsc; VE[k] = mat[3 * k + 1] + offsc; VF[k] = mat[3 * k + 2] + offsc;
		}
		uint8_t* marks = (uint8_t*)calloc(cells, 1);
		orc_edit* ed = (orc_edit*)malloc(sizeof(orc_edit) * (size_t)(nrow + ncol + 4));
		orc_btframe* stack = (orc_btframe*)malloc(sizeof(orc_btframe) * (size_t)(nrow + ncol + 4));
		size_t* cl = (size_t*)malloc(sizeof(size_t) * 2 * (size_t)(nrow + ncol + 4));
		int64_t* done = (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)(out[6] + 1));
		size_t ndone = 0;
		int nceil = (int)(sc->ncl_const + sc->ncl_lin * (double)nrow);
		if(nceil < 0) nceil = 0;
		size_t SQ = (size_t)nrow >> 4;
		if(SQ == 0) SQ = 1;
		for(int64_t c = 0; c < out[6]; c++) {
			size_t row = (size_t)cands[3 * c], col = (size_t)cands[3 * c + 1];
			int64_t csc = cands[3 * c + 2];
			int fate;
			if(csc < minsc) fate = 5;                          /* FILT_SCORE */
			else if(marks[row * ncol + col]) fate = 3;         /* FILT_START */
			else {
				int dom = 0;
				if(local) {
					for(size_t i = 0; i < ndone && !dom; i++) {
						size_t colhi = col, rowhi = row, rowlo = (size_t)done[2 * i], collo = (size_t)done[2 * i + 1];
						if(colhi < collo) { size_t t = colhi; colhi = collo; collo = t; }
						if(rowhi < rowlo) { size_t t = rowhi; rowhi = rowlo; rowlo = t; }
						if(colhi - collo <= SQ && rowhi - rowlo <= SQ) dom = 1;
					}
				}
				if(dom) fate = 4;                               /* FILT_DOMINATED */
				else {
					size_t ned = 0;
					int64_t a[7];
					int ok = orc_bt_one(VH, VE, VF, marks, rd, q33, nrow, rf, ncol, sc, local, triml, corel, corer,
					                    nceil, row, col, ed, &ned, a, stack, cl);
					if(local) { done[2 * ndone] = (int64_t)row; done[2 * ndone + 1] = (int64_t)col; ndone++; }
					fate = ok ? 1 : 2;
					if(ok) {
						if(!fw) {
							/* invertEdits: reverse, pos = len - pos - (readgap ? 0 : 1) */
							for(size_t i = 0; i < ned / 2; i++) { orc_edit t = ed[i]; ed[i] = ed[ned - 1 - i]; ed[ned - 1 - i] = t; }
							/* rdexrows_ = rows left after trimming (aligner_result.cpp:110-117) */
							int32_t sz = nrow - (int32_t)a[5] - (int32_t)a[6];
							for(size_t i = 0; i < ned; i++) ed[i].pos = sz - ed[i].pos - (ed[i].type == 1 ? 0 : 1);
						}
						if(na < maxaln) {
							int64_t* o = aln + 10 * (size_t)na;
							o[0] = c; o[1] = a[0]; o[2] = a[1]; o[3] = a[1]; o[4] = a[2]; o[5] = a[3]; o[6] = a[4];
							o[7] = (int64_t)ned;
							o[8] = fw ? a[5] : a[6]; o[9] = fw ? a[6] : a[5];
							for(size_t e = 0; e < ned && (int)e < maxedit; e++) {
								int32_t* q = edits + ((size_t)na * maxedit + e) * 4;
								q[0] = ed[e].pos; q[1] = ed[e].type; q[2] = ed[e].chr; q[3] = ed[e].qchr;
							}
						}
						na++;
					}
				}
			}
			if(c < capf) fates[c] = fate;
		}
		free(VH); free(VE); free(VF); free(marks); free(ed); free(stack); free(cl); free(done);
	}
	free(mat); free(cands);
	return na;
}

/* ---------------------------------------------------------------------- */
/* SwAligner::ungappedAlign (aligner_sw.cpp:286-494)                        */
/* ---------------------------------------------------------------------- */
/* rd/q33: the read as aligned (reverse-complemented when !fw); rf: reference
 * codes 0..4 of positions rfi .. rfi+len-1 (4 off the reference); reflen:
 * length of the reference.  out[10] = {ret, score, refoff, ns, refns, nedit,
 * trim5p, trim3p, 0, 0}; edits (pos, type, chr, qchr) x nedit. */
int orc_ungapped(const uint8_t* rd, const uint8_t* q33, int len, const uint8_t* rf, int64_t rfi, int64_t reflen,
                 int64_t minsc, const orc_scoring* sc, int ohang, int fw, int64_t* out, int32_t* edits) {
	memset(out, 0, 10 * sizeof(int64_t));
	int nceil = (int)(sc->ncl_const + sc->ncl_lin * (double)len);
	if(nceil < 0) nceil = 0;
	int64_t rff = rfi + len;
	int64_t leftNs = 0, rightNs = 0;
	if(rfi < 0) { if(!ohang) return 0; leftNs = -rfi; }
	if(rff > reflen) { if(!ohang) return 0; rightNs = rff - reflen; }
	if(leftNs + rightNs > nceil) return 0;
	int64_t score = 0;
	int ns = 0;
	size_t rowi = 0, rowf = (size_t)len - 1;
	if(!sc->local) {
		for(int i = 0; i < len; i++) {
			int refm = 1 << rf[i];
			if(rd[i] > 3 || refm > 15) ns++;
			score += score_of(sc, rd[i], refm, q33[i] - 33);
			if(score < minsc || ns > nceil) return 0;
		}
	} else {
		int64_t floorsc = 0, scoreMax = 0;
		size_t lastfloor = 0, sols = 0;
		rowi = (size_t)-1;
		for(int i = 0; i < len; i++) {
			int refm = 1 << rf[i];
			if(rd[i] > 3 || refm > 15) ns++;
			score += score_of(sc, rd[i], refm, q33[i] - 33);
			if(score >= minsc && score >= scoreMax) {
				scoreMax = score;
				rowf = (size_t)i;
				if(rowi != lastfloor) { rowi = lastfloor; sols++; }
			}
			if(score <= floorsc) { score = floorsc; lastfloor = (size_t)i + 1; }
		}
		if(ns > nceil || scoreMax < minsc) return 0;
		if(sols > 1) { out[0] = -1; return -1; }
		score = scoreMax;
	}
	int ned = 0, refns = 0;
	for(size_t i = rowi; i <= rowf; i++) {
		if(rf[i] > 3 || rd[i] != rf[i]) {
			int32_t* e = edits + 4 * ned;
			e[0] = (int32_t)i; e[1] = 3; e[2] = mask2dna_c(1 << rf[i]); e[3] = "ACGTN"[rd[i]];
			ned++;
			if(rf[i] > 3) refns++;
		}
	}
	size_t trimEnd = (size_t)len - 1 - rowf;
	/* setShape: shift by the rows trimmed at the top; invertEdits for !fw */
	for(int i = 0; i < ned; i++) edits[4 * i] -= (int32_t)rowi;
	if(!fw) {
		int32_t sz = len - (int32_t)rowi - (int32_t)trimEnd;
		for(int i = 0; i < ned / 2; i++)
			for(int k = 0; k < 4; k++) { int32_t t = edits[4 * i + k]; edits[4 * i + k] = edits[4 * (ned - 1 - i) + k]; edits[4 * (ned - 1 - i) + k] = t; }
		for(int i = 0; i < ned; i++) edits[4 * i] = sz - edits[4 * i] - 1;
	}
	out[0] = 1; out[1] = score; out[2] = rfi + (int64_t)rowi; out[3] = ns; out[4] = refns; out[5] = ned;
	out[6] = (int64_t)(fw ? rowi : trimEnd); out[7] = (int64_t)(fw ? trimEnd : rowi);
	return 1;
}

/* ---------------------------------------------------------------------- */
/* DP framing: DynProgFramer (dp_framer.cpp:81-129, 177-383),               */
/* PairedEndPolicy::otherMate (pe.cpp:161-352), Scoring::maxReadGaps /      */
/* maxRefGaps (scoring.cpp:42-98)                                           */
/* ---------------------------------------------------------------------- */
/* Gap budgets in closed form: the reference loops, converting matches of the
 * perfect score P into gaps while the score stays >= minsc; the k-th read gap
 * costs rdgo (k = 1) or rdge, the k-th reference gap also loses a match. */
static int64_t orc_gap_budget(int64_t P, int64_t minsc, int64_t first, int64_t step) {
	if(P < minsc) return -1;
	if(P - first < minsc) return 0;
	return 1 + (P - first - minsc) / step;
}

/* pe: {policy, minfrag, maxfrag, flip, dovetail, olap, expand}.
 * out[7] = {ok, fw, refl, ncol, triml, corel, corer}. */
void orc_frame(int kind, int64_t off, uint64_t rdlen, int64_t reflen, int64_t minsc, int fw, int anchor1,
               uint64_t alen, const orc_scoring* sc, const int32_t* pe, int64_t maxhalf, int trim_to_ref,
               int64_t* out) {
	memset(out, 0, 7 * sizeof(int64_t));
	const int64_t P = (int64_t)(rdlen * (uint64_t)sc->match);
	const int64_t rdgo = sc->rdg_const + sc->rdg_lin, rfgo = sc->rfg_const + sc->rfg_lin;
	const int64_t rdgaps = orc_gap_budget(P, minsc, rdgo, sc->rdg_lin);
	const int64_t rfgaps = orc_gap_budget(P, minsc, sc->match + rfgo, sc->match + sc->rfg_lin);
	double v = sc->ncl_const + sc->ncl_lin * (double)rdlen;
	int64_t nceil = v < 0.0 ? 0 : (int64_t)(int)v;
	if(nceil > (int64_t)rdlen) nceil = (int64_t)rdlen;
	/* the budgets are ints handed to size_t parameters */
	const uint64_t grd = (uint64_t)rdgaps, grf = (uint64_t)rfgaps;
	const uint64_t gmax = grd > grf ? grd : grf;
	uint64_t maxgap;
	int64_t refl, refr;
	int ofw = fw;
	if(kind == 0) {
		maxgap = gmax < (uint64_t)maxhalf ? gmax : (uint64_t)maxhalf;
		refl = (int64_t)((uint64_t)off - 2 * maxgap);
		refr = (int64_t)((uint64_t)off + (rdlen - 1) + 2 * maxgap);
	} else {
		/* pePolicyMateDir (pe.h:130-164): is the opposite mate to the left, on
		 * which strand */
		int left;
		switch(pe[0]) {
		case 1: left = anchor1 != fw; ofw = fw; break;
		case 2: left = anchor1 == fw; ofw = fw; break;
		case 3: left = !fw; ofw = !fw; break;
		default: left = fw; ofw = !fw; break;
		}
		const uint64_t len1 = anchor1 ? alen : rdlen, len2 = anchor1 ? rdlen : alen;
		const uint64_t a = anchor1 ? len1 : len2;   /* "length of opposite mate" as otherMate names it */
		uint64_t maxfrag = (uint64_t)pe[2], minfrag = pe[1] < 1 ? 1u : (uint64_t)pe[1];
		if(pe[6]) {
			if(len1 > maxfrag) maxfrag = len1;
			if(len2 > maxfrag) maxfrag = len2;
		} else if(len1 > maxfrag || len2 > maxfrag) {
			return;
		}
		const int64_t maxalcols = (int64_t)rdlen + rdgaps;
		int64_t ll, lr, rl, rr;
		if(left) {
			ll = (int64_t)((uint64_t)off + a - maxfrag);
			lr = (int64_t)((uint64_t)off + a - minfrag);
			rl = ll;
			rr = (int64_t)((uint64_t)off + maxfrag - 1);
			if(!pe[5]) {
				if(off - 1 < rr) rr = off - 1;
				if(rr < lr) lr = rr;
			} else if(!pe[4]) {
				const int64_t t = (int64_t)((uint64_t)off + a - 1);
				if(t < rr) rr = t;
			} else if(!pe[3] && maxalcols != -1) {
				const int64_t t = (int64_t)((uint64_t)off + a - 1 + (uint64_t)(maxalcols - 1));
				if(t < rr) rr = t;
			}
		} else {
			rr = (int64_t)((uint64_t)off + (maxfrag - 1));
			rl = (int64_t)((uint64_t)off + (minfrag - 1));
			ll = (int64_t)((uint64_t)off + a - maxfrag);
			lr = rr;
			if(!pe[5]) {
				const int64_t t = (int64_t)((uint64_t)off + a);
				if(t > ll) ll = t;
				if(ll > rl) rl = ll;
			} else if(!pe[4]) {
				if(off > ll) ll = off;
			} else if(!pe[3] && maxalcols != -1) {
				const int64_t t = off - maxalcols + 1;
				if(t > ll) ll = t;
			}
		}
		(void)lr;
		maxgap = gmax > (uint64_t)maxhalf ? gmax : (uint64_t)maxhalf;
		/* anchor to the left (opposite to the right): the opposite mate ends in
		 * [rl, rr]; anchor to the right: it starts in [ll, lr] */
		const int64_t st = left ? ll : (int64_t)((uint64_t)rl - (rdlen - 1));
		const int64_t en = left ? (int64_t)((uint64_t)lr + (rdlen - 1)) : rr;
		refl = (int64_t)((uint64_t)st - maxgap);
		refr = (int64_t)((uint64_t)en + maxgap);
	}
	int64_t maxns = trim_to_ref ? 0 : (nceil == (int64_t)rdlen ? nceil - 1 : nceil);
	uint64_t triml = 0, trimr = 0;
	if(refr >= reflen + maxns) trimr = (uint64_t)(refr - (reflen + maxns - 1));
	if(refl < -maxns) triml = (uint64_t)(-refl) - (uint64_t)maxns;
	const int64_t rl2 = (int64_t)((uint64_t)refl + triml), rr2 = (int64_t)((uint64_t)refr - trimr);
	if(rr2 < rl2) return;
	out[0] = 1;
	out[1] = ofw;
	out[2] = rl2;
	out[3] = rr2 - rl2 + 1;
	out[4] = (int64_t)triml;
	out[5] = (int64_t)maxgap;
	out[6] = kind == 0 ? (int64_t)(3 * maxgap) : (int64_t)((uint64_t)(refr - refl + 1) - maxgap - 1);
}
