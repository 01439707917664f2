/*
 * bt2g.h -- C ABI of the MI355X (gfx950) engines for bowtie2's seed-and-extend
 * hot path.  Drop-in boundary for the reference's per-thread C++ seams
 * (SURVEY.md section 8b); every entry point names the reference interface it
 * replaces.  Plain pointers and sizes only; no C++ or torch types cross it; no
 * exceptions escape it; every call returns a status (BT2G_OK == 0).
 *
 * Batching model: the reference calls its seams one read (one DP problem) at a
 * time from each worker thread; here the caller hands over a whole batch.  The
 * per-read results are exactly those of the reference call on that read.
 *
 *   reads   : n rows of `stride` bytes, codes 0..3 = A,C,G,T, 4 = N (Read::patFw)
 *   quals   : n rows of `stride` bytes, Phred+33 ASCII (Read::qual)
 *   lens    : n read lengths (<= stride, <= BT2G_MAX_READ_LEN)
 *
 * Two flavours of every batch call:
 *   <name>_dev(...)     all array arguments are device pointers (HBM-resident),
 *                      enqueued on `stream` (a hipStream_t; NULL = the null stream),
 *                      asynchronous.
 *   <name>(...)         same arguments as host pointers; copies in, runs, copies
 *                      out, synchronises.  For callers that keep data on the host.
 */
#ifndef BT2G_H_
#define BT2G_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BT2G_OK            0
#define BT2G_ERR_IO       -1
#define BT2G_ERR_FORMAT   -2
#define BT2G_ERR_HIP      -3
#define BT2G_ERR_ARG      -4
#define BT2G_ERR_NOMEM    -5
#define BT2G_ERR_OVERFLOW -6

/* Longest read the engines take (the reference checkpoints DPs of reads of
 * >= --cp-min (default 2000) bases; the checkpointed path stays on the CPU).
 * Reads up to 1024 bases go through the systolic fills; longer ones through
 * the one-problem-per-lane fills and a u16 score plane. */
#define BT2G_MAX_READ_LEN 2048

typedef struct bt2g_ctx bt2g_ctx;

/* Scoring scheme, same parameters as Scoring::Scoring (scoring.h:136-173) with
 * COST_MODEL_QUAL mismatches and COST_MODEL_CONSTANT N penalty (bowtie2
 * defaults: end-to-end {0,6,2,1,5,3,5,3,4,0}, --local {2,6,2,1,5,3,5,3,4,1}). */
typedef struct {
	int32_t match;      /* --ma, bonus for a match (0 in end-to-end mode) */
	int32_t mmp_max;    /* --mp MX */
	int32_t mmp_min;    /* --mp MN */
	int32_t npen;       /* --np */
	int32_t rdg_const;  /* --rdg open part */
	int32_t rdg_lin;    /* --rdg extend */
	int32_t rfg_const;  /* --rfg open part */
	int32_t rfg_lin;    /* --rfg extend */
	int32_t gapbar;     /* --gbar */
	int32_t local;      /* 1 = --local */
	double  ncl_const;  /* --n-ceil constant (L,0,0.15 default) */
	double  ncl_lin;    /* --n-ceil linear coefficient */
} bt2g_scoring;

/* Index arrays already in host memory (the arrays of Ebwt::readIntoMemory,
 * bt2_io.cpp:39-616, for the forward index and the mirror ".rev" index, plus
 * the unpacked reference of BitPairReference, reference.cpp:100-235). */
typedef struct {
	uint32_t len, zoff, ftab_chars, off_rate, line_rate;
	const uint32_t* fchr;      /* 5 */
	const uint8_t*  sides;     /* numSides * 64 */
	uint64_t        sides_bytes;
	const uint32_t* ftab;      /* 4^ftab_chars + 1 */
	const uint32_t* eftab;     /* 2 * ftab_chars */
	const uint32_t* offs;      /* SA sample, forward index only (NULL for mirror) */
	uint64_t        offs_len;
	const uint32_t* rstarts;   /* 3 * nfrag (forward index) */
	uint32_t        nfrag;
} bt2g_ebwt_mem;

typedef struct {
	bt2g_ebwt_mem fw, bw;
	const uint8_t*  ref_codes;   /* all references concatenated, codes 0..4 */
	const uint64_t* ref_starts;  /* nref + 1 offsets into ref_codes */
	uint32_t        nref;
} bt2g_index_mem;

/* ---- lifetime ---------------------------------------------------------- */

/* Load <base>.{1,2,rev.1,3,4}.bt2 and make the FM index (fw + mirror sides,
 * ftab/eftab, fchr, SA sample) and the reference resident in HBM of `device`.
 * Replaces Ebwt ctor + loadIntoMemory (bt2_search.cpp:5080-5097, 4870-4892) and
 * BitPairReference (bt2_search.cpp:4816-4832). */
int bt2g_open(const char* index_base, int device, bt2g_ctx** out);
/* Same from arrays already in host memory. */
int bt2g_open_mem(const bt2g_index_mem* m, int device, bt2g_ctx** out);
/* A second context on `base`'s device and index: its own stream and scratch,
 * no second copy of the index.  Every such context is closed before `base`:
 * bt2g_close(base) fails with BT2G_ERR_ARG while one is open.
 * Contexts are not thread-safe; one thread drives each (the drop-in binding
 * gives every dispatcher thread its own, integration/bt2g_seams.cpp). */
int bt2g_open_shared(bt2g_ctx* base, bt2g_ctx** out);
/* Scheduling priority of the context's streams: high != 0 -> the device's
 * highest stream priority (hipDeviceGetStreamPriorityRange), 0 -> the default.
 * For a caller that runs latency-bound searches beside throughput-bound
 * alignment on one device (the batch server's services; no reference
 * counterpart -- the reference has no device).  Call between calls, not during. */
int bt2g_set_priority(bt2g_ctx* ctx, int high);
/* Confine the context's stream to `num` of every `den` compute units (CU i is
 * used iff i % den < num; num >= den or den == 0: every CU, the default), so
 * that long launches on it leave CUs to other contexts' short ones (the batch
 * server's DP service beside its FM services).  Call between calls.  The
 * masked stream (hipExtStreamCreateWithCUMask) is a blocking stream (it
 * synchronises with the null stream) and gets an HSA queue of its own outside
 * the GPU_MAX_HW_QUEUES pool; it has no priority: combining this call with
 * bt2g_set_priority on one context fails with BT2G_ERR_ARG either way round. */
int bt2g_set_cu_share(bt2g_ctx* ctx, uint32_t num, uint32_t den);
/* Release a context (a shared one first, then the index owner). */
int bt2g_close(bt2g_ctx* ctx);
/* out: [len, zoff_fw, zoff_bw, fchr0..4, ftab_chars, off_rate, num_sides,
 *       nref, hbm_bytes]  (n <= 13 words written) */
int bt2g_info(bt2g_ctx* ctx, uint64_t* out, int n);
/* Last error message of this thread. */
const char* bt2g_last_error(void);

/* ---- FM engine ----------------------------------------------------------- */

/* SeedAligner::exactSweep (aligner_seed.h:1715-1726, aligner_seed.cpp:854-968)
 * for every read, both strands.  out: n x 8 u32 =
 *   {mineFw, mineRc, fw_top, fw_bot, rc_top, rc_bot, bwops, side_loads}
 * (top/bot = the exact end-to-end SA range when min edits == 0, else 0,0;
 * mineFw/mineRc are left 0 for a skipped strand). */
int bt2g_exact_sweep(bt2g_ctx* ctx, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t n,
                     uint32_t mine_max, int nofw, int norc, uint32_t* out);
int bt2g_exact_sweep_dev(bt2g_ctx* ctx, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t n,
                         uint32_t mine_max, int nofw, int norc, uint32_t* out, void* stream);

/* One exact-seed round: Seed::mmSeeds(0, seedlen) + instantiateSeeds(offset,
 * interval) + searchAllSeeds (aligner_seed.h:1667-1694, aligner_seed.cpp:498-718,
 * 1633-2033; bt2_search.cpp:3853-3906).  For read i, strand f (0 = fw, 1 = rc)
 * and seed s: out[((i*2+f)*maxseeds+s)*4 + {0..3}] = {topf, botf, topb, botb}
 * (all 0 when the seed has no hit or was filtered for an N).  nseeds[i] =
 * number of seed offsets (0 when the round is skipped, bt2_search.cpp:3866).
 * bwops[i] = FM ops of the read (== SeedSearchMetrics::bwops); loads[i] (optional,
 * may be NULL) = 64-B sides gathered for the read (roofline bytes). */
int bt2g_seed_search(bt2g_ctx* ctx, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t n,
                     uint32_t seedlen, uint32_t interval, uint32_t offset, uint32_t maxseeds,
                     uint32_t* out, int32_t* nseeds, uint32_t* bwops, uint32_t* loads);
int bt2g_seed_search_dev(bt2g_ctx* ctx, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t n,
                         uint32_t seedlen, uint32_t interval, uint32_t offset, uint32_t maxseeds,
                         uint32_t* out, int32_t* nseeds, uint32_t* bwops, uint32_t* loads, void* stream);

/* One 1-mismatch end-to-end hit (SeedResults::add1mmEe, aligner_seed.h:1248). */
typedef struct {
	uint32_t top, bot;   /* SA range in the forward BWT */
	int32_t  fw;         /* read orientation */
	int32_t  score;
	int32_t  pos;        /* Edit::pos, offset from the 5' end */
	int32_t  chr;        /* reference base 0..3 */
	int32_t  qchr;       /* read base 0..4 */
	int32_t  pad;
} bt2g_mm1;

/* SeedAligner::oneMmSearch with rep1mm=true, repex=false exactly as
 * bt2_search.cpp:3654-3667 calls it (aligner_seed.h:1731-1743,
 * aligner_seed.cpp:973-1323).  Hits are returned per read in the reference's
 * discovery order: hits[i*cap .. i*cap+counts[i]), counts[i] may exceed cap
 * (then BT2G_ERR_OVERFLOW is returned and cap of the hits are stored, which
 * ones unspecified: call again with cap >= counts[i] for the ordered list).
 * bwops and loads (optional) as for bt2g_seed_search. */
int bt2g_one_mm(bt2g_ctx* ctx, const uint8_t* reads, const uint8_t* quals, uint32_t stride, const uint32_t* lens,
                uint32_t n, const int32_t* minsc, const bt2g_scoring* sc, int nofw, int norc, uint32_t cap,
                bt2g_mm1* hits, int32_t* counts, uint32_t* bwops, uint32_t* loads);
int bt2g_one_mm_dev(bt2g_ctx* ctx, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                    const uint32_t* lens, uint32_t n, const int32_t* minsc, const bt2g_scoring* sc, int nofw,
                    int norc, uint32_t cap, bt2g_mm1* hits, int32_t* counts, uint32_t* bwops, uint32_t* loads,
                    void* stream);

/* Same search gated per read by the exactSweep output `sweep` (n x 8, from
 * bt2g_exact_sweep_dev) exactly as bt2_search.cpp:3476-3506,3640-3667 chains
 * them: no search when min(mineFw, mineRc) == 0; otherwise nofw = mineFw > 1,
 * norc = mineRc > 1 (counts[i] = 0 for skipped reads).  Fully asynchronous: an
 * overflow shows as counts[i] > cap. */
int bt2g_one_mm_gated_dev(bt2g_ctx* ctx, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                          const uint32_t* lens, uint32_t n, const int32_t* minsc, const bt2g_scoring* sc,
                          const uint32_t* sweep, uint32_t cap, bt2g_mm1* hits, int32_t* counts, uint32_t* bwops,
                          uint32_t* loads, void* stream);

/* bt2g_exact_sweep and, in the same call, bt2g_one_mm gated per read by the
 * sweep's result (nofw / norc: the reads' strand options, as for both calls):
 * one round trip for a read's two up-front searches (bt2_search.cpp:3453-3667).
 * With yfw = sweep[i*8] <= 1 && !nofw, yrc = sweep[i*8+1] <= 1 && !norc
 * (bt2_search.cpp:3649-3650), the 1-mm search of read i ran iff yfw || yrc --
 * and, with skip_exact, min(sweep[i*8], sweep[i*8+1]) != 0 (the rule of
 * bt2g_one_mm_gated_dev) -- as bt2g_one_mm on that read with nofw = !yfw,
 * norc = !yrc; counts[i] may exceed cap (no error: the caller asks again).
 * offs (optional, n x (2 + cap) x off_cap): Ebwt::getOffset of every row of
 * the exact ranges (slots 0, 1: fw, rc, when their mine is 0) and of the
 * stored 1-mm hits' ranges (slots 2..), for ranges of at most off_cap rows;
 * BT2G_OFF_MASK elsewhere -- the rows the extension of those hits resolves
 * first (GroupWalk2S, group_walk.h:862-1216), without a round trip.
 * mm_loads (optional, n): 64-B sides the 1-mm search gathered per read (0 where
 * it did not run; the sweep's own are sweep[i*8+7]). */
int bt2g_exact_sweep_1mm(bt2g_ctx* ctx, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                         const uint32_t* lens, uint32_t n, uint32_t mine_max, int nofw, int norc, int skip_exact,
                         const int32_t* minsc, const bt2g_scoring* sc, uint32_t cap, uint32_t* sweep,
                         bt2g_mm1* hits, int32_t* counts, uint32_t* bwops, uint32_t* mm_loads, uint32_t off_cap,
                         uint32_t* offs);

/* Ebwt::getOffset (bt2_idx.cpp:150-171): joined-text offset of each SA row.
 * loads (optional): 64-B sides gathered per row. */
int bt2g_get_offset(bt2g_ctx* ctx, const uint32_t* rows, uint32_t n, uint32_t* offs, uint32_t* loads);
int bt2g_get_offset_dev(bt2g_ctx* ctx, const uint32_t* rows, uint32_t n, uint32_t* offs, uint32_t* loads,
                        void* stream);

/* One seed-hit range to extend (SwDriver::extend's arguments,
 * aligner_sw_driver.cpp:299-312): the seed at `off` from the 5' end of the read
 * (fw) or of its reverse complement (!fw), `len` long, with SA range
 * [topf, botf) in the forward index and [topb, botb) in the mirror index. */
typedef struct {
	uint32_t read;       /* row in reads/lens */
	int32_t  fw;
	uint32_t off, len;
	uint32_t topf, botf, topb, botb;
} bt2g_ext_in;

typedef struct {
	uint32_t nlex, nrex; /* positions the hit extends to the left / right without an edit */
	uint32_t fmops;      /* LF steps taken (PerReadMetrics::nSdFmops increments) */
	uint32_t loads;      /* 64-B occurrence-table sides gathered (roofline bytes; not a reference output) */
} bt2g_ext_out;

/* SwDriver::extend (aligner_sw_driver.cpp:299-483), called by
 * prioritizeSATups (aligner_sw_driver.cpp:574-589) for every seed-hit range:
 * walks the range outward, left in the forward index and right in the mirror
 * index, while it stays the same size and agrees with the read. */
int bt2g_extend(bt2g_ctx* ctx, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t nreads,
                const bt2g_ext_in* in, uint32_t n, bt2g_ext_out* out);
int bt2g_extend_dev(bt2g_ctx* ctx, const uint8_t* reads, uint32_t stride, const uint32_t* lens,
                    const bt2g_ext_in* in, uint32_t n, bt2g_ext_out* out, void* stream);

/* bt2g_seed_search, and in the same call what the seed-extension stage asks of
 * the round's ranges (bt2g_exact_sweep_1mm does the same for the up-front
 * searches): ext (n x 2 x maxseeds, may be NULL) = SwDriver::extend of each
 * seed's range (as bt2g_extend with fw = strand 0, off = the seed's depth
 * s * interval + offset, len = min(seedlen, read length); prioritizeSATups,
 * aligner_sw_driver.cpp:574-589 asks it of every range it keeps), zeros where
 * the seed has no range; offs (n x 2 x maxseeds x off_cap, may be NULL) = the
 * offsets (Ebwt::getOffset) of rows topf .. botf-1 of every range of at most
 * off_cap rows, BT2G_OFF_MASK elsewhere (the rows GroupWalk2S::init resolves
 * for the ranges it takes, aligner_sw_driver.cpp:610-620 and 706-722). */
int bt2g_seed_search_ext(bt2g_ctx* ctx, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t n,
                         uint32_t seedlen, uint32_t interval, uint32_t offset, uint32_t maxseeds, uint32_t* out,
                         int32_t* nseeds, uint32_t* bwops, uint32_t* loads, bt2g_ext_out* ext, uint32_t off_cap,
                         uint32_t* offs);

/* ---- SW engine ----------------------------------------------------------- */

/* One dynamic-programming problem (SwAligner::initRead + initRef,
 * aligner_sw.cpp:34-271).  The reference window is either taken from the
 * resident reference (win_off < 0: columns refl .. refl+ncol-1 of reference
 * `refidx`, N outside it, plus the extra right column, aligner_sw.cpp:171-253)
 * or given explicitly as ncol+1 masks (1,2,4,8,16) at windows[win_off]. */
typedef struct {
	uint32_t read;       /* row in reads/quals/lens */
	int32_t  fw;         /* 1: align the read, 0: its reverse complement */
	int64_t  refl;       /* leftmost reference offset (may be < 0) */
	int64_t  win_off;    /* >= 0: offset of ncol+1 masks in `windows` */
	uint32_t refidx;
	uint32_t ncol;
	int32_t  minsc;
	uint32_t pad;
} bt2g_sw_problem;

/* Result of SwAligner::align (aligner_sw.cpp:500-729). */
typedef struct {
	int32_t  aligned;    /* return value of align() */
	int32_t  best;       /* `best` (MIN_I32 for MIN_I64) */
	int32_t  u8succ;     /* sse8succ_ */
	int32_t  i16succ;    /* sse16succ_ */
	int32_t  colstop;    /* colstop_ */
	int32_t  lastsolcol; /* lastsolcol_ */
	int32_t  ncand;      /* btncand_.size() (may exceed cap -> BT2G_ERR_OVERFLOW) */
	int32_t  flag;
} bt2g_sw_result;

/* DpBtCandidate (aligner_sw_nuc.h), sorted by the reference's total order. */
typedef struct {
	int32_t row, col, score;
} bt2g_sw_cand;

/* Fill + candidate gather for every problem: the u8/i16 end-to-end or local
 * fill chosen exactly as SwAligner::align does (u8 first when enable8; local
 * u8 saturation falls back to i16).  cands[p*cap ..] receives the sorted
 * candidate cells (cap: 1..8192 per problem).  mat (optional, NULL to skip): per problem
 * nrow*ncol*3 int16 H,E,F values in the fill's native domain, at mat_off[p]. */
int bt2g_sw_align(bt2g_ctx* ctx, const uint8_t* reads, const uint8_t* quals, uint32_t stride, const uint32_t* lens,
                  const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* windows, uint64_t windows_len,
                  const bt2g_scoring* sc, int enable8, uint32_t cap, bt2g_sw_result* res, bt2g_sw_cand* cands,
                  int16_t* mat, const uint64_t* mat_off);
int bt2g_sw_align_dev(bt2g_ctx* ctx, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                      const uint32_t* lens, const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* windows,
                      const bt2g_scoring* sc, int enable8, uint32_t cap, bt2g_sw_result* res, bt2g_sw_cand* cands,
                      int16_t* mat, const uint64_t* mat_off, void* stream);

/* Reserve persistent scratch for up to max_problems problems of width <=
 * max_cols, so bt2g_sw_align_dev neither allocates nor synchronises (problems
 * wider than max_cols then fail with result.flag = -3). */
int bt2g_reserve_sw(bt2g_ctx* ctx, uint32_t max_problems, uint32_t max_cols);

/* ---- SW backtrace (row A21) ------------------------------------------------ */

/* The DPRect fields the backtrace reads (dp_framer.h:62-93): columns trimmed
 * off the rectangle's left end and the inclusive range of "core" diagonals
 * (offsets from the untrimmed left end) an alignment must touch
 * (aligner_swsse_ee_u8.cpp:1764-1800).  Seed extension: corel = maxgap,
 * corer = 3*maxgap (dp_framer.cpp:116-125). */
typedef struct {
	int32_t triml, corel, corer, pad;
} bt2g_sw_rect;

/* One alignment returned by SwAligner::nextAlignment (aligner_sw.cpp:737-1146):
 * the SwResult/AlnRes fields that SAM output needs. */
typedef struct {
	int32_t cand;     /* index of the candidate cell in the sorted list (cural_) */
	int32_t score;    /* AlnScore::score_ */
	int32_t off;      /* rectangle column of the leftmost aligned reference char
	                     (reference offset = problem.refl + off) */
	int32_t ns;       /* AlnScore::ns_: read or reference Ns aligned */
	int32_t gaps;     /* AlnScore::gaps_ */
	int32_t refns;    /* AlnRes::refns_ */
	int32_t nedit;    /* edits in the alignment (> maxedit: only maxedit stored) */
	int32_t trim5p;   /* soft trimming (local mode), AlnRes::trimmed5p(true) */
	int32_t trim3p;
	int32_t pad;
} bt2g_sw_aln;

/* Edit (edit.h:58-110): pos from the read's 5' end after trimming; type 1 =
 * read gap, 2 = reference gap, 3 = mismatch; chr / qchr ASCII ('-' for gaps,
 * IUPAC mask2dna for reference masks). */
typedef struct {
	uint32_t pos;
	uint8_t  type, chr, qchr, pad;
} bt2g_edit;

/* SwAligner::align followed by the driver's loop of nextAlignment calls
 * (aligner_sw_driver.cpp:1157-1180: until done() or an empty result) for every
 * problem: the fill and candidates of bt2g_sw_align plus every alignment, in
 * the order the reference returns them.  rects may be NULL (triml 0, every
 * diagonal core).  Per problem p: naln[p] alignments at alns[p*maxaln ..]
 * (the loop stops after maxaln; naln[p] = -4 if the problem needs an i16
 * matrix but the reservation holds u8 only; -5 if its candidate list
 * overflowed cap, so that the list is not the reference's), edits of alignment k at
 * edits[(p*maxaln + k)*maxedit ..]; fates (optional, NULL to skip):
 * DpBtCandidate::fate of each candidate (aligner_sw_nuc.h:83-88) at
 * fates[p*cap ..].  Candidates below the problem's minsc are skipped
 * (FILT_SCORE) exactly as nextAlignment(minsc) does; a caller that tightens
 * minsc between calls (aligner_sw_driver.cpp:1252-1290) truncates the list,
 * since candidates are sorted by score. */
int bt2g_sw_align_bt(bt2g_ctx* ctx, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                     const uint32_t* lens, const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* windows,
                     uint64_t windows_len, const bt2g_sw_rect* rects, const bt2g_scoring* sc, int enable8,
                     uint32_t cap, bt2g_sw_result* res, bt2g_sw_cand* cands, uint32_t maxaln, uint32_t maxedit,
                     int32_t* naln, bt2g_sw_aln* alns, bt2g_edit* edits, int8_t* fates);
int bt2g_sw_align_bt_dev(bt2g_ctx* ctx, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                         const uint32_t* lens, const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* windows,
                         const bt2g_sw_rect* rects, const bt2g_scoring* sc, int enable8, uint32_t cap,
                         bt2g_sw_result* res, bt2g_sw_cand* cands, uint32_t maxaln, uint32_t maxedit,
                         int32_t* naln, bt2g_sw_aln* alns, bt2g_edit* edits, int8_t* fates, void* stream);

/* bt2g_sw_align_bt for host callers, with the variable-length outputs packed:
 * res, naln and alns (nprob x maxaln slots) as there; the sorted candidates of
 * every problem (min(ncand, cap) each), their fates (optional) and the edits of
 * every returned alignment (min(nedit, maxedit) each) back to back in problem
 * (and alignment) order in cands / fates / edits, which must hold nprob*cap,
 * nprob*cap and nprob*maxaln*maxedit entries; only the first totals[0]
 * candidates, totals[1] alignments and totals[2] edits are written.  Per-problem
 * offsets follow from res/naln/alns by prefix sums.  Same seams as
 * bt2g_sw_align_bt (aligner_sw.cpp:500-1146); what it saves is the copy of the
 * unused slots (~26 KB per 150 bp end-to-end DP at cap 512, maxaln 8). */
int bt2g_sw_align_bt_packed(bt2g_ctx* ctx, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                            const uint32_t* lens, const bt2g_sw_problem* probs, uint32_t nprob,
                            const uint8_t* windows, uint64_t windows_len, const bt2g_sw_rect* rects,
                            const bt2g_scoring* sc, int enable8, uint32_t cap, bt2g_sw_result* res, uint32_t maxaln,
                            uint32_t maxedit, int32_t* naln, bt2g_sw_aln* alns, bt2g_sw_cand* cands, int8_t* fates,
                            bt2g_edit* edits, uint64_t* totals);

/* Reserve the backtrace scratch (score plane + reportedThrough bits) for up to
 * max_problems problems of <= max_rows x max_cols, so bt2g_sw_align_bt_dev
 * neither allocates nor synchronises.  hbytes = 1 holds u8 fills only (end-to-end
 * with enable8 and minsc >= -254, the default 150 bp case), 2 holds any. */
int bt2g_reserve_sw_bt(bt2g_ctx* ctx, uint32_t max_problems, uint32_t max_rows, uint32_t max_cols, int hbytes);

/* ---- ungapped alignment (row A22) ----------------------------------------- */

/* One SwAligner::ungappedAlign call (aligner_sw.cpp:286-494, called from
 * aligner_sw_driver.cpp:1032-1073): the read (fw) or its reverse complement
 * (!fw) against reference `refidx` starting at offset `off` (may be < 0). */
typedef struct {
	uint32_t read;
	int32_t  fw;
	int64_t  off;
	uint32_t refidx;
	int32_t  minsc;
} bt2g_ug_problem;

typedef struct {
	int32_t ret;        /* ungappedAlign's return: 1 aligned, 0 not, -1 defer to DP (local) */
	int32_t score;
	int64_t refoff;     /* AlnRes::refoff() (coord.off + rowi) */
	int32_t ns, refns, nedit, trim5p, trim3p, pad;
} bt2g_ug_result;

/* ungappedAlign for n problems with the scoring scheme sc (local or
 * end-to-end); ohang = gReportOverhangs.  Edits of problem p (mismatches,
 * 5'->3' after trimming) at edits[p*maxedit ..], nedit may exceed maxedit. */
int bt2g_ungapped(bt2g_ctx* ctx, const uint8_t* reads, const uint8_t* quals, uint32_t stride, const uint32_t* lens,
                  const bt2g_ug_problem* probs, uint32_t n, const bt2g_scoring* sc, int ohang, uint32_t maxedit,
                  bt2g_ug_result* res, bt2g_edit* edits);
int bt2g_ungapped_dev(bt2g_ctx* ctx, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                      const uint32_t* lens, const bt2g_ug_problem* probs, uint32_t n, const bt2g_scoring* sc,
                      int ohang, uint32_t maxedit, bt2g_ug_result* res, bt2g_edit* edits, void* stream);

/* ---- DP framing (row A14) ------------------------------------------------ */

/* PairedEndPolicy (pe.h:166-330): mate orientation policy and fragment-length
 * constraints.  policy: PE_POLICY_FF 1, RR 2, FR 3, RF 4 (pe.h:30-35). */
typedef struct {
	int32_t policy;
	int32_t minfrag, maxfrag;   /* -I, -X */
	int32_t local;              /* unused by otherMate, kept for parity with the constructor */
	int32_t flip, dovetail, contain, olap, expand;   /* flippingOk_ .. expandToFit_ */
	int32_t pad;
} bt2g_pe_policy;

/* One rectangle to frame.  kind 0: seed extension,
 * DynProgFramer::frameSeedExtensionRect (dp_framer.cpp:81-129) around the
 * ungapped diagonal through `off`, as SwDriver::extendSeeds calls it
 * (aligner_sw_driver.cpp:992-1000, 1074-1084).  kind 1: mate search,
 * PairedEndPolicy::otherMate (pe.cpp:161-352) for the anchor alignment at `off`
 * followed by DynProgFramer::frameFindMateRect (dp_framer.h:155-197,
 * dp_framer.cpp:177-383), as SwDriver::extendSeedsPaired calls them
 * (aligner_sw_driver.cpp:1975-2024). */
typedef struct {
	int64_t  off;      /* kind 0: reference offset implied by the hit; kind 1: the anchor's refoff */
	uint32_t read;     /* the read of the DP: kind 0 the read itself, kind 1 the opposite mate */
	uint32_t refidx;
	int32_t  minsc;    /* minimum score of the DP (kind 1: ominsc_cur) */
	int32_t  fw;       /* kind 0: strand of the DP; kind 1: the anchor's strand */
	int32_t  kind;
	int32_t  anchor1;  /* kind 1: the anchor is mate 1 */
	uint32_t alen;     /* kind 1: length of the anchor mate */
	uint32_t pad;
} bt2g_frame_in;

/* Frame n rectangles.  Read and reference gap budgets are
 * Scoring::maxReadGaps / maxRefGaps (scoring.cpp:42-98) of the DP's minsc and
 * read length (the seed-hit branch of extendSeeds; its exact end-to-end
 * "eeMode" hits need no rectangle); the N budget is
 * min(nCeil(len), len) (bt2_search.cpp multiseedSearchWorker); trim_to_ref =
 * !--overhang.  Per input: ok[i] = 1 and a DP problem probs[i] (reference
 * window [rect.refl, rect.refr], strand: kind 0 fw, kind 1 otherMate's ofw) with
 * rects[i] {triml, corel, corer}, or ok[i] = 0 when otherMate finds no
 * concordant window or the rectangle is entirely trimmed.  pe may be NULL when
 * no input has kind 1. */
int bt2g_frame(bt2g_ctx* ctx, const bt2g_frame_in* in, uint32_t n, const uint32_t* lens, uint32_t nreads,
               const bt2g_scoring* sc, const bt2g_pe_policy* pe, int32_t maxhalf, int trim_to_ref,
               bt2g_sw_problem* probs, bt2g_sw_rect* rects, int32_t* ok);
int bt2g_frame_dev(bt2g_ctx* ctx, const bt2g_frame_in* in, uint32_t n, const uint32_t* lens,
                   const bt2g_scoring* sc, const bt2g_pe_policy* pe, int32_t maxhalf, int trim_to_ref,
                   bt2g_sw_problem* probs, bt2g_sw_rect* rects, int32_t* ok, void* stream);

/* ---- multi-GPU ----------------------------------------------------------- */
/* The only collective of the path: reads shard across ranks
 * (one process per GPU, a full index replica each) and the ranks sum a few
 * counters at the end -- RCCL over xGMI.  Where the reference has one process
 * (the server's OutputQueue / metrics, bt2_search.cpp:4913-4925 spawning every
 * worker in it) nothing needs reducing; these serve a sharded deployment.
 *   bt2g_comm_unique_id: one rank creates the communicator id (128 bytes) and
 *                        hands it to the others out of band;
 *   bt2g_comm_init:      every rank joins (collective; ctx's device);
 *   bt2g_allreduce_counts: counts[0..k) summed over the ranks, in place
 *                        (collective, synchronous on ctx's stream).
 * RCCL (librccl.so.1) is loaded on first use; BT2G_ERR_HIP if it is absent. */
#define BT2G_COMM_ID_BYTES 128
int bt2g_comm_unique_id(uint8_t* id);
int bt2g_comm_init(bt2g_ctx* ctx, int nranks, int rank, const uint8_t* id);
int bt2g_allreduce_counts(bt2g_ctx* ctx, uint64_t* counts, uint32_t k);

/* ---- measurement --------------------------------------------------------- */
/* Kernel timing with HIP events on the launch stream (off by default). */
int bt2g_set_profiling(bt2g_ctx* ctx, int on);
/* kernel ids: 0 exact_sweep, 1 seed_search, 2 one_mm, 3 get_offset / range offsets, 4 sw_align,
 * 5 sw_backtrace, 6 ungapped, 7 frame / the whole stream span of a bt2g_sw_align_bt_packed call;
 * host phases of a bt2g_sw_align_bt_packed call (wall time): 8 staging, 9 enqueueing, 10 waiting and
 * copying out; 11 the SW candidate sort (kernels, HIP events); 12 extend (k_extend, k_seed_extend) */
int bt2g_kernel_stats(bt2g_ctx* ctx, int kernel, uint64_t* launches, double* total_ms);
int bt2g_reset_stats(bt2g_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* BT2G_H_ */
