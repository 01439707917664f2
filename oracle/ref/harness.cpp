// oracle/ref/harness.cpp -- TEST INFRASTRUCTURE ONLY (never part of the product).
//
// A thin extern "C" wrapper, written for this repo, around the REFERENCE's own
// C++ classes (sfiligoi/bowtie2-server, compiled from /root/reference by
// oracle/ref/Makefile into oracle/_ref/libbt2ref.so).  It lets the Python tests
// and bench.py's cpu_baseline leg call the reference's exact code paths:
//
//   * Ebwt load            bt2_search.cpp:5080-5097, 4870-4892 (same ctor/load args)
//   * SeedAligner::exactSweep     aligner_seed.cpp:854
//   * SeedAligner::oneMmSearch    aligner_seed.cpp:973
//   * SeedAligner::instantiateSeeds/searchAllSeeds  aligner_seed.cpp:498,597
//   * SwAligner::initRead/initRef/align (+ btncand_)  aligner_sw.cpp:34,73,500
//   * Ebwt::getOffset             bt2_idx.cpp:150
//
// No reference source is copied here; everything is reached through the
// reference headers at build time.
#include <stdint.h>
#include <string.h>
#include <vector>
#include <string>
#include <algorithm>
#include "bt2_idx.h"
#include "reference.h"
#include "read.h"
#include "aligner_seed.h"
#include "aligner_cache.h"
#include "aligner_sw.h"
#include "scoring.h"
#include "simple_func.h"
#include "search_globals.h"
#include "random_source.h"
#include "dp_framer.h"
#include "pe.h"
#include "aligner_sw_driver.h"

// Globals normally defined by bt2_search.cpp (search_globals.h, aligner_seed_policy.h).
bool gReportOverhangs = false;
bool gNoMaqRound = false;
bool gStrandFix = true;
bool gRangeMode = false;
int gVerbose = 0;
int gQuiet = 1;
bool gNofw = false;
bool gNorc = false;
bool gMate1fw = true;
bool gMate2fw = false;
int gMinInsert = 0;
int gMaxInsert = 500;
int gGapBarrier = 4;
int gAllowRedundant = 0;
int gDefaultSeedLen = 22;
bool gFlippedMatesOK = false;
bool gDovetailMatesOK = false;
bool gContainMatesOK = true;
bool gOlapMatesOK = true;
bool gExpandToFrag = true;
bool gReportDiscordant = true;
bool gReportMixed = true;

namespace {

struct RefHandle {
	Ebwt* fw = nullptr;
	Ebwt* bw = nullptr;
	BitPairReference* refs = nullptr;
};

// Scoring exactly as bt2_search.cpp:5134-5148 builds it, parameterised.
struct ScoreParams {
	int32_t match;       // bonusMatch (0 e2e, 2 local)
	int32_t mmp_max;     // --mp MX (6)
	int32_t mmp_min;     // --mp MN (2)
	int32_t npen;        // --np (1)
	int32_t rdg_const;   // --rdg 5,3
	int32_t rdg_lin;
	int32_t rfg_const;   // --rfg 5,3
	int32_t rfg_lin;
	int32_t gapbar;      // --gbar (4)
	int32_t local;       // 1 = local mode
	double  ncl_const;   // --n-ceil L,0,0.15
	double  ncl_lin;
};

Scoring makeScoring(const ScoreParams& p) {
	SimpleFunc scoreMin;
	if(p.local) scoreMin.init(SIMPLE_FUNC_LOG, 20.0, 8.0);
	else        scoreMin.init(SIMPLE_FUNC_LINEAR, -0.6, -0.6);
	SimpleFunc nCeil;
	nCeil.init(SIMPLE_FUNC_LINEAR, 0.0, std::numeric_limits<double>::max(), p.ncl_const, p.ncl_lin);
	return Scoring(
		p.match, COST_MODEL_QUAL, p.mmp_max, p.mmp_min, scoreMin, nCeil,
		COST_MODEL_CONSTANT, p.npen, false,
		p.rdg_const, p.rfg_const, p.rdg_lin, p.rfg_lin, p.gapbar);
}

// Gives the harness read access to SwAligner's protected results.
struct SwAlignerX : public SwAligner {
	SwAlignerX() : SwAligner(NULL) {}
	const EList<DpBtCandidate>& cands() const { return btncand_; }
	size_t colstop() const { return colstop_; }
	size_t lastsolcol() const { return lastsolcol_; }
	bool u8succ() const { return sse8succ_; }
	bool i16succ() const { return sse16succ_; }
	size_t cural() const { return cural_; }
	EList<DpBtCandidate>& candsMut() { return btncand_; }
	const SSEMatrix& mat(bool u8, bool fw) const {
		if(u8) return fw ? sseU8fw_.mat_ : sseU8rc_.mat_;
		return fw ? sseI16fw_.mat_ : sseI16rc_.mat_;
	}
};

// Gives the harness read access to SeedAligner's FM-op counter (bwops_).
struct SeedAlignerX : public SeedAligner {
	uint64_t ops() const { return bwops_; }
};

} // namespace

extern "C" {

void* bt2ref_open(const char* base) {
	RefHandle* h = new RefHandle();
	std::string b(base);
	h->fw = new Ebwt(b, 0, -1, true, -1, 0, false, false, false, false, true, true, true,
	                 false, false, false, false);
	h->fw->loadIntoMemory(0, -1, true, true, true, false, false);
	h->bw = new Ebwt(b + ".rev", 0, 1, false, -1, 0, false, false, false, false, false, true, false,
	                 false, false, false, false);
	h->bw->loadIntoMemory(0, 1, false, true, false, false, false);
	h->refs = new BitPairReference(b, false, false, NULL, NULL, false, false, false, false, false, false);
	return h;
}

void bt2ref_close(void* vh) {
	RefHandle* h = (RefHandle*)vh;
	delete h->fw; delete h->bw; delete h->refs; delete h;
}

// out: [len, zOff_fw, zOff_bw, fchr0..4, ftabChars, offRate, numSides, nPat, nFrag]
void bt2ref_info(void* vh, uint64_t* out) {
	RefHandle* h = (RefHandle*)vh;
	const EbwtParams& e = h->fw->eh();
	out[0] = e.len(); out[1] = h->fw->zOff(); out[2] = h->bw->zOff();
	for(int i = 0; i < 5; i++) out[3 + i] = h->fw->fchr()[i];
	out[8] = e.ftabChars(); out[9] = e.offRate(); out[10] = e.numSides();
	out[11] = h->fw->nPat(); out[12] = h->fw->nFrag();
}

// Ebwt::contains on fw and (reversed string) on the mirror -> SA ranges.
// seq: ASCII ACGT.  Returns 1 iff found in fw.
int bt2ref_contains(void* vh, const char* seq, uint32_t* out4) {
	RefHandle* h = (RefHandle*)vh;
	BTDnaString s(seq, true);
	TIndexOffU tf = 0, bf = 0, tb = 0, bb = 0;
	bool ok = h->fw->contains(s, &tf, &bf);
	s.reverse();
	h->bw->contains(s, &tb, &bb);
	out4[0] = tf; out4[1] = bf; out4[2] = tb; out4[3] = bb;
	return ok ? 1 : 0;
}

// One bidirectional LF step on index `which` (0 fw, 1 mirror) from range [top,bot)
// with mirror range starting at topp: INIT_LOCS + mapBiLFEx (aligner_seed.h:1847,
// bt2_idx.h:2372) or, for a 1-row range, mapLF1 (bt2_idx.h:2451).
void bt2ref_bilf(void* vh, int which, uint32_t top, uint32_t bot, uint32_t topp,
                 uint32_t* t4, uint32_t* b4, uint32_t* tp4, uint32_t* bp4) {
	RefHandle* h = (RefHandle*)vh;
	const Ebwt* e = which ? h->bw : h->fw;
	TIndexOffU t[4] = {0,0,0,0}, b[4] = {0,0,0,0};
	TIndexOffU tp[4] = {topp,topp,topp,topp}, bp[4] = {topp + (bot - top), topp + (bot - top), topp + (bot - top), topp + (bot - top)};
	SideLocus tloc, bloc;
	INIT_LOCS(top, bot, tloc, bloc, *e);
	if(bloc.valid()) {
		e->mapBiLFEx(tloc, bloc, t, b, tp, bp);
	} else {
		TIndexOffU row = top;
		int c = e->mapLF1(row, tloc);
		if(c >= 0) { t[c] = row; b[c] = row + 1; }
		for(int i = 0; i < 4; i++) { tp[i] = topp; bp[i] = topp + ((int)i == c ? 1 : 0); }
	}
	for(int i = 0; i < 4; i++) { t4[i] = t[i]; b4[i] = b[i]; tp4[i] = tp[i]; bp4[i] = bp[i]; }
}

uint32_t bt2ref_ftab_lohi(void* vh, int which, uint32_t i, uint32_t* bot) {
	RefHandle* h = (RefHandle*)vh;
	const Ebwt* e = which ? h->bw : h->fw;
	TIndexOffU t = 0, b = 0;
	e->ftabLoHi(i, t, b);
	*bot = b;
	return t;
}

uint32_t bt2ref_get_offset(void* vh, uint32_t row) {
	RefHandle* h = (RefHandle*)vh;
	return h->fw->getOffset(row);
}

// Fetch 2-bit reference bases [off, off+len) of reference `refidx` (values 0..4).
int bt2ref_get_stretch(void* vh, uint32_t refidx, uint64_t off, uint64_t len, uint8_t* dst) {
	RefHandle* h = (RefHandle*)vh;
	for(uint64_t i = 0; i < len; i++) dst[i] = (uint8_t)h->refs->getBase(refidx, off + i);
	return 0;
}

// Length of reference `refidx` (BitPairReference::approxLen, Ns included).
uint64_t bt2ref_ref_len(void* vh, uint32_t refidx) {
	RefHandle* h = (RefHandle*)vh;
	return (uint64_t)h->refs->approxLen(refidx);
}

// SeedAligner::exactSweep over n reads (ASCII seq/qual, NUL-terminated).
// out per read: mineFw, mineRc, nelt, exact fw [top,bot), exact rc [top,bot), bwops
void bt2ref_exact_sweep_fr(void* vh, int n, const char** seqs, const char** quals,
                           int mineMax, int nofw, int norc, uint64_t* out);

void bt2ref_exact_sweep(void* vh, int n, const char** seqs, const char** quals,
                        int mineMax, uint64_t* out /* 8 per read */) {
	bt2ref_exact_sweep_fr(vh, n, seqs, quals, mineMax, 0, 0, out);
}

// The same with --nofw / --norc.
void bt2ref_exact_sweep_fr(void* vh, int n, const char** seqs, const char** quals,
                           int mineMax, int nofw, int norc, uint64_t* out /* 8 per read */) {
	RefHandle* h = (RefHandle*)vh;
	SeedAlignerX al;
	SeedResults sr;
	SeedSearchMetrics met;
	ScoreParams sp = {0, 6, 2, 1, 5, 3, 5, 3, 4, 0, 0.0, 0.15};
	Scoring sc = makeScoring(sp);
	for(int i = 0; i < n; i++) {
		Read rd("r", seqs[i], quals[i]);
		sr.clear();
		sr.nextRead(rd);
		size_t mineFw = 0, mineRc = 0;
		met.reset();
		uint64_t ops0 = al.ops();
		size_t nelt = al.exactSweep(*h->fw, rd, sc, nofw != 0, norc != 0, (size_t)mineMax,
		                            mineFw, mineRc, true, sr, met);
		uint64_t* o = out + 8 * (size_t)i;
		o[0] = mineFw; o[1] = mineRc; o[2] = nelt;
		EEHit f = sr.exactFwEEHit(), r = sr.exactRcEEHit();
		o[3] = f.top; o[4] = f.bot; o[5] = r.top; o[6] = r.bot;
		o[7] = al.ops() - ops0;  // exactSweep adds to bwops_ only (aligner_seed.cpp:808-818)
	}
}

// SeedAligner::oneMmSearch (rep1mm, no repex, as bt2_search.cpp:3654-3667).
// Writes hits in discovery order: 6 words each (top, bot, fw, score, edit pos, edit chr|readc<<8).
// counts[i] = number of hits for read i (capped at cap per read).  out stride = cap*6.
void bt2ref_one_mm_sc(void* vh, int n, const char** seqs, const char** quals,
                      const int64_t* minsc, int local, int nofw, int norc,
                      int cap, int64_t* out, int32_t* counts, uint64_t* bwops, const void* spp);

void bt2ref_one_mm(void* vh, int n, const char** seqs, const char** quals,
                   const int64_t* minsc, int local, int nofw, int norc,
                   int cap, int64_t* out, int32_t* counts, uint64_t* bwops) {
	bt2ref_one_mm_sc(vh, n, seqs, quals, minsc, local, nofw, norc, cap, out, counts, bwops, NULL);
}

// The same with a scoring scheme (ScoreParams*; NULL: the defaults of `local`).
void bt2ref_one_mm_sc(void* vh, int n, const char** seqs, const char** quals,
                      const int64_t* minsc, int local, int nofw, int norc,
                      int cap, int64_t* out, int32_t* counts, uint64_t* bwops, const void* spp) {
	RefHandle* h = (RefHandle*)vh;
	SeedAlignerX al;
	SeedResults sr;
	SeedSearchMetrics met;
	ScoreParams sp = {local ? 2 : 0, 6, 2, 1, 5, 3, 5, 3, 4, local, 0.0, 0.15};
	if(spp) sp = *(const ScoreParams*)spp;
	Scoring sc = makeScoring(sp);
	for(int i = 0; i < n; i++) {
		Read rd("r", seqs[i], quals[i]);
		sr.clear();
		sr.nextRead(rd);
		met.reset();
		uint64_t ops0 = al.ops();
		al.oneMmSearch(h->fw, h->bw, rd, sc, minsc[i], nofw != 0, norc != 0, local != 0,
		               false, true, sr, met);
		const EList<EEHit>& hits = sr.mm1EEHits();
		int k = 0;
		for(size_t j = 0; j < hits.size() && k < cap; j++, k++) {
			int64_t* o = out + ((size_t)i * cap + k) * 6;
			o[0] = hits[j].top; o[1] = hits[j].bot; o[2] = hits[j].fw ? 1 : 0;
			o[3] = hits[j].score;
			o[4] = hits[j].e1.pos; o[5] = (int64_t)hits[j].e1.chr | ((int64_t)hits[j].e1.qchr << 8);
		}
		counts[i] = (int32_t)hits.size();
		bwops[i] = al.ops() - ops0;
	}
}

// Exact-seed search exactly as one seed round of bt2_search.cpp:3853-3906:
// Seed::mmSeeds(0, seedlen) -> instantiateSeeds(offset, interval) -> searchAllSeeds.
// out per read, per strand (fw then rc), per seed offset index (up to maxseeds):
//   topf, botf, topb, botb  (all 0 when the seed had no hit / was filtered)
// nseeds[i] = number of seed offsets instantiated for read i; bwops[i] = FM ops.
void bt2ref_seed_search(void* vh, int n, const char** seqs, const char** quals,
                        int seedlen, int interval, int offset, int maxseeds,
                        uint32_t* out, int32_t* nseeds, uint64_t* bwops) {
	RefHandle* h = (RefHandle*)vh;
	SeedAligner al;
	SeedResults sr;
	SeedSearchMetrics met;
	PerReadMetrics prm;
	ScoreParams sp = {0, 6, 2, 1, 5, 3, 5, 3, 4, 0, 0.0, 0.15};
	Scoring sc = makeScoring(sp);
	// Engine-level parity: a current-read cache large enough never to run out.
	// The server's default (--seed-cache-sz 20 MB, bt2_search.cpp:484) drops a
	// seed hit when its SA range no longer fits the per-read pool
	// (aligner_cache.cpp:82-96) -- giant ranges of e.g. poly-A 22-mers at hg38
	// scale; that resource limit is reproduced by the drop-in server, which runs
	// the reference's own cache code (integration/bt2g_seams.cpp), not here.
	// (one per thread, kept across calls -- ca.nextRead() clears it for every
	// read: the CPU stand-in server calls this once per read, and a 1 GB block
	// made and freed per call was an mmap / munmap pair per read whose TLB
	// shootdowns slowed every thread of that server)
	static thread_local AlignmentCache scCurrent((size_t)1 << 30, false);
	AlignmentCacheIface ca(&scCurrent, NULL, NULL);
	EList<Seed> seeds;
	Constraint gc = Constraint::penaltyFuncBased(sc.scoreMin);
	EList<SATuple> satups;
	for(int i = 0; i < n; i++) {
		Read rd("r", seqs[i], quals[i]);
		uint32_t* o = out + (size_t)i * 2 * maxseeds * 4;
		memset(o, 0, sizeof(uint32_t) * 2 * maxseeds * 4);
		nseeds[i] = 0; bwops[i] = 0;
		// bt2_search.cpp:3866-3869: the round is skipped when the offset drives
		// the first seed off the end of the read.
		if(offset > 0 && (size_t)(seedlen + offset) > rd.length()) continue;
		sr.clear();
		sr.nextRead(rd);
		ca.nextRead();
		met.reset(); prm.reset();
		seeds.clear();
		Seed::mmSeeds(0, seedlen, seeds, gc);
		std::pair<int, int> instFw, instRc;
		al.instantiateSeeds(seeds, (size_t)offset, interval, rd, sc, false, false, ca, sr, met,
		                    instFw, instRc);
		al.searchAllSeeds(seeds, h->fw, h->bw, rd, sc, ca, sr, met, prm);
		int ns = (int)sr.numOffs();
		nseeds[i] = ns;
		bwops[i] = met.bwops;
		for(int fwi = 0; fwi < 2; fwi++) {
			bool fw = fwi == 0;
			for(int s = 0; s < ns && s < maxseeds; s++) {
				const QVal& qv = sr.hitsAtOffIdx(fw, s);
				if(!qv.valid() || qv.empty()) continue;
				satups.clear();
				size_t nrange = 0, nelt = 0;
				ca.queryQval(qv, satups, nrange, nelt);
				if(satups.size() == 0) continue;
				uint32_t* q = o + ((size_t)fwi * maxseeds + s) * 4;
				q[0] = satups[0].topf; q[1] = satups[0].topf + (uint32_t)satups[0].offs.size();
				q[2] = satups[0].topb; q[3] = satups[0].topb + (uint32_t)satups[0].offs.size();
			}
		}
	}
}

// SwAligner fill + gather for one DP problem, exactly as bt2_dp.cpp:720-744 drives it.
// rfmask: ncol+1 reference masks (1,2,4,8 or 16=N); the extra one is the column
// right of the rectangle (aligner_sw.cpp:174-176).
// out: [0]=aligned(0/1) [1]=best [2]=u8succ [3]=i16succ [4]=colstop [5]=lastsolcol [6]=ncand
// cands: up to cap triples (row, col, score), in the reference's sorted order.
// mat (optional, nrow*ncol*3 int32: H,E,F of the successful matrix, or NULL).
int bt2ref_sw(const char* seq, const char* qual, int fw, const uint8_t* rfmask, int ncol,
              int64_t minsc, const ScoreParams* sp, int enable8, int cap,
              int64_t* out, int64_t* cands, int32_t* mat) {
	Scoring sc = makeScoring(*sp);
	BTDnaString rdfw(seq, true), rdrc;
	BTString qufw(qual), qurc;
	rdrc = rdfw; rdrc.reverseComp();
	qurc = qufw; qurc.reverse();
	SwAlignerX sw;
	sw.initRead(rdfw, rdrc, qufw, qurc, 0, rdfw.length(), sc);
	std::vector<char> rf(ncol + 16, 0);
	for(int i = 0; i <= ncol; i++) rf[i] = (char)rfmask[i];
	DPRect rect;
	rect.refl = 0; rect.refr = ncol - 1; rect.refl_pretrim = 0; rect.refr_pretrim = ncol - 1;
	rect.triml = rect.trimr = 0; rect.corel = 0; rect.corer = 0; rect.maxgap = 0;
	sw.initRef(fw != 0, 0, rect, rf.data(), 0, (size_t)ncol, (TRefOff)ncol + 1000, sc, minsc,
	           enable8 != 0, 2000, 4, false, true);
	TAlScore best = std::numeric_limits<TAlScore>::min();
	bool aligned = sw.align(best);
	out[0] = aligned ? 1 : 0; out[1] = best;
	out[2] = sw.u8succ(); out[3] = sw.i16succ();
	out[4] = (int64_t)sw.colstop(); out[5] = (int64_t)sw.lastsolcol();
	const EList<DpBtCandidate>& c = sw.cands();
	out[6] = (int64_t)c.size();
	for(size_t i = 0; i < c.size() && (int)i < cap; i++) {
		cands[3 * i] = c[i].row; cands[3 * i + 1] = c[i].col; cands[3 * i + 2] = c[i].score;
	}
	if(mat != NULL && (sw.u8succ() || sw.i16succ())) {
		const SSEMatrix& m = sw.mat(sw.u8succ(), fw != 0);
		size_t nrow = rdfw.length();
		for(size_t r = 0; r < nrow; r++)
			for(int cc = 0; cc < ncol; cc++) {
				int32_t* p = mat + 3 * (r * ncol + cc);
				p[0] = m.helt(r, cc); p[1] = m.eelt(r, cc); p[2] = m.felt(r, cc);
			}
	}
	return 0;
}

} // extern "C"

// ---- batch entry points used by bench.py's cpu_baseline leg -----------------
extern "C" {

void bt2ref_get_offsets(void* vh, int n, const uint32_t* rows, uint32_t* out) {
	RefHandle* h = (RefHandle*)vh;
	for(int i = 0; i < n; i++) out[i] = h->fw->getOffset(rows[i]);
}

// SwAligner::initRead/initRef/align for n problems (one SwAligner reused, as a
// worker thread does).  rf: concatenated ncol+1 masks, rf_off[i] its start.
// out: n x 7 (aligned, best, u8succ, i16succ, colstop, lastsolcol, ncand).
void bt2ref_sw_batch(int n, const char** seqs, const char** quals, const uint8_t* fws, const uint8_t* rf,
                     const int64_t* rf_off, const int32_t* ncols, const int64_t* minsc, const ScoreParams* sp,
                     int64_t* out) {
	Scoring sc = makeScoring(*sp);
	SwAlignerX sw;
	BTDnaString rdfw, rdrc;
	BTString qufw, qurc;
	std::vector<char> buf;
	const char* last = nullptr;
	for(int i = 0; i < n; i++) {
		if(seqs[i] != last) {
			rdfw.install(seqs[i], true);
			rdrc = rdfw; rdrc.reverseComp();
			qufw.install(quals[i]);
			qurc = qufw; qurc.reverse();
			sw.initRead(rdfw, rdrc, qufw, qurc, 0, rdfw.length(), sc);
			last = seqs[i];
		}
		int ncol = ncols[i];
		buf.assign(rf + rf_off[i], rf + rf_off[i] + ncol + 1);
		buf.resize(ncol + 16, 0);
		DPRect rect;
		rect.refl = 0; rect.refr = ncol - 1; rect.refl_pretrim = 0; rect.refr_pretrim = ncol - 1;
		rect.triml = rect.trimr = 0; rect.corel = 0; rect.corer = 0; rect.maxgap = 0;
		sw.initRef(fws[i] != 0, 0, rect, buf.data(), 0, (size_t)ncol, (TRefOff)ncol + 1000, sc, minsc[i],
		           true, 2000, 4, false, true);
		TAlScore best = std::numeric_limits<TAlScore>::min();
		bool aligned = sw.align(best);
		int64_t* o = out + 7 * (size_t)i;
		o[0] = aligned; o[1] = best; o[2] = sw.u8succ(); o[3] = sw.i16succ();
		o[4] = (int64_t)sw.colstop(); o[5] = (int64_t)sw.lastsolcol(); o[6] = (int64_t)sw.cands().size();
	}
}

// oneMmSearch gated by exactSweep exactly as bt2_search.cpp:3640-3667 chains them.
// sweep: n x 8 from bt2ref_exact_sweep (mineFw, mineRc, ...).  counts[i] = hits.
void bt2ref_one_mm_gated(void* vh, int n, const char** seqs, const char** quals, const int64_t* minsc,
                         const uint64_t* sweep, int32_t* counts, int local) {
	RefHandle* h = (RefHandle*)vh;
	SeedAligner al;
	SeedResults sr;
	SeedSearchMetrics met;
	ScoreParams sp = {local ? 2 : 0, 6, 2, 1, 5, 3, 5, 3, 4, local, 0.0, 0.15};
	Scoring sc = makeScoring(sp);
	for(int i = 0; i < n; i++) {
		counts[i] = 0;
		uint64_t mfw = sweep[8 * (size_t)i], mrc = sweep[8 * (size_t)i + 1];
		if(std::min(mfw, mrc) == 0) continue;
		bool yfw = mfw <= 1, yrc = mrc <= 1;
		if(!(yfw || yrc)) continue;
		Read rd("r", seqs[i], quals[i]);
		sr.clear();
		sr.nextRead(rd);
		al.oneMmSearch(h->fw, h->bw, rd, sc, minsc[i], !yfw, !yrc, local != 0, false, true, sr, met);
		counts[i] = (int32_t)sr.mm1EEHits().size();
	}
}

// As bt2ref_one_mm_gated, also returning the hits in discovery order (6 words
// each, as bt2ref_one_mm: top, bot, fw, score, edit pos, edit chr | qchr << 8;
// chr / qchr ASCII) at out[(i*cap + k)*6].
void bt2ref_one_mm_gated_hits(void* vh, int n, const char** seqs, const char** quals, const int64_t* minsc,
                              const uint64_t* sweep, int32_t* counts, int local, int cap, int64_t* out) {
	RefHandle* h = (RefHandle*)vh;
	SeedAligner al;
	SeedResults sr;
	SeedSearchMetrics met;
	ScoreParams sp = {local ? 2 : 0, 6, 2, 1, 5, 3, 5, 3, 4, local, 0.0, 0.15};
	Scoring sc = makeScoring(sp);
	for(int i = 0; i < n; i++) {
		counts[i] = 0;
		uint64_t mfw = sweep[8 * (size_t)i], mrc = sweep[8 * (size_t)i + 1];
		if(std::min(mfw, mrc) == 0) continue;
		bool yfw = mfw <= 1, yrc = mrc <= 1;
		if(!(yfw || yrc)) continue;
		Read rd("r", seqs[i], quals[i]);
		sr.clear();
		sr.nextRead(rd);
		al.oneMmSearch(h->fw, h->bw, rd, sc, minsc[i], !yfw, !yrc, local != 0, false, true, sr, met);
		const EList<EEHit>& hits = sr.mm1EEHits();
		counts[i] = (int32_t)hits.size();
		for(size_t j = 0; j < hits.size() && (int)j < cap; j++) {
			int64_t* o = out + ((size_t)i * cap + j) * 6;
			o[0] = hits[j].top; o[1] = hits[j].bot; o[2] = hits[j].fw ? 1 : 0; o[3] = hits[j].score;
			o[4] = hits[j].e1.pos; o[5] = (int64_t)hits[j].e1.chr | ((int64_t)hits[j].e1.qchr << 8);
		}
	}
}

// Ebwt::joinedToTextOff (bt2_idx.cpp:54) for n joined offsets with hit length
// qlens[i]: out[3i..] = {tidx (-1 when rejected as straddling), textoff, tlen}.
void bt2ref_joined_to_text_off(void* vh, int n, const uint32_t* offs, const uint32_t* qlens, int reject,
                               int64_t* out) {
	RefHandle* h = (RefHandle*)vh;
	for(int i = 0; i < n; i++) {
		TIndexOffU tidx = 0, toff = 0, tlen = 0;
		bool straddled = false;
		h->fw->joinedToTextOff(qlens[i], offs[i], tidx, toff, tlen, reject != 0, straddled);
		int64_t* o = out + 3 * (size_t)i;
		o[0] = tidx == OFF_MASK ? -1 : (int64_t)tidx; o[1] = toff; o[2] = tlen;
	}
}

} // extern "C"

// ---- backtrace (row 8a A21) --------------------------------------------------
extern "C" {

// SwAligner::align followed by the nextAlignment loop of SwDriver::extendSeeds
// (aligner_sw_driver.cpp:1157-1180: call until done() or an empty result), on a
// rectangle with the given trim / core diagonals (dp_framer.cpp:116-125).
// Alignments in the order returned, up to maxaln, 10 words each:
//   {cand index, score, off (rectangle column of the leftmost aligned ref
//    char), refoff, ns, gaps, refns, nedit, trim5p(soft), trim3p(soft)}
// edits[(k*maxedit + e)*4 + {pos, type, chr, qchr}] (ASCII chr/qchr, 5'->3').
// fates[i] = btncand_[i].fate after the loop (first capf candidates).
// Returns the number of alignments.
int bt2ref_sw_bt(const char* seq, const char* qual, int fw, const uint8_t* rfmask, int ncol, int64_t minsc,
                 const ScoreParams* sp, int enable8, int triml, int corel, int corer, int maxaln, int maxedit,
                 int64_t* out, int64_t* aln, int32_t* edits, int32_t* fates, int capf) {
	Scoring sc = makeScoring(*sp);
	BTDnaString rdfw(seq, true), rdrc;
	BTString qufw(qual), qurc;
	rdrc = rdfw; rdrc.reverseComp();
	qurc = qufw; qurc.reverse();
	SwAlignerX sw;
	sw.initRead(rdfw, rdrc, qufw, qurc, 0, rdfw.length(), sc);
	std::vector<char> rf(ncol + 16, 0);
	for(int i = 0; i <= ncol; i++) rf[i] = (char)rfmask[i];
	DPRect rect;
	rect.refl = 0; rect.refr = ncol - 1; rect.refl_pretrim = -triml; rect.refr_pretrim = ncol - 1;
	rect.triml = triml; rect.trimr = 0; rect.corel = corel; rect.corer = corer; rect.maxgap = 0;
	sw.initRef(fw != 0, 0, rect, rf.data(), 0, (size_t)ncol, (TRefOff)ncol + 1000, sc, minsc,
	           enable8 != 0, 2000, 4, false, true);
	TAlScore best = std::numeric_limits<TAlScore>::min();
	bool aligned = sw.align(best);
	out[0] = aligned ? 1 : 0; out[1] = best;
	out[2] = sw.u8succ(); out[3] = sw.i16succ();
	out[4] = (int64_t)sw.colstop(); out[5] = (int64_t)sw.lastsolcol(); out[6] = (int64_t)sw.cands().size();
	int na = 0;
	if(aligned) {
		RandomSource rnd;
		rnd.init(0);
		SwResult res;
		while(!sw.done()) {
			res.reset();
			sw.nextAlignment(res, minsc, rnd);
			if(res.empty()) break;
			if(na < maxaln) {
				const AlnRes& a = res.alres;
				int64_t* o = aln + 10 * (size_t)na;
				o[0] = (int64_t)sw.cural() - 1;
				o[1] = a.score().score();
				o[2] = a.refoff();
				o[3] = a.refoff();
				o[4] = a.score().ns();
				o[5] = a.score().gaps();
				o[6] = (int64_t)a.refNs();
				o[7] = (int64_t)a.ned().size();
				o[8] = (int64_t)a.trimmed5p(true);
				o[9] = (int64_t)a.trimmed3p(true);
				for(size_t e = 0; e < a.ned().size() && (int)e < maxedit; e++) {
					int32_t* q = edits + ((size_t)na * maxedit + e) * 4;
					q[0] = (int32_t)a.ned()[e].pos; q[1] = a.ned()[e].type;
					q[2] = a.ned()[e].chr; q[3] = a.ned()[e].qchr;
				}
			}
			na++;
		}
		const EList<DpBtCandidate>& c = sw.cands();
		for(size_t i = 0; i < c.size() && (int)i < capf; i++) fates[i] = c[i].fate;
	}
	return na;
}

} // extern "C"

// ---- batch backtrace for bench.py's cpu_baseline leg -------------------------
extern "C" {

// As bt2ref_sw_batch plus the SwDriver nextAlignment loop on every aligned
// problem (seed-extension rectangle: triml 0, core diagonals [corel, corer]).
// out: n x 8 = {aligned, ncand, naln, cand0, score0, off0, nedit0, edit checksum}
// with the checksum over all alignments k and their edits e:
//   sum (k+1) * (pos*131 + type*31 + chr*7 + qchr)   (mod 2^63)
// As bt2ref_sw_bt_batch with a DPRect per problem: rects n x 4 = {triml,
// corel, corer, 0} (bt2g_sw_rect; the window is the trimmed rectangle).
void bt2ref_sw_bt_batch_rects(int n, const char** seqs, const char** quals, const uint8_t* fws, const uint8_t* rf,
                              const int64_t* rf_off, const int32_t* ncols, const int64_t* minsc,
                              const ScoreParams* sp, const int32_t* rects, int64_t* out) {
	Scoring sc = makeScoring(*sp);
	SwAlignerX sw;
	BTDnaString rdfw, rdrc;
	BTString qufw, qurc;
	std::vector<char> buf;
	const char* last = nullptr;
	RandomSource rnd;
	rnd.init(0);
	SwResult res;
	for(int i = 0; i < n; i++) {
		if(seqs[i] != last) {
			rdfw.install(seqs[i], true);
			rdrc = rdfw; rdrc.reverseComp();
			qufw.install(quals[i]);
			qurc = qufw; qurc.reverse();
			sw.initRead(rdfw, rdrc, qufw, qurc, 0, rdfw.length(), sc);
			last = seqs[i];
		}
		int ncol = ncols[i];
		buf.assign(rf + rf_off[i], rf + rf_off[i] + ncol + 1);
		buf.resize(ncol + 16, 0);
		DPRect rect;
		const int32_t* rc = rects + 4 * (size_t)i;
		rect.refl = 0; rect.refr = ncol - 1; rect.refl_pretrim = -(int64_t)rc[0]; rect.refr_pretrim = ncol - 1;
		rect.triml = (size_t)rc[0]; rect.trimr = 0; rect.corel = (size_t)rc[1]; rect.corer = (size_t)rc[2];
		rect.maxgap = 0;
		sw.initRef(fws[i] != 0, 0, rect, buf.data(), 0, (size_t)ncol, (TRefOff)ncol + 1000, sc, minsc[i],
		           true, 2000, 4, false, true);
		TAlScore best = std::numeric_limits<TAlScore>::min();
		bool aligned = sw.align(best);
		int64_t* o = out + 8 * (size_t)i;
		memset(o, 0, 8 * sizeof(int64_t));
		o[0] = aligned; o[1] = (int64_t)sw.cands().size();
		if(!aligned) continue;
		int64_t na = 0;
		uint64_t ck = 0;
		while(!sw.done()) {
			res.reset();
			sw.nextAlignment(res, minsc[i], rnd);
			if(res.empty()) break;
			const AlnRes& a = res.alres;
			if(na == 0) {
				o[3] = (int64_t)sw.cural() - 1; o[4] = a.score().score(); o[5] = a.refoff();
				o[6] = (int64_t)a.ned().size();
			}
			for(size_t e = 0; e < a.ned().size(); e++) {
				const Edit& ed = a.ned()[e];
				ck += (uint64_t)(na + 1) * ((uint64_t)ed.pos * 131 + (uint64_t)ed.type * 31 +
				                            (uint64_t)ed.chr * 7 + (uint64_t)ed.qchr);
			}
			na++;
		}
		o[2] = na;
		o[7] = (int64_t)(ck & 0x7fffffffffffffffULL);
	}
}

void bt2ref_sw_bt_batch(int n, const char** seqs, const char** quals, const uint8_t* fws, const uint8_t* rf,
                        const int64_t* rf_off, const int32_t* ncols, const int64_t* minsc, const ScoreParams* sp,
                        int corel, int corer, int64_t* out) {
	std::vector<int32_t> rects(4 * (size_t)n);
	for(int i = 0; i < n; i++) { rects[4 * i] = 0; rects[4 * i + 1] = corel; rects[4 * i + 2] = corer; rects[4 * i + 3] = 0; }
	bt2ref_sw_bt_batch_rects(n, seqs, quals, fws, rf, rf_off, ncols, minsc, sp, rects.data(), out);
}

} // extern "C"

// ---- ungapped alignment (row 8a A22) -----------------------------------------
extern "C" {

// SwAligner::ungappedAlign (aligner_sw.cpp:286-494) for n reads against the
// loaded index's reference, each at (refidx[i], off[i]) on strand fw[i], with
// the read (fw) or its reverse complement (as aligner_sw_driver.cpp:1034-1043).
// out: n x 10 = {ret, score, refoff, ns, refns, nedit, trim5p, trim3p, 0, 0};
// edits[(i*maxedit + e)*4 + {pos, type, chr, qchr}].
void bt2ref_ungapped(void* vh, int n, const char** seqs, const char** quals, const uint8_t* fws,
                     const uint32_t* refidx, const int64_t* off, const int64_t* minsc, const ScoreParams* sp,
                     int ohang, int maxedit, int64_t* out, int32_t* edits) {
	RefHandle* h = (RefHandle*)vh;
	Scoring sc = makeScoring(*sp);
	SwAligner sw(NULL);
	SwResult res;
	for(int i = 0; i < n; i++) {
		BTDnaString rdfw(seqs[i], true), rdrc = rdfw;
		rdrc.reverseComp();
		BTString qfw(quals[i]), qrc = qfw;
		qrc.reverse();
		bool fw = fws[i] != 0;
		Coord coord((TRefId)refidx[i], (TRefOff)off[i], fw);
		size_t tlen = h->refs->approxLen(refidx[i]);
		res.reset();
		int ret = sw.ungappedAlign(fw ? rdfw : rdrc, fw ? qfw : qrc, coord, *h->refs, tlen, sc, ohang != 0,
		                           minsc[i], res);
		int64_t* o = out + 10 * (size_t)i;
		memset(o, 0, 10 * sizeof(int64_t));
		o[0] = ret;
		if(ret == 1) {
			const AlnRes& a = res.alres;
			o[1] = a.score().score(); o[2] = a.refoff(); o[3] = a.score().ns(); o[4] = (int64_t)a.refNs();
			o[5] = (int64_t)a.ned().size(); o[6] = (int64_t)a.trimmed5p(true); o[7] = (int64_t)a.trimmed3p(true);
			for(size_t e = 0; e < a.ned().size() && (int)e < maxedit; e++) {
				int32_t* q = edits + ((size_t)i * maxedit + e) * 4;
				q[0] = (int32_t)a.ned()[e].pos; q[1] = a.ned()[e].type; q[2] = a.ned()[e].chr; q[3] = a.ned()[e].qchr;
			}
		}
	}
}

} // extern "C"

extern "C" {

// DP framing exactly as SwDriver calls it: seed extension (kind 0,
// aligner_sw_driver.cpp:992-1000, 1074-1084) and mate search (kind 1,
// aligner_sw_driver.cpp:1975-2024: maxReadGaps/maxRefGaps of ominsc, otherMate
// with maxalcols = orows + oreadGaps, frameFindMateRect(!oleft, ...)).
// in: n x 8 int64 {kind, off, rdlen, reflen, minsc, fw, anchor1, alen}
// pe: {policy, minfrag, maxfrag, flip, dovetail, olap, expand}
// out: n x 7 {ok, fw, refl, ncol, triml, corel, corer}
void bt2ref_frame(int n, const int64_t* in, const ScoreParams* sp, const int32_t* pe, int maxhalf, int trim_to_ref,
                  int64_t* out) {
	Scoring sc = makeScoring(*sp);
	DynProgFramer fr(trim_to_ref != 0);
	PairedEndPolicy pepol(pe[0], (size_t)pe[2], (size_t)pe[1], sp->local != 0, pe[3] != 0, pe[4] != 0, true,
	                      pe[5] != 0, pe[6] != 0);
	for(int i = 0; i < n; i++) {
		const int64_t* x = in + 8 * (size_t)i;
		int64_t* o = out + 7 * (size_t)i;
		memset(o, 0, 7 * sizeof(int64_t));
		const int kind = (int)x[0];
		const int64_t off = x[1];
		const size_t rdlen = (size_t)x[2];
		const int64_t reflen = x[3], minsc = x[4];
		const bool fw = x[5] != 0, anchor1 = x[6] != 0;
		const size_t alen = (size_t)x[7];
		int nceil = std::min((int)sc.nCeil.f<int>((double)rdlen), (int)rdlen);
		int readGaps = sc.maxReadGaps(minsc, rdlen);
		int refGaps = sc.maxRefGaps(minsc, rdlen);
		DPRect rect;
		bool found;
		bool ofw = fw;
		if(kind == 0) {
			found = fr.frameSeedExtensionRect(off, rdlen, reflen, readGaps, refGaps, (size_t)nceil, (size_t)maxhalf,
			                                  rect);
		} else {
			bool oleft = false;
			int64_t oll = 0, olr = 0, orl = 0, orr = 0;
			found = pepol.otherMate(anchor1, fw, off, rdlen + readGaps, (size_t)reflen, anchor1 ? alen : rdlen,
			                        anchor1 ? rdlen : alen, oleft, oll, olr, orl, orr, ofw);
			if(found)
				found = fr.frameFindMateRect(!oleft, oll, olr, orl, orr, rdlen, reflen, readGaps, refGaps,
				                             (size_t)nceil, (size_t)maxhalf, rect);
		}
		if(!found) continue;
		o[0] = 1; o[1] = ofw; o[2] = rect.refl; o[3] = rect.refr - rect.refl + 1;
		o[4] = (int64_t)rect.triml; o[5] = (int64_t)rect.corel; o[6] = (int64_t)rect.corer;
	}
}

} // extern "C"

// SwDriver::extend (aligner_sw_driver.cpp:299-483, protected) on seed-hit
// ranges: per range {fw, off, len} and {topf, botf, topb, botb}; out per range
// {nlex, nrex, nSdFmops increments}.
namespace {
struct SwDriverX : public SwDriver {
	SwDriverX() : SwDriver(1 << 20) {}
	void ext(const Read& rd, const Ebwt& f, const Ebwt* b, uint32_t tf, uint32_t bf, uint32_t tb, uint32_t bb, bool fw,
	         size_t off, size_t len, PerReadMetrics& prm, size_t& nlex, size_t& nrex) {
		extend(rd, f, b, tf, bf, tb, bb, fw, off, len, prm, nlex, nrex);
	}
};
}  // namespace

extern "C" {
void bt2ref_extend(void* vh, int n, const char** seqs, const char** quals, const int32_t* fw, const uint32_t* off,
                   const uint32_t* len, const uint32_t* tb, uint32_t* out) {
	RefHandle* h = (RefHandle*)vh;
	SwDriverX sd;
	for(int i = 0; i < n; i++) {
		Read rd("r", seqs[i], quals[i]);
		PerReadMetrics prm;
		prm.reset();
		size_t nlex = 0, nrex = 0;
		sd.ext(rd, *h->fw, h->bw, tb[4 * i], tb[4 * i + 1], tb[4 * i + 2], tb[4 * i + 3], fw[i] != 0, off[i], len[i], prm,
		       nlex, nrex);
		out[3 * i] = (uint32_t)nlex;
		out[3 * i + 1] = (uint32_t)nrex;
		out[3 * i + 2] = (uint32_t)prm.nSdFmops;
	}
}
} // extern "C"
