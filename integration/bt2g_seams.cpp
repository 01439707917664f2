// integration/bt2g_seams.cpp -- the reference-side binding of the bt2g C ABI.
//
// What a bowtie2 maintainer adds to put the MI355X engines under the
// reference's own host code: definitions of the per-thread seams that
// multiseedSearchWorker (bt2_search.cpp:3050-4197) and SwDriver
// (aligner_sw_driver.cpp:756-2100) call, each served by one bt2g_* call and
// the bookkeeping the reference does around that seam.  The reference's
// driver, RNG, SeedResults/AlignmentCache, SwDriver state machine, AlnSinkWrap,
// MAPQ and SAM writer run unchanged, so SAM equality between the stock server
// and this build shows that every GPU call returned exactly what the
// reference's own seam would have returned on the reference's own schedule.
//
// Linking (integration/Makefile): the reference objects plus this file, with
// `-Wl,--wrap=<seam>` so that calls from the other translation units
// (bt2_search.cpp, aligner_sw_driver.cpp) reach __wrap_<seam> below, and
// __real_<seam> is the reference's CPU implementation, used only for work the
// engines do not take (reads longer than BT2G_MAX_READ_LEN, DPs of reads at or
// above the checkpointing threshold cminlen -- SURVEY.md 2 row 6 -- and
// mismatch seeds, -N 1).  Every such fallback is counted; the counts are
// written to $BT2G_ADAPTER_STATS.
//
// Seams (reference file:line):
//   SeedAligner::exactSweep      aligner_seed.cpp:854-968    -> bt2g_exact_sweep
//   SeedAligner::oneMmSearch     aligner_seed.cpp:973-1323   -> bt2g_one_mm
//   SeedAligner::searchAllSeeds  aligner_seed.cpp:597-718    -> bt2g_seed_search
//   SwAligner::ungappedAlign     aligner_sw.cpp:286-494      -> bt2g_ungapped
//   SwAligner::align             aligner_sw.cpp:500-729      -> bt2g_sw_align_bt (fill, gather, sort,
//   SwAligner::nextAlignment     aligner_sw.cpp:737-1146        and every backtrace, with candidate fates)
//
// The GPU context is opened on first use from $BT2G_INDEX (the index base the
// server was started with) on device $BT2G_DEVICE (default 0).  Calls are
// serialised by one mutex: this binding demonstrates the drop-in and its
// exactness; it is not the throughput path (bench.py batches instead).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <signal.h>
#include <unistd.h>
#include <fcntl.h>
#include <atomic>
#include <mutex>
#include <vector>
#include <limits>

#include "aligner_seed.h"
#include "aligner_cache.h"
#include "aligner_sw.h"
#include "read.h"
#include "scoring.h"
#include "bt2g.h"

namespace {

std::mutex g_mu;
bt2g_ctx* g_ctx = nullptr;

enum { ST_EXACT, ST_1MM, ST_SEEDS, ST_UG, ST_DP, ST_N };
const char* const ST_NAMES[ST_N] = {"exact_sweep", "one_mm", "seed_search", "ungapped", "sw_dp"};
std::atomic<uint64_t> g_gpu[ST_N], g_cpu[ST_N];
char g_stats_path[4096];

void write_stats() {
	if(!g_stats_path[0]) return;
	char buf[1024];
	int n = 0;
	n += snprintf(buf + n, sizeof(buf) - n, "{");
	for(int i = 0; i < ST_N; i++)
		n += snprintf(buf + n, sizeof(buf) - n, "%s\"%s\": [%llu, %llu]", i ? ", " : "", ST_NAMES[i],
		              (unsigned long long)g_gpu[i].load(), (unsigned long long)g_cpu[i].load());
	n += snprintf(buf + n, sizeof(buf) - n, "}\n");
	int fd = open(g_stats_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
	if(fd >= 0) {
		ssize_t w = write(fd, buf, (size_t)n);
		(void)w;
		close(fd);
	}
}

void on_term(int) {
	write_stats();
	_exit(0);
}

void count(int st, bool gpu) {
	uint64_t t = (gpu ? g_gpu[st] : g_cpu[st]).fetch_add(1) + 1;
	if((t & 1023) == 0) write_stats();
}

void die(const char* what, int rc) {
	fprintf(stderr, "bt2g adapter: %s failed (%d): %s\n", what, rc, bt2g_last_error());
	throw 1;   // the reference's error convention (bt2_search.cpp:5598-5620)
}

// Opened lazily under g_mu.
bt2g_ctx* ctx() {
	if(g_ctx) return g_ctx;
	const char* base = getenv("BT2G_INDEX");
	if(!base) {
		fprintf(stderr, "bt2g adapter: BT2G_INDEX is not set\n");
		throw 1;
	}
	const char* dev = getenv("BT2G_DEVICE");
	const char* sp = getenv("BT2G_ADAPTER_STATS");
	if(sp) {
		strncpy(g_stats_path, sp, sizeof(g_stats_path) - 1);
		signal(SIGTERM, on_term);
	}
	int rc = bt2g_open(base, dev ? atoi(dev) : 0, &g_ctx);
	if(rc) die("bt2g_open", rc);
	return g_ctx;
}

// bt2g_scoring of a reference Scoring object (scoring.h:442-460).  Only the
// models the engines implement: quality-aware mismatches, constant N penalty.
bool to_scoring(const Scoring& sc, bt2g_scoring& o) {
	if(sc.mmcostType != COST_MODEL_QUAL || sc.npenType != COST_MODEL_CONSTANT || sc.matchType != COST_MODEL_CONSTANT)
		return false;
	if(sc.nCeil.getMin() != 0.0) return false;
	o.match = sc.monotone ? 0 : sc.matchConst;
	o.mmp_max = sc.mmpMax;
	o.mmp_min = sc.mmpMin;
	o.npen = sc.npen;
	o.rdg_const = sc.rdGapConst;
	o.rdg_lin = sc.rdGapLinear;
	o.rfg_const = sc.rfGapConst;
	o.rfg_lin = sc.rfGapLinear;
	o.gapbar = sc.gapbar;
	o.local = sc.monotone ? 0 : 1;
	o.ncl_const = sc.nCeil.getConst();
	o.ncl_lin = sc.nCeil.getCoeff();
	return true;
}

// A read as one row of codes (0..4) and Phred+33 qualities.
struct Row {
	std::vector<uint8_t> codes, quals;
	uint32_t len = 0;
	void set(const BTDnaString& s, const BTString& q) {
		len = (uint32_t)s.length();
		codes.resize(len ? len : 1);
		quals.resize(len ? len : 1);
		for(uint32_t i = 0; i < len; i++) {
			codes[i] = (uint8_t)s[i];
			quals[i] = (uint8_t)q[i];
		}
	}
	// forward read from the strand-specific one the driver holds
	void set_fw_of(const BTDnaString& s, const BTString& q, bool fw) {
		set(s, q);
		if(!fw) {
			for(uint32_t i = 0, j = len ? len - 1 : 0; i < j; i++, j--) {
				std::swap(codes[i], codes[j]);
				std::swap(quals[i], quals[j]);
			}
			for(uint32_t i = 0; i < len; i++) codes[i] = codes[i] > 3 ? 4 : (uint8_t)(3 - codes[i]);
		}
	}
};

// AlnRes from an engine alignment: edits already in their final (5'->3',
// post-trim) positions, so they are shifted by the leading trim before
// setShape, which subtracts it (aligner_result.cpp:101-108).
void fill_alnres(AlnRes& a, const bt2g_edit* ed, uint32_t nedit, int64_t score, int64_t ns, int64_t gaps,
                 int basesAligned, TRefId refidx, TRefOff refoff, TRefOff reflen, bool fw, size_t rdlen,
                 size_t trim5p, size_t trim3p, size_t refns) {
	a.reset();
	const size_t trimBeg = fw ? trim5p : trim3p;
	EList<Edit>& ned = a.ned();
	for(uint32_t e = 0; e < nedit; e++)
		ned.push_back(Edit(ed[e].pos + (uint32_t)trimBeg, ed[e].chr, ed[e].qchr, ed[e].type));
	a.setScore(AlnScore(score, basesAligned, (int)nedit, ns, gaps));
	a.setShape(refidx, refoff, reflen, fw, rdlen, true, 0, 0, true, trim5p, trim3p);
	a.setRefNs(refns);
}

// Per-SwAligner state between align() and the nextAlignment() calls.
struct DpState {
	bool gpu = false;          // served by the engine (else the reference's CPU path)
	bool u8 = false;           // u8 fill succeeded (RNG re-seed rule, aligner_sw.cpp:877 vs 932)
	std::vector<int8_t> fates; // engine's DpBtCandidate::fate per candidate
	std::vector<bt2g_sw_aln> alns;
	std::vector<bt2g_edit> edits;
	uint32_t maxedit = 0;
	int32_t naln = 0;
	uint32_t next = 0;         // next engine alignment to hand out
};

thread_local std::vector<std::pair<const void*, DpState>> t_dp;

DpState& dp_state(const void* sw) {
	for(auto& p : t_dp)
		if(p.first == sw) return p.second;
	t_dp.emplace_back(sw, DpState());
	return t_dp.back().second;
}

// Protected-member access (no added members: same layout as the base).
struct SeedAlignerAcc : public SeedAligner {
	void set_state(const Ebwt* f, const Ebwt* b, const Scoring* s, const Read* r) {
		ebwtFw_ = f; ebwtBw_ = b; sc_ = s; read_ = r; bwops_ = bwedits_ = 0;
	}
	void add_ops(uint64_t n) { bwops_ += n; }
	uint64_t ops() const { return bwops_; }
};

struct SwAlignerAcc : public SwAligner {
	bool gpu_align(TAlScore& best, bool& served);
	bool gpu_next(SwResult& res, TAlScore minsc, RandomSource& rnd, DpState& st);
	size_t rdlen() const { return rdf_ - rdi_; }
	size_t cminlen() const { return cperMinlen_; }
};

const uint32_t MAXALN0 = 64;

}  // namespace

extern "C" {

// ---- the reference's CPU implementations (renamed by --wrap) ---------------
size_t __real__ZN11SeedAligner10exactSweepERK4EbwtRK4ReadRK7ScoringbbmRmS9_bR11SeedResultsR17SeedSearchMetrics(
	SeedAligner*, const Ebwt&, const Read&, const Scoring&, bool, bool, size_t, size_t&, size_t&, bool, SeedResults&,
	SeedSearchMetrics&);
bool __real__ZN11SeedAligner11oneMmSearchEPK4EbwtS2_RK4ReadRK7ScoringlbbbbbR11SeedResultsR17SeedSearchMetrics(
	SeedAligner*, const Ebwt*, const Ebwt*, const Read&, const Scoring&, int64_t, bool, bool, bool, bool, bool,
	SeedResults&, SeedSearchMetrics&);
void __real__ZN11SeedAligner14searchAllSeedsERK5EListI4SeedLi128EEPK4EbwtS7_RK4ReadRK7ScoringR19AlignmentCacheIfaceR11SeedResultsR17SeedSearchMetricsR14PerReadMetrics(
	SeedAligner*, const EList<Seed>&, const Ebwt*, const Ebwt*, const Read&, const Scoring&, AlignmentCacheIface&,
	SeedResults&, SeedSearchMetrics&, PerReadMetrics&);
int __real__ZN9SwAligner13ungappedAlignERK20SDnaStringExpandableILi1024ELi2EERK17SStringExpandableIcLi1024ELi2ELi0EERK5CoordRK16BitPairReferencemRK7ScoringblR8SwResult(
	SwAligner*, const BTDnaString&, const BTString&, const Coord&, const BitPairReference&, size_t, const Scoring&,
	bool, TAlScore, SwResult&);
bool __real__ZN9SwAligner5alignERl(SwAligner*, TAlScore&);
bool __real__ZN9SwAligner13nextAlignmentER8SwResultlR12RandomSource(SwAligner*, SwResult&, TAlScore, RandomSource&);

// ---- SeedAligner::exactSweep (aligner_seed.cpp:854-968) ---------------------
size_t __wrap__ZN11SeedAligner10exactSweepERK4EbwtRK4ReadRK7ScoringbbmRmS9_bR11SeedResultsR17SeedSearchMetrics(
	SeedAligner* self, const Ebwt& ebwt, const Read& read, const Scoring& sc, bool nofw, bool norc, size_t mineMax,
	size_t& mineFw, size_t& mineRc, bool repex, SeedResults& hits, SeedSearchMetrics& met) {
	const size_t len = read.length();
	if(!repex || len == 0 || len > BT2G_MAX_READ_LEN) {
		count(ST_EXACT, false);
		return __real__ZN11SeedAligner10exactSweepERK4EbwtRK4ReadRK7ScoringbbmRmS9_bR11SeedResultsR17SeedSearchMetrics(
			self, ebwt, read, sc, nofw, norc, mineMax, mineFw, mineRc, repex, hits, met);
	}
	Row r;
	r.set(read.patFw, read.qual);
	uint32_t out[8];
	{
		std::lock_guard<std::mutex> lk(g_mu);
		int rc = bt2g_exact_sweep(ctx(), r.codes.data(), r.len, &r.len, 1, (uint32_t)mineMax, nofw, norc, out);
		if(rc) die("bt2g_exact_sweep", rc);
	}
	count(ST_EXACT, true);
	// outputs exactly as the tail of exactSweep (aligner_seed.cpp:944-967)
	if(!nofw) mineFw = out[0];
	if(!norc) mineRc = out[1];
	static_cast<SeedAlignerAcc*>(self)->add_ops(out[6]);
	size_t nelt = 0;
	const int64_t score = (int64_t)len * sc.match();
	if(!nofw && out[0] == 0 && out[3] > out[2]) {
		hits.addExactEeFw(out[2], out[3], NULL, NULL, true, score);
		nelt += out[3] - out[2];
	}
	if(!norc && out[1] == 0 && out[5] > out[4]) {
		hits.addExactEeRc(out[4], out[5], NULL, NULL, false, score);
		nelt += out[5] - out[4];
	}
	return nelt;
}

// ---- SeedAligner::oneMmSearch (aligner_seed.cpp:973-1323) --------------------
// The engine returns the hits in the reference's discovery order; each goes to
// SeedResults::add1mmEe exactly as aligner_seed.cpp:1283 does.  The return
// value is unused by the caller (bt2_search.cpp:3654).
bool __wrap__ZN11SeedAligner11oneMmSearchEPK4EbwtS2_RK4ReadRK7ScoringlbbbbbR11SeedResultsR17SeedSearchMetrics(
	SeedAligner* self, const Ebwt* ebwtFw, const Ebwt* ebwtBw, const Read& read, const Scoring& sc, int64_t minsc,
	bool nofw, bool norc, bool local, bool repex, bool rep1mm, SeedResults& hits, SeedSearchMetrics& met) {
	const size_t len = read.length();
	bt2g_scoring bs;
	if(repex || !rep1mm || len < 2 || len > BT2G_MAX_READ_LEN || !to_scoring(sc, bs) || local != !sc.monotone ||
	   minsc < std::numeric_limits<int32_t>::min() || minsc > std::numeric_limits<int32_t>::max()) {
		count(ST_1MM, false);
		return __real__ZN11SeedAligner11oneMmSearchEPK4EbwtS2_RK4ReadRK7ScoringlbbbbbR11SeedResultsR17SeedSearchMetrics(
			self, ebwtFw, ebwtBw, read, sc, minsc, nofw, norc, local, repex, rep1mm, hits, met);
	}
	Row r;
	r.set(read.patFw, read.qual);
	int32_t ms = (int32_t)minsc, cnt = 0;
	uint32_t ops = 0;
	std::vector<bt2g_mm1> h(64);
	{
		std::lock_guard<std::mutex> lk(g_mu);
		int rc = bt2g_one_mm(ctx(), r.codes.data(), r.quals.data(), r.len, &r.len, 1, &ms, &bs, nofw, norc,
		                     (uint32_t)h.size(), h.data(), &cnt, &ops, nullptr);
		if(rc == BT2G_ERR_OVERFLOW) {
			h.resize((size_t)cnt);
			rc = bt2g_one_mm(ctx(), r.codes.data(), r.quals.data(), r.len, &r.len, 1, &ms, &bs, nofw, norc,
			                 (uint32_t)h.size(), h.data(), &cnt, &ops, nullptr);
		}
		if(rc) die("bt2g_one_mm", rc);
	}
	count(ST_1MM, true);
	static_cast<SeedAlignerAcc*>(self)->add_ops(ops);
	for(int32_t k = 0; k < cnt; k++) {
		Edit e((uint32_t)h[k].pos, h[k].chr, h[k].qchr, EDIT_TYPE_MM, false);
		hits.add1mmEe(h[k].top, h[k].bot, &e, NULL, h[k].fw != 0, h[k].score);
	}
	return cnt > 0;
}

// ---- SeedAligner::searchAllSeeds (aligner_seed.cpp:597-718) ------------------
// One bt2g_seed_search of the read for the round's offsets (instantiateSeeds
// already ran: sr.idx2off), then the reference's cache protocol per
// instantiated seed, in the order searchAllSeeds runs it: strand fw then rc,
// seed offsets ascending; SeedSearchCache::addOnTheFly for a hit (reportHit,
// aligner_seed.cpp:1576-1630), beginAlign / addAllCached / finishAlign, and
// SeedResults::add.
void __wrap__ZN11SeedAligner14searchAllSeedsERK5EListI4SeedLi128EEPK4EbwtS7_RK4ReadRK7ScoringR19AlignmentCacheIfaceR11SeedResultsR17SeedSearchMetricsR14PerReadMetrics(
	SeedAligner* self, const EList<Seed>& seeds, const Ebwt* ebwtFw, const Ebwt* ebwtBw, const Read& read,
	const Scoring& pens, AlignmentCacheIface& cache, SeedResults& sr, SeedSearchMetrics& met, PerReadMetrics& prm) {
	const size_t len = read.length();
	const size_t nof = sr.numOffs();
	bool ok = len > 0 && len <= BT2G_MAX_READ_LEN && nof > 0 && ebwtBw != NULL;
	for(size_t j = 0; ok && j < seeds.size(); j++) ok = seeds[j].type == SEED_TYPE_EXACT;
	if(!ok) {
		count(ST_SEEDS, false);
		__real__ZN11SeedAligner14searchAllSeedsERK5EListI4SeedLi128EEPK4EbwtS7_RK4ReadRK7ScoringR19AlignmentCacheIfaceR11SeedResultsR17SeedSearchMetricsR14PerReadMetrics(
			self, seeds, ebwtFw, ebwtBw, read, pens, cache, sr, met, prm);
		return;
	}
	SeedAlignerAcc* al = static_cast<SeedAlignerAcc*>(self);
	al->set_state(ebwtFw, ebwtBw, &pens, &read);
	const uint32_t seedlen = (uint32_t)std::min<size_t>((size_t)seeds[0].len, len);
	const uint32_t off = (uint32_t)sr.idx2off(0);
	uint32_t per = nof > 1 ? (uint32_t)(sr.idx2off(1) - sr.idx2off(0))
	                       : (uint32_t)(len > off + seedlen ? len - off - seedlen + 1 : 1);
	Row r;
	r.set(read.patFw, read.qual);
	std::vector<uint32_t> out(2 * nof * 4);
	int32_t ns = 0;
	uint32_t ops = 0;
	{
		std::lock_guard<std::mutex> lk(g_mu);
		int rc = bt2g_seed_search(ctx(), r.codes.data(), r.len, &r.len, 1, (uint32_t)seeds[0].len, per, off,
		                          (uint32_t)nof, out.data(), &ns, &ops, nullptr);
		if(rc) die("bt2g_seed_search", rc);
	}
	if((size_t)ns != nof) {
		fprintf(stderr, "bt2g adapter: seed offsets differ (engine %d, reference %zu)\n", ns, nof);
		throw 1;
	}
	count(ST_SEEDS, true);
	al->add_ops(ops);
	uint64_t possearches = 0, seedsearches = 0, ooms = 0;
	for(int fwi = 0; fwi < 2; fwi++) {
		const bool fw = fwi == 0;
		for(size_t i = 0; i < nof; i++) {
			EList<InstantiatedSeed>& iss = sr.instantiatedSeeds(fw, i);
			if(iss.empty()) continue;
			possearches++;
			seedsearches += iss.size();
			const BTDnaString& seq = sr.seqs(fw)[i];
			SeedSearchCache srcache(seq, sr.quals(fw)[i]);
			const uint32_t* q = &out[((size_t)fwi * nof + i) * 4];
			if(q[1] > q[0]) srcache.addOnTheFly(seq, q[0], q[1], q[2], q[3]);
			if(srcache.beginAlign(cache) == -1) { ooms++; continue; }
			if(!srcache.addAllCached()) { ooms++; continue; }
			srcache.finishAlign();
			if(srcache.qvValid()) sr.add(srcache.getQv(), cache.current(), (uint32_t)i, fw);
		}
	}
	// per-read and search metrics as aligner_seed.cpp:697-717
	prm.nSeedRanges = sr.numRanges();
	prm.nSeedElts = sr.numElts();
	prm.nSeedRangesFw = sr.numRangesFw();
	prm.nSeedRangesRc = sr.numRangesRc();
	prm.nSeedEltsFw = sr.numEltsFw();
	prm.nSeedEltsRc = sr.numEltsRc();
	prm.seedMedian = (uint64_t)(sr.medianHitsPerSeed() + 0.5);
	prm.seedMean = (uint64_t)sr.averageHitsPerSeed();
	prm.nSdFmops += al->ops();
	met.seedsearch += seedsearches;
	met.nrange += sr.numRanges();
	met.nelt += sr.numElts();
	met.possearch += possearches;
	met.ooms += ooms;
	met.bwops += al->ops();
}

// ---- SwAligner::ungappedAlign (aligner_sw.cpp:286-494) -----------------------
int __wrap__ZN9SwAligner13ungappedAlignERK20SDnaStringExpandableILi1024ELi2EERK17SStringExpandableIcLi1024ELi2ELi0EERK5CoordRK16BitPairReferencemRK7ScoringblR8SwResult(
	SwAligner* self, const BTDnaString& rd, const BTString& qu, const Coord& coord, const BitPairReference& refs,
	size_t reflen, const Scoring& sc, bool ohang, TAlScore minsc, SwResult& res) {
	const size_t len = rd.length();
	bt2g_scoring bs;
	if(len == 0 || len > BT2G_MAX_READ_LEN || !to_scoring(sc, bs) ||
	   minsc < std::numeric_limits<int32_t>::min() || minsc > std::numeric_limits<int32_t>::max()) {
		count(ST_UG, false);
		return __real__ZN9SwAligner13ungappedAlignERK20SDnaStringExpandableILi1024ELi2EERK17SStringExpandableIcLi1024ELi2ELi0EERK5CoordRK16BitPairReferencemRK7ScoringblR8SwResult(
			self, rd, qu, coord, refs, reflen, sc, ohang, minsc, res);
	}
	const bool fw = coord.fw();
	Row r;
	r.set_fw_of(rd, qu, fw);
	bt2g_ug_problem p;
	memset(&p, 0, sizeof(p));
	p.read = 0;
	p.fw = fw ? 1 : 0;
	p.off = coord.off();
	p.refidx = (uint32_t)coord.ref();
	p.minsc = (int32_t)minsc;
	bt2g_ug_result o;
	std::vector<bt2g_edit> ed(len + 1);
	{
		std::lock_guard<std::mutex> lk(g_mu);
		int rc = bt2g_ungapped(ctx(), r.codes.data(), r.quals.data(), r.len, &r.len, &p, 1, &bs, ohang ? 1 : 0,
		                       (uint32_t)ed.size(), &o, ed.data());
		if(rc) die("bt2g_ungapped", rc);
	}
	count(ST_UG, true);
	res.alres.reset();
	if(o.ret != 1) return o.ret;
	// AlnScore(score, len - #edits, #edits, ns, 0) and setShape as aligner_sw.cpp:466-481
	fill_alnres(res.alres, ed.data(), (uint32_t)o.nedit, o.score, o.ns, 0, (int)(len - (size_t)o.nedit),
	            coord.ref(), o.refoff, (TRefOff)reflen, fw, len, (size_t)o.trim5p, (size_t)o.trim3p, (size_t)o.refns);
	return 1;
}

// ---- SwAligner::align + nextAlignment (aligner_sw.cpp:500-1146) ---------------
bool __wrap__ZN9SwAligner5alignERl(SwAligner* self, TAlScore& best) {
	SwAlignerAcc* s = static_cast<SwAlignerAcc*>(self);
	bool served = false;
	bool ret = s->gpu_align(best, served);
	if(served) return ret;
	dp_state(self).gpu = false;
	count(ST_DP, false);
	return __real__ZN9SwAligner5alignERl(self, best);
}

bool __wrap__ZN9SwAligner13nextAlignmentER8SwResultlR12RandomSource(SwAligner* self, SwResult& res, TAlScore minsc,
                                                                    RandomSource& rnd) {
	DpState& st = dp_state(self);
	if(!st.gpu) return __real__ZN9SwAligner13nextAlignmentER8SwResultlR12RandomSource(self, res, minsc, rnd);
	return static_cast<SwAlignerAcc*>(self)->gpu_next(res, minsc, rnd, st);
}

}  // extern "C"

// align(): the engine's fill + gather + sort and the whole nextAlignment loop
// of this DP, on the window initRef built (rf_[rfi_ .. rff_] plus the extra
// right column, aligner_sw.cpp:171-253) and the DPRect's trim and core
// diagonals.  SwAligner state is set as align() leaves it (btncand_ sorted,
// cural_ 0, sse8succ_/sse16succ_), so done() and numAlignmentsReported() work.
bool SwAlignerAcc::gpu_align(TAlScore& best, bool& served) {
	served = false;
	const size_t rdlen = rdf_ - rdi_;
	const size_t ncol = (size_t)(rff_ - rfi_);
	bt2g_scoring bs;
	if(rdi_ != 0 || rdlen != rdfw_->length() || rdlen == 0 || rdlen > BT2G_MAX_READ_LEN || rdlen >= cperMinlen_ ||
	   ncol == 0 || !to_scoring(*sc_, bs) || minsc_ < std::numeric_limits<int32_t>::min() ||
	   minsc_ > std::numeric_limits<int32_t>::max())
		return false;
	DpState& st = dp_state(this);
	Row r;
	r.set(*rdfw_, *qufw_);
	bt2g_sw_problem p;
	memset(&p, 0, sizeof(p));
	p.read = 0;
	p.fw = fw_ ? 1 : 0;
	p.refl = 0;
	p.win_off = 0;
	p.refidx = (uint32_t)refidx_;
	p.ncol = (uint32_t)ncol;
	p.minsc = (int32_t)minsc_;
	bt2g_sw_rect rect;
	rect.triml = (int32_t)rect_->triml;
	rect.corel = (int32_t)rect_->corel;
	rect.corer = (int32_t)rect_->corer;
	rect.pad = 0;
	std::vector<uint8_t> win(ncol + 1);
	for(size_t i = 0; i <= ncol; i++) win[i] = (uint8_t)rf_[rfi_ + i];
	bt2g_sw_result o;
	uint32_t cap = 1024;
	uint32_t maxaln = MAXALN0;
	const uint32_t maxedit = (uint32_t)(2 * rdlen + 8);
	std::vector<bt2g_sw_cand> cands;
	for(;;) {
		cands.assign(cap, bt2g_sw_cand());
		st.fates.assign(cap, 0);
		st.alns.assign(maxaln, bt2g_sw_aln());
		st.edits.assign((size_t)maxaln * maxedit, bt2g_edit());
		int rc;
		{
			std::lock_guard<std::mutex> lk(g_mu);
			rc = bt2g_sw_align_bt(ctx(), r.codes.data(), r.quals.data(), r.len, &r.len, &p, 1, win.data(), win.size(),
			                      &rect, &bs, (enable8_ && !readSse16_) ? 1 : 0, cap, &o, cands.data(), maxaln,
			                      maxedit, &st.naln, st.alns.data(), st.edits.data(), st.fates.data());
		}
		if(rc == BT2G_ERR_OVERFLOW && o.ncand > (int32_t)cap) { cap = (uint32_t)o.ncand; continue; }
		if(rc) die("bt2g_sw_align_bt", rc);
		if(st.naln == (int32_t)maxaln && maxaln < (uint32_t)o.ncand) { maxaln = (uint32_t)o.ncand; continue; }
		break;
	}
	if(st.naln < 0) {
		fprintf(stderr, "bt2g adapter: sw_align_bt status %d\n", st.naln);
		throw 1;
	}
	served = true;
	count(ST_DP, true);
	st.gpu = true;
	st.maxedit = maxedit;
	st.next = 0;
	// SwAligner::align's own state (aligner_sw.cpp:505-512, 677-729)
	state_ = 2;   // STATE_ALIGNED (private enum, aligner_sw.h:197-201)
	btncand_.clear();
	btncanddone_.clear();
	btncanddoneSucc_ = btncanddoneFail_ = 0;
	sse8succ_ = o.u8succ != 0;
	sse16succ_ = o.i16succ != 0;
	st.u8 = sse8succ_;
	colstop_ = (size_t)o.colstop;
	lastsolcol_ = (size_t)o.lastsolcol;
	cural_ = 0;
	best = o.best == std::numeric_limits<int32_t>::min() ? std::numeric_limits<TAlScore>::min() : (TAlScore)o.best;
	if(!o.aligned) return false;
	for(int32_t i = 0; i < o.ncand; i++) btncand_.push_back(DpBtCandidate(cands[i].row, cands[i].col, cands[i].score));
	return !btncand_.empty();
}

// nextAlignment(): walk the candidate list as aligner_sw.cpp:758-1140 does,
// with the engine's fate for each candidate: a score below `minsc` is
// FILT_SCORE (the caller may have tightened minsc, aligner_sw_driver.cpp:
// 1252-1290; candidates are sorted by score, so every later one is filtered
// too and the engine's marks for earlier ones are unchanged); FILT_START and
// FILT_DOMINATED consume no randomness; every tried candidate draws
// rnd.nextU32() and re-seeds rnd as the u8 / i16 branches do.
bool SwAlignerAcc::gpu_next(SwResult& res, TAlScore minsc, RandomSource& rnd, DpState& st) {
	if(done()) {
		res.reset();
		return false;
	}
	const size_t candsz = btncand_.size();
	while(cural_ < candsz) {
		DpBtCandidate& c = btncand_[cural_];
		if(c.score < minsc) {
			c.fate = BT_CAND_FATE_FILT_SCORE;
			nbtfiltsc_++;
			cural_++;
			continue;
		}
		const int f = st.fates[cural_];
		if(f == BT_CAND_FATE_FILT_START) { c.fate = f; nbtfiltst_++; cural_++; continue; }
		if(f == BT_CAND_FATE_FILT_DOMINATED) { c.fate = f; nbtfiltdo_++; cural_++; continue; }
		if(f != BT_CAND_FATE_SUCCEEDED && f != BT_CAND_FATE_FAILED) {
			fprintf(stderr, "bt2g adapter: candidate %zu of %zu has no engine fate (%d)\n", cural_, candsz, f);
			throw 1;
		}
		const uint32_t reseed = rnd.nextU32() + 1;
		res.reset();
		rnd.init(st.u8 ? reseed + 1 : reseed);
		c.fate = f;
		if(!sc_->monotone) {
			btncanddone_.push_back(c);
			if(f == BT_CAND_FATE_SUCCEEDED) btncanddoneSucc_++; else btncanddoneFail_++;
		}
		if(f == BT_CAND_FATE_FAILED) { cural_++; continue; }
		if(st.next >= (uint32_t)st.naln) {
			fprintf(stderr, "bt2g adapter: engine returned %d alignments, reference wants more\n", st.naln);
			throw 1;
		}
		const bt2g_sw_aln& a = st.alns[st.next];
		if(a.cand != (int32_t)cural_ || a.nedit > (int32_t)st.maxedit) {
			fprintf(stderr, "bt2g adapter: alignment %u is candidate %d, expected %zu\n", st.next, a.cand, cural_);
			throw 1;
		}
		const bt2g_edit* ed = &st.edits[(size_t)st.next * st.maxedit];
		st.next++;
		const size_t rdlen = rdf_ - rdi_;
		// backtraceNucleotides*: setScore / setShape / setRefNs (aligner_swsse_ee_u8.cpp:1822-1847)
		const int based = (int)(rdlen - (size_t)a.trim5p - (size_t)a.trim3p - (size_t)a.nedit);
		fill_alnres(res.alres, ed, (uint32_t)a.nedit, a.score, a.ns, a.gaps, based, refidx_,
		            (TRefOff)a.off + rfi_ + rect_->refl, reflen_, fw_, rdlen, (size_t)a.trim5p, (size_t)a.trim3p,
		            (size_t)a.refns);
		cural_++;
		return true;
	}
	return false;
}
