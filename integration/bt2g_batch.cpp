// integration/bt2g_batch.cpp -- the batch-first host driver: the reference's
// per-read search worker restated as resumable per-read state machines that
// a few driver threads advance in lockstep over whole-batch engine calls.
//
// The reference aligns one read at a time per worker thread
// (multiseedSearchWorker, bt2_search.cpp:3050-4197): exact sweep, the 1-mm
// search, each seed round, and between them SwDriver::extendSeeds
// (aligner_sw_driver.cpp:756-1297), which walks the seed hits in an RNG-driven
// order, resolves their reference offsets, frames and solves a DP per new
// diagonal and reports alignments, tightening the minimum score as it goes.
// Every engine seam is one round trip for one read.  Here each driver thread
// owns hundreds of reads in flight ("slots"); every slot runs the worker's
// decision logic until it needs an engine result, then parks with a request;
// once every runnable slot has parked, the thread issues ONE engine call per
// stage for all of them (exact sweep, 1-mm search, seed search, seed-hit
// extension, SA-row resolution, ungapped alignment, DP fill + backtrace) and
// resumes them.  Nothing the reference decides changes: each slot executes
// the reference's statements in the reference's order with its own RNG,
// SeedResults, AlignmentCache, SwDriver state and AlnSinkWrap, so the SAM
// records are the reference's.  The per-read pieces that do not wait on an
// engine run as the reference's own code (AlnSinkWrap::nextRead / report /
// finishRead with MAPQ and SAM, SeedResults / AlignmentCache bookkeeping,
// rankSeedHits, SwDriver::eeSaTups and prioritizeSATups with their RNG
// draws); what is restated are the two control loops that do wait:
//
//   Driver::step_read   multiseedSearchWorker's per-read body, unpaired
//                       (bt2_search.cpp:3266-4160)
//   SwDriverB::ext_step SwDriver::extendSeeds (aligner_sw_driver.cpp:756-1297)
//
// and the replay of SwAligner::nextAlignment's RNG draws from the engine's
// candidate fates (aligner_sw.cpp:737-1146).
//
// DP speculation: once a read's seed hits are prioritised and their rows
// resolved, the DPs its extension loop can ask for are known up to the loop's
// random visit order (one per new diagonal, framed at the current minimum
// score).  The first DP the loop needs goes to the engine together with up to
// BT2G_SPEC_DPS - 1 of the others; the loop then takes each DP from that
// table when the problem is the same.  A result computed at a lower minimum
// score serves a tightened one in end-to-end mode: the candidate list at
// minsc' >= minsc is the prefix of the list at minsc (gatherCells keeps
// last-row cells >= minsc, sorted by score, aligner_swsse_ee_u8.cpp:1176-1208),
// the walks of that prefix do not depend on later candidates, align()'s
// `best` does not depend on minsc, and the candidates past the prefix are
// FILT_SCORE in nextAlignment (aligner_sw.cpp:760-764), consuming no
// randomness -- provided both scores pick the same fill width (u8 iff
// minsc >= -254, aligner_sw.cpp:518).  Local mode reuses exact matches only.
//
// Hook: the worker threads bt2_search.cpp:4913-4925 spawns
// (std::thread(multiseedSearchWorker, &tps[i])) become driver threads
// (std::thread::_M_start_thread wrapped); -p N gives N drivers.  The options
// multiseedSearchWorker reads are file-static in bt2_search.cpp; the Makefile
// recipe (objcopy --globalize-symbol) makes those symbols visible.
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <pthread.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <limits>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <typeinfo>
#include <vector>

#include "aligner_cache.h"
#include "aligner_seed.h"
#include "aligner_sw.h"
#include "aligner_sw_driver.h"
#include "aln_sink.h"
#include "dp_framer.h"
#include "pat.h"
#include "read.h"
#include "scoring.h"
#include "simple_func.h"
#include "unique.h"
#include "bt2g.h"
#include "bt2g_gw_spec.h"
#include "bt2g_refspec.h"

// ---- the worker's options: file-static in bt2_search.cpp ------------------------
// (names and types as declared at bt2_search.cpp:89-264, 1861-1872; the Makefile
// globalizes exactly these symbols of bt2_search.o)
extern bool        R_localAlign          __asm__("_ZL10localAlign");
extern SimpleFunc  R_scoreMin            __asm__("_ZL8scoreMin");
extern SimpleFunc  R_nCeil               __asm__("_ZL5nCeil");
extern SimpleFunc  R_msIval              __asm__("_ZL6msIval");
extern size_t      R_maxDpStreak         __asm__("_ZL11maxDpStreak");
extern size_t      R_maxMateStreak       __asm__("_ZL13maxMateStreak");
extern size_t      R_maxDp               __asm__("_ZL5maxDp");
extern size_t      R_maxUg               __asm__("_ZL5maxUg");
extern size_t      R_maxIters            __asm__("_ZL8maxIters");
extern size_t      R_maxItersIncr        __asm__("_ZL12maxItersIncr");
extern size_t      R_maxStreakIncr       __asm__("_ZL13maxStreakIncr");
extern uint32_t    R_khits               __asm__("_ZL5khits");
extern uint32_t    R_mhits               __asm__("_ZL5mhits");
extern bool        R_msample             __asm__("_ZL7msample");
extern bool        R_allHits             __asm__("_ZL7allHits");
extern int         R_mapqv               __asm__("_ZL5mapqv");
extern bool        R_bwaSwLike           __asm__("_ZL9bwaSwLike");
extern float       R_bwaSwLikeC          __asm__("_ZL10bwaSwLikeC");
extern float       R_bwaSwLikeT          __asm__("_ZL10bwaSwLikeT");
extern size_t      R_nSeedRounds         __asm__("_ZL11nSeedRounds");
extern bool        R_doExactUpFront      __asm__("_ZL14doExactUpFront");
extern bool        R_do1mmUpFront        __asm__("_ZL12do1mmUpFront");
extern bool        R_seedSumm            __asm__("_ZL8seedSumm");
extern int         R_multiseedMms        __asm__("_ZL12multiseedMms");
extern int         R_multiseedLen        __asm__("_ZL12multiseedLen");
extern size_t      R_maxhalf             __asm__("_ZL7maxhalf");
extern bool        R_doUngapped          __asm__("_ZL10doUngapped");
extern bool        R_doExtend            __asm__("_ZL8doExtend");
extern bool        R_enable8             __asm__("_ZL7enable8");
extern size_t      R_cminlen             __asm__("_ZL7cminlen");
extern size_t      R_cpow2               __asm__("_ZL5cpow2");
extern bool        R_doTri               __asm__("_ZL5doTri");
extern int         R_tighten             __asm__("_ZL7tighten");
extern size_t      R_seedBoostThresh     __asm__("_ZL15seedBoostThresh");
extern bool        R_qcFilter            __asm__("_ZL8qcFilter");
extern bool        R_scUnMapped          __asm__("_ZL10scUnMapped");
extern bool        R_xeq                 __asm__("_ZL3xeq");
extern bool        R_sam_print_xt        __asm__("_ZL12sam_print_xt");
extern uint32_t    R_skipReads           __asm__("_ZL9skipReads");
extern uint64_t    R_qUpto               __asm__("_ZL5qUpto");
extern float       R_sampleFrac          __asm__("_ZL10sampleFrac");
extern bool        R_arbitraryRandom     __asm__("_ZL15arbitraryRandom");
extern bool        R_msNoCache           __asm__("_ZL9msNoCache");
extern uint32_t    R_seedCacheCurrentMB  __asm__("_ZL18seedCacheCurrentMB");
extern uint32_t    R_exactCacheCurrentMB __asm__("_ZL19exactCacheCurrentMB");
extern Ebwt*       R_ebwtFw              __asm__("_ZL16multiseed_ebwtFw");
extern Ebwt*       R_ebwtBw              __asm__("_ZL16multiseed_ebwtBw");
extern Scoring*    R_sc                  __asm__("_ZL12multiseed_sc");
extern BitPairReference* R_refs          __asm__("_ZL14multiseed_refs");
extern PatternSourceServiceFactory* R_factory __asm__("_ZL27multiseed_readahead_factory");
extern int         R_metricsIval         __asm__("_ZL11metricsIval");
extern bool        R_metricsPerRead      __asm__("_ZL14metricsPerRead");
extern bool        R_metricsStderr       __asm__("_ZL13metricsStderr");
extern OutFileBuf* R_metricsOfb          __asm__("_ZL20multiseed_metricsOfb");
extern std::string R_logDps              __asm__("_ZL6logDps");
extern std::string R_logDpsOpp           __asm__("_ZL9logDpsOpp");
extern bool gReportDiscordant;           // bt2_search.cpp:127-128 (global there)
extern bool gReportMixed;

namespace {

typedef PatternSourceServiceFactory::ReadElement ReadElement;

uint64_t now_us() {
	return (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
		std::chrono::steady_clock::now().time_since_epoch()).count();
}

size_t env_or(const char* name, size_t dflt) {
	const char* e = getenv(name);
	return e && atol(e) > 0 ? (size_t)atol(e) : dflt;
}

[[noreturn]] void die(const char* what, int rc) {
	fprintf(stderr, "bt2g batch: %s failed (%d): %s\n", what, rc, bt2g_last_error());
	fflush(stderr);
	abort();
}

// ---- process-wide state ------------------------------------------------------
std::mutex g_mu;
bt2g_ctx* g_base = nullptr;                 // index owner on the first device
std::vector<bt2g_ctx*> g_bases;             // one per device ($BT2G_DEVICES)
bool g_stub = false;

// counters ($BT2G_ADAPTER_STATS, written on SIGTERM and every 64 k reads)
enum { K_EXACT, K_1MM, K_SEEDS, K_EXT, K_OFF, K_UG, K_DP, K_N };
const char* const K_NAMES[K_N] = {"exact_sweep", "one_mm", "seed_search", "extend", "get_offset", "ungapped", "sw_dp"};
std::atomic<uint64_t> g_req[K_N], g_calls[K_N], g_call_us[K_N], g_cpu[K_N];
std::atomic<uint64_t> g_reads{0}, g_rounds{0}, g_round_us{0}, g_cpu_us{0}, g_gpu_us{0};
std::atomic<uint64_t> g_dp_spec{0}, g_dp_used{0}, g_dp_reuse{0}, g_dp_miss{0};
char g_stats_path[4096];

void write_stats() {
	if(!g_stats_path[0]) return;
	char buf[4096];
	int n = snprintf(buf, sizeof(buf), "{\"driver\": \"batch\", \"reads\": %llu, \"rounds\": %llu, \"round_ms\": %.1f, "
	                 "\"cpu_ms\": %.1f, \"gpu_ms\": %.1f, \"dp\": [%llu, %llu, %llu, %llu]",
	                 (unsigned long long)g_reads.load(), (unsigned long long)g_rounds.load(),
	                 g_round_us.load() / 1000.0, g_cpu_us.load() / 1000.0, g_gpu_us.load() / 1000.0,
	                 (unsigned long long)g_dp_spec.load(), (unsigned long long)g_dp_used.load(),
	                 (unsigned long long)g_dp_reuse.load(), (unsigned long long)g_dp_miss.load());
	for(int k = 0; k < K_N; k++)
		n += snprintf(buf + n, sizeof(buf) - n, ", \"%s\": [%llu, %llu, %llu, %.1f]", K_NAMES[k],
		              (unsigned long long)g_req[k].load(), (unsigned long long)g_cpu[k].load(),
		              (unsigned long long)g_calls[k].load(), g_call_us[k].load() / 1000.0);
	n += snprintf(buf + n, sizeof(buf) - n, "}\n");
	FILE* f = fopen(g_stats_path, "w");
	if(f) {
		fwrite(buf, 1, (size_t)n, f);
		fclose(f);
	}
}

void on_term(int) {
	write_stats();
	_exit(0);
}

// Environment of the engines, set before any thread starts (static
// initialiser): the runtime reads it at its first HIP call.
struct EnvInit {
	EnvInit() {
		setenv("BT2G_SYNC", "poll", 0);
		const char* hq = getenv("BT2G_HW_QUEUES");
		long q = hq ? atol(hq) : 16;
		if(q < 1) q = 1;
		if(q > 32) q = 32;                      // the runtime refuses more
		char b[16];
		snprintf(b, sizeof(b), "%ld", q);
		setenv("GPU_MAX_HW_QUEUES", b, 1);
		if(const char* sp = getenv("BT2G_ADAPTER_STATS")) {
			strncpy(g_stats_path, sp, sizeof(g_stats_path) - 1);
			signal(SIGTERM, on_term);
		}
	}
} g_env_init;

std::vector<int> devices() {
	std::vector<int> d;
	if(const char* e = getenv("BT2G_DEVICES")) {
		for(const char* p = e; *p;) {
			char* end = nullptr;
			long v = strtol(p, &end, 10);
			if(end == p) break;
			d.push_back((int)v);
			p = *end == ',' ? end + 1 : end;
		}
	}
	if(d.empty()) {
		const char* dev = getenv("BT2G_DEVICE");
		d.push_back(dev ? atoi(dev) : 0);
	}
	return d;
}

// The index replicas, opened once (the first driver thread), one per device.
void open_bases() {
	std::lock_guard<std::mutex> lk(g_mu);
	if(g_base) return;
	const char* base = getenv("BT2G_INDEX");
	if(!base) {
		fprintf(stderr, "bt2g batch: BT2G_INDEX is not set\n");
		abort();
	}
	const std::vector<int> devs = devices();
	g_bases.assign(devs.size(), nullptr);
	std::vector<int> rcs(devs.size(), 0);
	std::vector<std::thread> ld;
	for(size_t i = 0; i < devs.size(); i++)
		ld.emplace_back([&, i] { rcs[i] = bt2g_open(base, devs[i], &g_bases[i]); });
	for(std::thread& t : ld) t.join();
	for(size_t i = 0; i < devs.size(); i++)
		if(rcs[i]) die("bt2g_open", rcs[i]);
	g_base = g_bases[0];
}

// bt2g_scoring of a reference Scoring object (scoring.h:442-460); only the
// models the engines implement.
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

// AlnRes from an engine alignment: edits in their final (5'->3', post-trim)
// positions, shifted by the leading trim before setShape, which subtracts it
// (aligner_result.cpp:101-108).
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

// ---- per-read tables the reference's own SwDriver code fills ---------------
// SwDriver::extend results of the read being prioritised (bt2g_extend), and the
// ranges GroupWalk2S::init is handed by eeSaTups / prioritizeSATups (their rows
// are then resolved by bt2g_get_offset).  Set by the driver thread around the
// reference call; no engine wait happens inside it.
struct GwRange {
	TIndexOffU topf;
	size_t size;
	TSlice offs;
};
struct RefTables {
	bool ext_on = false;
	std::vector<bt2g_ext_in> ext_keys;
	std::vector<bt2g_ext_out> ext_vals;
	size_t ext_next = 0;
	bool gw_on = false;
	std::vector<GwRange> gw;
};
thread_local RefTables* t_tab = nullptr;
thread_local std::atomic<uint64_t>* t_cpu_ext = nullptr;

// One engine DP: SwAligner::initRead + initRef + align and every
// nextAlignment walk of it (bt2g_sw_align_bt), keyed by the problem.
struct DpRes {
	int32_t fw = 0;
	uint32_t refidx = 0;
	int64_t refl = 0;
	uint32_t ncol = 0;
	bt2g_sw_rect rect{};
	int32_t minsc = 0;
	TRefOff tlen = 0;
	bool ready = false, cpu = false;
	bt2g_sw_result o{};
	int32_t naln = 0;
	uint32_t maxedit = 0;
	std::vector<bt2g_sw_cand> cands;
	std::vector<int8_t> fates;
	std::vector<bt2g_sw_aln> alns;
	std::vector<bt2g_edit> edits;
	DPRect drect;          // for the CPU path (reads the engine does not take)
};

bool u8_regime(int64_t minsc) { return R_enable8 && minsc >= -254; }

struct Driver;
struct Slot;

// ---- SwDriver::extendSeeds as a resumable state machine -----------------------
// (aligner_sw_driver.cpp:756-1297, unpaired).  Members of the reference's
// SwDriver (satpos_, gws_, rands_, eehits_, seenDiags1_, redAnchor_, res*_)
// are used as the reference uses them; the loop's locals live here so that
// it can stop where it needs an engine result and resume there.
enum { EXTEND_BLOCKED = 0 };
enum { FOUND_NONE_ = 0, FOUND_EE_, FOUND_UNGAPPED_ };

struct SwDriverB : public SwDriver {
	explicit SwDriverB(size_t bytes) : SwDriver(bytes) {}

	// extendSeeds arguments (bt2_search.cpp:3559-3593 / 3741-3775 / 4017-4051)
	int seedmms = 0, seedlen = 0, seedival = 0;
	TAlScore* minsc = nullptr;
	int nceil = 0;
	size_t maxIters = 0, maxUg = 0, maxDp = 0, maxUgStreak = 0, maxDpStreak = 0;
	bool* exhaustive = nullptr;
	// loop state
	int pc = 0;
	bool all = false, eeMode = false, firstEe = false, firstExtend = false;
	size_t nonz = 0, nelt = 0, neltLeft = 0, rows = 0, eltsDone = 0, rdlen = 0;
	TAlScore perfectScore = 0;
	size_t i = 0, riter = 0;
	bool is_small = false, fw = false, first = false;
	uint32_t rdoff = 0, seedhitlen = 0;
	TIndexOffU tidx = 0, toff = 0, tlen = 0;
	int64_t refoff = 0;
	Coord refcoord;
	int readGaps = 0, refGaps = 0;
	bool ungapped = false;
	int state = FOUND_NONE_;
	bool found = false;
	DPRect rect;
	int ug_ret = 0;
	// the DP in replay (the reference's SwAligner after align())
	DpRes* dp = nullptr;
	size_t cural = 0;
	uint32_t dp_next = 0;
	size_t dp_next_edit = 0;
	bool firstInner = true;
	bool cpu_dp = false;       // replayed by the driver thread's own SwAligner

	int ext_step(Driver& d, Slot& s);
	bool replay_next(Driver& d, Slot& s, SwResult& res);
	bool need_dp(Driver& d, Slot& s, int& out);
	void speculate(Driver& d, Slot& s, std::vector<DpRes*>& out, size_t k);

	// protected reference members, for the driver
	EList<SATupleAndPos, 16>& sp() { return satpos_; }
};

// One read in flight.  Owns the reference's per-read objects a worker thread
// owns (bt2_search.cpp:3086-3176), reused read after read.
struct Elem {
	ReadElement re;
	int live = 0;
	explicit Elem(const ReadElement& r) : re(r) {}
};

enum {
	P_START = 0, P_AFTER_EXACT, P_AFTER_EXT_EXACT, P_1MM, P_AFTER_1MM, P_AFTER_EXT_1MM, P_ROUND, P_AFTER_SEEDS,
	P_ROUND_EXT, P_AFTER_EXT_SEEDS, P_FINISH
};

struct Slot {
	Slot(const ReportingParams& rp, Mapq& mapq, size_t tid)
		: scCurrent((uint64_t)R_seedCacheCurrentMB * 1024 * 1024, false),
		  ca(&scCurrent, NULL, NULL),
		  sd((size_t)R_exactCacheCurrentMB * 1024 * 1024),
		  msinkwrap(rp, mapq, tid) {}
	AlignmentCache scCurrent;
	AlignmentCacheIface ca;
	SwDriverB sd;
	SeedResults shs[2];
	AlnSinkWrap msinkwrap;
	RandomSource rnd;
	PerReadMetrics prm;
	EList<Seed> seeds;
	Constraint gc = Constraint::penaltyFuncBased(R_scoreMin);   // (a Seed points at it)
	EList<uint32_t> offIdx2off;
	RefTables tab;

	// the read
	Elem* el = nullptr;
	Read* rd = nullptr;
	Read* rdb = nullptr;     // the buffer's mate-2 slot (empty: unpaired)
	TReadId rdid = 0;
	AlnSink* msink = nullptr;

	// multiseedSearchWorker's per-read locals (bt2_search.cpp:3283-3451, 3814-3823)
	int pc = P_START;
	size_t rdlen = 0;
	TAlScore minsc = 0;
	bool nfilt[2] = {true, true}, scfilt[2] = {true, true}, lenfilt[2] = {true, true}, qcfilt[2] = {true, true};
	bool filt = true, nofw = false, norc = false, done = false, exhaustive[2] = {false, false};
	bool yfw = false, yrc = false;
	int nceil = 0, interval = 0;
	size_t streak = 0, mxDp = 0, mxUg = 0, mxIter = 0, nrounds = 0, nelt = 0;
	size_t minedfw = 0, minedrc = 0;
	int seedlen = 0;
	size_t roundi = 0, offset = 0;
	size_t seedsTried = 0, seedsTriedMS[4] = {0, 0, 0, 0};
	size_t nUniqueSeeds = 0, nRepeatSeeds = 0, seedHitTot = 0;
	size_t nUniqueSeedsMS[4] = {0, 0, 0, 0}, nRepeatSeedsMS[4] = {0, 0, 0, 0}, seedHitTotMS[4] = {0, 0, 0, 0};
	uint64_t valid_fw = 0, valid_rc = 0;   // seeds instantiated this round (instantiateSeeds, aligner_seed.cpp:556-580)
	std::vector<uint64_t> valid_big;       // (reads with more than 64 seed offsets per strand)

	// engine results
	uint32_t sweep[8] = {0};
	bool mm_asked = false;
	int32_t mm_minsc = 0;
	int mm_nofw = 0, mm_norc = 0;
	std::vector<bt2g_mm1> mm;
	int32_t mm_cnt = 0;
	uint32_t mm_ops = 0;
	// seed search (the round-0 one asked with the exact sweep: its arguments are
	// known when the read is set up)
	bool sd_ready = false;
	uint32_t sd_L = 0, sd_per = 0, sd_off = 0, sd_nof = 0;
	std::vector<uint32_t> sd_out;      // [strand][offset][topf, botf, topb, botb]
	int32_t sd_ns = 0;
	uint32_t sd_ops = 0;
	// pending requests of this slot's extension loop
	std::vector<bt2g_ext_in> ext_in;
	std::vector<bt2g_ext_out> ext_out;
	std::vector<uint32_t> off_rows, off_vals;
	std::vector<std::pair<size_t, size_t>> off_where;
	bt2g_ug_problem ug_p{};
	bt2g_ug_result ug_r{};
	std::vector<bt2g_edit> ug_ed;
	// the read's DP table (speculative and asked DPs)
	std::vector<std::unique_ptr<DpRes>> dps;
	size_t ndps = 0;
	DpRes* new_dp() {
		if(ndps == dps.size()) dps.emplace_back(new DpRes());
		DpRes* r = dps[ndps++].get();
		r->ready = r->cpu = false;
		r->naln = 0;
		return r;
	}
	// per-round row in the engine call's read pack
	uint64_t row_stamp = ~0ull;
	uint32_t row = 0;
};

// Reads packed as rows of one engine call.
struct Pack {
	std::vector<uint8_t> codes, quals;
	std::vector<uint32_t> lens;
	uint32_t stride = 0;
	void reset(uint32_t s) {
		stride = s;
		codes.clear();
		quals.clear();
		lens.clear();
	}
	uint32_t add(const Read& r) {
		const uint32_t L = (uint32_t)std::min<size_t>(r.length(), stride);
		const size_t o = codes.size();
		codes.resize(o + stride, 4);
		quals.resize(o + stride, 'I');
		for(uint32_t i = 0; i < L; i++) {
			codes[o + i] = (uint8_t)r.patFw[i];
			quals[o + i] = (uint8_t)r.qual[i];
		}
		lens.push_back(L);
		return (uint32_t)lens.size() - 1;
	}
	uint32_t n() const { return (uint32_t)lens.size(); }
};

// ---- one driver thread --------------------------------------------------------
struct Driver {
	explicit Driver(int tid_) : tid(tid_), swcpu(nullptr) {}
	int tid;
	bt2g_ctx* ctx = nullptr;
	const Scoring* sc = nullptr;
	bt2g_scoring bsc{};
	bool bsc_ok = false;
	const Ebwt* ebwtFw = nullptr;
	const Ebwt* ebwtBw = nullptr;
	const BitPairReference* ref = nullptr;
	std::unique_ptr<ReportingParams> rp;
	std::unique_ptr<Mapq> mapq;
	// per-thread reference objects (CPU paths; metrics)
	SeedAligner al;
	SwAligner swcpu;
	SeedSearchMetrics sdm;
	WalkMetrics wlm;
	SwMetrics swmSeed;
	ReportingMetrics rpm;
	// slots
	std::vector<std::unique_ptr<Slot>> all;
	std::vector<Slot*> freel, run, next;
	size_t active = 0;
	// reads in: a feeder thread pops the factory's ready queue for this driver
	std::mutex in_mu;
	std::condition_variable in_cv, room_cv;
	std::deque<Elem*> inbox;
	size_t held = 0, max_held = 64;
	// requests of this round
	std::vector<Slot*> rq[K_N];
	std::vector<std::pair<Slot*, DpRes*>> rq_dp;
	uint64_t stamp = 0;
	size_t spec_k = 16;

	void feeder();
	void run_loop();
	void admit(Elem* e);
	void release(Slot* s);
	void step_read(Slot& s);
	void setup_read(Slot& s);
	void gpu_phase();
	void prefetch_seeds(Slot& s);

	// engine calls of a round
	int call_exact();
	int call_1mm();
	int call_seeds();
	int call_ext();
	int call_off();
	int call_ug();
	int call_dp();
	int run_dp(const std::vector<std::pair<Slot*, DpRes*>>& v, uint32_t cap, uint32_t maxaln);
	void cpu_dp(Slot& s, DpRes& r);

	// helpers
	bool seeds_valid(const Slot& s, bool fw, size_t i) const;
	void set_valid(Slot& s, bool fw, size_t i);
	void resolve_rows_request(Slot& s);
	int after_seeds(Slot& s);
};

uint32_t row_of(Pack& pk, Slot& s, uint64_t stamp) {
	if(s.row_stamp != stamp) {
		s.row_stamp = stamp;
		s.row = pk.add(*s.rd);
	}
	return s.row;
}

// ---- the engine calls of one round ---------------------------------------------
int Driver::call_exact() {
	// grouped by (nofw, norc): batch-wide arguments of bt2g_exact_sweep
	std::vector<Slot*>& v = rq[K_EXACT];
	if(v.empty()) return 0;
	thread_local Pack pk;
	thread_local std::vector<uint32_t> out;
	for(int g = 0; g < 4; g++) {
		const bool nf = (g & 2) != 0, nr = (g & 1) != 0;
		std::vector<Slot*> sub;
		uint32_t stride = 1;
		for(Slot* s : v)
			if(s->nofw == nf && s->norc == nr) {
				sub.push_back(s);
				stride = std::max<uint32_t>(stride, (uint32_t)s->rdlen);
			}
		if(sub.empty()) continue;
		pk.reset(stride);
		for(Slot* s : sub) pk.add(*s->rd);
		out.resize(8 * sub.size());
		const uint64_t t0 = now_us();
		int rc = bt2g_exact_sweep(ctx, pk.codes.data(), pk.stride, pk.lens.data(), pk.n(), 2, nf ? 1 : 0, nr ? 1 : 0,
		                          out.data());
		g_call_us[K_EXACT] += now_us() - t0;
		g_calls[K_EXACT]++;
		if(rc) die("bt2g_exact_sweep", rc);
		for(size_t i = 0; i < sub.size(); i++) memcpy(sub[i]->sweep, &out[8 * i], sizeof(sub[i]->sweep));
	}
	g_req[K_EXACT] += v.size();
	return 0;
}

int Driver::call_1mm() {
	std::vector<Slot*>& v = rq[K_1MM];
	if(v.empty()) return 0;
	thread_local Pack pk;
	thread_local std::vector<int32_t> ms, cnt;
	thread_local std::vector<uint32_t> ops;
	thread_local std::vector<bt2g_mm1> h;
	for(int g = 0; g < 4; g++) {
		const int nf = (g >> 1) & 1, nr = g & 1;
		std::vector<Slot*> sub;
		uint32_t stride = 1;
		for(Slot* s : v)
			if(s->mm_nofw == nf && s->mm_norc == nr) {
				sub.push_back(s);
				stride = std::max<uint32_t>(stride, (uint32_t)s->rdlen);
			}
		if(sub.empty()) continue;
		uint32_t cap = 16;
		for(int pass = 0; pass < 2 && !sub.empty(); pass++) {
			pk.reset(stride);
			const size_t n = sub.size();
			ms.resize(n);
			cnt.resize(n);
			ops.resize(n);
			h.resize(n * (size_t)cap);
			for(size_t i = 0; i < n; i++) {
				pk.add(*sub[i]->rd);
				ms[i] = sub[i]->mm_minsc;
			}
			const uint64_t t0 = now_us();
			int rc = bt2g_one_mm(ctx, pk.codes.data(), pk.quals.data(), pk.stride, pk.lens.data(), (uint32_t)n, ms.data(),
			                     &bsc, nf, nr, cap, h.data(), cnt.data(), ops.data(), nullptr);
			g_call_us[K_1MM] += now_us() - t0;
			g_calls[K_1MM]++;
			if(rc && rc != BT2G_ERR_OVERFLOW) die("bt2g_one_mm", rc);
			std::vector<Slot*> again;
			uint32_t cap2 = cap;
			for(size_t i = 0; i < n; i++) {
				Slot* s = sub[i];
				if(cnt[i] > (int32_t)cap) {        // more hits than the slots: all of them, in order, next pass
					again.push_back(s);
					cap2 = std::max<uint32_t>(cap2, (uint32_t)cnt[i]);
					continue;
				}
				s->mm_cnt = cnt[i];
				s->mm_ops = ops[i];
				s->mm.assign(&h[i * cap], &h[i * cap] + cnt[i]);
			}
			sub.swap(again);
			cap = cap2;
		}
		if(!sub.empty()) die("bt2g_one_mm (rerun)", BT2G_ERR_OVERFLOW);
	}
	g_req[K_1MM] += v.size();
	return 0;
}

int Driver::call_seeds() {
	std::vector<Slot*>& v = rq[K_SEEDS];
	if(v.empty()) return 0;
	thread_local Pack pk;
	thread_local std::vector<uint32_t> out, ops;
	thread_local std::vector<int32_t> ns;
	std::vector<bool> taken(v.size(), false);
	for(size_t a = 0; a < v.size(); a++) {
		if(taken[a]) continue;
		Slot* s0 = v[a];
		std::vector<Slot*> sub;
		uint32_t stride = 1, maxs = 1;
		for(size_t b = a; b < v.size(); b++) {
			Slot* s = v[b];
			if(taken[b] || s->sd_L != s0->sd_L || s->sd_per != s0->sd_per || s->sd_off != s0->sd_off) continue;
			taken[b] = true;
			sub.push_back(s);
			stride = std::max<uint32_t>(stride, (uint32_t)s->rdlen);
			maxs = std::max(maxs, s->sd_nof);
		}
		pk.reset(stride);
		for(Slot* s : sub) pk.add(*s->rd);
		const size_t n = sub.size();
		out.resize(n * 2 * maxs * 4);
		ops.resize(n);
		ns.resize(n);
		const uint64_t t0 = now_us();
		int rc = bt2g_seed_search(ctx, pk.codes.data(), pk.stride, pk.lens.data(), (uint32_t)n, s0->sd_L, s0->sd_per,
		                          s0->sd_off, maxs, out.data(), ns.data(), ops.data(), nullptr);
		g_call_us[K_SEEDS] += now_us() - t0;
		g_calls[K_SEEDS]++;
		if(rc) die("bt2g_seed_search", rc);
		for(size_t i = 0; i < n; i++) {
			Slot* s = sub[i];
			s->sd_ns = ns[i];
			s->sd_ops = ops[i];
			s->sd_out.assign(2 * (size_t)s->sd_nof * 4, 0);
			for(int f = 0; f < 2; f++)
				for(uint32_t k = 0; k < s->sd_nof && k < maxs; k++)
					memcpy(&s->sd_out[((size_t)f * s->sd_nof + k) * 4], &out[((i * 2 + f) * maxs + k) * 4], 16);
			s->sd_ready = true;
		}
	}
	g_req[K_SEEDS] += v.size();
	return 0;
}

int Driver::call_ext() {
	std::vector<Slot*>& v = rq[K_EXT];
	if(v.empty()) return 0;
	thread_local Pack pk;
	thread_local std::vector<bt2g_ext_in> in;
	thread_local std::vector<bt2g_ext_out> out;
	uint32_t stride = 1;
	for(Slot* s : v) stride = std::max<uint32_t>(stride, (uint32_t)s->rdlen);
	pk.reset(stride);
	in.clear();
	for(Slot* s : v) {
		const uint32_t r = pk.add(*s->rd);
		for(const bt2g_ext_in& q : s->ext_in) {
			in.push_back(q);
			in.back().read = r;
		}
	}
	out.resize(in.size());
	const uint64_t t0 = now_us();
	int rc = bt2g_extend(ctx, pk.codes.data(), pk.stride, pk.lens.data(), pk.n(), in.data(), (uint32_t)in.size(),
	                     out.data());
	g_call_us[K_EXT] += now_us() - t0;
	g_calls[K_EXT]++;
	if(rc) die("bt2g_extend", rc);
	size_t k = 0;
	for(Slot* s : v) {
		s->ext_out.assign(out.begin() + k, out.begin() + k + s->ext_in.size());
		k += s->ext_in.size();
	}
	g_req[K_EXT] += v.size();
	return 0;
}

int Driver::call_off() {
	std::vector<Slot*>& v = rq[K_OFF];
	if(v.empty()) return 0;
	thread_local std::vector<uint32_t> rows, offs;
	rows.clear();
	for(Slot* s : v) rows.insert(rows.end(), s->off_rows.begin(), s->off_rows.end());
	offs.resize(rows.size());
	const uint64_t t0 = now_us();
	int rc = bt2g_get_offset(ctx, rows.data(), (uint32_t)rows.size(), offs.data(), nullptr);
	g_call_us[K_OFF] += now_us() - t0;
	g_calls[K_OFF]++;
	if(rc) die("bt2g_get_offset", rc);
	size_t k = 0;
	for(Slot* s : v) {
		// into the ranges' offset slots in the cache, where the reference's walks leave them
		for(size_t j = 0; j < s->off_rows.size(); j++) {
			const std::pair<size_t, size_t>& w = s->off_where[j];
			s->tab.gw[w.first].offs[w.second] = offs[k + j];
		}
		k += s->off_rows.size();
		s->tab.gw.clear();
	}
	g_req[K_OFF] += v.size();
	return 0;
}

int Driver::call_ug() {
	std::vector<Slot*>& v = rq[K_UG];
	if(v.empty()) return 0;
	thread_local Pack pk;
	thread_local std::vector<bt2g_ug_problem> P;
	thread_local std::vector<bt2g_ug_result> R;
	thread_local std::vector<bt2g_edit> E;
	uint32_t stride = 1;
	for(Slot* s : v) stride = std::max<uint32_t>(stride, (uint32_t)s->rdlen);
	pk.reset(stride);
	P.resize(v.size());
	for(size_t i = 0; i < v.size(); i++) {
		P[i] = v[i]->ug_p;
		P[i].read = pk.add(*v[i]->rd);
	}
	const uint32_t maxedit = stride + 1;
	R.resize(v.size());
	E.resize(v.size() * (size_t)maxedit);
	const uint64_t t0 = now_us();
	int rc = bt2g_ungapped(ctx, pk.codes.data(), pk.quals.data(), pk.stride, pk.lens.data(), P.data(), (uint32_t)v.size(),
	                       &bsc, gReportOverhangs ? 1 : 0, maxedit, R.data(), E.data());
	g_call_us[K_UG] += now_us() - t0;
	g_calls[K_UG]++;
	if(rc) die("bt2g_ungapped", rc);
	for(size_t i = 0; i < v.size(); i++) {
		v[i]->ug_r = R[i];
		const int32_t ne = R[i].ret == 1 ? std::min<int32_t>(std::max<int32_t>(R[i].nedit, 0), (int32_t)maxedit) : 0;
		v[i]->ug_ed.assign(&E[i * maxedit], &E[i * maxedit] + ne);
	}
	g_req[K_UG] += v.size();
	return 0;
}

// Fill + gather + the nextAlignment loop for every DP of the batch
// (bt2g_sw_align_bt_packed).  A DP whose candidate list outgrew `cap`, or that
// may have more than `maxaln` alignments, runs again alone with room for all;
// one with more candidates than the engine takes goes to the CPU when used.
int Driver::run_dp(const std::vector<std::pair<Slot*, DpRes*>>& v, uint32_t cap, uint32_t maxaln) {
	struct B {
		Pack pk;
		std::vector<bt2g_sw_problem> P;
		std::vector<bt2g_sw_rect> RC;
		std::vector<bt2g_sw_result> R;
		std::vector<int32_t> NA;
		std::vector<bt2g_sw_aln> A;
		std::vector<bt2g_sw_cand> C;
		std::vector<int8_t> F;
		std::vector<bt2g_edit> E;
	};
	thread_local B b;
	uint32_t stride = 1;
	for(auto& q : v) stride = std::max<uint32_t>(stride, (uint32_t)q.first->rdlen);
	b.pk.reset(stride);
	const uint64_t st = ++stamp;
	const size_t n = v.size();
	b.P.resize(n);
	b.RC.resize(n);
	for(size_t i = 0; i < n; i++) {
		const DpRes& r = *v[i].second;
		bt2g_sw_problem& p = b.P[i];
		memset(&p, 0, sizeof(p));
		p.read = row_of(b.pk, *v[i].first, st);
		p.fw = r.fw;
		p.refl = r.refl;
		p.win_off = -1;                 // the engine's HBM-resident reference (initRef's window)
		p.refidx = r.refidx;
		p.ncol = r.ncol;
		p.minsc = r.minsc;
		b.RC[i] = r.rect;
	}
	const uint32_t maxedit = 2 * stride + 8;
	b.R.resize(n);
	b.NA.resize(n);
	b.A.resize(n * (size_t)maxaln);
	if(b.C.size() < n * (size_t)cap) {
		b.C.resize(n * (size_t)cap);
		b.F.resize(n * (size_t)cap);
	}
	if(b.E.size() < n * (size_t)maxaln * maxedit) b.E.resize(n * (size_t)maxaln * maxedit);
	uint64_t tot[3] = {0, 0, 0};
	const uint64_t t0 = now_us();
	int rc = bt2g_sw_align_bt_packed(ctx, b.pk.codes.data(), b.pk.quals.data(), b.pk.stride, b.pk.lens.data(), b.P.data(),
	                                 (uint32_t)n, nullptr, 0, b.RC.data(), &bsc, R_enable8 ? 1 : 0, cap, b.R.data(),
	                                 maxaln, maxedit, b.NA.data(), b.A.data(), b.C.data(), b.F.data(), b.E.data(), tot);
	g_call_us[K_DP] += now_us() - t0;
	g_calls[K_DP]++;
	if(rc && rc != BT2G_ERR_OVERFLOW) die("bt2g_sw_align_bt_packed", rc);
	std::vector<std::pair<Slot*, DpRes*>> again;
	uint32_t cap2 = cap, maxaln2 = maxaln;
	size_t oc = 0, oe = 0;
	for(size_t i = 0; i < n; i++) {
		DpRes& r = *v[i].second;
		const bt2g_sw_result& o = b.R[i];
		const uint32_t nc = (uint32_t)std::min<int64_t>(std::max<int32_t>(o.ncand, 0), cap);
		const uint32_t na = (uint32_t)std::min<int64_t>(std::max<int32_t>(b.NA[i], 0), maxaln);
		uint32_t ne = 0;
		for(uint32_t k = 0; k < na; k++)
			ne += (uint32_t)std::min<int64_t>(std::max<int32_t>(b.A[i * maxaln + k].nedit, 0), maxedit);
		const size_t c0 = oc, e0 = oe;
		oc += nc;
		oe += ne;
		if(o.ncand > 8192) {            // beyond the engine's candidate capacity: the CPU, when used
			r.cpu = true;
			r.ready = true;
			continue;
		}
		if(o.ncand > (int32_t)cap || (b.NA[i] == (int32_t)maxaln && o.ncand > (int32_t)maxaln)) {
			again.push_back(v[i]);
			cap2 = std::max<uint32_t>(cap2, (uint32_t)o.ncand);
			maxaln2 = std::max<uint32_t>(maxaln2, (uint32_t)o.ncand);
			continue;
		}
		if(b.NA[i] < 0) die("bt2g_sw_align_bt_packed (status)", b.NA[i]);
		r.o = o;
		r.naln = b.NA[i];
		r.maxedit = maxedit;
		r.cands.assign(b.C.begin() + c0, b.C.begin() + c0 + nc);
		r.fates.assign(b.F.begin() + c0, b.F.begin() + c0 + nc);
		r.alns.assign(b.A.begin() + i * maxaln, b.A.begin() + i * maxaln + na);
		r.edits.assign(b.E.begin() + e0, b.E.begin() + e0 + ne);
		r.ready = true;
	}
	if(oc != tot[0] || oe != tot[2]) {
		fprintf(stderr, "bt2g batch: packed DP outputs %llu/%llu, expected %zu/%zu\n", (unsigned long long)tot[0],
		        (unsigned long long)tot[2], oc, oe);
		abort();
	}
	if(!again.empty()) return run_dp(again, cap2, maxaln2);
	return 0;
}

int Driver::call_dp() {
	if(rq_dp.empty()) return 0;
	g_req[K_DP] += rq_dp.size();
	// long reads (> 1024 bases) batch apart: a batch is padded to its longest read
	std::vector<std::pair<Slot*, DpRes*>> sh, lg;
	for(auto& q : rq_dp) (q.first->rdlen > 1024 ? lg : sh).push_back(q);
	const uint32_t cap = R_localAlign ? 2048 : 512;
	if(!sh.empty()) run_dp(sh, cap, 8);
	if(!lg.empty()) run_dp(lg, cap, 8);
	return 0;
}

// A DP the engine does not take (reads at or above --cp-min, longer than
// BT2G_MAX_READ_LEN, or more candidates than the engine holds): the
// reference's own SwAligner, when the extension loop reaches it
// (aligner_sw_driver.cpp:1104-1139).
void Driver::cpu_dp(Slot& s, DpRes& r) {
	const Read& rd = *s.rd;
	swcpu.reset();
	swcpu.initRead(rd.patFw, rd.patRc, rd.qual, rd.qualRev, 0, rd.length(), *sc);
	size_t nsInLeftShift = 0;
	swcpu.initRef(r.fw != 0, r.refidx, r.drect, const_cast<BitPairReference&>(*ref), r.tlen, *sc, r.minsc, R_enable8,
	              R_cminlen, R_cpow2, R_doTri, true, 0, nsInLeftShift);
	TAlScore best = std::numeric_limits<TAlScore>::min();
	r.o.aligned = swcpu.align(best) ? 1 : 0;
	r.o.best = best == std::numeric_limits<TAlScore>::min() ? std::numeric_limits<int32_t>::min() : (int32_t)best;
	g_cpu[K_DP]++;
}

// ---- the extension loop ----------------------------------------------------------
enum {
	X_START = 0, X_AFTER_EE_ROWS, X_AFTER_EXT, X_AFTER_PRIO_ROWS, X_AFTER_UG, X_AFTER_DP
};

// The DP the loop needs now (framed at the current minsc): from the read's
// table, or requested with up to spec_k - 1 speculative others.  Returns true
// when it is available (d.dp set), false when the slot must wait.
bool SwDriverB::need_dp(Driver& d, Slot& s, int& out) {
	(void)out;
	const int64_t ms = *minsc;
	const int32_t nc = (int32_t)(rect.refr + 1 - rect.refl);
	for(size_t k = 0; k < s.ndps; k++) {
		DpRes* r = s.dps[k].get();
		if(!r->ready || r->fw != (fw ? 1 : 0) || r->refidx != (uint32_t)tidx || r->refl != rect.refl ||
		   r->ncol != (uint32_t)nc || r->rect.triml != (int32_t)rect.triml || r->rect.corel != (int32_t)rect.corel ||
		   r->rect.corer != (int32_t)rect.corer)
			continue;
		bool ok = r->minsc == ms;
		if(!ok && !R_localAlign && r->minsc < ms && u8_regime(r->minsc) == u8_regime(ms)) ok = true;
		if(!ok) continue;
		dp = r;
		g_dp_used++;
		if(r->minsc != ms) g_dp_reuse++;
		return true;
	}
	g_dp_miss++;
	DpRes* r = s.new_dp();
	r->fw = fw ? 1 : 0;
	r->refidx = (uint32_t)tidx;
	r->refl = rect.refl;
	r->ncol = (uint32_t)nc;
	r->rect.triml = (int32_t)rect.triml;
	r->rect.corel = (int32_t)rect.corel;
	r->rect.corer = (int32_t)rect.corer;
	r->rect.pad = 0;
	r->minsc = (int32_t)ms;
	r->tlen = tlen;
	r->drect = rect;
	const bool engine = d.bsc_ok && rdlen > 0 && rdlen <= BT2G_MAX_READ_LEN && rdlen < R_cminlen &&
	                    ms >= std::numeric_limits<int32_t>::min() && ms <= std::numeric_limits<int32_t>::max();
	if(!engine) {
		r->cpu = true;
		r->ready = true;
		dp = r;
		return true;
	}
	std::vector<DpRes*> spec;
	if(d.spec_k > 1) speculate(d, s, spec, d.spec_k - 1);
	d.rq_dp.emplace_back(&s, r);
	for(DpRes* q : spec) d.rq_dp.emplace_back(&s, q);
	g_dp_spec += spec.size();
	dp = r;
	return false;
}

// Up to k more DPs this extension loop may ask for at the current minsc: one
// per element of the prioritised ranges whose row is resolved, on a diagonal
// not yet seen, framed exactly as the loop frames it
// (aligner_sw_driver.cpp:937-1097).
void SwDriverB::speculate(Driver& d, Slot& s, std::vector<DpRes*>& out, size_t k) {
	const int64_t ms = *minsc;
	if(eeMode) return;
	const int rg = d.sc->maxReadGaps(ms, rdlen), fg = d.sc->maxRefGaps(ms, rdlen);
	if(R_doUngapped && rg == 0 && fg == 0) return;
	DynProgFramer dpframe(!gReportOverhangs);
	struct Diag { uint32_t t; int64_t o; bool f; };
	std::vector<Diag> seen;
	for(size_t ii = 0; ii < gws_.size() && out.size() < k; ii++) {
		const SATupleAndPos& p = satpos_[ii];
		const bool f = p.pos.fw;
		uint32_t ro = p.pos.rdoff;
		if(!f) ro = (uint32_t)(rdlen - ro - p.pos.seedlen);
		for(size_t e = 0; e < p.sat.size() && out.size() < k; e++) {
			const TIndexOffU off = p.sat.offs[e];
			if(off == OFF_MASK) continue;
			TIndexOffU ti = 0, to = 0, tl = 0;
			bool straddled = false;
			d.ebwtFw->joinedToTextOff(p.sat.key.len, off, ti, to, tl, false, straddled);
			if(ti == OFF_MASK) continue;
			const int64_t ro64 = (int64_t)to - ro;
			Coord c(ti, ro64, f);
			if(seenDiags1_.locusPresent(c)) continue;
			bool dup = (ti == tidx && ro64 == refoff && f == fw);
			for(const Diag& x : seen) dup = dup || (x.t == ti && x.o == ro64 && x.f == f);
			if(dup) continue;
			seen.push_back(Diag{(uint32_t)ti, ro64, f});
			DPRect r;
			if(!dpframe.frameSeedExtensionRect(ro64, rdlen, tl, rg, fg, (size_t)nceil, R_maxhalf, r)) continue;
			const int32_t nc = (int32_t)(r.refr + 1 - r.refl);
			bool have = false;
			for(size_t q = 0; q < s.ndps && !have; q++) {
				const DpRes* x = s.dps[q].get();
				have = x->fw == (f ? 1 : 0) && x->refidx == (uint32_t)ti && x->refl == r.refl && x->ncol == (uint32_t)nc &&
				       x->rect.triml == (int32_t)r.triml && x->rect.corel == (int32_t)r.corel &&
				       x->rect.corer == (int32_t)r.corer && x->minsc == (int32_t)ms;
			}
			if(have) continue;
			DpRes* q = s.new_dp();
			q->fw = f ? 1 : 0;
			q->refidx = (uint32_t)ti;
			q->refl = r.refl;
			q->ncol = (uint32_t)nc;
			q->rect.triml = (int32_t)r.triml;
			q->rect.corel = (int32_t)r.corel;
			q->rect.corer = (int32_t)r.corer;
			q->rect.pad = 0;
			q->minsc = (int32_t)ms;
			q->tlen = tl;
			q->drect = r;
			out.push_back(q);
		}
	}
}

// nextAlignment(): the candidate list walked as aligner_sw.cpp:758-1140 walks
// it, with the engine's fate for each candidate: below `minsc` FILT_SCORE
// (the caller may have tightened it since align()); FILT_START and
// FILT_DOMINATED consume no randomness; every tried candidate draws
// rnd.nextU32() and re-seeds rnd as the u8 / i16 branches do.
bool SwDriverB::replay_next(Driver& d, Slot& s, SwResult& res) {
	if(cpu_dp) return d.swcpu.nextAlignment(res, *minsc, s.rnd);
	DpRes& r = *dp;
	const size_t candsz = r.cands.size();
	const bool u8 = r.o.u8succ != 0;
	while(cural < candsz) {
		const bt2g_sw_cand& c = r.cands[cural];
		if(c.score < *minsc) {
			cural++;
			continue;
		}
		const int f = r.fates[cural];
		if(f == BT_CAND_FATE_FILT_START || f == BT_CAND_FATE_FILT_DOMINATED) {
			cural++;
			continue;
		}
		if(f != BT_CAND_FATE_SUCCEEDED && f != BT_CAND_FATE_FAILED) {
			fprintf(stderr, "bt2g batch: candidate %zu of %zu has no engine fate (%d)\n", cural, candsz, f);
			abort();
		}
		const uint32_t reseed = s.rnd.nextU32() + 1;
		res.reset();
		s.rnd.init(u8 ? reseed + 1 : reseed);
		if(f == BT_CAND_FATE_FAILED) {
			cural++;
			continue;
		}
		if(dp_next >= (uint32_t)r.naln) {
			fprintf(stderr, "bt2g batch: engine returned %d alignments, reference wants more\n", r.naln);
			abort();
		}
		const bt2g_sw_aln& a = r.alns[dp_next];
		if(a.cand != (int32_t)cural || a.nedit > (int32_t)r.maxedit) {
			fprintf(stderr, "bt2g batch: alignment %u is candidate %d, expected %zu\n", dp_next, a.cand, cural);
			abort();
		}
		const bt2g_edit* ed = r.edits.data() + dp_next_edit;
		dp_next_edit += (size_t)a.nedit;
		dp_next++;
		// backtraceNucleotides*: setScore / setShape / setRefNs (aligner_swsse_ee_u8.cpp:1822-1847)
		const int based = (int)(rdlen - (size_t)a.trim5p - (size_t)a.trim3p - (size_t)a.nedit);
		fill_alnres(res.alres, ed, (uint32_t)a.nedit, a.score, a.ns, a.gaps, based, (TRefId)r.refidx,
		            (TRefOff)a.off + r.refl, (TRefOff)r.tlen, r.fw != 0, rdlen, (size_t)a.trim5p, (size_t)a.trim3p,
		            (size_t)a.refns);
		cural++;
		return true;
	}
	res.reset();
	return false;
}

// The read's rows handed to GroupWalk2S::init by the call that just returned,
// as one engine request (bt2g_get_offset == Ebwt::getOffset, bt2_idx.cpp:150-171).
void Driver::resolve_rows_request(Slot& s) {
	const size_t MAX_ROWS = 8192;          // per read (the rest: Ebwt::getOffset in advanceElement)
	s.off_rows.clear();
	s.off_where.clear();
	for(size_t r = 0; r < s.tab.gw.size(); r++) {
		GwRange& x = s.tab.gw[r];
		for(size_t j = 0; j < x.size && s.off_rows.size() < MAX_ROWS; j++)
			if(x.offs[j] == OFF_MASK) {
				s.off_rows.push_back((uint32_t)(x.topf + j));
				s.off_where.emplace_back(r, j);
			}
	}
	if(s.off_rows.empty()) {
		s.tab.gw.clear();
		return;
	}
	rq[K_OFF].push_back(&s);
}

int SwDriverB::ext_step(Driver& d, Slot& s) {
	AlnSinkWrap* msink = &s.msinkwrap;
	const Read& rd = *s.rd;
	const Scoring& sc = *d.sc;
	const Ebwt& ebwtFw = *d.ebwtFw;
	const BitPairReference& ref = *d.ref;
	switch(pc) {
	case X_START: break;
	case X_AFTER_EE_ROWS: goto after_ee_rows;
	case X_AFTER_EXT: goto after_ext;
	case X_AFTER_PRIO_ROWS: goto after_prio_rows;
	case X_AFTER_UG: goto after_ug;
	case X_AFTER_DP: goto after_dp;
	default: abort();
	}
	// aligner_sw_driver.cpp:792-823
	all = msink->allHits();
	rdlen = rd.length();
	perfectScore = sc.perfectScore(rdlen);
	nonz = s.shs[0].nonzeroOffsets();
	eeMode = s.shs[0].numE2eHits() > 0;
	firstEe = true;
	firstExtend = true;
	s.prm.nEeFail = 0;
	s.prm.nUgFail = 0;
	s.prm.nDpFail = 0;
	nelt = 0;
	neltLeft = 0;
	rows = rdlen;
	eltsDone = 0;
	s.ndps = 0;
	while(true) {
		if(eeMode) {
			if(firstEe) {
				firstEe = false;
				s.tab.gw.clear();
				s.tab.gw_on = true;
				t_tab = &s.tab;
				eeMode = eeSaTups(rd, s.shs[0], ebwtFw, ref, s.rnd, d.wlm, d.swmSeed, nelt, maxIters, all);
				s.tab.gw_on = false;
				t_tab = nullptr;
				d.resolve_rows_request(s);
				if(!s.off_rows.empty()) {
					pc = X_AFTER_EE_ROWS;
					return EXTEND_BLOCKED;
				}
			after_ee_rows:;
			} else {
				eeMode = false;
			}
		}
		if(!eeMode) {
			if(nonz == 0) return EXTEND_EXHAUSTED_CANDIDATES;
			if(*minsc == perfectScore) return EXTEND_PERFECT_SCORE;
			if(firstExtend) {
				nelt = 0;
				// every range the loop at aligner_sw_driver.cpp:519-604 visits, in its
				// order, extended on the engine first (SwDriver::extend reads them)
				s.ext_in.clear();
				if(R_doExtend && d.ebwtBw != NULL && rdlen > 0 && rdlen <= BT2G_MAX_READ_LEN) {
					EList<SATuple, 16>& sat = satups_;
					for(size_t k = 0; k < nonz; k++) {
						bool f = true;
						uint32_t offidx = 0, ro = 0, sl = 0;
						QVal qv = s.shs[0].hitsByRank(k, offidx, ro, f, sl);
						size_t nr = 0, ne = 0;
						sat.clear();
						s.ca.queryQval(qv, sat, nr, ne);
						for(size_t j = 0; j < sat.size(); j++) {
							const TIndexOffU sz = (TIndexOffU)sat[j].size();
							bt2g_ext_in x;
							x.read = 0;
							x.fw = f ? 1 : 0;
							x.off = ro;
							x.len = sl;
							x.topf = sat[j].topf;
							x.botf = sat[j].topf + sz;
							x.topb = sat[j].topb;
							x.botb = sat[j].topb + sz;
							if(sz > 0 && ro + sl <= rdlen) s.ext_in.push_back(x);
						}
					}
					sat.clear();
				}
				if(!s.ext_in.empty()) {
					d.rq[K_EXT].push_back(&s);
					pc = X_AFTER_EXT;
					return EXTEND_BLOCKED;
				}
				s.ext_out.clear();
			after_ext:
				s.tab.ext_on = !s.ext_in.empty();
				s.tab.ext_keys.swap(s.ext_in);
				s.tab.ext_vals.swap(s.ext_out);
				s.tab.ext_next = 0;
				s.tab.gw.clear();
				s.tab.gw_on = true;
				t_tab = &s.tab;
				t_cpu_ext = &g_cpu[K_EXT];
				prioritizeSATups(rd, s.shs[0], ebwtFw, d.ebwtBw, ref, seedmms, maxIters, R_doExtend, true, true, 5, s.ca,
				                 s.rnd, d.wlm, s.prm, nelt, all);
				s.tab.ext_on = false;
				s.tab.gw_on = false;
				t_tab = nullptr;
				d.resolve_rows_request(s);
				if(!s.off_rows.empty()) {
					pc = X_AFTER_PRIO_ROWS;
					return EXTEND_BLOCKED;
				}
			after_prio_rows:
				neltLeft = nelt;
				firstExtend = false;
			}
			if(neltLeft == 0) break;    // finished examining gapped candidates
		}
		for(i = 0; i < gws_.size(); i++) {
			if(eeMode && eehits_[i].score < *minsc) return EXTEND_PERFECT_SCORE;
			is_small = satpos_[i].sat.size() < 5;
			fw = satpos_[i].pos.fw;
			rdoff = satpos_[i].pos.rdoff;
			seedhitlen = satpos_[i].pos.seedlen;
			if(!fw) rdoff = (uint32_t)(rdlen - rdoff - seedhitlen);
			first = true;
			riter = 0;
			while(!rands_[i].done() && (first || is_small || eeMode)) {
				riter++;
				if(*minsc == perfectScore) {
					if(!eeMode || eehits_[i].score < perfectScore) return EXTEND_PERFECT_SCORE;
				} else if(eeMode && eehits_[i].score < *minsc) {
					break;
				}
				if(s.prm.nExDps >= maxDp || s.prm.nMateDps >= maxDp) return EXTEND_EXCEEDED_HARD_LIMIT;
				if(s.prm.nExUgs >= maxUg || s.prm.nMateUgs >= maxUg) return EXTEND_EXCEEDED_HARD_LIMIT;
				if(s.prm.nExIters >= maxIters) return EXTEND_EXCEEDED_HARD_LIMIT;
				s.prm.nExIters++;
				first = false;
				{
					// resolve the next element's offset (aligner_sw_driver.cpp:924-952)
					WalkResult wr;
					const size_t elt = rands_[i].next(s.rnd);
					SARangeWithOffs<TSlice> sa;
					sa.topf = satpos_[i].sat.topf;
					sa.len = satpos_[i].sat.key.len;
					sa.offs = satpos_[i].sat.offs;
					gws_[i].advanceElement((TIndexOffU)elt, ebwtFw, ref, sa, gwstate_, wr, d.wlm, s.prm);
					eltsDone++;
					if(!eeMode) neltLeft--;
					tidx = 0;
					toff = 0;
					tlen = 0;
					bool straddled = false;
					ebwtFw.joinedToTextOff(wr.elt.len, wr.toff, tidx, toff, tlen, eeMode, straddled);
				}
				if(tidx == OFF_MASK) continue;   // the seed hit straddled a reference boundary
				refoff = (int64_t)toff - rdoff;
				refcoord.init(tidx, refoff, fw);
				if(seenDiags1_.locusPresent(refcoord)) {
					s.prm.nRedundants++;
					d.swmSeed.rshit++;
					continue;
				}
				readGaps = 0;
				refGaps = 0;
				ungapped = false;
				if(!eeMode) {
					readGaps = sc.maxReadGaps(*minsc, rdlen);
					refGaps = sc.maxRefGaps(*minsc, rdlen);
					ungapped = (readGaps == 0 && refGaps == 0);
				}
				state = FOUND_NONE_;
				found = false;
				if(eeMode) {
					resEe_.reset();
					resEe_.alres.reset();
					const EEHit& h = eehits_[i];
					resEe_.alres.setScore(AlnScore(h.score, (int)(rdlen - h.mms()), h.mms(), h.ns(), 0));
					resEe_.alres.setShape(refcoord.ref(), refcoord.off(), tlen, fw, rdlen, true, 0, 0, true, 0, 0);
					resEe_.alres.setRefNs(h.refns());
					if(h.mms() > 0) resEe_.alres.ned().push_back(h.e1);
					state = FOUND_EE_;
					found = true;
					Interval refival(refcoord, 1);
					seenDiags1_.add(refival);
				} else if(R_doUngapped && ungapped) {
					resUngap_.reset();
					if(d.bsc_ok && rdlen > 0 && rdlen <= BT2G_MAX_READ_LEN) {
						memset(&s.ug_p, 0, sizeof(s.ug_p));
						s.ug_p.fw = fw ? 1 : 0;
						s.ug_p.off = refcoord.off();
						s.ug_p.refidx = (uint32_t)refcoord.ref();
						s.ug_p.minsc = (int32_t)*minsc;
						d.rq[K_UG].push_back(&s);
						pc = X_AFTER_UG;
						return EXTEND_BLOCKED;
					after_ug:
						resUngap_.alres.reset();
						ug_ret = s.ug_r.ret;
						if(s.ug_r.ret == 1)
							fill_alnres(resUngap_.alres, s.ug_ed.data(), (uint32_t)s.ug_r.nedit, s.ug_r.score, s.ug_r.ns, 0,
							            (int)(rdlen - (size_t)s.ug_r.nedit), refcoord.ref(), s.ug_r.refoff, (TRefOff)tlen,
							            fw, rdlen, (size_t)s.ug_r.trim5p, (size_t)s.ug_r.trim3p, (size_t)s.ug_r.refns);
					} else {
						d.swcpu.reset();
						ug_ret = d.swcpu.ungappedAlign(fw ? rd.patFw : rd.patRc, fw ? rd.qual : rd.qualRev, refcoord, ref, tlen,
						                               sc, gReportOverhangs, *minsc, resUngap_);
						g_cpu[K_UG]++;
					}
					Interval refival(refcoord, 1);
					seenDiags1_.add(refival);
					s.prm.nExUgs++;
					if(ug_ret == 0) {
						s.prm.nExUgFails++;
						s.prm.nUgFail++;
						if(s.prm.nUgFail >= maxUgStreak) return EXTEND_EXCEEDED_SOFT_LIMIT;
						d.swmSeed.ungapfail++;
						continue;
					} else if(ug_ret == -1) {
						s.prm.nExUgFails++;
						s.prm.nUgFail++;
						if(s.prm.nUgFail >= maxUgStreak) return EXTEND_EXCEEDED_SOFT_LIMIT;
						d.swmSeed.ungapnodec++;
					} else {
						s.prm.nExUgSuccs++;
						s.prm.nUgLastSucc = s.prm.nExUgs - 1;
						if(s.prm.nUgFail > s.prm.nUgFailStreak) s.prm.nUgFailStreak = s.prm.nUgFail;
						s.prm.nUgFail = 0;
						found = true;
						state = FOUND_UNGAPPED_;
						d.swmSeed.ungapsucc++;
					}
				}
				if(state == FOUND_NONE_) {
					DynProgFramer dpframe(!gReportOverhangs);
					found = dpframe.frameSeedExtensionRect(refoff, rows, tlen, readGaps, refGaps, (size_t)nceil, R_maxhalf,
					                                       rect);
					seenDiags1_.add(Interval(refcoord, 1));
					if(!found) continue;
				}
				if(state == FOUND_NONE_) {
					{
						Interval refival(tidx, 0, fw, 0);
						rect.initIval(refival);
						seenDiags1_.add(refival);
					}
					{
						int unused = 0;
						if(!need_dp(d, s, unused)) {
							pc = X_AFTER_DP;
							return EXTEND_BLOCKED;
						}
					}
				after_dp:
					// SwAligner::align's outcome (aligner_sw.cpp:677-729) at this minsc
					cpu_dp = dp->cpu;
					cural = 0;
					dp_next = 0;
					dp_next_edit = 0;
					if(cpu_dp) {
						dp->minsc = (int32_t)*minsc;
						d.cpu_dp(s, *dp);
						found = dp->o.aligned != 0;
					} else {
						found = false;
						if(dp->o.aligned)
							for(const bt2g_sw_cand& c : dp->cands)
								if(c.score >= *minsc) {
									found = true;
									break;
								}
					}
					d.swmSeed.tallyGappedDp(readGaps, refGaps);
					s.prm.nExDps++;
					if(!found) {
						s.prm.nExDpFails++;
						s.prm.nDpFail++;
						if(s.prm.nDpFail >= maxDpStreak) return EXTEND_EXCEEDED_SOFT_LIMIT;
						const TAlScore bestCell = dp->o.best == std::numeric_limits<int32_t>::min()
						                              ? std::numeric_limits<TAlScore>::min()
						                              : (TAlScore)dp->o.best;
						if(bestCell > std::numeric_limits<TAlScore>::min() && bestCell > s.prm.bestLtMinscMate1)
							s.prm.bestLtMinscMate1 = bestCell;
						continue;     // look for more anchor alignments
					} else {
						s.prm.nExDpSuccs++;
						s.prm.nDpLastSucc = s.prm.nExDps - 1;
						if(s.prm.nDpFail > s.prm.nDpFailStreak) s.prm.nDpFailStreak = s.prm.nDpFail;
						s.prm.nDpFail = 0;
					}
				}
				// aligner_sw_driver.cpp:1161-1287
				firstInner = true;
				while(true) {
					SwResult* res = NULL;
					if(state == FOUND_EE_) {
						if(!firstInner) break;
						res = &resEe_;
					} else if(state == FOUND_UNGAPPED_) {
						if(!firstInner) break;
						res = &resUngap_;
					} else {
						resGap_.reset();
						if(cpu_dp ? d.swcpu.done() : cural == dp->cands.size()) break;
						replay_next(d, s, resGap_);
						found = !resGap_.empty();
						if(!found) break;
						res = &resGap_;
					}
					firstInner = false;
					Interval refival(tidx, 0, fw, tlen);
					if(gReportOverhangs && !refival.containsIgnoreOrient(res->alres.refival())) {
						res->alres.clipOutside(true, 0, tlen);
						if(res->alres.refExtent() == 0) continue;
					}
					if(!refival.overlapsIgnoreOrient(res->alres.refival())) continue;
					if(redAnchor_.overlap(res->alres)) continue;
					redAnchor_.add(res->alres);
					res->alres.setParams(seedmms, seedlen, seedival, *minsc);
					if(msink->report(0, &res->alres, NULL)) return EXTEND_POLICY_FULFILLED;
					if(R_tighten > 0 && msink->Mmode() && msink->hasSecondBestUnp1()) {
						TAlScore& m = *minsc;
						if(R_tighten == 1) {
							if(msink->bestUnp1() >= m) {
								m = msink->bestUnp1();
								if(m < perfectScore && msink->bestUnp1() == msink->secondBestUnp1()) m++;
							}
						} else if(R_tighten == 2) {
							if(msink->secondBestUnp1() >= m) {
								m = msink->secondBestUnp1();
								if(m < perfectScore) m++;
							}
						} else {
							TAlScore diff = msink->bestUnp1() - msink->secondBestUnp1();
							TAlScore bot = msink->secondBestUnp1() + ((diff * 3) / 4);
							if(bot >= m) {
								m = bot;
								if(m < perfectScore) m++;
							}
						}
					}
				}
			}
		}
	}
	return EXTEND_EXHAUSTED_CANDIDATES;
}

}  // namespace

// ---- the reference's SwDriver / GroupWalk2S pieces, served from the tables ------
extern "C" {
void bt2g_real__ZN8SwDriver6extendERK4ReadRK4EbwtPS4_jjjjbmmR14PerReadMetricsRmS9_(
	SwDriver*, const Read&, const Ebwt&, const Ebwt*, TIndexOffU, TIndexOffU, TIndexOffU, TIndexOffU, bool, size_t,
	size_t, PerReadMetrics&, size_t&, size_t&);
void bt2g_real__ZN8SwDriver16prioritizeSATupsERK4ReadR11SeedResultsRK4EbwtPS6_RK16BitPairReferenceimbbbmR19AlignmentCacheIfaceR12RandomSourceR11WalkMetricsR14PerReadMetricsRmb(
	SwDriver*, const Read&, SeedResults&, const Ebwt&, const Ebwt*, const BitPairReference&, int, size_t, bool, bool, bool,
	size_t, AlignmentCacheIface&, RandomSource&, WalkMetrics&, PerReadMetrics&, size_t&, bool);
bool bt2g_real__ZN8SwDriver8eeSaTupsERK4ReadR11SeedResultsRK4EbwtRK16BitPairReferenceR12RandomSourceR11WalkMetricsR9SwMetricsRmmb(
	SwDriver*, const Read&, SeedResults&, const Ebwt&, const BitPairReference&, RandomSource&, WalkMetrics&, SwMetrics&,
	size_t&, size_t, bool);
}

void SwDriver::prioritizeSATups(const Read& read, SeedResults& sh, const Ebwt& ebwtFw, const Ebwt* ebwtBw,
                                const BitPairReference& ref, int seedmms, size_t maxelt, bool doExtend, bool lensq,
                                bool szsq, size_t nsm, AlignmentCacheIface& ca, RandomSource& rnd, WalkMetrics& wlm,
                                PerReadMetrics& prm, size_t& nelt_out, bool all) {
	bt2g_real__ZN8SwDriver16prioritizeSATupsERK4ReadR11SeedResultsRK4EbwtPS6_RK16BitPairReferenceimbbbmR19AlignmentCacheIfaceR12RandomSourceR11WalkMetricsR14PerReadMetricsRmb(
		this, read, sh, ebwtFw, ebwtBw, ref, seedmms, maxelt, doExtend, lensq, szsq, nsm, ca, rnd, wlm, prm, nelt_out, all);
}

bool SwDriver::eeSaTups(const Read& rd, SeedResults& sh, const Ebwt& ebwt, const BitPairReference& ref,
                        RandomSource& rnd, WalkMetrics& wlm, SwMetrics& swmSeed, size_t& nelt_out, size_t maxelt,
                        bool all) {
	return bt2g_real__ZN8SwDriver8eeSaTupsERK4ReadR11SeedResultsRK4EbwtRK16BitPairReferenceR12RandomSourceR11WalkMetricsR9SwMetricsRmmb(
		this, rd, sh, ebwt, ref, rnd, wlm, swmSeed, nelt_out, maxelt, all);
}

// SwDriver::extend (aligner_sw_driver.cpp:299-483) from the engine's results for
// this read (asked in the same order prioritizeSATups calls it), else the CPU.
void SwDriver::extend(const Read& rd, const Ebwt& ebwtFw, const Ebwt* ebwtBw, TIndexOffU topf, TIndexOffU botf,
                      TIndexOffU topb, TIndexOffU botb, bool fw, size_t off, size_t len, PerReadMetrics& prm,
                      size_t& nlex, size_t& nrex) {
	RefTables* t = t_tab;
	if(t && t->ext_on) {
		const std::vector<bt2g_ext_in>& K = t->ext_keys;
		const size_t n = K.size();
		for(size_t c = 0; c < n; c++) {
			const size_t i = (t->ext_next + c) % n;
			const bt2g_ext_in& k = K[i];
			if(k.topf == topf && k.botf == botf && k.topb == topb && k.botb == botb && (k.fw != 0) == fw && k.off == off &&
			   k.len == len) {
				nlex += t->ext_vals[i].nlex;
				nrex += t->ext_vals[i].nrex;
				prm.nSdFmops += t->ext_vals[i].fmops;
				t->ext_next = i + 1;
				return;
			}
		}
	}
	if(t_cpu_ext) (*t_cpu_ext)++;
	bt2g_real__ZN8SwDriver6extendERK4ReadRK4EbwtPS4_jjjjbmmR14PerReadMetricsRmS9_(
		this, rd, ebwtFw, ebwtBw, topf, botf, topb, botb, fw, off, len, prm, nlex, nrex);
}

template <>
void GroupWalk2S<TSlice, 16>::init(const Ebwt& ebwtFw, const BitPairReference& ref, SARangeWithOffs<TSlice>& sa,
                                   RandomSource& rnd, WalkMetrics& met) {
	(void)ebwtFw; (void)ref; (void)rnd; (void)met;
	reset();
	elt_ += sa.size();
	// the range's offset slots as the cache would hold them before any walk
	// (AlignmentCache::addOnTheFlyImpl only reserves them, bt2g_refspec.h)
	static_cast<bt2gref::TSliceAcc&>(sa.offs).fill(OFF_MASK);
	if(t_tab && t_tab->gw_on) t_tab->gw.push_back(GwRange{sa.topf, sa.size(), sa.offs});
}

template <>
bool GroupWalk2S<TSlice, 16>::advanceElement(TIndexOffU elt, const Ebwt& ebwtFw, const BitPairReference& ref,
                                             SARangeWithOffs<TSlice>& sa, GroupWalkState& gws, WalkResult& res,
                                             WalkMetrics& met, PerReadMetrics& prm) {
	(void)ref; (void)gws; (void)prm;
	if(sa.offs[elt] == OFF_MASK) {       // not batched: the reference's getOffset on the CPU
		sa.offs[elt] = ebwtFw.getOffset(sa.topf + elt);
		g_cpu[K_OFF]++;
	}
	met.reports++;
	res.init(0, false, 0, elt, sa.topf + elt, (TIndexOffU)sa.len, sa.offs[elt]);
	rep_++;
	return true;
}

namespace {

// ---- multiseedSearchWorker's per-read body (bt2_search.cpp:3266-4160), unpaired
bool Driver::seeds_valid(const Slot& s, bool fw, size_t i) const {
	if(i < 64) return ((fw ? s.valid_fw : s.valid_rc) >> i) & 1;
	const size_t k = (i - 64) * 2 + (fw ? 0 : 1);
	return k / 64 < s.valid_big.size() && ((s.valid_big[k / 64] >> (k % 64)) & 1);
}

void Driver::set_valid(Slot& s, bool fw, size_t i) {
	if(i < 64) {
		(fw ? s.valid_fw : s.valid_rc) |= 1ull << i;
		return;
	}
	const size_t k = (i - 64) * 2 + (fw ? 0 : 1);
	if(s.valid_big.size() <= k / 64) s.valid_big.resize(k / 64 + 1, 0);
	s.valid_big[k / 64] |= 1ull << (k % 64);
}

// Per-read setup (bt2_search.cpp:3266-3451).
void Driver::setup_read(Slot& s) {
	s.prm.reset();
	s.prm.doFmString = false;
	if(R_sam_print_xt) gettimeofday(&s.prm.tv_beg, &s.prm.tz_beg);
	s.ca.nextRead();
	const Read& rd = *s.rd;
	s.rdlen = rd.length();
	s.msinkwrap.nextRead(s.msink, s.rd, NULL, s.rdid, sc->qualitiesMatter());
	TAlScore minsc = std::numeric_limits<TAlScore>::max();
	if(R_bwaSwLike) {
		float a = (float)sc->match(30);
		float T = R_bwaSwLikeT, c = R_bwaSwLikeC;
		minsc = (TAlScore)max<float>(a * T, a * c * log(s.rdlen));
	} else {
		minsc = R_scoreMin.f<TAlScore>(s.rdlen);
		if(R_localAlign) {
			if(minsc < 0) minsc = 0;
		} else {
			if(minsc > 0) minsc = 0;
		}
	}
	s.minsc = minsc;
	size_t readns[2] = {0, 0};
	sc->nFilterPair(&rd.patFw, NULL, readns[0], readns[1], s.nfilt[0], s.nfilt[1]);
	s.scfilt[0] = sc->scoreFilter(minsc, s.rdlen);
	s.scfilt[1] = sc->scoreFilter(std::numeric_limits<TAlScore>::max(), 0);
	s.lenfilt[0] = s.lenfilt[1] = true;
	if(s.rdlen <= (size_t)R_multiseedMms || s.rdlen < 2) s.lenfilt[0] = false;
	if(s.rdlen < 2) s.lenfilt[0] = false;
	s.qcfilt[0] = s.qcfilt[1] = true;
	if(R_qcFilter) {
		s.qcfilt[0] = (rd.filter != '0');
		s.qcfilt[1] = (s.rdb->filter != '0');
	}
	s.filt = s.nfilt[0] && s.scfilt[0] && s.lenfilt[0] && s.qcfilt[0];
	s.prm.nFilt += (s.filt ? 0 : 1) + ((s.nfilt[1] && s.scfilt[1] && s.lenfilt[1] && s.qcfilt[1]) ? 0 : 1);
	s.sd.nextRead(false, s.rdlen, 0);
	s.minedfw = s.minedrc = 0;
	s.nofw = gNofw;
	s.norc = gNorc;
	s.nceil = std::min(R_nCeil.f<int>((double)s.rdlen), (int)s.rdlen);
	s.exhaustive[0] = s.exhaustive[1] = false;
	s.rnd.init(rd.seed);      // (pairPostFilt is false for an unpaired read)
	s.interval = std::max(R_msIval.f<int>((double)s.rdlen), 1);
	s.streak = R_maxDpStreak;
	s.mxDp = R_maxDp;
	s.mxUg = R_maxUg;
	s.mxIter = R_maxIters;
	if(R_allHits) {
		s.streak = s.mxDp = s.mxUg = s.mxIter = std::numeric_limits<size_t>::max();
	} else if(R_khits > 1) {
		s.streak += (R_khits - 1) * R_maxStreakIncr;
		s.mxDp += (R_khits - 1) * R_maxItersIncr;
		s.mxUg += (R_khits - 1) * R_maxItersIncr;
		s.mxIter += (R_khits - 1) * R_maxItersIncr;
	}
	s.prm.maxDPFails = s.streak;
	s.nrounds = R_nSeedRounds;
	if(s.filt) {
		s.shs[0].clear();
		s.shs[0].nextRead(rd);
	}
	s.done = !s.filt;
	s.nelt = 0;
	s.sd_ready = false;
	s.mm_asked = false;
	s.seedlen = R_multiseedLen;
	s.seedsTried = 0;
	for(int k = 0; k < 4; k++) s.seedsTriedMS[k] = s.nUniqueSeedsMS[k] = s.nRepeatSeedsMS[k] = s.seedHitTotMS[k] = 0;
	s.nUniqueSeeds = s.nRepeatSeeds = s.seedHitTot = 0;
	s.ndps = 0;
}

// (the engine takes the read?)
bool engine_read(const Slot& s) { return s.rdlen > 0 && s.rdlen <= BT2G_MAX_READ_LEN; }

// instantiateSeeds (aligner_seed.cpp:498-587) for exact seeds: offsets,
// sequences and qualities into SeedResults; which seeds instantiate (an N
// disqualifies an exact seed: Constraint::canN, aligner_seed.h:88-92).
// Returns the number instantiated.
int instantiate(Driver& d, Slot& s) {
	const Read& rd = *s.rd;
	const int len = s.seeds[0].len;
	int nseeds = 1;
	if((int)rd.length() - (int)s.offset > len) nseeds += ((int)rd.length() - (int)s.offset - len) / s.interval;
	s.offIdx2off.clear();
	for(int i = 0; i < nseeds; i++) s.offIdx2off.push_back(s.interval * i + (int)s.offset);
	SeedResults& sr = s.shs[0];
	sr.reset(rd, s.offIdx2off, nseeds);
	s.valid_fw = s.valid_rc = 0;
	s.valid_big.clear();
	int ninst = 0;
	int inst_fw = 0, inst_rc = 0;
	for(int fwi = 0; fwi < 2; fwi++) {
		const bool fw = fwi == 0;
		if((fw && s.nofw) || (!fw && s.norc)) continue;
		for(int i = 0; i < nseeds; i++) {
			const int depth = i * s.interval + (int)s.offset;
			const int sl = std::min<int>(len, (int)rd.length());
			d.al.instantiateSeq(rd, sr.seqs(fw)[i], sr.quals(fw)[i], sl, depth, fw);
			bool ok = true;
			const BTDnaString& q = sr.seqs(fw)[i];
			for(int k = 0; k < sl && ok; k++) ok = (int)q[k] < 4;
			if(ok) {
				d.set_valid(s, fw, (size_t)i);
				ninst++;
				(fw ? inst_fw : inst_rc)++;
			} else {
				d.sdm.filteredseed++;
			}
		}
	}
	s.seedsTriedMS[0] = (size_t)inst_fw;
	s.seedsTriedMS[1] = (size_t)inst_rc;
	return ninst;
}

// searchAllSeeds' cache protocol and metrics (aligner_seed.cpp:597-718) over
// the engine's seed ranges: strand fw then rc, offsets ascending;
// SeedSearchCache::addOnTheFly for a hit (reportHit, aligner_seed.cpp:1576-1630),
// beginAlign / addAllCached / finishAlign, SeedResults::add.
int Driver::after_seeds(Slot& s) {
	SeedResults& sr = s.shs[0];
	const size_t nof = sr.numOffs();
	if((size_t)s.sd_ns != nof) {
		fprintf(stderr, "bt2g batch: seed offsets differ (engine %d, reference %zu)\n", s.sd_ns, nof);
		abort();
	}
	uint64_t possearches = 0, seedsearches = 0, ooms = 0;
	for(int fwi = 0; fwi < 2; fwi++) {
		const bool fw = fwi == 0;
		for(size_t i = 0; i < nof; i++) {
			if(!seeds_valid(s, fw, i)) continue;
			possearches++;
			seedsearches++;
			const BTDnaString& seq = sr.seqs(fw)[i];
			SeedSearchCache srcache(seq, sr.quals(fw)[i]);
			const uint32_t* q = &s.sd_out[((size_t)fwi * nof + i) * 4];
			if(q[1] > q[0]) srcache.addOnTheFly(seq, q[0], q[1], q[2], q[3]);
			if(srcache.beginAlign(s.ca) == -1) {
				ooms++;
				continue;
			}
			if(!srcache.addAllCached()) {
				ooms++;
				continue;
			}
			srcache.finishAlign();
			if(srcache.qvValid()) sr.add(srcache.getQv(), s.ca.current(), (uint32_t)i, fw);
		}
	}
	s.prm.nSeedRanges = sr.numRanges();
	s.prm.nSeedElts = sr.numElts();
	s.prm.nSeedRangesFw = sr.numRangesFw();
	s.prm.nSeedRangesRc = sr.numRangesRc();
	s.prm.nSeedEltsFw = sr.numEltsFw();
	s.prm.nSeedEltsRc = sr.numEltsRc();
	s.prm.seedMedian = (uint64_t)(sr.medianHitsPerSeed() + 0.5);
	s.prm.seedMean = (uint64_t)sr.averageHitsPerSeed();
	s.prm.nSdFmops += s.sd_ops;
	sdm.seedsearch += seedsearches;
	sdm.nrange += sr.numRanges();
	sdm.nelt += sr.numElts();
	sdm.possearch += possearches;
	sdm.ooms += ooms;
	sdm.bwops += s.sd_ops;
	return 0;
}

// Start one extendSeeds call (bt2_search.cpp:3559-3593 and its two twins).
void start_ext(Slot& s, int seedmms, int seedlen, int seedival) {
	SwDriverB& x = s.sd;
	x.pc = X_START;
	x.seedmms = seedmms;
	x.seedlen = seedlen;
	x.seedival = seedival;
	x.minsc = &s.minsc;
	x.nceil = s.nceil;
	x.maxIters = s.mxIter;
	x.maxUg = s.mxUg;
	x.maxDp = s.mxDp;
	x.maxUgStreak = s.streak;
	x.maxDpStreak = s.streak;
	x.exhaustive = &s.exhaustive[0];
}

// extendSeeds' return code as the worker handles it (bt2_search.cpp:3601-3629).
void after_ext(Driver& d, Slot& s, int ret, bool perfect_check) {
	if(ret == EXTEND_EXHAUSTED_CANDIDATES) {
	} else if(ret == EXTEND_POLICY_FULFILLED) {
		if(s.msinkwrap.state().doneWithMate(true)) s.done = true;
	} else if(ret == EXTEND_PERFECT_SCORE) {
		s.done = true;
	} else if(ret == EXTEND_EXCEEDED_HARD_LIMIT) {
		s.done = true;
	} else if(ret == EXTEND_EXCEEDED_SOFT_LIMIT) {
	} else {
		fprintf(stderr, "Bad return value: %d\n", ret);
		throw 1;
	}
	if(perfect_check && !s.done) {
		const TAlScore perfectScore = d.sc->perfectScore(s.rdlen);
		if(s.minsc == perfectScore) s.done = true;
	}
}

void Driver::step_read(Slot& s) {
	const Read& rd = *s.rd;
	int ret = 0;
	switch(s.pc) {
	case P_START: break;
	case P_AFTER_EXACT: goto after_exact;
	case P_AFTER_EXT_EXACT: goto after_ext_exact;
	case P_AFTER_1MM: goto after_1mm;
	case P_AFTER_EXT_1MM: goto after_ext_1mm;
	case P_AFTER_SEEDS: goto after_seeds_l;
	case P_AFTER_EXT_SEEDS: goto after_ext_seeds;
	default: abort();
	}
	setup_read(s);
	// exact end-to-end alignments (bt2_search.cpp:3453-3482)
	if(R_doExactUpFront) {
		if(!(!s.filt || s.done || s.msinkwrap.state().doneWithMate(true))) {
			swmSeed.exatts++;
			if(engine_read(s)) {
				rq[K_EXACT].push_back(&s);
				prefetch_seeds(s);
				s.pc = P_AFTER_EXACT;
				return;
			}
			s.nelt = al.exactSweep(*ebwtFw, rd, *sc, s.nofw, s.norc, 2, s.minedfw, s.minedrc, true, s.shs[0], sdm);
			g_cpu[K_EXACT]++;
			goto exact_done;
		after_exact:
			{
				const uint32_t* out = s.sweep;
				if(!s.nofw) s.minedfw = out[0];
				if(!s.norc) s.minedrc = out[1];
				sdm.bwops += out[6];
				size_t nelt = 0;
				const int64_t score = (int64_t)s.rdlen * sc->match();
				if(!s.nofw && out[0] == 0 && out[3] > out[2]) {
					s.shs[0].addExactEeFw(out[2], out[3], NULL, NULL, true, score);
					nelt += out[3] - out[2];
				}
				if(!s.norc && out[1] == 0 && out[5] > out[4]) {
					s.shs[0].addExactEeRc(out[4], out[5], NULL, NULL, false, score);
					nelt += out[5] - out[4];
				}
				s.nelt = nelt;
			}
		exact_done:
			{
				size_t bestmin = std::min(s.minedfw, s.minedrc);
				if(bestmin == 0) sdm.bestmin0++;
				else if(bestmin == 1) sdm.bestmin1++;
				else sdm.bestmin2++;
			}
		}
		if(!R_seedSumm) {
			if(s.nelt == 0) {
				s.shs[0].clearExactE2eHits();
			} else if(s.msinkwrap.state().doneWithMate(true)) {
				s.shs[0].clearExactE2eHits();
				s.done = true;
			} else {
				start_ext(s, -1, 0, 0);
				ret = s.sd.ext_step(*this, s);
				if(ret == EXTEND_BLOCKED) {
					s.pc = P_AFTER_EXT_EXACT;
					return;
				}
				goto have_ext_exact;
			after_ext_exact:
				ret = s.sd.ext_step(*this, s);
				if(ret == EXTEND_BLOCKED) return;
			have_ext_exact:
				s.shs[0].clearExactE2eHits();
				after_ext(*this, s, ret, true);
			}
		}
	}
	// 1-mismatch end-to-end alignments (bt2_search.cpp:3633-3813)
	if(R_do1mmUpFront && !R_seedSumm) {
		if(!s.filt || s.done) {
			s.shs[0].clear1mmE2eHits();
			s.nelt = 0;
		} else {
			s.nelt = 0;
			s.yfw = s.minedfw <= 1 && !s.nofw;
			s.yrc = s.minedrc <= 1 && !s.norc;
			if(s.yfw || s.yrc) {
				swmSeed.mm1atts++;
				if(engine_read(s) && bsc_ok && s.minsc >= std::numeric_limits<int32_t>::min() &&
				   s.minsc <= std::numeric_limits<int32_t>::max() && R_localAlign == !sc->monotone) {
					s.mm_nofw = s.yfw ? 0 : 1;
					s.mm_norc = s.yrc ? 0 : 1;
					s.mm_minsc = (int32_t)s.minsc;
					rq[K_1MM].push_back(&s);
					s.pc = P_AFTER_1MM;
					return;
				after_1mm:
					sdm.bwops += s.mm_ops;
					for(int32_t k = 0; k < s.mm_cnt; k++) {
						const bt2g_mm1& h = s.mm[k];
						Edit e((uint32_t)h.pos, h.chr, h.qchr, EDIT_TYPE_MM, false);
						s.shs[0].add1mmEe(h.top, h.bot, &e, NULL, h.fw != 0, h.score);
					}
				} else {
					al.oneMmSearch(ebwtFw, ebwtBw, rd, *sc, s.minsc, !s.yfw, !s.yrc, R_localAlign, false, true, s.shs[0], sdm);
					g_cpu[K_1MM]++;
				}
				s.nelt = s.shs[0].num1mmE2eHits();
			}
		}
		if(s.nelt > 0) {
			if(s.msinkwrap.state().doneWithMate(true)) {
				s.done = true;
			} else {
				start_ext(s, -1, 0, 0);
				ret = s.sd.ext_step(*this, s);
				if(ret == EXTEND_BLOCKED) {
					s.pc = P_AFTER_EXT_1MM;
					return;
				}
				goto have_ext_1mm;
			after_ext_1mm:
				ret = s.sd.ext_step(*this, s);
				if(ret == EXTEND_BLOCKED) return;
			have_ext_1mm:
				s.shs[0].clear1mmE2eHits();
				after_ext(*this, s, ret, true);
			}
		}
	}
	// seed rounds (bt2_search.cpp:3814-4090)
	s.seedlen = R_multiseedLen;
	s.nrounds = std::min<size_t>(s.nrounds, (size_t)s.interval);
	for(s.roundi = 0; s.roundi < R_nSeedRounds; s.roundi++) {
		s.ca.nextRead();
		s.shs[0].clearSeeds();
		s.shs[1].clearSeeds();
		if(s.done || s.msinkwrap.state().doneWithMate(true)) {
			s.done = true;
		} else if(s.roundi >= s.nrounds || s.interval <= (int)s.roundi) {
			// not doing this round
		} else {
			s.offset = ((size_t)s.interval * s.roundi) / s.nrounds;
			swmSeed.sdatts++;
			s.seeds.clear();
			Seed::mmSeeds(R_multiseedMms, s.seedlen, s.seeds, s.gc);
			if(s.offset > 0 && s.seeds[0].len + s.offset > rd.length()) goto round_summary;
			if(!engine_read(s) || R_multiseedMms != 0 || ebwtBw == NULL) {
				// the reference's own seed search on the host (instantiateSeeds +
				// searchAllSeeds, bt2_search.cpp:3873-3913)
				std::pair<int, int> instFw, instRc;
				std::pair<int, int> inst = al.instantiateSeeds(s.seeds, s.offset, s.interval, rd, *sc, s.nofw, s.norc, s.ca,
				                                               s.shs[0], sdm, instFw, instRc);
				if(inst.first + inst.second == 0) {
					s.done = true;
					goto round_summary;
				}
				s.seedsTried += (inst.first + inst.second);
				s.seedsTriedMS[0] = instFw.first + instFw.second;
				s.seedsTriedMS[1] = instRc.first + instRc.second;
				al.searchAllSeeds(s.seeds, ebwtFw, ebwtBw, rd, *sc, s.ca, s.shs[0], sdm, s.prm);
				g_cpu[K_SEEDS]++;
			} else {
				{
					const int inst = instantiate(*this, s);
					if(inst == 0) {
						s.done = true;
						goto round_summary;
					}
					s.seedsTried += (size_t)inst;
				}
				if(!(s.sd_ready && s.sd_L == (uint32_t)s.seeds[0].len && s.sd_per == (uint32_t)s.interval &&
				     s.sd_off == (uint32_t)s.offset && s.sd_nof == (uint32_t)s.shs[0].numOffs())) {
					s.sd_ready = false;
					s.sd_L = (uint32_t)s.seeds[0].len;
					s.sd_per = (uint32_t)s.interval;
					s.sd_off = (uint32_t)s.offset;
					s.sd_nof = (uint32_t)s.shs[0].numOffs();
					rq[K_SEEDS].push_back(&s);
					s.pc = P_AFTER_SEEDS;
					return;
				}
			after_seeds_l:
				s.sd_ready = false;
				after_seeds(s);
			}
			if(s.shs[0].empty()) s.done = true;
		}
	round_summary:
		if(!s.shs[0].empty()) {
			s.nUniqueSeeds += s.shs[0].numUniqueSeeds();
			s.nUniqueSeedsMS[0] += s.shs[0].numUniqueSeedsStrand(true);
			s.nUniqueSeedsMS[1] += s.shs[0].numUniqueSeedsStrand(false);
			s.nRepeatSeeds += s.shs[0].numRepeatSeeds();
			s.nRepeatSeedsMS[0] += s.shs[0].numRepeatSeedsStrand(true);
			s.nRepeatSeedsMS[1] += s.shs[0].numRepeatSeedsStrand(false);
			s.seedHitTot += s.shs[0].numElts();
			s.seedHitTotMS[0] += s.shs[0].numEltsFw();
			s.seedHitTotMS[1] += s.shs[0].numEltsRc();
			swmSeed.sdsucc++;
		}
		if(s.done || s.msinkwrap.state().doneWithMate(true)) {
			s.done = true;
		} else if(!R_seedSumm && !s.shs[0].empty()) {
			s.shs[0].rankSeedHits(s.rnd, s.msinkwrap.allHits());
			start_ext(s, R_multiseedMms, s.seedlen, s.interval);
			ret = s.sd.ext_step(*this, s);
			if(ret == EXTEND_BLOCKED) {
				s.pc = P_AFTER_EXT_SEEDS;
				return;
			}
			goto have_ext_seeds;
		after_ext_seeds:
			ret = s.sd.ext_step(*this, s);
			if(ret == EXTEND_BLOCKED) return;
		have_ext_seeds:
			after_ext(*this, s, ret, false);
		}
		if(!s.done && s.shs[0].averageHitsPerSeed() < R_seedBoostThresh) s.done = true;
	}
	// per-read seed statistics (bt2_search.cpp:4091-4124) and the SAM record
	if(s.seedsTried > 0) {
		s.prm.seedPctUnique = (float)s.nUniqueSeeds / s.seedsTried;
		s.prm.seedPctRep = (float)s.nRepeatSeeds / s.seedsTried;
		s.prm.seedHitAvg = (float)s.seedHitTot / s.seedsTried;
	} else {
		s.prm.seedPctUnique = -1.0f;
		s.prm.seedPctRep = -1.0f;
		s.prm.seedHitAvg = -1.0f;
	}
	for(int k = 0; k < 4; k++) {
		if(s.seedsTriedMS[k] > 0) {
			s.prm.seedPctUniqueMS[k] = (float)s.nUniqueSeedsMS[k] / s.seedsTriedMS[k];
			s.prm.seedPctRepMS[k] = (float)s.nRepeatSeedsMS[k] / s.seedsTriedMS[k];
			s.prm.seedHitAvgMS[k] = (float)s.seedHitTotMS[k] / s.seedsTriedMS[k];
		} else {
			s.prm.seedPctUniqueMS[k] = -1.0f;
			s.prm.seedPctRepMS[k] = -1.0f;
			s.prm.seedHitAvgMS[k] = -1.0f;
		}
	}
	{
		size_t totnucs = 0;
		if(s.filt) {
			size_t len = s.rdlen;
			if(!s.nofw && !s.norc) len *= 2;
			totnucs += len;
		}
		s.prm.seedsPerNuc = totnucs > 0 ? ((float)s.seedsTried / totnucs) : -1;
		for(int k = 0; k < 4; k++) s.prm.seedsPerNucMS[k] = totnucs > 0 ? ((float)s.seedsTriedMS[k] / totnucs) : -1;
	}
	s.msinkwrap.finishRead(&s.shs[0], &s.shs[1], s.exhaustive[0], s.exhaustive[1], s.nfilt[0], s.nfilt[1], s.scfilt[0],
	                       s.scfilt[1], s.lenfilt[0], s.lenfilt[1], s.qcfilt[0], s.qcfilt[1], s.rnd, rpm, s.prm, *sc,
	                       !R_seedSumm, R_seedSumm, R_scUnMapped, R_xeq);
	s.pc = P_FINISH;
}

}  // namespace

namespace {

// The first seed round's search, asked with the exact sweep: its arguments are
// functions of the read and the server's options (round 0: offset 0, the
// read's interval, bt2_search.cpp:3814-3906).  The round takes it only if its
// own arguments are the same (checked in step_read).
void Driver::prefetch_seeds(Slot& s) {
	if(R_seedSumm || R_nSeedRounds == 0 || R_multiseedMms != 0 || ebwtBw == NULL) return;
	const int L = R_multiseedLen;
	int nseeds = 1;
	if((int)s.rdlen > L) nseeds += ((int)s.rdlen - L) / s.interval;
	s.sd_L = (uint32_t)L;
	s.sd_per = (uint32_t)s.interval;
	s.sd_off = 0;
	s.sd_nof = (uint32_t)nseeds;
	s.sd_ready = false;
	rq[K_SEEDS].push_back(&s);
}

void Driver::gpu_phase() {
	call_exact();
	call_seeds();
	call_1mm();
	call_ext();
	call_off();
	call_ug();
	call_dp();
	for(int k = 0; k < K_N; k++) rq[k].clear();
	rq_dp.clear();
}

void Driver::feeder() {
	pthread_setname_np(pthread_self(), "bt2g-feed");
	for(;;) {
		{
			std::unique_lock<std::mutex> lk(in_mu);
			room_cv.wait(lk, [this] { return held < max_held; });
			held++;
		}
		ReadElement re = R_factory->nextReadPair();      // blocks until a connection has reads
		Elem* e = new Elem(re);
		{
			std::lock_guard<std::mutex> lk(in_mu);
			inbox.push_back(e);
		}
		in_cv.notify_one();
	}
}

void finish_elem(Driver& d, Elem* e) {
	R_factory->returnUnready(e->re);      // back to its connection (PSFactory::ReadAhead's destructor)
	delete e;
	{
		std::lock_guard<std::mutex> lk(d.in_mu);
		d.held--;
	}
	d.room_cv.notify_one();
}

// The reads of one buffer, in the order the reference's worker takes them
// (bt2_search.cpp:3201-3211, 4174: the buffer is read to its end).
void Driver::admit(Elem* e) {
	PatternSourcePerThread* ps = e->re.ps;
	e->live = 1;
	bool first = true;
	do {
		if(!first) e->re.nextReadPair();
		first = false;
		if(!e->re.readResult.first) continue;
		Read& ra = ps->read_a();
		if(!ps->read_b().empty()) {
			fprintf(stderr, "bt2g batch: paired reads are served by the fiber drop-in (bowtie2-align-server-gpu)\n");
			abort();
		}
		if(ra.rdid < R_skipReads || ra.rdid >= R_qUpto) continue;
		Slot* s;
		if(freel.empty()) {
			all.emplace_back(new Slot(*rp, *mapq, (size_t)tid));
			s = all.back().get();
		} else {
			s = freel.back();
			freel.pop_back();
		}
		s->el = e;
		s->rd = &ra;
		s->rdb = &ps->read_b();
		s->rdid = ra.rdid;
		s->msink = &ps->msink();
		s->pc = P_START;
		e->live++;
		active++;
		run.push_back(s);
	} while(ps->nextReadPairReady());
	if(--e->live == 0) finish_elem(*this, e);
}

void Driver::release(Slot* s) {
	Elem* e = s->el;
	s->el = nullptr;
	active--;
	freel.push_back(s);
	if(((++g_reads) & 0xffff) == 0) write_stats();
	if(--e->live == 0) finish_elem(*this, e);
}

void Driver::run_loop() {
	open_bases();
	const size_t ndev = g_bases.size();
	int rc = bt2g_open_shared(g_bases[(size_t)tid % ndev], &ctx);
	if(rc) die("bt2g_open_shared", rc);
	sc = R_sc;
	ebwtFw = R_ebwtFw;
	ebwtBw = R_ebwtBw;
	ref = R_refs;
	bsc_ok = to_scoring(*sc, bsc);
	rp.reset(new ReportingParams(R_allHits ? std::numeric_limits<THitInt>::max() : R_khits, R_mhits, 0, R_msample,
	                             gReportDiscordant, gReportMixed));
	mapq.reset(new_mapq(R_mapqv, R_scoreMin, *sc));
	max_held = env_or("BT2G_BATCH_ELEMS", 64);
	spec_k = env_or("BT2G_SPEC_DPS", 16);
	{
		char nm[16];
		snprintf(nm, sizeof(nm), "bt2g-drv%d", tid);
		pthread_setname_np(pthread_self(), nm);
	}
	std::thread(&Driver::feeder, this).detach();
	for(;;) {
		std::deque<Elem*> got;
		{
			std::unique_lock<std::mutex> lk(in_mu);
			if(active == 0) in_cv.wait(lk, [this] { return !inbox.empty(); });
			got.swap(inbox);
		}
		for(Elem* e : got) admit(e);
		const uint64_t t0 = now_us();
		for(size_t k = 0; k < run.size(); k++) {
			Slot* s = run[k];
			step_read(*s);
			if(s->pc == P_FINISH) release(s);
			else next.push_back(s);
		}
		run.clear();
		const uint64_t t1 = now_us();
		gpu_phase();
		const uint64_t t2 = now_us();
		run.swap(next);
		g_rounds++;
		g_cpu_us += t1 - t0;
		g_gpu_us += t2 - t1;
		g_round_us += t2 - t0;
	}
}

// The options this driver restates (the rest of the worker's behaviour for
// them would need code it does not have): checked once, loudly.
void check_options() {
	const char* why = nullptr;
	if(R_arbitraryRandom) why = "--non-deterministic";
	else if(R_sampleFrac < 1.0f) why = "--sample";
	else if(R_metricsIval > 0 && (R_metricsOfb != NULL || R_metricsStderr)) why = "--met-file/--met-stderr";
	else if(R_metricsPerRead) why = "--met-read";
	else if(!R_logDps.empty() || !R_logDpsOpp.empty()) why = "--log-dp";
	if(why) {
		fprintf(stderr, "bt2g batch: %s is not supported by the batch driver (use bowtie2-align-server-gpu)\n", why);
		abort();
	}
}

void batch_worker(thread_tracking_pair* tp) {
	static std::once_flag once;
	std::call_once(once, check_options);
	Driver* d = new Driver(tp->tid);           // lives as long as the server
	d->run_loop();
}

}  // namespace

// ---- the worker spawn (bt2_search.cpp:4913-4925) -------------------------------
// std::thread(multiseedSearchWorker, (void*)&tps[i]): a thread whose state is a
// void(*)(void*) call with its argument becomes a driver thread on that
// argument (thread_tracking_pair: its tid is the AlnSinkWrap / OutputQueue
// thread id).  Every other thread (listener, connections) starts as usual.
extern "C" {
void __real__ZNSt6thread15_M_start_threadESt10unique_ptrINS_6_StateESt14default_deleteIS1_EEPFvvE(
	std::thread* self, std::unique_ptr<std::thread::_State> st, void (*dep)());

void __wrap__ZNSt6thread15_M_start_threadESt10unique_ptrINS_6_StateESt14default_deleteIS1_EEPFvvE(
	std::thread* self, std::unique_ptr<std::thread::_State> st, void (*dep)()) {
	static const char* const WORKER = "NSt6thread11_State_implINS_8_InvokerISt5tupleIJPFvPvES3_EEEEEE";
	if(!st || strcmp(typeid(*st).name(), WORKER) != 0) {
		__real__ZNSt6thread15_M_start_threadESt10unique_ptrINS_6_StateESt14default_deleteIS1_EEPFvvE(self, std::move(st),
		                                                                                              dep);
		return;
	}
	// _State_impl<_Invoker<tuple<void(*)(void*), void*>>>: the vtable pointer, then
	// the tuple, whose elements libstdc++ lays out last-first (checked below)
	static const bool layout_ok = [] {
		std::tuple<void (*)(void*), void*> t((void (*)(void*))0x1111, (void*)0x2222);
		return *(void**)((char*)&t) == (void*)0x2222 && *(void**)((char*)&t + sizeof(void*)) == (void*)0x1111;
	}();
	if(!layout_ok) {
		fprintf(stderr, "bt2g batch: unexpected std::thread state layout\n");
		abort();
	}
	thread_tracking_pair* tp = *(thread_tracking_pair**)((char*)st.get() + sizeof(void*));
	st.reset();
	std::thread t([tp] { batch_worker(tp); });
	self->swap(t);
}
}  // extern "C"
