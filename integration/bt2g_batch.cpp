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
//   Driver::step_read          multiseedSearchWorker's per-read body, unpaired
//                              and paired (bt2_search.cpp:3266-4160)
//   SwDriverB::ext_step        SwDriver::extendSeeds (aligner_sw_driver.cpp:756-1297)
//   SwDriverB::ext_step_paired SwDriver::extendSeedsPaired, mate search included
//                              (aligner_sw_driver.cpp:1385-2402)
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
#include <sched.h>
#include <signal.h>
#include <execinfo.h>
#include <unistd.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/syscall.h>

#include <algorithm>
#include <array>
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
#include <unordered_map>
#include <vector>

#include "aligner_cache.h"
#include "aligner_seed.h"
#include "aligner_sw.h"
#include "aligner_sw_driver.h"
#include "aln_sink.h"
#include "dp_framer.h"
#include "pat.h"
#include "pe.h"
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
extern bool gReportDiscordant;           // bt2_search.cpp:118-128 (globals there)
extern bool gReportMixed;
extern bool gMate1fw, gMate2fw, gFlippedMatesOK, gDovetailMatesOK, gContainMatesOK, gOlapMatesOK, gExpandToFrag;
extern int gMinInsert, gMaxInsert;

extern "C" void bt2g_prof_thread(int role);   // bt2g_prof.cpp: CPU samples of this thread ($BT2G_SAMPLE)
extern "C" void bt2g_prof_role(int role);     // (samples tagged 3: stepping reads, 1: engine calls)

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
// service workers' busy time per kind (a call's packing and unpacking included)
std::atomic<uint64_t> g_svc_us[K_N];
std::atomic<uint64_t> g_reads{0}, g_rounds{0}, g_round_us{0}, g_cpu_us{0}, g_gpu_us{0};
std::atomic<uint64_t> g_dp_spec{0}, g_dp_used{0}, g_dp_reuse{0}, g_dp_miss{0};
std::atomic<uint64_t> g_mm_pf{0}, g_mm_pf_used{0};   // 1-mm searches prefetched with the sweep / taken
std::atomic<uint64_t> g_rows_pf{0};                   // SA rows resolved with the sweep or the seeds
std::atomic<uint64_t> g_ext_pf{0};
std::atomic<uint64_t> g_ext_spec{0};                   // seed ranges extended in the seed call (bt2g_seed_search_ext)
std::atomic<uint64_t> g_gw_inits{0}, g_gw_elts{0}, g_gw_adv{0};   // (diagnostic) GroupWalk2S inits, their elements, advanceElement calls
std::atomic<uint64_t> g_dp_pre_us{0}, g_dp_post_us{0};   // the DP service's host work around its calls
std::atomic<uint64_t> g_dp_again{0};                   // DPs run again (candidates, alignments or edits over the room)                    // extend requests answered by the seed call
// rounds per read: total and a histogram (bin b: [2^b, 2^(b+1)))
std::atomic<uint64_t> g_steps{0}, g_steps_hist[16];
// reads in flight summed over rounds; drivers' time with no read in flight
std::atomic<uint64_t> g_inflight{0}, g_idle_us{0}, g_slots{0};
// slot footprints at release (bin b: [2^b, 2^(b+1)) KiB) and slots rebuilt for size
std::atomic<uint64_t> g_slot_mem_hist[16], g_slots_rebuilt{0}, g_slots_live{0};
std::atomic<uint64_t> g_pool_trims{0}, g_pool_trim_pages{0};   // pool_trim calls and pages handed back
// $BT2G_PHASES=1 (diagnostics): the drivers' CPU by phase of the per-read logic,
// inclusive TSC cycles and calls, summed into the stats once per round
enum { PH_STEP, PH_SETUP, PH_ADMIT, PH_RELEASE, PH_INST, PH_AFTER_SEEDS, PH_RANK, PH_EESAT, PH_PRIO, PH_ROWS,
       PH_NEXTELT, PH_NEEDDP, PH_DPFOUND, PH_REPLAY, PH_REDUND, PH_REPORT, PH_FINISH, PH_SUBMIT, PH_N };
const char* const PH_NAMES[PH_N] = {"step", "setup_read", "admit", "release", "instantiate", "after_seeds",
                                    "rankSeedHits", "eeSaTups", "prioritizeSATups", "rows_request", "next_element",
                                    "need_dp", "dp_found", "replay_next", "redundant", "report", "finishRead",
                                    "submit_wait"};
bool phases_on() {
	static const bool on = [] { const char* e = getenv("BT2G_PHASES"); return e && *e == '1'; }();
	return on;
}
thread_local uint64_t t_ph[PH_N], t_phn[PH_N];
std::atomic<uint64_t> g_ph[PH_N], g_phn[PH_N];
std::atomic<uint64_t> g_tsc0{0}, g_us0{0};
struct Ph {
	int id;
	uint64_t t0;
	explicit Ph(int i) : id(i), t0(phases_on() ? __builtin_ia32_rdtsc() : 0) {}
	~Ph() {
		if(t0) {
			t_ph[id] += __builtin_ia32_rdtsc() - t0;
			t_phn[id]++;
		}
	}
};
void ph_flush() {
	if(!phases_on()) return;
	for(int k = 0; k < PH_N; k++) {
		if(t_phn[k]) {
			g_ph[k] += t_ph[k];
			g_phn[k] += t_phn[k];
			t_ph[k] = t_phn[k] = 0;
		}
	}
}
char g_stats_path[4096];

int svc_stats(char* buf, size_t cap);   // the services' kernel times and work (below)

void write_stats() {
	if(!g_stats_path[0]) return;
	char buf[16384];
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
	n += snprintf(buf + n, sizeof(buf) - n, ", \"ext_speculative\": %llu", (unsigned long long)g_ext_spec.load());
	n += snprintf(buf + n, sizeof(buf) - n, ", \"gw\": [%llu, %llu, %llu]", (unsigned long long)g_gw_inits.load(),
	              (unsigned long long)g_gw_elts.load(), (unsigned long long)g_gw_adv.load());
	n += snprintf(buf + n, sizeof(buf) - n, ", \"one_mm_prefetch\": [%llu, %llu], \"rows_prefetched\": %llu, \"ext_prefetched\": %llu"
	              ", \"dp_host_ms\": [%.1f, %.1f], \"dp_again\": %llu",
	              (unsigned long long)g_mm_pf.load(), (unsigned long long)g_mm_pf_used.load(),
	              (unsigned long long)g_rows_pf.load(), (unsigned long long)g_ext_pf.load(), g_dp_pre_us.load() / 1000.0,
	              g_dp_post_us.load() / 1000.0, (unsigned long long)g_dp_again.load());
	n += snprintf(buf + n, sizeof(buf) - n, ", \"svc_busy_ms\": [");
	for(int k = 0; k < K_N; k++)
		n += snprintf(buf + n, sizeof(buf) - n, "%s%.1f", k ? ", " : "", g_svc_us[k].load() / 1000.0);
	n += snprintf(buf + n, sizeof(buf) - n, "]");
	n += snprintf(buf + n, sizeof(buf) - n, ", \"inflight_sum\": %llu, \"idle_ms\": %.1f, \"slots\": %llu",
	              (unsigned long long)g_inflight.load(), g_idle_us.load() / 1000.0, (unsigned long long)g_slots.load());
	if(phases_on() && g_tsc0.load()) {
		// TSC cycles -> ns from the TSC and the steady clock since the first round
		const double ns_per_cyc = (now_us() - g_us0.load()) * 1e3 / (double)(__builtin_ia32_rdtsc() - g_tsc0.load());
		n += snprintf(buf + n, sizeof(buf) - n, ", \"phases_ms\": {");
		for(int k = 0; k < PH_N; k++)
			n += snprintf(buf + n, sizeof(buf) - n, "%s\"%s\": [%.1f, %llu]", k ? ", " : "", PH_NAMES[k],
			              g_ph[k].load() * ns_per_cyc / 1e6, (unsigned long long)g_phn[k].load());
		n += snprintf(buf + n, sizeof(buf) - n, "}");
	}
	n += snprintf(buf + n, sizeof(buf) - n, ", \"pool_trims\": [%llu, %llu]", (unsigned long long)g_pool_trims.load(),
	              (unsigned long long)g_pool_trim_pages.load());
	n += snprintf(buf + n, sizeof(buf) - n, ", \"slots_live\": %llu, \"slots_rebuilt\": %llu, \"slot_kib_hist\": [",
	              (unsigned long long)g_slots_live.load(), (unsigned long long)g_slots_rebuilt.load());
	for(int b = 0; b < 16; b++)
		n += snprintf(buf + n, sizeof(buf) - n, "%s%llu", b ? ", " : "", (unsigned long long)g_slot_mem_hist[b].load());
	n += snprintf(buf + n, sizeof(buf) - n, "]");
	n += snprintf(buf + n, sizeof(buf) - n, ", \"steps\": %llu, \"steps_hist\": [", (unsigned long long)g_steps.load());
	for(int b = 0; b < 16; b++)
		n += snprintf(buf + n, sizeof(buf) - n, "%s%llu", b ? ", " : "", (unsigned long long)g_steps_hist[b].load());
	n += snprintf(buf + n, sizeof(buf) - n, "]");
	n += svc_stats(buf + n, sizeof(buf) - n);
	n += snprintf(buf + n, sizeof(buf) - n, "}\n");
	FILE* f = fopen(g_stats_path, "w");
	if(f) {
		fwrite(buf, 1, (size_t)n, f);
		fclose(f);
	}
}

extern "C" void bt2g_alloc_stats_dump();
extern "C" long long bt2g_alloc_thread_net();    // bt2g_alloc.cpp: this thread's allocated - freed bytes
extern "C" void bt2g_alloc_site_scope(int on);   // bt2g_alloc.cpp ($BT2G_ALLOC_SITES)   // bt2g_alloc.cpp ($BT2G_ALLOC_STATS)

// $BT2G_EXIT_CLEAN=1: SIGTERM ends the process through exit() (atexit handlers
// run: a profiler preloaded into the server writes its trace), from a thread
// of its own rather than the signal handler.
std::atomic<bool> g_term{false};
bool exit_clean() {
	static const bool on = [] { const char* e = getenv("BT2G_EXIT_CLEAN"); return e && *e == '1'; }();
	return on;
}

void on_term(int) {
	if(exit_clean()) {
		g_term.store(true);
		return;
	}
	write_stats();
	bt2g_alloc_stats_dump();
	_exit(0);
}

void term_watch() {
	while(!g_term.load()) usleep(10000);
	write_stats();
	bt2g_alloc_stats_dump();
	exit(0);
}

// A fault in a driver thread: its stack on stderr (the server's log), then die.
void on_fault(int sig) {
	void* pcs[64];
	const int n = backtrace(pcs, 64);
	char msg[64];
	const int k = snprintf(msg, sizeof(msg), "bt2g batch: signal %d, stack:\n", sig);
	if(write(2, msg, (size_t)k) < 0) {}
	backtrace_symbols_fd(pcs, n, 2);
	signal(sig, SIG_DFL);
	raise(sig);
}

// $BT2G_PIN_CPUS: run the server's threads on that many CPUs of its affinity
// mask ("auto", the default: as many as the cgroup's CPU quota, cpu.max, when
// the mask is larger -- the GPU box gives a 16-CPU quota over a 256-CPU mask,
// and threads spread over 256 CPUs burn the quota in bursts and are then
// throttled together for the rest of the period; "0": no pinning).
void pin_cpus() {
	// (default "auto" since round 6: r06f, one lease, 2 x 3 passes each: 263.6 / 268.6 k
	// aligned reads/s pinned against 246.7 / 240.8 k spread, 41 vs 51 us of server
	// CPU per read -- threads that stay on 16 CPUs keep their slots in 2 L3s)
	const char* e = getenv("BT2G_PIN_CPUS");
	if(!e) e = "auto";
	if(!*e || !strcmp(e, "0")) return;
	long n = atol(e);
	if(!strcmp(e, "auto")) {
		n = 0;
		if(FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
			char q[64] = {0};
			unsigned long period = 0;
			if(fscanf(f, "%63s %lu", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0)
				n = (long)((strtoul(q, nullptr, 10) + period - 1) / period);
			fclose(f);
		}
	}
	cpu_set_t set;
	if(n <= 0 || sched_getaffinity(0, sizeof(set), &set) != 0 || CPU_COUNT(&set) <= n) return;
	cpu_set_t pin;
	CPU_ZERO(&pin);
	long k = 0;
	for(int c = 0; c < CPU_SETSIZE && k < n; c++)
		if(CPU_ISSET(c, &set)) {
			CPU_SET(c, &pin);
			k++;
		}
	if(sched_setaffinity(0, sizeof(pin), &pin) == 0) fprintf(stderr, "bt2g batch: threads pinned to %ld CPUs\n", k);
}

// Environment of the engines, set before any thread starts (static
// initialiser): the runtime reads it at its first HIP call.
struct EnvInit {
	EnvInit() {
		pin_cpus();
		setenv("BT2G_SYNC", "poll", 0);
		const char* hq = getenv("BT2G_HW_QUEUES");
		// (16 for ~20 streams -- six DP workers and two per other kind, each with its
		// own context and stream: r04r measured 190 k reads/s with 16 and 214 k with
		// 32 on different runs, but r04ae with 32 ran every service kernel slower,
		// the 1-mm work queue 6x, and the server at 123 k against r04ab's 205 k)
		long q = hq ? atol(hq) : 16;
		if(q < 1) q = 1;
		if(q > 32) q = 32;                      // the runtime refuses more
		char b[16];
		snprintf(b, sizeof(b), "%ld", q);
		setenv("GPU_MAX_HW_QUEUES", b, 1);
		signal(SIGSEGV, on_fault);
		signal(SIGBUS, on_fault);
		signal(SIGABRT, on_fault);
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
	bool fresh;          // every row asked (or taken from a call that resolved it), none read first
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
	DpRes() {
		cands.reserve(128);
		fates.reserve(128);
		alns.reserve(8);
		edits.reserve(256);
	}
	int mate = 0;          // the read of the DP (its row in the slot)
	int32_t fw = 0;
	uint32_t refidx = 0;
	int64_t refl = 0;
	uint32_t ncol = 0;
	bt2g_sw_rect rect{};
	int32_t minsc = 0;
	TRefOff tlen = 0;
	bool extend = true;    // seed extension (else mate search), SwAligner::initRef's `extend`
	bool ready = false, cpu = false;
	bt2g_sw_result o{};
	int32_t naln = 0;
	uint32_t maxedit = 0;
	std::vector<bt2g_sw_cand> cands;
	std::vector<int8_t> fates;
	std::vector<bt2g_sw_aln> alns;
	std::vector<bt2g_edit> edits;
	DPRect drect;          // for the CPU path (reads the engine does not take)
	bool same_problem(int m, bool f, uint32_t ti, const DPRect& r) const {
		return mate == m && fw == (f ? 1 : 0) && refidx == ti && refl == r.refl &&
		       ncol == (uint32_t)(r.refr + 1 - r.refl) && rect.triml == (int32_t)r.triml &&
		       rect.corel == (int32_t)r.corel && rect.corer == (int32_t)r.corer;
	}
};

bool u8_regime(int64_t minsc) { return R_enable8 && minsc >= -254; }

// The SwAligner after align(): the engine's candidate list replayed by
// nextAlignment (or, for a DP the engine does not take, the driver thread's
// own SwAligner).
struct Replay {
	DpRes* dp = nullptr;
	size_t cural = 0;
	uint32_t next = 0;
	size_t next_edit = 0;
	bool cpu = false;
	void start(DpRes* d) {
		dp = d;
		cural = 0;
		next = 0;
		next_edit = 0;
		cpu = d->cpu;
	}
};

struct Driver;
struct Slot;

// ---- a slot's 20 MB cache pools ---------------------------------------------------
// Each slot owns the two ds.h Pools a worker thread owns (AlignmentCache's for the
// current read's seed hits, aligner_cache.h:474, and SwDriver's for end-to-end hit
// offsets, aligner_sw_driver.h:308).  Their pages are committed as a read first
// writes them -- AlignmentCache::addOnTheFlyImpl writes an OFF_MASK entry for every
// element of a seed's SA range (aligner_cache.cpp:85-91), up to the whole 20 MB for
// a read in a high-copy repeat -- and a pool keeps them: a worker thread of the
// stock server holds two such pools, but ~14 k slots would each keep the
// high-water mark of every read they served (r05a: +10 GB of host memory per pass
// of 1 M reads, 79 GB in these pools after 7).  So when a read has used more than
// POOL_KEEP pages of a pool, the pages past that are handed back to the kernel
// (MADV_DONTNEED: zero pages on the next touch; a pool's pages are always
// written before they are read).  The cost is a page fault per 16 KB the next heavy
// read writes, against the ~4 k entries it writes there.
// Pool's own fields (ds.h:3145-3149) are private: read through the rule that an
// explicit instantiation may name any member.
template<typename Tag, typename Tag::type M> struct PoolPeek {
	friend typename Tag::type peek(Tag) { return M; }
};
struct PoolSuper { typedef uint8_t* Pool::*type; friend type peek(PoolSuper); };
struct PoolCur { typedef size_t Pool::*type; friend type peek(PoolCur); };
template struct PoolPeek<PoolSuper, &Pool::super_pages>;
template struct PoolPeek<PoolCur, &Pool::cur_>;
// EIvalMergeListBinned's bins (ival_list.h:296), for clearing only the bins a read used
struct DiagBins { typedef EList<EIvalMergeList> EIvalMergeListBinned::*type; friend type peek(DiagBins); };
template struct PoolPeek<DiagBins, &EIvalMergeListBinned::bins_>;

// pages (16 KB each, CACHE_PAGE_SZ) a pool keeps ($BT2G_POOL_KEEP_PAGES, default 64).
// r06e, one lease, 2 x 3 passes each: 16 pages 228.5 / 249.0 k aligned reads/s at
// 54.3 / 47.4 us of server CPU per read and 42.2 GB RSS; 64 pages 253.5 / 250.2 k at
// 46.5 / 48.0 us and 49.3 GB -- the trim's madvise and the pages' refaults were 4 %
// of the server's CPU samples (r06c)
size_t pool_keep() {
	static const size_t k = env_or("BT2G_POOL_KEEP_PAGES", 64);
	return k;
}

// After a read: the pages the pool handed out beyond pool_keep() go back.
void pool_trim(Pool& p) {
	const size_t used = p.*peek(PoolCur());
	const size_t POOL_KEEP = pool_keep();
	if(used <= POOL_KEEP) return;
	uint8_t* base = p.*peek(PoolSuper());
	const uintptr_t lo = ((uintptr_t)base + POOL_KEEP * CACHE_PAGE_SZ + 4095) & ~(uintptr_t)4095;
	const uintptr_t hi = ((uintptr_t)base + used * CACHE_PAGE_SZ) & ~(uintptr_t)4095;
	if(hi <= lo) return;
	(void)madvise((void*)lo, hi - lo, MADV_DONTNEED);
	g_pool_trims++;
	g_pool_trim_pages += used - POOL_KEEP;
}

// Random1toN (random_util.h:32-215, random_util.cpp: swap list below 128
// elements or without replacement, else a seen list converted to a swap list
// past max(16, 0.1 n) draws) with the same draws and the same answers, but its
// swap list kept sparse: the list is the identity except where a draw swapped,
// so only those (position, value) pairs are stored.  The reference fills the
// whole list (up to 127 entries, and an EList growth) at a range's first draw
// -- 6 % of the drivers' CPU in r06c's profile, for ~1-2 draws per range.
struct R1N {
	size_t n = 0, cur = 0, thresh = 0;
	bool swaplist = false, converted = false;
	std::vector<std::pair<size_t, size_t>> sw;    // swap-list entries that are not the identity
	std::vector<size_t> seen, list;               // seen list; the materialised list after a conversion
	void init(size_t n_, bool withoutReplacement) {
		n = n_;
		converted = false;
		swaplist = n_ < 128 || withoutReplacement;
		cur = 0;
		sw.clear();
		seen.clear();
		list.clear();
		thresh = std::max<size_t>(16, (size_t)(0.10f * n_));
	}
	void reset() {
		n = cur = thresh = 0;
		swaplist = converted = false;
		sw.clear();
		seen.clear();
		list.clear();
	}
	bool inited() const { return n > 0; }
	void setDone() { cur = n; }
	bool done() const { return inited() && cur >= n; }
	size_t get(size_t i) const {
		if(converted) return list[i];
		for(const auto& p : sw)
			if(p.first == i) return p.second;
		return i;
	}
	void set(size_t i, size_t v) {
		if(converted) {
			list[i] = v;
			return;
		}
		for(auto& p : sw)
			if(p.first == i) {
				p.second = v;
				return;
			}
		sw.emplace_back(i, v);
	}
	size_t next(RandomSource& rnd) {
		if(cur == 0 && !converted && n == 1) {
			cur = 1;
			return 0;
		}
		if(swaplist) {
			const size_t r = cur + (rnd.nextU32() % (n - cur));
			const size_t vr = get(r);
			if(r != cur) set(r, get(cur));       // (position cur is never read again)
			cur++;
			return vr;
		}
		size_t rn = 0;
		for(bool again = true; again;) {
			rn = rnd.nextU32() % n;
			again = std::find(seen.begin(), seen.end(), rn) != seen.end();
		}
		seen.push_back(rn);
		cur++;
		if(seen.size() >= thresh && cur < n) {
			std::sort(seen.begin(), seen.end());
			list.clear();
			list.reserve(n - cur);
			size_t prev = 0;
			for(size_t x : seen) {
				for(size_t j = prev; j < x; j++) list.push_back(j);
				prev = x + 1;
			}
			for(size_t j = prev; j < n; j++) list.push_back(j);
			seen.clear();
			cur = 0;
			n = list.size();
			converted = true;
			swaplist = true;
		}
		return rn;
	}
};

// ---- SwDriver::extendSeeds / extendSeedsPaired as resumable state machines ----
// (aligner_sw_driver.cpp:756-1297 and 1385-2402).  Members of the reference's
// SwDriver (satpos_, gws_, rands_, eehits_, seenDiags*_, red*_, res*_,
// mateStreaks_) are used as the reference uses them; the loops' locals live
// here so that a loop can stop where it needs an engine result and resume
// there.
// RedundantAlns (aligner_result.h:1657-1692, aligner_result.cpp:929-1010)
// restated flat: the reference keeps one sorted set of (ref, strand, ref offset,
// read row) cells per read row and inserts ~150 of them per reported alignment;
// here an alignment is its [left, right) reference interval per read row, kept
// in one array per read, and overlap() compares a candidate's intervals row by
// row with those of the same reference and strand.  Same cells, same answers:
// the intervals are computed by the reference's own walk over the edits
// (including its invertEdits round trip for reverse-strand alignments).
struct RedFlat {
	struct Aln {
		TRefId ref;
		bool fw;
		size_t row0;                      // first read row
		size_t nrow;
		size_t at;                        // its intervals in iv
	};
	std::vector<Aln> alns;
	std::vector<std::pair<TRefOff, TRefOff>> iv, tmp;
	void reset() {
		alns.clear();
		iv.clear();
		last = nullptr;
	}
	// the cells of res: per row, [left, right) (aligner_result.cpp:930-969)
	static size_t cells(const AlnRes& res, std::vector<std::pair<TRefOff, TRefOff>>& out) {
		TRefOff left = res.refoff(), right;
		const size_t len = res.readExtentRows();
		const size_t start = res.trimmedLeft(true);
		if(!res.fw()) const_cast<AlnRes&>(res).invertEdits();
		const EList<Edit>& ned = res.ned();
		size_t nedidx = 0;
		for(size_t i = start; i < start + len; i++) {
			size_t diff = 1;
			right = left + 1;
			while(nedidx < ned.size() && ned[nedidx].pos == i) {
				if(ned[nedidx].isRefGap()) diff = 0;
				nedidx++;
			}
			if(i < start + len - 1) {
				size_t nx = nedidx;
				while(nx < ned.size() && ned[nx].pos == i + 1) {
					if(ned[nx].isReadGap()) right++;
					nx++;
				}
			}
			out.emplace_back(left, right);
			left = right + diff - 1;
		}
		if(!res.fw()) const_cast<AlnRes&>(res).invertEdits();
		return start;
	}
	const AlnRes* last = nullptr;         // the alignment whose cells tmp holds (overlap, then add)
	size_t last_row0 = 0;
	bool overlap(const AlnRes& res) {
		tmp.clear();
		const size_t row0 = cells(res, tmp);
		last = &res;
		last_row0 = row0;
		const size_t row1 = row0 + tmp.size();
		for(const Aln& a : alns) {
			if(a.ref != res.refid() || a.fw != res.fw()) continue;
			const size_t lo = std::max(row0, a.row0), hi = std::min(row1, a.row0 + a.nrow);
			for(size_t r = lo; r < hi; r++) {
				const std::pair<TRefOff, TRefOff>& x = tmp[r - row0];
				const std::pair<TRefOff, TRefOff>& y = iv[a.at + (r - a.row0)];
				if(std::max(x.first, y.first) < std::min(x.second, y.second)) return true;
			}
		}
		return false;
	}
	// (every call follows overlap() on the same, unchanged alignment: its cells
	// are taken from tmp instead of walked again)
	void add(const AlnRes& res) {
		Aln a;
		a.ref = res.refid();
		a.fw = res.fw();
		a.at = iv.size();
		if(last == &res) {
			iv.insert(iv.end(), tmp.begin(), tmp.end());
			a.row0 = last_row0;
		} else {
			a.row0 = cells(res, iv);
		}
		last = nullptr;
		a.nrow = iv.size() - a.at;
		alns.push_back(a);
	}
};

enum { EXTEND_BLOCKED = 0 };
enum { FOUND_NONE_ = 0, FOUND_EE_, FOUND_UNGAPPED_ };
enum { X_START = 0, X_AFTER_EE_ROWS, X_AFTER_EXT, X_AFTER_PRIO_ROWS, X_AFTER_UG, X_AFTER_DP, X_AFTER_MDP };

struct SwDriverB : public SwDriver {
	explicit SwDriverB(size_t bytes) : SwDriver(bytes) {}
	Pool& ee_pool() { return pool_; }
	RedFlat redA, redM1, redM2;            // redAnchor_, redMate1_, redMate2_ (RedFlat above)
	// SwDriver::nextRead (aligner_sw_driver.h:422-441) with the flat redundancy sets
	// seenDiags1_ / seenDiags2_ with the bins each read added to (bin = the
	// reference id's low 7 bits, ival_list.h:232-236): the next read clears
	// those bins only, the same state as EIvalMergeListBinned::reset's clear of
	// all 128 (r05s: the two resets were ~5 % of the drivers' samples; a read
	// touches a few bins)
	uint64_t sd_used[2][2] = {{0, 0}, {0, 0}};
	void sd_add(int which, const Interval& iv) {
		const size_t bin = iv.ref() & ~(0xffffffff << EIvalMergeListBinned::NBIN);
		sd_used[which][bin >> 6] |= 1ull << (bin & 63);
		(which ? seenDiags2_ : seenDiags1_).add(iv);
	}
	void sd_clear(int which) {
		EList<EIvalMergeList>& bins = (which ? seenDiags2_ : seenDiags1_).*peek(DiagBins());
		for(int w = 0; w < 2; w++) {
			for(uint64_t m = sd_used[which][w]; m; m &= m - 1) bins[w * 64 + __builtin_ctzll(m)].clear();
			sd_used[which][w] = 0;
		}
	}
	void next_read() {
		redA.reset();
		sd_clear(0);
		sd_clear(1);
		seedExRangeFw_[0].clear();
		seedExRangeFw_[1].clear();
		seedExRangeRc_[0].clear();
		seedExRangeRc_[1].clear();
		redM1.reset();
		redM2.reset();
	}

	// extendSeeds / extendSeedsPaired arguments (bt2_search.cpp:3505-3593 and twins)
	int mate = 0;                  // the anchor mate (0: mate 1)
	bool paired = false, anchor1 = true, oppFilt = false;
	int seedmms = 0, seedlen = 0, seedival = 0;
	TAlScore* minsc = nullptr;
	TAlScore* ominsc = nullptr;
	int nceil = 0, onceil = 0;
	bool nofw = false, norc = false;
	size_t maxIters = 0, maxUg = 0, maxDp = 0, maxEeStreak = 0, maxUgStreak = 0, maxDpStreak = 0, maxMateStreak = 0;
	bool swMateImmediately = true;
	bool* exhaustive = nullptr;
	// loop state
	int pc = X_START;
	bool all = false, eeMode = false, firstEe = false, firstExtend = false;
	size_t nonz = 0, nelt = 0, neltLeft = 0, rows = 0, orows = 0, eltsDone = 0, rdlen = 0, ordlen = 0;
	TAlScore perfectScore = 0, operfectScore = 0, bestPairScore = 0;
	size_t i = 0;
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
	Replay a;                      // the anchor's DP (SwAligner swa)
	bool firstInner = true;
	int res_kind = 0;              // the anchor result in hand: FOUND_EE_ / FOUND_UNGAPPED_ / FOUND_NONE_ (resGap_)
	// the opposite mate (extendSeedsPaired)
	Replay o;                      // the opposite mate's DP (SwAligner oswa)
	bool foundConcordant = false, foundMate = false, didAnchor = false;
	TRefOff off = 0;
	TAlScore ominsc_cur = 0;
	int oreadGaps = 0, orefGaps = 0;
	bool oleft = false, ofw = false;
	int64_t oll = 0, olr = 0, orl = 0, orr = 0;
	DPRect orect;

	SwResult* res_ptr() { return res_kind == FOUND_EE_ ? &resEe_ : res_kind == FOUND_UNGAPPED_ ? &resUngap_ : &resGap_; }
	EIvalMergeListBinned& seenDiags() { return anchor1 ? seenDiags1_ : seenDiags2_; }

	// SwDriver::prioritizeSATups restated flat (prio_flat, below): the picks as
	// (range in satpos2_, element) pairs, materialised only as the loop reaches them
	struct PrioEnt {
		uint32_t src, elt;     // satpos2_ index; element, or WHOLE (a small range, all of it)
		int32_t rnd;           // WHOLE: its Random1toN in rands_ (-1 until the loop gets there)
		uint8_t done;          // one element: given out
	};
	static constexpr uint32_t WHOLE = 0xFFFFFFFFu;
	std::vector<PrioEnt> pe_;
	bool lazy_ = false;        // the loop's ranges are pe_ (else satpos_/rands_/gws_, eeSaTups)
	void prio_flat(const Read& read, SeedResults& sh, const Ebwt& ebwtFw, const Ebwt* ebwtBw, int seedmms,
	               size_t maxelt, bool doExtend, AlignmentCacheIface& ca, RandomSource& rnd, PerReadMetrics& prm,
	               size_t& nelt_out, bool all, RefTables& tab);
	size_t n_ent() const { return lazy_ ? pe_.size() : gws_.size(); }
	size_t ent_size(size_t k) const {
		if(!lazy_) return satpos_[k].sat.size();
		return pe_[k].elt == WHOLE ? satpos2_[pe_[k].src].sat.size() : 1;
	}
	const SeedPos& ent_pos(size_t k) const { return lazy_ ? satpos2_[pe_[k].src].pos : satpos_[k].pos; }
	TIndexOffU ent_topf(size_t k) const {
		if(!lazy_) return satpos_[k].sat.topf;
		return satpos2_[pe_[k].src].sat.topf + (pe_[k].elt == WHOLE ? 0 : pe_[k].elt);
	}
	uint32_t ent_len(size_t k) const { return lazy_ ? satpos2_[pe_[k].src].sat.key.len : satpos_[k].sat.key.len; }
	TSlice ent_offs(size_t k) const {
		if(!lazy_) return satpos_[k].sat.offs;
		const SATupleAndPos& p = satpos2_[pe_[k].src];
		if(pe_[k].elt == WHOLE) return p.sat.offs;
		TSlice o;
		o.init(p.sat.offs, pe_[k].elt, pe_[k].elt + 1);
		return o;
	}
	TIndexOffU ent_off(size_t k, size_t e) const {
		if(!lazy_) return satpos_[k].sat.offs[e];
		const SATupleAndPos& p = satpos2_[pe_[k].src];
		return p.sat.offs[(pe_[k].elt == WHOLE ? 0 : pe_[k].elt) + e];
	}
	std::vector<R1N> lr_, lr2_;   // the lazy path's Random1toNs: picks' small ranges; prio_flat's (rands2_)
	size_t nlr_ = 0;              // lr_ entries in use
	R1N& ent_rand(size_t k, bool all_) {
		PrioEnt& e = pe_[k];
		if(e.rnd < 0) {           // a small range's Random1toN, made when first needed (init draws nothing)
			if(nlr_ == lr_.size()) lr_.emplace_back();
			lr_[nlr_].init(satpos2_[e.src].sat.size(), all_);
			e.rnd = (int32_t)nlr_++;
		}
		return lr_[e.rnd];
	}
	bool ent_done(size_t k) {
		if(!lazy_) return rands_[k].done();
		if(pe_[k].elt != WHOLE) return pe_[k].done != 0;
		return ent_rand(k, all).done();
	}
	size_t ent_next(size_t k, RandomSource& rnd) {
		if(!lazy_) return rands_[k].next(rnd);
		if(pe_[k].elt != WHOLE) {   // Random1toN of one: 0, no draw (random_util.h:88-94)
			pe_[k].done = 1;
			return 0;
		}
		return ent_rand(k, all).next(rnd);
	}
	void ent_set_done(size_t k) {
		if(!lazy_) rands_[k].setDone();
		else if(pe_[k].elt != WHOLE) pe_[k].done = 1;
		else ent_rand(k, all).setDone();
	}
	int ext_step(Driver& d, Slot& s);          // extendSeeds
	int ext_step_paired(Driver& d, Slot& s);   // extendSeedsPaired
	bool need_dp(Driver& d, Slot& s, int m, bool f, TIndexOffU ti, TRefOff tl, const DPRect& r, TAlScore ms,
	             bool extend, bool spec, bool force_cpu, Replay& rp);
	void speculate(Driver& d, Slot& s, std::vector<DpRes*>& out, size_t k);
	bool replay_next(Driver& d, Slot& s, Replay& rp, bool opp, TAlScore ms, SwResult& res);
	bool replay_done(Driver& d, const Replay& rp, bool opp) const;
	bool dp_found(Driver& d, Slot& s, Replay& rp, bool opp, TAlScore ms, TAlScore& bestCell);
};

// A connection's read buffer the driver took from the factory's ready queue
// (PSFactory::ReadAhead's element).  Its reads are copied into slots and the
// buffer goes back to its connection soon -- but a connection ends (its
// AlnSinkSam and OutputQueue are destroyed, pat.cpp:2016-2086) once every
// buffer of it has come back after its input ran out, so one buffer per
// connection, the latest, is held until every read of the connection taken so
// far has finished (Conn below).
struct Elem {
	ReadElement re;
	const void* conn = nullptr;     // the connection: its AlnSink
	explicit Elem(const ReadElement& r) : re(r) {}
};

// Per connection: buffers taken and not returned + reads in flight, and the
// held buffer.
struct Conn {
	long live = 0;
	Elem* last = nullptr;
};

// Buffer elements are made by a driver's feeder and freed by whichever driver
// returns the buffer: recycled through one pool rather than the allocator (a
// block freed on another thread than it was made on travels through the
// allocator's shared depot).
std::mutex g_elem_mu;
std::vector<Elem*> g_elem_pool;
Elem* elem_new(const ReadElement& re) {
	Elem* e = nullptr;
	{
		std::lock_guard<std::mutex> lk(g_elem_mu);
		if(!g_elem_pool.empty()) {
			e = g_elem_pool.back();
			g_elem_pool.pop_back();
		}
	}
	if(!e) return new Elem(re);
	e->~Elem();                               // (ReadElement holds a reference: rebuilt in place)
	return new (e) Elem(re);
}
void elem_free(Elem* e) {
	std::lock_guard<std::mutex> lk(g_elem_mu);
	g_elem_pool.push_back(e);
}
std::mutex g_conn_mu;
std::unordered_map<const void*, Conn> g_conns;

enum {
	P_START = 0, P_AFTER_EXACT, P_EXT_EXACT, P_1MM, P_AFTER_1MM, P_EXT_1MM, P_ROUND, P_AFTER_SEEDS, P_EXT_SEEDS,
	P_FINISH
};

// Engine results of one mate.
struct MateRes {
	// (result vectors sized up front: the services' workers fill them, and a
	// vector grown on one worker and regrown on another moves its blocks between
	// threads through the allocator's shared depot)
	MateRes() {
		mm.reserve(64);
		sd_out.reserve(256);
		sd_ext.reserve(64);
		pf_rows.reserve(160);
		sd_rows.reserve(160);
	}
	uint32_t sweep[8] = {0};
	bool sweep_asked = false;
	int32_t mm_minsc = 0;
	int mm_nofw = 0, mm_norc = 0;
	bool mm_asked = false;
	// the 1-mm search prefetched with the exact sweep (bt2g_exact_sweep_1mm):
	// pf_want set when the sweep is asked, pf_ok when it ran within the cap;
	// taken only for the identical request (flags and minsc)
	bool pf_want = false, pf_ok = false;
	int pf_nofw = 0, pf_norc = 0;
	int32_t pf_minsc = 0;
	// (row, offset) of the rows of the small exact / 1-mm ranges, resolved in the
	// same call, sorted by row: resolve_rows_request takes them from here
	std::vector<std::pair<uint32_t, uint32_t>> pf_rows;
	std::vector<bt2g_mm1> mm;
	int32_t mm_cnt = 0;
	uint32_t mm_ops = 0;
	// seed search (a round's; round 0's asked with the exact sweep, its arguments
	// being known when the read is set up)
	bool sd_ready = false;
	uint32_t sd_L = 0, sd_per = 0, sd_off = 0, sd_nof = 0;
	std::vector<uint32_t> sd_out;      // [strand][offset][topf, botf, topb, botb]
	// with the seed search (bt2g_seed_search_ext): SwDriver::extend of each seed's
	// range ([strand][offset]; empty when not asked) and the (row, offset) of the
	// small ranges' rows, sorted by row (the seed-extension stage's two requests)
	std::vector<bt2g_ext_out> sd_ext;
	std::vector<std::pair<uint32_t, uint32_t>> sd_rows;
	int32_t sd_ns = 0;
	uint32_t sd_ops = 0;
	// row in this round's engine call
	uint64_t row_stamp = ~0ull;
	uint32_t row = 0;
	// seeds instantiated this round (instantiateSeeds, aligner_seed.cpp:556-580)
	uint64_t valid_fw = 0, valid_rc = 0;
	std::vector<uint64_t> valid_big;   // (reads with more than 64 seed offsets per strand)
};

// One read (pair) in flight.  Owns the reference's per-read objects a worker
// thread owns (bt2_search.cpp:3086-3176), reused read after read.
struct Slot {
	Slot(const ReportingParams& rp, Mapq& mapq, size_t tid)
		: scCurrent((uint64_t)R_seedCacheCurrentMB * 1024 * 1024, false),
		  ca(&scCurrent, NULL, NULL),
		  sd((size_t)R_exactCacheCurrentMB * 1024 * 1024),
		  msinkwrap(rp, mapq, tid) {
		ext_in.reserve(64);
		ext_out.reserve(64);
		off_rows.reserve(1024);
		off_vals.reserve(1024);
		off_where.reserve(1024);
		ug_ed.reserve(64);
		dps.reserve(64);
	}
	AlignmentCache scCurrent;
	AlignmentCacheIface ca;
	SwDriverB sd;
	SeedResults shs[2];
	AlnSinkWrap msinkwrap;
	RandomSource rnd;
	PerReadMetrics prm;
	EList<Seed> seeds[2];
	Constraint gc = Constraint::penaltyFuncBased(R_scoreMin);   // (a Seed points at it)
	EList<uint32_t> offIdx2off;
	RefTables tab;

	// the read (pair): copies of the buffer's reads
	Read rdbuf[2];
	const void* conn = nullptr;
	Read* rds[2] = {&rdbuf[0], &rdbuf[1]};
	TReadId rdid = 0;
	AlnSink* msink = nullptr;
	bool paired = false;

	// multiseedSearchWorker's per-read locals (bt2_search.cpp:3283-3451, 3814-3823)
	int pc = P_START;
	uint32_t nsteps = 0;         // rounds this read was stepped in
	size_t rdlens[2] = {0, 0};
	TAlScore minsc[2] = {0, 0};
	bool nfilt[2] = {true, true}, scfilt[2] = {true, true}, lenfilt[2] = {true, true}, qcfilt[2] = {true, true};
	bool filt[2] = {true, true}, nofw[2] = {false, false}, norc[2] = {false, false}, done[2] = {false, false};
	bool exhaustive[2] = {false, false}, yfw[2] = {false, false}, yrc[2] = {false, false};
	int nceil[2] = {0, 0}, interval[2] = {0, 0}, seedlens[2] = {0, 0};
	size_t streak[2] = {0, 0}, mtStreak[2] = {0, 0}, mxDp[2] = {0, 0}, mxUg[2] = {0, 0}, mxIter[2] = {0, 0};
	size_t nrounds[2] = {0, 0}, nelt[2] = {0, 0}, minedfw[2] = {0, 0}, minedrc[2] = {0, 0};
	size_t matemap[2] = {0, 1};
	size_t matei = 0, roundi = 0;
	size_t seedsTried = 0, seedsTriedMS[4] = {0, 0, 0, 0};
	size_t nUniqueSeeds = 0, nRepeatSeeds = 0, seedHitTot = 0;
	size_t nUniqueSeedsMS[4] = {0, 0, 0, 0}, nRepeatSeedsMS[4] = {0, 0, 0, 0}, seedHitTotMS[4] = {0, 0, 0, 0};
	size_t round_off[2] = {0, 0};       // this round's seed offset per mate
	bool round_go[2] = {false, false};  // (the round searches this mate unless an earlier one stops it)

	MateRes mr[2];
	// pending requests of the extension loop (its anchor: sd.mate)
	std::vector<bt2g_ext_in> ext_in;
	std::vector<bt2g_ext_out> ext_out;
	std::vector<uint32_t> off_rows, off_vals;
	std::vector<std::pair<size_t, size_t>> off_where;
	bt2g_ug_problem ug_p{};
	bt2g_ug_result ug_r{};
	std::vector<bt2g_edit> ug_ed;
	// bytes this slot's objects grew by since it was built (allocations minus frees
	// on the driver thread while it was stepped; the construction's ~150 KB and
	// two 20 MB pools, ds.h Pool, mostly untouched, not counted): past $BT2G_SLOT_MAX_KB the slot is
	// rebuilt when its read finishes, so a slot does not keep the high-water
	// mark of every read it ever served (ELists keep their capacity)
	long long mem = 0;
	size_t idx = 0;                  // position in Driver::all
	// the read's DP table (asked and speculative DPs)
	std::vector<std::unique_ptr<DpRes>> dps;
	size_t ndps = 0;
	DpRes* new_dp() {
		if(ndps == dps.size()) dps.emplace_back(new DpRes());
		DpRes* r = dps[ndps++].get();
		r->ready = r->cpu = false;
		r->naln = 0;
		return r;
	}
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

struct Rq {
	Slot* s;
	int m;         // mate
};

// ---- engine services -------------------------------------------------------------
// The engine calls of a round, by kind.  With $BT2G_SERVICES (default on) each
// kind has a thread of its own per device (a context and stream of its own):
// the drivers hand it their requests of the round and wait; it takes whatever
// every driver has pending, makes ONE call for all of it and returns the
// results to the slots.  So a round's calls of the different kinds run at the
// same time (a round waits for its slowest kind, not for their sum), and the
// calls carry the requests of every driver (fewer, bigger launches, and one
// stream per kind instead of one per driver and kind).  Off: a driver makes
// its calls itself, one after another, on its own context.
struct Driver;
// A driver's reads are split in two lanes ($BT2G_LANES; default 2, --local 1): while one lane's
// requests are with the services, the driver steps the other lane's reads, so
// a round costs max(stepping, waiting) instead of their sum.
struct Lane {
	std::vector<Rq> rq[K_N];                        // this lane's requests of its round, by kind
	std::vector<std::pair<Slot*, DpRes*>> rq_dp;
	std::vector<Slot*> run, next;                   // its reads to step, and those stepped
	int outstanding = 0;                            // kinds handed to services (Driver::out_mu)
	Driver* d = nullptr;
};
struct Svc {
	int kind = 0;
	bt2g_ctx* ctx = nullptr;
	bool cu_masked = false;     // the DP worker's stream is on a CU share by default (--local)
	const bt2g_scoring* bsc = nullptr;
	uint64_t stamp = 0;
	// the kind's queue (its first worker's): drivers with requests of this kind;
	// the kind's workers ($BT2G_SVC_WORKERS, DP $BT2G_DP_WORKERS) each take what is
	// pending when they are free, on contexts of their own
	Svc* q = this;
	std::vector<Svc*> workers;
	std::mutex mu;
	std::condition_variable cv;
	std::vector<Lane*> pending;
	// $BT2G_KPROF=1: the engine's per-launch kernel times (HIP events on the
	// context's stream, bt2g_set_profiling) by kernel id, cumulative; and the
	// algorithmic work of the calls -- FM kinds: bytes (64 B per occurrence-table
	// side gathered + the read bytes walked, bench.py's figures), DP: cells
	std::mutex st_mu;
	uint64_t k_launch[16] = {};     // bt2g_kernel_stats ids 0-15
	double k_ms[16] = {};
	std::atomic<uint64_t> work{0}, items{0};
	// algorithmic work by kernel id (same figures, per kernel of a fused call: the
	// sweep's call also runs the 1-mm search (id 2), the seed call the ranges'
	// extension (id 12)); and the seed ranges extended ahead vs. taken
	std::atomic<uint64_t> kwork[16] = {}, kitems[16] = {};
	void loop();
	void run(std::vector<Rq>& v, std::vector<std::pair<Slot*, DpRes*>>& dp);
	// the calls
	void call_exact(std::vector<Rq>& v);
	void call_1mm(std::vector<Rq>& v);
	void call_seeds(std::vector<Rq>& v);
	void call_ext(std::vector<Rq>& v);
	void call_off(std::vector<Rq>& v);
	void call_ug(std::vector<Rq>& v);
	void call_dp(std::vector<std::pair<Slot*, DpRes*>>& v);
	void run_dp(const std::vector<std::pair<Slot*, DpRes*>>& v, uint32_t cap, uint32_t maxaln, uint32_t me);
	uint32_t row_of(Pack& pk, Slot& s, int m);
};

std::atomic<uint64_t> g_stamp{0};
std::atomic<bool> g_paired_seen{false};   // a read pair was admitted (Driver::admit)

// $BT2G_MM_PREFETCH=0: no 1-mm search with the exact sweep
bool mm_prefetch_on() {
	static const bool on = [] { const char* e = getenv("BT2G_MM_PREFETCH"); return !(e && *e == '0'); }();
	return on;
}

// $BT2G_SEED_PREFETCH=0: the seed search without its ranges' extension and rows
bool seed_prefetch_on() {
	static const bool on = [] { const char* e = getenv("BT2G_SEED_PREFETCH"); return !(e && *e == '0'); }();
	return on;
}

bool kprof_on() {
	static const bool on = [] { const char* e = getenv("BT2G_KPROF"); return e && *e == '1'; }();
	return on;
}

// The calls' algorithmic work by kernel id (bytes, DP cells): with $BT2G_KPROF,
// or alone with $BT2G_KWORK=1 -- a rocprofv3 --pmc pass of the same command
// then sets the counters' HBM bytes against the work of the same dispatches
// (bench.py pmc_ratio) without the engines' own HIP events under the profiler.
bool kwork_on() {
	static const bool on = [] { const char* e = getenv("BT2G_KWORK"); return kprof_on() || (e && *e == '1'); }();
	return on;
}

bool services_on() {
	static const bool on = [] { const char* e = getenv("BT2G_SERVICES"); return !(e && *e == '0'); }();
	return on;
}

// ---- one driver thread --------------------------------------------------------
struct Driver {
	explicit Driver(int tid_) : tid(tid_), swcpu(nullptr), oswcpu(nullptr) {}
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
	std::unique_ptr<PairedEndPolicy> pepol;
	// per-thread reference objects (CPU paths; metrics)
	SeedAligner al;
	SwAligner swcpu, oswcpu;
	SeedSearchMetrics sdm;
	WalkMetrics wlm;
	SwMetrics swmSeed, swmMate;
	ReportingMetrics rpm;
	// slots
	std::vector<std::unique_ptr<Slot>> all;
	std::vector<Slot*> freel;
	Lane lanes[2];
	Lane* cur = &lanes[0];               // the lane being stepped (admitted reads join it)
	size_t active = 0;
	// reads in: a feeder thread pops the factory's ready queue for this driver
	std::mutex in_mu;
	std::condition_variable in_cv, room_cv;
	std::vector<Elem*> inbox, got;   // (swapped each round: no allocation once grown)
	size_t max_slots = 1024;         // reads in flight per driver ($BT2G_BATCH_SLOTS)
	long long slot_max = 1 << 20;     // a slot's bytes past which it is rebuilt ($BT2G_SLOT_MAX_KB)
	std::atomic<size_t> active_a{0}; // `active` for the feeder
	// requests of this round: the stepping lane's lists
	std::vector<Rq>* rq = lanes[0].rq;
	std::vector<std::pair<Slot*, DpRes*>>* rq_dp = &lanes[0].rq_dp;
	size_t spec_k = 8;
	// the engine calls: the device's services, or (services off) the driver's own
	Svc* svc[K_N] = {};
	Svc own;
	std::mutex out_mu;
	std::condition_variable out_cv;
	void svc_done(Lane* l);

	void feeder();
	void run_loop();
	void admit(Elem* e);
	void release(Slot* s);
	void step_read(Slot& s);
	void setup_read(Slot& s);
	void submit(Lane& l);
	void wait(Lane& l);
	void prefetch_seeds(Slot& s, int mate);
	void cpu_dp(Slot& s, DpRes& r, SwAligner& sw);

	// helpers
	bool seeds_valid(const MateRes& m, bool fw, size_t i) const;
	void set_valid(MateRes& m, bool fw, size_t i);
	void resolve_rows_request(Slot& s);
	void take_offsets(Slot& s);
	void after_seeds(Slot& s, int mate);
	int instantiate(Slot& s, int mate, size_t offset);
	bool engine_read(const Slot& s, int m) const { return s.rdlens[m] > 0 && s.rdlens[m] <= BT2G_MAX_READ_LEN; }
	int ext(Slot& s) { return s.sd.paired ? s.sd.ext_step_paired(*this, s) : s.sd.ext_step(*this, s); }
};

uint32_t Svc::row_of(Pack& pk, Slot& s, int m) {
	MateRes& x = s.mr[m];
	if(x.row_stamp != stamp) {
		x.row_stamp = stamp;
		x.row = pk.add(*s.rds[m]);
	}
	return x.row;
}

// ---- the engine calls of one round ---------------------------------------------
// (grouped by each call's batch-wide arguments)
void Svc::call_exact(std::vector<Rq>& v) {
	if(v.empty()) return;
	thread_local Pack pk;
	thread_local std::vector<uint32_t> out;
	thread_local std::vector<int32_t> ms, cnt;
	thread_local std::vector<uint32_t> ops, offs, mld;
	thread_local std::vector<bt2g_mm1> h;
	const uint32_t cap = 16, off_cap = 8;
	for(int g = 0; g < 8; g++) {
		// (reads grouped by their strand options, and by whether their 1-mm search
		// rides along: bt2g_exact_sweep_1mm)
		const bool nf = (g & 2) != 0, nr = (g & 1) != 0, pf = (g & 4) != 0;
		std::vector<Rq> sub;
		uint32_t stride = 1;
		for(const Rq& q : v)
			if(q.s->nofw[q.m] == nf && q.s->norc[q.m] == nr && q.s->mr[q.m].pf_want == pf) {
				sub.push_back(q);
				stride = std::max<uint32_t>(stride, (uint32_t)q.s->rdlens[q.m]);
			}
		if(sub.empty()) continue;
		pk.reset(stride);
		for(const Rq& q : sub) pk.add(*q.s->rds[q.m]);
		out.resize(8 * sub.size());
		const uint64_t t0 = now_us();
		int rc;
		if(pf) {
			const size_t n = sub.size();
			ms.resize(n);
			cnt.resize(n);
			ops.resize(n);
			h.resize(n * (size_t)cap);
			const size_t per = (size_t)(2 + cap) * off_cap;
			offs.resize(n * per);
			for(size_t i = 0; i < n; i++) ms[i] = sub[i].s->mr[sub[i].m].pf_minsc;
			mld.resize(n);
			rc = bt2g_exact_sweep_1mm(ctx, pk.codes.data(), pk.quals.data(), pk.stride, pk.lens.data(), (uint32_t)n, 2,
			                          nf ? 1 : 0, nr ? 1 : 0, 0, ms.data(), bsc, cap, out.data(), h.data(), cnt.data(),
			                          ops.data(), kwork_on() ? mld.data() : nullptr, off_cap, offs.data());
			if(kwork_on() && !rc) {
				// the 1-mm search's bytes: 64 B per side + the read and its qualities walked
				// per strand (as call_1mm counts them); the reads it ran on
				uint64_t w = 0, k = 0;
				for(size_t i = 0; i < n; i++)
					if(mld[i]) {
						w += 64ull * mld[i] + 4ull * pk.lens[i];
						k++;
					}
				kwork[2] += w;
				kitems[2] += k;
			}
			for(size_t i = 0; i < n && !rc; i++) {
				MateRes& x = sub[i].s->mr[sub[i].m];
				// the resolved rows of the small ranges (slots: fw, rc exact ranges, 1-mm hits)
				x.pf_rows.clear();
				for(uint32_t slot = 0; slot < 2 + cap; slot++) {
					uint32_t top = 0, bot = 0;
					if(slot < 2) {
						if(out[8 * i + slot] == 0) { top = out[8 * i + 2 + 2 * slot]; bot = out[8 * i + 3 + 2 * slot]; }
					} else if((int32_t)(slot - 2) < std::min<int32_t>(cnt[i], (int32_t)cap)) {
						top = h[i * cap + slot - 2].top;
						bot = h[i * cap + slot - 2].bot;
					}
					if(bot <= top || bot - top > off_cap) continue;
					for(uint32_t j = 0; j < bot - top; j++) {
						const uint32_t o = offs[i * per + (size_t)slot * off_cap + j];
						if(o != OFF_MASK) x.pf_rows.emplace_back(top + j, o);
					}
				}
				std::sort(x.pf_rows.begin(), x.pf_rows.end());
				// the gate bt2g_exact_sweep_1mm applied (include/bt2g.h)
				const uint32_t mfw = out[8 * i], mrc = out[8 * i + 1];
				const bool yfw = mfw <= 1 && !nf, yrc = mrc <= 1 && !nr;
				const bool ran = yfw || yrc;
				x.pf_ok = ran && cnt[i] <= (int32_t)cap;
				if(!x.pf_ok) continue;
				g_mm_pf++;
				x.pf_nofw = yfw ? 0 : 1;
				x.pf_norc = yrc ? 0 : 1;
				x.mm_cnt = cnt[i];
				x.mm_ops = ops[i];
				x.mm.assign(&h[i * cap], &h[i * cap] + cnt[i]);
			}
		} else {
			rc = bt2g_exact_sweep(ctx, pk.codes.data(), pk.stride, pk.lens.data(), pk.n(), 2, nf ? 1 : 0, nr ? 1 : 0,
			                      out.data());
		}
		g_call_us[K_EXACT] += now_us() - t0;
		g_calls[K_EXACT]++;
		if(rc) die("bt2g_exact_sweep", rc);
		uint64_t w = 0;
		for(size_t i = 0; i < sub.size(); i++) {
			memcpy(sub[i].s->mr[sub[i].m].sweep, &out[8 * i], 8 * sizeof(uint32_t));
			w += 64ull * out[8 * i + 7] + 2ull * pk.lens[i];
		}
		work += w;
		items += sub.size();
		kwork[0] += w;
		kitems[0] += sub.size();
	}
	g_req[K_EXACT] += v.size();
}

void Svc::call_1mm(std::vector<Rq>& v) {
	if(v.empty()) return;
	thread_local Pack pk;
	thread_local std::vector<int32_t> ms, cnt;
	thread_local std::vector<uint32_t> ops;
	thread_local std::vector<bt2g_mm1> h;
	thread_local std::vector<uint32_t> ld;
	for(int g = 0; g < 4; g++) {
		const int nf = (g >> 1) & 1, nr = g & 1;
		std::vector<Rq> sub;
		uint32_t stride = 1;
		for(const Rq& q : v)
			if(q.s->mr[q.m].mm_nofw == nf && q.s->mr[q.m].mm_norc == nr) {
				sub.push_back(q);
				stride = std::max<uint32_t>(stride, (uint32_t)q.s->rdlens[q.m]);
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
				pk.add(*sub[i].s->rds[sub[i].m]);
				ms[i] = sub[i].s->mr[sub[i].m].mm_minsc;
			}
			const uint64_t t0 = now_us();
			ld.resize(n);
			int rc = bt2g_one_mm(ctx, pk.codes.data(), pk.quals.data(), pk.stride, pk.lens.data(), (uint32_t)n, ms.data(),
			                     bsc, nf, nr, cap, h.data(), cnt.data(), ops.data(), kwork_on() ? ld.data() : nullptr);
			if(kwork_on()) {
				uint64_t w = 0;
				for(size_t i = 0; i < n; i++) w += 64ull * ld[i] + 4ull * pk.lens[i];
				work += w;
				items += n;
				kwork[2] += w;
				kitems[2] += n;
			}
			g_call_us[K_1MM] += now_us() - t0;
			g_calls[K_1MM]++;
			if(rc && rc != BT2G_ERR_OVERFLOW) die("bt2g_one_mm", rc);
			std::vector<Rq> again;
			uint32_t cap2 = cap;
			for(size_t i = 0; i < n; i++) {
				MateRes& x = sub[i].s->mr[sub[i].m];
				if(cnt[i] > (int32_t)cap) {        // more hits than the slots: all of them, in order, next pass
					again.push_back(sub[i]);
					cap2 = std::max<uint32_t>(cap2, (uint32_t)cnt[i]);
					continue;
				}
				x.mm_cnt = cnt[i];
				x.mm_ops = ops[i];
				x.mm.assign(&h[i * cap], &h[i * cap] + cnt[i]);
			}
			sub.swap(again);
			cap = cap2;
		}
		if(!sub.empty()) die("bt2g_one_mm (rerun)", BT2G_ERR_OVERFLOW);
	}
	g_req[K_1MM] += v.size();
}

void Svc::call_seeds(std::vector<Rq>& v) {
	if(v.empty()) return;
	thread_local Pack pk;
	thread_local std::vector<uint32_t> out, ops, ld, offs;
	thread_local std::vector<bt2g_ext_out> ext;
	thread_local std::vector<int32_t> ns;
	const bool pf = seed_prefetch_on();
	const uint32_t OFF_CAP = 8;
	std::vector<bool> taken(v.size(), false);
	for(size_t a = 0; a < v.size(); a++) {
		if(taken[a]) continue;
		const MateRes& x0 = v[a].s->mr[v[a].m];
		std::vector<Rq> sub;
		uint32_t stride = 1, maxs = 1;
		for(size_t b = a; b < v.size(); b++) {
			const MateRes& x = v[b].s->mr[v[b].m];
			if(taken[b] || x.sd_L != x0.sd_L || x.sd_per != x0.sd_per || x.sd_off != x0.sd_off) continue;
			taken[b] = true;
			sub.push_back(v[b]);
			stride = std::max<uint32_t>(stride, (uint32_t)v[b].s->rdlens[v[b].m]);
			maxs = std::max(maxs, x.sd_nof);
		}
		pk.reset(stride);
		for(const Rq& q : sub) pk.add(*q.s->rds[q.m]);
		const size_t n = sub.size();
		out.resize(n * 2 * maxs * 4);
		ops.resize(n);
		ns.resize(n);
		const uint64_t t0 = now_us();
		ld.resize(n);
		if(pf) {
			ext.resize(n * 2 * maxs);
			offs.resize(n * 2 * maxs * OFF_CAP);
		}
		int rc = bt2g_seed_search_ext(ctx, pk.codes.data(), pk.stride, pk.lens.data(), (uint32_t)n, x0.sd_L, x0.sd_per,
		                              x0.sd_off, maxs, out.data(), ns.data(), ops.data(), kwork_on() ? ld.data() : nullptr,
		                              pf ? ext.data() : nullptr, OFF_CAP, pf ? offs.data() : nullptr);
		if(kwork_on()) {
			uint64_t w = 0;
			for(size_t i = 0; i < n; i++) w += 64ull * ld[i] + (uint64_t)std::max(ns[i], 0) * 2u * (x0.sd_L + 12u);
			work += w;
			items += n;
			kwork[1] += w;
			kitems[1] += n;
		}
		if(pf && !rc) {
			// the ranges' extension (k_seed_extend): 64 B per side gathered + one read
			// byte per LF step; every range with a hit, asked or not
			uint64_t w = 0, k = 0;
			for(size_t g = 0; g < n * 2 * maxs; g++)
				if(ext[g].fmops) {
					w += 64ull * ext[g].loads + ext[g].fmops;
					k++;
				}
			g_ext_spec += k;
			if(kwork_on()) {
				kwork[12] += w;
				kitems[12] += k;
			}
		}
		g_call_us[K_SEEDS] += now_us() - t0;
		g_calls[K_SEEDS]++;
		if(rc) die("bt2g_seed_search", rc);
		for(size_t i = 0; i < n; i++) {
			MateRes& x = sub[i].s->mr[sub[i].m];
			x.sd_ns = ns[i];
			x.sd_ops = ops[i];
			x.sd_out.assign(2 * (size_t)x.sd_nof * 4, 0);
			for(int f = 0; f < 2; f++)
				for(uint32_t k = 0; k < x.sd_nof && k < maxs; k++)
					memcpy(&x.sd_out[((size_t)f * x.sd_nof + k) * 4], &out[((i * 2 + f) * maxs + k) * 4], 16);
			x.sd_ext.clear();
			x.sd_rows.clear();
			if(pf) {
				x.sd_ext.assign(2 * (size_t)x.sd_nof, bt2g_ext_out{0, 0, 0, 0});
				for(int f = 0; f < 2; f++)
					for(uint32_t k = 0; k < x.sd_nof && k < maxs; k++) {
						const size_t g = (i * 2 + f) * maxs + k;
						x.sd_ext[(size_t)f * x.sd_nof + k] = ext[g];
						const uint32_t top = out[g * 4], bot = out[g * 4 + 1];
						if(bot > top && bot - top <= OFF_CAP)
							for(uint32_t j = 0; j < bot - top; j++)
								if(offs[g * OFF_CAP + j] != OFF_MASK) x.sd_rows.emplace_back(top + j, offs[g * OFF_CAP + j]);
					}
				std::sort(x.sd_rows.begin(), x.sd_rows.end());
			}
			x.sd_ready = true;
		}
	}
	g_req[K_SEEDS] += v.size();
}

void Svc::call_ext(std::vector<Rq>& v) {
	if(v.empty()) return;
	thread_local Pack pk;
	thread_local std::vector<bt2g_ext_in> in;
	thread_local std::vector<bt2g_ext_out> out;
	uint32_t stride = 1;
	for(const Rq& q : v) stride = std::max<uint32_t>(stride, (uint32_t)q.s->rdlens[q.m]);
	pk.reset(stride);
	in.clear();
	for(const Rq& q : v) {
		const uint32_t r = pk.add(*q.s->rds[q.m]);
		for(const bt2g_ext_in& x : q.s->ext_in) {
			in.push_back(x);
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
	if(kwork_on()) {
		uint64_t w = 0;
		for(const bt2g_ext_out& o : out) w += 64ull * o.loads + o.fmops;
		kwork[12] += w;
		kitems[12] += out.size();
	}
	size_t k = 0;
	for(const Rq& q : v) {
		q.s->ext_out.assign(out.begin() + k, out.begin() + k + q.s->ext_in.size());
		k += q.s->ext_in.size();
	}
	g_req[K_EXT] += v.size();
}

void Svc::call_off(std::vector<Rq>& v) {
	if(v.empty()) return;
	thread_local std::vector<uint32_t> rows, offs, ld;
	rows.clear();
	for(const Rq& q : v) rows.insert(rows.end(), q.s->off_rows.begin(), q.s->off_rows.end());
	offs.resize(rows.size());
	const uint64_t t0 = now_us();
	ld.resize(rows.size());
	int rc = bt2g_get_offset(ctx, rows.data(), (uint32_t)rows.size(), offs.data(), kwork_on() ? ld.data() : nullptr);
	if(kwork_on()) {
		uint64_t w = 0;
		for(uint32_t x : ld) w += 64ull * x + 12u;
		work += w;
		items += rows.size();
		kwork[3] += w;
		kitems[3] += rows.size();
	}
	g_call_us[K_OFF] += now_us() - t0;
	g_calls[K_OFF]++;
	if(rc) die("bt2g_get_offset", rc);
	// each read's offsets as one contiguous copy: its driver puts them where the
	// reference's walks leave them when it resumes the read (take_offsets).
	// (round 6: the scatter into the slots' cache pages had run here, ~1 ms per
	// call of ~50 k rows, between the kernel and the answer every driver of the
	// call was waiting for -- 87 % of this service's CPU in r06c's profile)
	size_t k = 0;
	for(const Rq& q : v) {
		Slot* s = q.s;
		const size_t m = s->off_rows.size();
		s->off_vals.assign(offs.begin() + (std::ptrdiff_t)k, offs.begin() + (std::ptrdiff_t)(k + m));
		k += m;
	}
	g_req[K_OFF] += v.size();
}

void Svc::call_ug(std::vector<Rq>& v) {
	if(v.empty()) return;
	thread_local Pack pk;
	thread_local std::vector<bt2g_ug_problem> P;
	thread_local std::vector<bt2g_ug_result> R;
	thread_local std::vector<bt2g_edit> E;
	uint32_t stride = 1;
	for(const Rq& q : v) stride = std::max<uint32_t>(stride, (uint32_t)q.s->rdlens[q.m]);
	pk.reset(stride);
	P.resize(v.size());
	for(size_t i = 0; i < v.size(); i++) {
		P[i] = v[i].s->ug_p;
		P[i].read = pk.add(*v[i].s->rds[v[i].m]);
	}
	const uint32_t maxedit = stride + 1;
	R.resize(v.size());
	E.resize(v.size() * (size_t)maxedit);
	const uint64_t t0 = now_us();
	int rc = bt2g_ungapped(ctx, pk.codes.data(), pk.quals.data(), pk.stride, pk.lens.data(), P.data(), (uint32_t)v.size(),
	                       bsc, gReportOverhangs ? 1 : 0, maxedit, R.data(), E.data());
	g_call_us[K_UG] += now_us() - t0;
	g_calls[K_UG]++;
	if(rc) die("bt2g_ungapped", rc);
	for(size_t i = 0; i < v.size(); i++) {
		v[i].s->ug_r = R[i];
		const int32_t ne = R[i].ret == 1 ? std::min<int32_t>(std::max<int32_t>(R[i].nedit, 0), (int32_t)maxedit) : 0;
		v[i].s->ug_ed.assign(&E[i * maxedit], &E[i * maxedit] + ne);
	}
	g_req[K_UG] += v.size();
}

// Fill + gather + the nextAlignment loop for every DP of the batch
// (bt2g_sw_align_bt_packed).  A DP whose candidate list outgrew `cap`, or that
// may have more than `maxaln` alignments, runs again alone with room for all;
// one with more candidates than the engine takes goes to the CPU when used.
void Svc::run_dp(const std::vector<std::pair<Slot*, DpRes*>>& v, uint32_t cap, uint32_t maxaln, uint32_t me) {
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
	const uint64_t tpre = now_us();
	uint32_t stride = 1;
	for(auto& q : v) stride = std::max<uint32_t>(stride, (uint32_t)q.first->rdlens[q.second->mate]);
	b.pk.reset(stride);
	stamp = g_stamp.fetch_add(1) + 1;   // (unique over the kind's workers: a slot's rows are per call)
	const size_t n = v.size();
	b.P.resize(n);
	b.RC.resize(n);
	for(size_t i = 0; i < n; i++) {
		const DpRes& r = *v[i].second;
		bt2g_sw_problem& p = b.P[i];
		memset(&p, 0, sizeof(p));
		p.read = row_of(b.pk, *v[i].first, r.mate);
		p.fw = r.fw;
		p.refl = r.refl;
		p.win_off = -1;                 // the engine's HBM-resident reference (initRef's window)
		p.refidx = r.refidx;
		p.ncol = r.ncol;
		p.minsc = r.minsc;
		b.RC[i] = r.rect;
	}
	if(kwork_on()) {
		uint64_t cells = 0;
		for(size_t i = 0; i < n; i++) cells += (uint64_t)b.pk.lens[b.P[i].read] * b.P[i].ncol;
		work += cells;
		items += n;
		kwork[4] += cells;
		kitems[4] += n;
	}
	// edits stored per alignment: `me` (0: all an alignment can have, 2 x stride + 8);
	// an alignment with more runs again with room for all (the engine reports
	// the true count).  The output blocks are sized nprob x maxaln x maxedit:
	// the full bound made ~20 KB of pinned staging per DP
	const uint32_t full = 2 * stride + 8;
	const uint32_t maxedit = me && me < full ? me : full;
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
	g_dp_pre_us += t0 - tpre;
	int rc = bt2g_sw_align_bt_packed(ctx, b.pk.codes.data(), b.pk.quals.data(), b.pk.stride, b.pk.lens.data(), b.P.data(),
	                                 (uint32_t)n, nullptr, 0, b.RC.data(), bsc, R_enable8 ? 1 : 0, cap, b.R.data(),
	                                 maxaln, maxedit, b.NA.data(), b.A.data(), b.C.data(), b.F.data(), b.E.data(), tot);
	const uint64_t t1 = now_us();
	g_call_us[K_DP] += t1 - t0;
	g_calls[K_DP]++;
	if(rc && rc != BT2G_ERR_OVERFLOW) die("bt2g_sw_align_bt_packed", rc);
	std::vector<std::pair<Slot*, DpRes*>> again;
	uint32_t cap2 = cap, maxaln2 = maxaln, me2 = me;
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
		bool trunc = false;
		for(uint32_t k = 0; k < na; k++) trunc = trunc || b.A[i * maxaln + k].nedit > (int32_t)maxedit;
		if(o.ncand > (int32_t)cap || (b.NA[i] == (int32_t)maxaln && o.ncand > (int32_t)maxaln) || trunc) {
			again.push_back(v[i]);
			if(o.ncand > (int32_t)cap) cap2 = std::max<uint32_t>(cap2, (uint32_t)o.ncand);
			if(b.NA[i] == (int32_t)maxaln && o.ncand > (int32_t)maxaln)
				maxaln2 = std::max<uint32_t>(maxaln2, (uint32_t)o.ncand);
			if(trunc) me2 = 0;
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
	g_dp_post_us += now_us() - t1;
	if(oc != tot[0] || oe != tot[2]) {
		fprintf(stderr, "bt2g batch: packed DP outputs %llu/%llu, expected %zu/%zu\n", (unsigned long long)tot[0],
		        (unsigned long long)tot[2], oc, oe);
		abort();
	}
	if(!again.empty()) {
		g_dp_again += again.size();
		run_dp(again, cap2, maxaln2, me2);
	}
}

void Svc::call_dp(std::vector<std::pair<Slot*, DpRes*>>& v) {
	if(v.empty()) return;
	g_req[K_DP] += v.size();
	// long reads (> 1024 bases) batch apart: a batch is padded to its longest read;
	// and DPs wider than twice their read (mate searches, ~150 x 700) apart from the
	// rest: the engine picks the walk for a whole call by its widest DP, and one
	// wide DP would send a call's seed extensions to the H-plane walk (r04v
	// paired: 14.5 ms DP calls) instead of the decision plane + workgroup walk
	// DPs wider than the engine's decision-plane ratio ($BT2G_DEC_RATIO, default 6,
	// the same variable and default as bt2g_api.cpp dec_ratio) go in calls of their
	// own too: one of them would send a whole call of mate searches to the H plane
	std::vector<std::pair<Slot*, DpRes*>> sh, wide, wider, lg;
	static const size_t ratio = env_or("BT2G_DEC_RATIO", 6);
	for(auto& q : v) {
		const size_t len = q.first->rdlens[q.second->mate], nc = q.second->ncol;
		(len > 1024 ? lg : nc > ratio * len ? wider : nc > 2 * len ? wide : sh).push_back(q);
	}
	const uint32_t cap = R_localAlign ? 2048 : 512;
	static const uint32_t me = (uint32_t)env_or("BT2G_DP_MAXEDIT", 48);
	if(!sh.empty()) run_dp(sh, cap, 8, me);
	if(!wide.empty()) run_dp(wide, cap, 8, me);
	if(!wider.empty()) run_dp(wider, cap, 8, me);
	if(!lg.empty()) run_dp(lg, cap, 8, me);
}

// A DP the engine does not take (reads at or above --cp-min, longer than
// BT2G_MAX_READ_LEN, or more candidates than the engine holds): the
// reference's own SwAligner, when the extension loop reaches it
// (aligner_sw_driver.cpp:1104-1139, 2029-2079).
void Driver::cpu_dp(Slot& s, DpRes& r, SwAligner& sw) {
	const Read& rd = *s.rds[r.mate];
	sw.reset();
	sw.initRead(rd.patFw, rd.patRc, rd.qual, rd.qualRev, 0, rd.length(), *sc);
	size_t nsInLeftShift = 0;
	sw.initRef(r.fw != 0, r.refidx, r.drect, const_cast<BitPairReference&>(*ref), r.tlen, *sc, r.minsc, R_enable8,
	           R_cminlen, R_cpow2, R_doTri, r.extend, 0, nsInLeftShift);
	TAlScore best = std::numeric_limits<TAlScore>::min();
	r.o.aligned = sw.align(best) ? 1 : 0;
	r.o.best = best == std::numeric_limits<TAlScore>::min() ? std::numeric_limits<int32_t>::min() : (int32_t)best;
	g_cpu[K_DP]++;
}

// ---- the extension loops ---------------------------------------------------------

// The DP the loop needs now: from the read's table, or requested (with up to
// spec_k - 1 speculative others for a seed extension).  Returns true when it is
// available (rp started), false when the slot must wait for this round's
// engine call.
//
// force_cpu: a mate search under an anchor the driver thread's own SwAligner
// is replaying -- no wait may come between (another slot would take that
// SwAligner), so the mate DP runs on the CPU too.
bool SwDriverB::need_dp(Driver& d, Slot& s, int m, bool f, TIndexOffU ti, TRefOff tl, const DPRect& r, TAlScore ms,
                        bool extend, bool spec, bool force_cpu, Replay& rp) {
	for(size_t k = 0; k < s.ndps && !force_cpu; k++) {
		DpRes* x = s.dps[k].get();
		if(!x->ready || !x->same_problem(m, f, (uint32_t)ti, r)) continue;
		bool ok = x->minsc == ms;
		if(!ok && !R_localAlign && !x->cpu && x->minsc < ms && u8_regime(x->minsc) == u8_regime(ms)) ok = true;
		if(!ok) continue;
		rp.start(x);
		g_dp_used++;
		if(x->minsc != ms) g_dp_reuse++;
		return true;
	}
	g_dp_miss++;
	DpRes* x = s.new_dp();
	x->mate = m;
	x->fw = f ? 1 : 0;
	x->refidx = (uint32_t)ti;
	x->refl = r.refl;
	x->ncol = (uint32_t)(r.refr + 1 - r.refl);
	x->rect.triml = (int32_t)r.triml;
	x->rect.corel = (int32_t)r.corel;
	x->rect.corer = (int32_t)r.corer;
	x->rect.pad = 0;
	x->minsc = (int32_t)ms;
	x->tlen = tl;
	x->extend = extend;
	x->drect = r;
	const size_t len = s.rdlens[m];
	const bool engine = !force_cpu && d.bsc_ok && len > 0 && len <= BT2G_MAX_READ_LEN && len < R_cminlen &&
	                    ms >= std::numeric_limits<int32_t>::min() && ms <= std::numeric_limits<int32_t>::max();
	if(!engine) {
		x->cpu = true;
		x->ready = true;
		rp.start(x);
		return true;
	}
	d.rq_dp->emplace_back(&s, x);
	if(spec && d.spec_k > 1) {
		std::vector<DpRes*> more;
		speculate(d, s, more, d.spec_k - 1);
		for(DpRes* q : more) d.rq_dp->emplace_back(&s, q);
		g_dp_spec += more.size();
	}
	rp.dp = x;
	return false;
}

// Up to k more seed-extension DPs this loop may ask for at the current minsc:
// one per element of the prioritised ranges whose row is resolved, on a
// diagonal not yet seen, framed exactly as the loop frames it
// (aligner_sw_driver.cpp:937-1097).
void SwDriverB::speculate(Driver& d, Slot& s, std::vector<DpRes*>& out, size_t k) {
	const int64_t ms = *minsc;
	if(eeMode) return;
	const int rg = d.sc->maxReadGaps(ms, rdlen), fg = d.sc->maxRefGaps(ms, rdlen);
	if(R_doUngapped && rg == 0 && fg == 0) return;
	DynProgFramer dpframe(!gReportOverhangs);
	struct Diag { uint32_t t; int64_t o; bool f; };
	std::vector<Diag> seen;
	// (speculation never changes a result -- a speculative DP serves only the same
	// problem asked later -- so where it looks is a matter of cost only)
	// (from the loop's current range i: the loop has left the ranges before it,
	// aligner_sw_driver.cpp:883-1030; r05i: resuming instead at a cursor past every
	// element examined so far asked 41 % more DPs for the same reads -- it skips
	// the elements whose rows the loop resolves as it goes, the ones it asks next)
	for(size_t ii = i; ii < n_ent() && out.size() < k; ii++) {
		const SeedPos& pos = ent_pos(ii);
		const bool f = pos.fw;
		uint32_t ro = pos.rdoff;
		if(!f) ro = (uint32_t)(rdlen - ro - pos.seedlen);
		const size_t esz = ent_size(ii);
		for(size_t e = 0; e < esz && out.size() < k; e++) {
			const TIndexOffU so = ent_off(ii, e);
			if(so == OFF_MASK) continue;
			TIndexOffU ti = 0, to = 0, tl = 0;
			bool straddled = false;
			d.ebwtFw->joinedToTextOff(ent_len(ii), so, ti, to, tl, false, straddled);
			if(ti == OFF_MASK) continue;
			const int64_t ro64 = (int64_t)to - ro;
			Coord c(ti, ro64, f);
			if(seenDiags().locusPresent(c)) continue;
			bool dup = (ti == tidx && ro64 == refoff && f == fw);
			for(const Diag& x : seen) dup = dup || (x.t == ti && x.o == ro64 && x.f == f);
			if(dup) continue;
			seen.push_back(Diag{(uint32_t)ti, ro64, f});
			DPRect r;
			if(!dpframe.frameSeedExtensionRect(ro64, rdlen, tl, rg, fg, (size_t)nceil, R_maxhalf, r)) continue;
			bool have = false;
			for(size_t q = 0; q < s.ndps && !have; q++) {
				const DpRes* x = s.dps[q].get();
				have = x->same_problem(mate, f, (uint32_t)ti, r) && x->minsc == (int32_t)ms;
			}
			if(have) continue;
			DpRes* q = s.new_dp();
			q->mate = mate;
			q->fw = f ? 1 : 0;
			q->refidx = (uint32_t)ti;
			q->refl = r.refl;
			q->ncol = (uint32_t)(r.refr + 1 - r.refl);
			q->rect.triml = (int32_t)r.triml;
			q->rect.corel = (int32_t)r.corel;
			q->rect.corer = (int32_t)r.corer;
			q->rect.pad = 0;
			q->minsc = (int32_t)ms;
			q->tlen = tl;
			q->extend = true;
			q->drect = r;
			out.push_back(q);
		}
	}
}

// SwAligner::align's outcome (aligner_sw.cpp:677-729) at minsc `ms` from the
// table entry (computed at a minsc <= ms, same fill width: see the header).
bool SwDriverB::dp_found(Driver& d, Slot& s, Replay& rp, bool opp, TAlScore ms, TAlScore& bestCell) {
	DpRes& r = *rp.dp;
	if(rp.cpu) {
		r.minsc = (int32_t)ms;
		d.cpu_dp(s, r, opp ? d.oswcpu : d.swcpu);
		bestCell = r.o.best == std::numeric_limits<int32_t>::min() ? std::numeric_limits<TAlScore>::min()
		                                                            : (TAlScore)r.o.best;
		return r.o.aligned != 0;
	}
	bestCell = r.o.best == std::numeric_limits<int32_t>::min() ? std::numeric_limits<TAlScore>::min()
	                                                            : (TAlScore)r.o.best;
	if(!r.o.aligned) return false;
	for(const bt2g_sw_cand& c : r.cands)
		if(c.score >= ms) return true;
	return false;
}

bool SwDriverB::replay_done(Driver& d, const Replay& rp, bool opp) const {
	if(rp.cpu) return (opp ? d.oswcpu : d.swcpu).done();
	return rp.cural == rp.dp->cands.size();
}

// nextAlignment(): the candidate list walked as aligner_sw.cpp:758-1140 walks
// it, with the engine's fate for each candidate: below `ms` FILT_SCORE (the
// caller may have tightened it since align()); FILT_START and FILT_DOMINATED
// consume no randomness; every tried candidate draws rnd.nextU32() and
// re-seeds rnd as the u8 / i16 branches do.
bool SwDriverB::replay_next(Driver& d, Slot& s, Replay& rp, bool opp, TAlScore ms, SwResult& res) {
	if(rp.cpu) return (opp ? d.oswcpu : d.swcpu).nextAlignment(res, ms, s.rnd);
	DpRes& r = *rp.dp;
	const size_t candsz = r.cands.size();
	const bool u8 = r.o.u8succ != 0;
	const size_t len = s.rdlens[r.mate];
	while(rp.cural < candsz) {
		const bt2g_sw_cand& c = r.cands[rp.cural];
		if(c.score < ms) {
			rp.cural++;
			continue;
		}
		const int f = r.fates[rp.cural];
		if(f == BT_CAND_FATE_FILT_START || f == BT_CAND_FATE_FILT_DOMINATED) {
			rp.cural++;
			continue;
		}
		if(f != BT_CAND_FATE_SUCCEEDED && f != BT_CAND_FATE_FAILED) {
			fprintf(stderr, "bt2g batch: candidate %zu of %zu has no engine fate (%d)\n", rp.cural, candsz, f);
			abort();
		}
		const uint32_t reseed = s.rnd.nextU32() + 1;
		res.reset();
		s.rnd.init(u8 ? reseed + 1 : reseed);
		if(f == BT_CAND_FATE_FAILED) {
			rp.cural++;
			continue;
		}
		if(rp.next >= (uint32_t)r.naln) {
			fprintf(stderr, "bt2g batch: engine returned %d alignments, reference wants more\n", r.naln);
			abort();
		}
		const bt2g_sw_aln& a = r.alns[rp.next];
		if(a.cand != (int32_t)rp.cural || a.nedit > (int32_t)r.maxedit) {
			fprintf(stderr, "bt2g batch: alignment %u is candidate %d, expected %zu\n", rp.next, a.cand, rp.cural);
			abort();
		}
		const bt2g_edit* ed = r.edits.data() + rp.next_edit;
		rp.next_edit += (size_t)a.nedit;
		rp.next++;
		// backtraceNucleotides*: setScore / setShape / setRefNs (aligner_swsse_ee_u8.cpp:1822-1847)
		const int based = (int)(len - (size_t)a.trim5p - (size_t)a.trim3p - (size_t)a.nedit);
		fill_alnres(res.alres, ed, (uint32_t)a.nedit, a.score, a.ns, a.gaps, based, (TRefId)r.refidx,
		            (TRefOff)a.off + r.refl, (TRefOff)r.tlen, r.fw != 0, len, (size_t)a.trim5p, (size_t)a.trim3p,
		            (size_t)a.refns);
		rp.cural++;
		return true;
	}
	res.reset();
	return false;
}

// The rows handed to GroupWalk2S::init by the call that just returned, as one
// engine request (bt2g_get_offset == Ebwt::getOffset, bt2_idx.cpp:150-171).
void Driver::resolve_rows_request(Slot& s) {
	const size_t MAX_ROWS = 8192;          // per read (the rest: Ebwt::getOffset in advanceElement)
	s.off_rows.clear();
	s.off_where.clear();
	const std::vector<std::pair<uint32_t, uint32_t>>* known[4] = {&s.mr[0].pf_rows, &s.mr[1].pf_rows, &s.mr[0].sd_rows,
	                                                               &s.mr[1].sd_rows};
	// the offsets of range x's rows that the sweep's or the seed call's small ranges
	// already brought (sorted (row, offset) lists), matched by a merge over the
	// range's rows: a read whose rows are all known makes no rows request -- no
	// round.  (round 6: was a binary search in each list per row, ~6 % of the
	// drivers' CPU; asking every row instead made 24 % more rounds, r06d)
	thread_local std::vector<uint32_t> kv;
	auto match = [&](TIndexOffU topf, size_t size) {
		kv.assign(size, OFF_MASK);
		for(const auto* L : known) {
			if(L->empty() || L->back().first < topf || L->front().first >= topf + size) continue;
			for(auto it = std::lower_bound(L->begin(), L->end(), std::make_pair((uint32_t)topf, 0u));
			    it != L->end() && it->first < topf + size; ++it)
				kv[it->first - topf] = it->second;
		}
	};
	for(size_t r = 0; r < s.tab.gw.size(); r++) {
		GwRange& x = s.tab.gw[r];
		if(x.fresh) {
			// (prio_flat's picks: nothing was written for them -- every row is
			// asked, or taken from a call that resolved it; past MAX_ROWS marked
			// unresolved, for advanceElement's CPU path)
			match(x.topf, x.size);
			for(size_t j = 0; j < x.size; j++) {
				if(kv[j] != OFF_MASK) {
					x.offs[j] = kv[j];
					g_rows_pf++;
				} else if(s.off_rows.size() < MAX_ROWS) {
					s.off_rows.push_back((uint32_t)(x.topf + j));
					s.off_where.emplace_back(r, j);
				} else {
					x.offs[j] = OFF_MASK;
				}
			}
			continue;
		}
		bool matched = false;
		for(size_t j = 0; j < x.size && s.off_rows.size() < MAX_ROWS; j++)
			if(x.offs[j] == OFF_MASK) {
				if(!matched) {
					match(x.topf, x.size);
					matched = true;
				}
				if(kv[j] != OFF_MASK) {
					x.offs[j] = kv[j];
					g_rows_pf++;
					continue;
				}
				s.off_rows.push_back((uint32_t)(x.topf + j));
				s.off_where.emplace_back(r, j);
			}
	}
	if(s.off_rows.empty()) {
		s.tab.gw.clear();
		return;
	}
	rq[K_OFF].push_back(Rq{&s, s.sd.mate});
}

// The preamble of both loops' first pass: eeSaTups for end-to-end hits, or
// SwDriver::extend for every seed-hit range + prioritizeSATups; then the rows
// they hand GroupWalk2S resolved.  Expanded into each loop (below) so that
// their resume points stay in one function each.
#define BT2GB_EE_SETUP(LABEL_ROWS)                                                                     \
	lazy_ = false;                                                                                     \
	s.tab.gw.clear();                                                                                  \
	s.tab.gw_on = true;                                                                                \
	t_tab = &s.tab;                                                                                    \
	{                                                                                                  \
		Ph ph_(PH_EESAT);                                                                              \
		eeMode = eeSaTups(rd, s.shs[mate], ebwtFw, ref, s.rnd, d.wlm, d.swmSeed, nelt, maxIters, all); \
	}                                                                                                  \
	s.tab.gw_on = false;                                                                               \
	t_tab = nullptr;                                                                                   \
	{                                                                                                  \
		Ph ph_(PH_ROWS);                                                                               \
		d.resolve_rows_request(s);                                                                     \
	}                                                                                                  \
	if(!s.off_rows.empty()) {                                                                          \
		pc = X_AFTER_EE_ROWS;                                                                          \
		return EXTEND_BLOCKED;                                                                         \
	}                                                                                                  \
	LABEL_ROWS:;

// every range the loop at aligner_sw_driver.cpp:519-604 visits, in its order,
// extended on the engine first (SwDriver::extend below reads the results)
static void ext_request(Driver& d, Slot& s, SwDriverB& x) {
	s.ext_in.clear();
	const size_t len = s.rdlens[x.mate];
	if(!(R_doExtend && d.ebwtBw != NULL && len > 0 && len <= BT2G_MAX_READ_LEN)) return;
	EList<SATuple, 16> sat;
	for(size_t k = 0; k < x.nonz; k++) {
		bool f = true;
		uint32_t offidx = 0, ro = 0, sl = 0;
		QVal qv = s.shs[x.mate].hitsByRank(k, offidx, ro, f, sl);
		size_t nr = 0, ne = 0;
		sat.clear();
		s.ca.queryQval(qv, sat, nr, ne);
		for(size_t j = 0; j < sat.size(); j++) {
			const TIndexOffU sz = (TIndexOffU)sat[j].size();
			bt2g_ext_in q;
			q.read = 0;
			q.fw = f ? 1 : 0;
			q.off = ro;
			q.len = sl;
			q.topf = sat[j].topf;
			q.botf = sat[j].topf + sz;
			q.topb = sat[j].topb;
			q.botb = sat[j].topb + sz;
			if(sz > 0 && ro + sl <= len) s.ext_in.push_back(q);
		}
	}
}

// The extend requests of ext_request answered from the seed call's results
// (MateRes::sd_ext) when every one of them is a seed of the round's search with
// the same range; else false and the engine is asked.
static bool ext_from_seeds(Slot& s, size_t mate) {
	const MateRes& x = s.mr[mate];
	if(x.sd_ext.size() != 2 * (size_t)x.sd_nof || x.sd_per == 0) return false;
	const uint32_t L = std::min<uint32_t>(x.sd_L, (uint32_t)s.rdlens[mate]);
	s.ext_out.resize(s.ext_in.size());
	for(size_t i = 0; i < s.ext_in.size(); i++) {
		const bt2g_ext_in& q = s.ext_in[i];
		if(q.off < x.sd_off || (q.off - x.sd_off) % x.sd_per != 0 || q.len != L) return false;
		const size_t k = (q.off - x.sd_off) / x.sd_per, f = q.fw ? 0 : 1;
		if(k >= x.sd_nof) return false;
		const uint32_t* o = &x.sd_out[(f * x.sd_nof + k) * 4];
		if(o[0] != q.topf || o[1] != q.botf || o[2] != q.topb || o[3] != q.botb) return false;
		s.ext_out[i] = x.sd_ext[f * x.sd_nof + k];
	}
	g_ext_pf += s.ext_in.size();
	return true;
}

// $BT2G_PRIO_REF=1: the reference's prioritizeSATups and GroupWalk2S objects
// instead of prio_flat (A/B; the SAM is the same either way)
static bool prio_ref() {
	static const bool on = [] { const char* e = getenv("BT2G_PRIO_REF"); return e && *e == '1'; }();
	return on;
}

// SwDriver::prioritizeSATups (aligner_sw_driver.cpp:490-738), restated for the
// batch driver.  Kept exactly: the seed-hit ranges and their order (hitsByRank,
// queryQval), the ranges an earlier extension covers (seedmms 0), the
// extensions (SwDriver::extend, served from the seed call's table), the sort,
// then the picks -- the first nsmall ranges whole (nsm 5), then single
// elements of the rest drawn by RowSampler (lengths and sizes squared) and
// each range's Random1toN, with the same draws from rnd in the same order, up
// to maxelt elements.  Changed: a pick is recorded as (range, element) in pe_;
// the SATuple, Random1toN and GroupWalk2S the reference builds for every pick
// are not built (the loop examines ~6 of a read's ~45 picks, r05r: 3.19 M
// GroupWalk2S::init for 0.43 M advanceElement over 70 k reads), and the picks'
// rows go to the rows request straight from pe_ (GwRange::fresh).  Random1toN::
// init draws nothing, so a small range's chooser is made when the loop gets to it.
void SwDriverB::prio_flat(const Read& read, SeedResults& sh, const Ebwt& ebwtFw, const Ebwt* ebwtBw, int seedmms,
                          size_t maxelt, bool doExtend, AlignmentCacheIface& ca, RandomSource& rnd,
                          PerReadMetrics& prm, size_t& nelt_out, bool all_, RefTables& tab) {
	const size_t nsm = 5;
	const int matei = read.mate <= 1 ? 0 : 1;
	satups_.clear();
	gws_.clear();
	rands_.clear();
	rands2_.clear();
	nlr_ = 0;
	satpos_.clear();
	satpos2_.clear();
	pe_.clear();
	lazy_ = true;
	size_t nrange = 0, nelt = 0, nsmall = 0;
	const size_t nz = sh.nonzeroOffsets();
	for(size_t h = 0; h < nz; h++) {
		bool hfw = true;
		uint32_t offidx = 0, hoff = 0, hlen = 0;
		QVal qv = sh.hitsByRank(h, offidx, hoff, hfw, hlen);
		ca.queryQval(qv, satups_, nrange, nelt);
		EList<ExtendRange>& exr = hfw ? seedExRangeFw_[matei] : seedExRangeRc_[matei];
		for(size_t j = 0; j < satups_.size(); j++) {
			const size_t sz = satups_[j].size();
			if(seedmms == 0) {
				// inside an extension already made, from a range no bigger: skipped
				bool covered = false;
				for(size_t k = 0; k < exr.size() && !covered; k++)
					covered = exr[k].off <= hoff && exr[k].off + exr[k].len >= (size_t)hoff + hlen && sz <= exr[k].sz;
				if(covered) {
					nrange--;
					nelt -= sz;
					continue;
				}
			}
			satpos2_.expand();
			SATupleAndPos& p = satpos2_.back();
			p.sat = satups_[j];
			p.origSz = sz;
			p.pos.init(hfw, offidx, hoff, hlen);
			if(sz <= nsm) nsmall++;
			size_t nlex = 0, nrex = 0;
			if(doExtend)
				extend(read, ebwtFw, ebwtBw, p.sat.topf, (TIndexOffU)(p.sat.topf + sz), p.sat.topb,
				       (TIndexOffU)(p.sat.topb + sz), hfw, hoff, hlen, prm, nlex, nrex);
			p.nlex = nlex;
			p.nrex = nrex;
			if(seedmms == 0 && (nlex > 0 || nrex > 0)) {
				exr.expand();
				exr.back().off = hoff - (hfw ? nlex : nrex);
				exr.back().len = hlen + nlex + nrex;
				exr.back().sz = sz;
			}
		}
		satups_.clear();
	}
	nelt_out = nelt;
	satpos2_.sort();
	size_t added = 0;
	for(size_t j = 0; j < nsmall && added < maxelt; j++) {
		pe_.push_back(PrioEnt{(uint32_t)j, WHOLE, -1, 0});
		added += satpos2_[j].sat.size();
	}
	if(added < maxelt && nsmall != satpos2_.size()) {
		rowsamp_.init(satpos2_, nsmall, satpos2_.size(), true, true);
		if(lr2_.size() < satpos2_.size()) lr2_.resize(satpos2_.size());
		for(size_t j = 0; j < satpos2_.size(); j++) lr2_[j].reset();
		while(added < maxelt && added < nelt) {
			const size_t ri = rowsamp_.next(rnd) + nsmall;
			R1N& rr = lr2_[ri];
			if(!rr.inited()) rr.init(satpos2_[ri].sat.size(), all_);
			const size_t r = rr.next(rnd);
			if(rr.done()) rowsamp_.finishedRange(ri - nsmall);
			pe_.push_back(PrioEnt{(uint32_t)ri, (uint32_t)r, -1, 0});
			added++;
		}
	}
	nelt_out = added;
	// the picks' rows, for the rows request (resolve_rows_request)
	tab.gw.clear();
	tab.gw.reserve(pe_.size());
	for(size_t k = 0; k < pe_.size(); k++)
		tab.gw.push_back(GwRange{ent_topf(k), ent_size(k), ent_offs(k), true});
}

// GroupWalk2S::advanceElement as the drop-in serves it (the specialisation
// below) for a prio_flat pick: the row's offset from the rows request, or
// Ebwt::getOffset on the CPU for a row past the request's cap.
static inline void adv_flat(TIndexOffU elt, const Ebwt& ebwtFw, SARangeWithOffs<TSlice>& sa, WalkResult& res,
                            WalkMetrics& met) {
	if(sa.offs[elt] == OFF_MASK) {
		sa.offs[elt] = ebwtFw.getOffset(sa.topf + elt);
		g_cpu[K_OFF]++;
	}
	met.reports++;
	res.init(0, false, 0, elt, sa.topf + elt, (TIndexOffU)sa.len, sa.offs[elt]);
}

#define BT2GB_PRIO_SETUP(LABEL_EXT, LABEL_ROWS)                                                        \
	ext_request(d, s, *this);                                                                          \
	if(!s.ext_in.empty() && ext_from_seeds(s, mate)) goto LABEL_EXT;                                   \
	if(!s.ext_in.empty()) {                                                                            \
		d.rq[K_EXT].push_back(Rq{&s, mate});                                                           \
		pc = X_AFTER_EXT;                                                                              \
		return EXTEND_BLOCKED;                                                                         \
	}                                                                                                  \
	s.ext_out.clear();                                                                                 \
	LABEL_EXT:                                                                                         \
	s.tab.ext_on = !s.ext_in.empty();                                                                  \
	s.tab.ext_keys.swap(s.ext_in);                                                                     \
	s.tab.ext_vals.swap(s.ext_out);                                                                    \
	s.tab.ext_next = 0;                                                                                \
	s.tab.gw.clear();                                                                                  \
	s.tab.gw_on = true;                                                                                \
	t_tab = &s.tab;                                                                                    \
	t_cpu_ext = &g_cpu[K_EXT];                                                                         \
	{                                                                                                  \
		Ph ph_(PH_PRIO);                                                                               \
		if(prio_ref()) {                                                                               \
			lazy_ = false;                                                                             \
			prioritizeSATups(rd, s.shs[mate], ebwtFw, d.ebwtBw, ref, seedmms, maxIters, R_doExtend, true, \
			                 true, 5, s.ca, s.rnd, d.wlm, s.prm, nelt, all);                           \
		} else {                                                                                       \
			prio_flat(rd, s.shs[mate], ebwtFw, d.ebwtBw, seedmms, maxIters, R_doExtend, s.ca, s.rnd,   \
			          s.prm, nelt, all, s.tab);                                                        \
		}                                                                                              \
	}                                                                                                  \
	s.tab.ext_on = false;                                                                              \
	s.tab.gw_on = false;                                                                               \
	t_tab = nullptr;                                                                                   \
	{                                                                                                  \
		Ph ph_(PH_ROWS);                                                                               \
		d.resolve_rows_request(s);                                                                     \
	}                                                                                                  \
	if(!s.off_rows.empty()) {                                                                          \
		pc = X_AFTER_PRIO_ROWS;                                                                        \
		return EXTEND_BLOCKED;                                                                         \
	}                                                                                                  \
	LABEL_ROWS:;

// Resolve the next element's offset and its reference coordinates
// (aligner_sw_driver.cpp:924-952, 1626-1651).
#define BT2GB_NEXT_ELEMENT()                                                                           \
	{                                                                                                  \
		Ph ph_(PH_NEXTELT);                                                                            \
		WalkResult wr;                                                                                 \
		const size_t elt = ent_next(i, s.rnd);                                                         \
		SARangeWithOffs<TSlice> sa;                                                                    \
		sa.topf = ent_topf(i);                                                                         \
		sa.len = ent_len(i);                                                                           \
		sa.offs = ent_offs(i);                                                                         \
		if(lazy_) adv_flat((TIndexOffU)elt, ebwtFw, sa, wr, d.wlm);                                    \
		else gws_[i].advanceElement((TIndexOffU)elt, ebwtFw, ref, sa, gwstate_, wr, d.wlm, s.prm);     \
		eltsDone++;                                                                                    \
		BT2GB_NELT_DEC;                                                                                \
		tidx = 0;                                                                                      \
		toff = 0;                                                                                      \
		tlen = 0;                                                                                      \
		bool straddled = false;                                                                        \
		ebwtFw.joinedToTextOff(wr.elt.len, wr.toff, tidx, toff, tlen, eeMode, straddled);              \
	}

// Ask the engine for the ungapped alignment at refcoord (or run the
// reference's on the CPU) and leave ungappedAlign's return in ug_ret
// (aligner_sw_driver.cpp:1033-1043, 1742-1752).
#define BT2GB_UNGAPPED(LABEL)                                                                          \
	resUngap_.reset();                                                                                 \
	if(d.bsc_ok && rdlen > 0 && rdlen <= BT2G_MAX_READ_LEN) {                                          \
		memset(&s.ug_p, 0, sizeof(s.ug_p));                                                            \
		s.ug_p.fw = fw ? 1 : 0;                                                                        \
		s.ug_p.off = refcoord.off();                                                                   \
		s.ug_p.refidx = (uint32_t)refcoord.ref();                                                      \
		s.ug_p.minsc = (int32_t)*minsc;                                                                \
		d.rq[K_UG].push_back(Rq{&s, mate});                                                            \
		pc = X_AFTER_UG;                                                                               \
		return EXTEND_BLOCKED;                                                                         \
	LABEL:                                                                                             \
		resUngap_.alres.reset();                                                                       \
		ug_ret = s.ug_r.ret;                                                                           \
		if(s.ug_r.ret == 1)                                                                            \
			fill_alnres(resUngap_.alres, s.ug_ed.data(), (uint32_t)s.ug_r.nedit, s.ug_r.score, s.ug_r.ns, 0, \
			            (int)(rdlen - (size_t)s.ug_r.nedit), refcoord.ref(), s.ug_r.refoff, (TRefOff)tlen, fw, \
			            rdlen, (size_t)s.ug_r.trim5p, (size_t)s.ug_r.trim3p, (size_t)s.ug_r.refns);           \
	} else {                                                                                           \
		d.swcpu.reset();                                                                               \
		ug_ret = d.swcpu.ungappedAlign(fw ? rd.patFw : rd.patRc, fw ? rd.qual : rd.qualRev, refcoord, ref, tlen, \
		                               sc, gReportOverhangs, *minsc, resUngap_);                        \
		g_cpu[K_UG]++;                                                                                 \
	}

// The report and -M tightening after an unpaired alignment
// (aligner_sw_driver.cpp:1245-1285).
static void tighten_unp(SwDriverB& x, AlnSinkWrap* msink) {
	if(R_tighten > 0 && msink->Mmode() && msink->hasSecondBestUnp1()) {
		TAlScore& m = *x.minsc;
		if(R_tighten == 1) {
			if(msink->bestUnp1() >= m) {
				m = msink->bestUnp1();
				if(m < x.perfectScore && msink->bestUnp1() == msink->secondBestUnp1()) m++;
			}
		} else if(R_tighten == 2) {
			if(msink->secondBestUnp1() >= m) {
				m = msink->secondBestUnp1();
				if(m < x.perfectScore) m++;
			}
		} else {
			TAlScore diff = msink->bestUnp1() - msink->secondBestUnp1();
			TAlScore bot = msink->secondBestUnp1() + ((diff * 3) / 4);
			if(bot >= m) {
				m = bot;
				if(m < x.perfectScore) m++;
			}
		}
	}
}

// The paired score a concordant alignment must now reach under -M tightening
// (aligner_sw_driver.cpp:1455-1473, 1948-1966, 2226-2244).
static bool pair_floor(const SwDriverB& x, AlnSinkWrap* msink, TAlScore& ps) {
	if(!(R_tighten > 0 && msink->Mmode() && msink->hasSecondBestPair())) return false;
	if(R_tighten == 1) {
		ps = msink->bestPair();
	} else if(R_tighten == 2) {
		ps = msink->secondBestPair();
	} else {
		TAlScore diff = msink->bestPair() - msink->secondBestPair();
		ps = msink->secondBestPair() + (diff * 3) / 4;
	}
	if(R_tighten == 1 && ps < x.bestPairScore && msink->bestPair() == msink->secondBestPair()) ps++;
	if(R_tighten >= 2 && ps < x.bestPairScore) ps++;
	return true;
}

#define BT2GB_NELT_DEC if(!eeMode) neltLeft--

// SwDriver::extendSeeds (aligner_sw_driver.cpp:756-1297).
int SwDriverB::ext_step(Driver& d, Slot& s) {
	AlnSinkWrap* msink = &s.msinkwrap;
	const Read& rd = *s.rds[mate];
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
	nonz = s.shs[mate].nonzeroOffsets();
	eeMode = s.shs[mate].numE2eHits() > 0;
	firstEe = true;
	firstExtend = true;
	s.prm.nEeFail = 0;
	s.prm.nUgFail = 0;
	s.prm.nDpFail = 0;
	nelt = 0;
	neltLeft = 0;
	rows = rdlen;
	eltsDone = 0;
	while(true) {
		if(eeMode) {
			if(firstEe) {
				firstEe = false;
				BT2GB_EE_SETUP(after_ee_rows)
			} else {
				eeMode = false;
			}
		}
		if(!eeMode) {
			if(nonz == 0) return EXTEND_EXHAUSTED_CANDIDATES;
			if(*minsc == perfectScore) return EXTEND_PERFECT_SCORE;
			if(firstExtend) {
				nelt = 0;
				BT2GB_PRIO_SETUP(after_ext, after_prio_rows)
				neltLeft = nelt;
				firstExtend = false;
			}
			if(neltLeft == 0) break;    // finished examining gapped candidates
		}
		for(i = 0; i < n_ent(); i++) {
			if(eeMode && eehits_[i].score < *minsc) return EXTEND_PERFECT_SCORE;
			is_small = ent_size(i) < 5;
			fw = ent_pos(i).fw;
			rdoff = ent_pos(i).rdoff;
			seedhitlen = ent_pos(i).seedlen;
			if(!fw) rdoff = (uint32_t)(rdlen - rdoff - seedhitlen);
			first = true;
			while(!ent_done(i) && (first || is_small || eeMode)) {
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
				BT2GB_NEXT_ELEMENT()
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
					sd_add(0, Interval(refcoord, 1));
				} else if(R_doUngapped && ungapped) {
					BT2GB_UNGAPPED(after_ug)
					sd_add(0, Interval(refcoord, 1));
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
					sd_add(0, Interval(refcoord, 1));
					if(!found) continue;
				}
				if(state == FOUND_NONE_) {
					{
						Interval refival(tidx, 0, fw, 0);
						rect.initIval(refival);
						sd_add(0, refival);
					}
					{
						Ph ph(PH_NEEDDP);
						if(!need_dp(d, s, mate, fw, tidx, tlen, rect, *minsc, true, true, false, a)) {
							pc = X_AFTER_DP;
							return EXTEND_BLOCKED;
						}
					}
				after_dp:
					a.start(a.dp);
					{
						TAlScore bestCell = std::numeric_limits<TAlScore>::min();
						{
							Ph ph(PH_DPFOUND);
							found = dp_found(d, s, a, false, *minsc, bestCell);
						}
						d.swmSeed.tallyGappedDp(readGaps, refGaps);
						s.prm.nExDps++;
						if(!found) {
							s.prm.nExDpFails++;
							s.prm.nDpFail++;
							if(s.prm.nDpFail >= maxDpStreak) return EXTEND_EXCEEDED_SOFT_LIMIT;
							if(bestCell > std::numeric_limits<TAlScore>::min() && bestCell > s.prm.bestLtMinscMate1)
								s.prm.bestLtMinscMate1 = bestCell;
							continue;     // look for more anchor alignments
						}
					}
					s.prm.nExDpSuccs++;
					s.prm.nDpLastSucc = s.prm.nExDps - 1;
					if(s.prm.nDpFail > s.prm.nDpFailStreak) s.prm.nDpFailStreak = s.prm.nDpFail;
					s.prm.nDpFail = 0;
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
						if(replay_done(d, a, false)) break;
						{
							Ph ph(PH_REPLAY);
							replay_next(d, s, a, false, *minsc, resGap_);
						}
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
					{
						Ph ph(PH_REDUND);
						if(redA.overlap(res->alres)) continue;
						redA.add(res->alres);
					}
					res->alres.setParams(seedmms, seedlen, seedival, *minsc);
					{
						Ph ph(PH_REPORT);
						if(msink->report(0, anchor1 ? &res->alres : NULL, anchor1 ? NULL : &res->alres))
							return EXTEND_POLICY_FULFILLED;
					}
					tighten_unp(*this, msink);
				}
			}
		}
	}
	return EXTEND_EXHAUSTED_CANDIDATES;
}

#undef BT2GB_NELT_DEC
#define BT2GB_NELT_DEC neltLeft--

// SwDriver::extendSeedsPaired (aligner_sw_driver.cpp:1385-2402), with
// swMateImmediately and reportImmediately true as multiseedSearchWorker calls it.
int SwDriverB::ext_step_paired(Driver& d, Slot& s) {
	AlnSinkWrap* msink = &s.msinkwrap;
	const Read& rd = *s.rds[mate];
	const Read& ord = *s.rds[mate ^ 1];
	const Scoring& sc = *d.sc;
	const Ebwt& ebwtFw = *d.ebwtFw;
	const BitPairReference& ref = *d.ref;
	const PairedEndPolicy& pepol = *d.pepol;
	const bool mixed = gReportMixed, discord = gReportDiscordant;
	switch(pc) {
	case X_START: break;
	case X_AFTER_EE_ROWS: goto after_ee_rows;
	case X_AFTER_EXT: goto after_ext;
	case X_AFTER_PRIO_ROWS: goto after_prio_rows;
	case X_AFTER_UG: goto after_ug;
	case X_AFTER_DP: goto after_dp;
	case X_AFTER_MDP: goto after_mdp;
	default: abort();
	}
	// aligner_sw_driver.cpp:1435-1504
	all = msink->allHits();
	rdlen = rd.length();
	ordlen = ord.length();
	perfectScore = sc.perfectScore(rdlen);
	operfectScore = sc.perfectScore(ordlen);
	bestPairScore = perfectScore + operfectScore;
	{
		TAlScore ps;
		if(pair_floor(*this, msink, ps)) {
			TAlScore nc = ps - operfectScore;
			if(nc > *minsc) *minsc = nc;
		}
	}
	nonz = s.shs[mate].nonzeroOffsets();
	eeMode = s.shs[mate].numE2eHits() > 0;
	firstEe = true;
	firstExtend = true;
	s.prm.nEeFail = 0;
	s.prm.nUgFail = 0;
	s.prm.nDpFail = 0;
	nelt = 0;
	neltLeft = 0;
	rows = rdlen;
	orows = ordlen;
	eltsDone = 0;
	while(true) {
		if(eeMode) {
			if(firstEe) {
				firstEe = false;
				BT2GB_EE_SETUP(after_ee_rows)
				neltLeft = nelt;
				mateStreaks_.resize(n_ent());
				mateStreaks_.fill(0);
			} else {
				eeMode = false;
			}
		}
		if(!eeMode) {
			if(nonz == 0) return EXTEND_EXHAUSTED_CANDIDATES;
			if(msink->Mmode() && *minsc == perfectScore) return EXTEND_PERFECT_SCORE;
			if(firstExtend) {
				nelt = 0;
				BT2GB_PRIO_SETUP(after_ext, after_prio_rows)
				neltLeft = nelt;
				firstExtend = false;
				mateStreaks_.resize(n_ent());
				mateStreaks_.fill(0);
			}
			if(neltLeft == 0) break;
		}
		for(i = 0; i < n_ent(); i++) {
			if(eeMode && eehits_[i].score < *minsc) return EXTEND_PERFECT_SCORE;
			is_small = ent_size(i) < 5;
			fw = ent_pos(i).fw;
			rdoff = ent_pos(i).rdoff;
			seedhitlen = ent_pos(i).seedlen;
			if(!fw) rdoff = (uint32_t)(rdlen - rdoff - seedhitlen);
			first = true;
			while(!ent_done(i) && (first || is_small || eeMode)) {
				if(*minsc == perfectScore) {
					if(!eeMode || eehits_[i].score < perfectScore) return EXTEND_PERFECT_SCORE;
				} else if(eeMode && eehits_[i].score < *minsc) {
					break;
				}
				if(s.prm.nExDps >= maxDp || s.prm.nMateDps >= maxDp) return EXTEND_EXCEEDED_HARD_LIMIT;
				if(s.prm.nExUgs >= maxUg || s.prm.nMateUgs >= maxUg) return EXTEND_EXCEEDED_HARD_LIMIT;
				if(s.prm.nExIters >= maxIters) return EXTEND_EXCEEDED_HARD_LIMIT;
				if(eeMode && s.prm.nEeFail >= maxEeStreak) return EXTEND_EXCEEDED_SOFT_LIMIT;
				if(!eeMode && s.prm.nDpFail >= maxDpStreak) return EXTEND_EXCEEDED_SOFT_LIMIT;
				if(!eeMode && s.prm.nUgFail >= maxUgStreak) return EXTEND_EXCEEDED_SOFT_LIMIT;
				if(mateStreaks_[i] >= maxMateStreak) {
					ent_set_done(i);           // don't try this seed range anymore
					break;
				}
				s.prm.nExIters++;
				first = false;
				BT2GB_NEXT_ELEMENT()
				if(tidx == OFF_MASK) continue;
				refoff = (int64_t)toff - rdoff;
				refcoord.init(tidx, refoff, fw);
				if(seenDiags().locusPresent(refcoord)) {
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
					sd_add(anchor1 ? 0 : 1, Interval(refcoord, 1));
					s.prm.nExEes++;
					s.prm.nEeFail++;        // failed until proven successful
					s.prm.nExEeFails++;
				} else if(R_doUngapped && ungapped) {
					BT2GB_UNGAPPED(after_ug)
					sd_add(anchor1 ? 0 : 1, Interval(refcoord, 1));
					s.prm.nExUgs++;
					s.prm.nUgFail++;        // failed until proven successful
					s.prm.nExUgFails++;
					if(ug_ret == 0) {
						d.swmSeed.ungapfail++;
						continue;
					} else if(ug_ret == -1) {
						d.swmSeed.ungapnodec++;
					} else {
						found = true;
						state = FOUND_UNGAPPED_;
						d.swmSeed.ungapsucc++;
					}
				}
				if(state == FOUND_NONE_) {
					DynProgFramer dpframe(!gReportOverhangs);
					found = dpframe.frameSeedExtensionRect(refoff, rows, tlen, readGaps, refGaps, (size_t)nceil, R_maxhalf,
					                                       rect);
					sd_add(anchor1 ? 0 : 1, Interval(refcoord, 1));
					if(!found) continue;
				}
				if(state == FOUND_NONE_) {
					{
						Interval refival(tidx, 0, fw, 0);
						rect.initIval(refival);
						sd_add(anchor1 ? 0 : 1, refival);
					}
					{
						Ph ph(PH_NEEDDP);
						if(!need_dp(d, s, mate, fw, tidx, tlen, rect, *minsc, true, true, false, a)) {
							pc = X_AFTER_DP;
							return EXTEND_BLOCKED;
						}
					}
				after_dp:
					a.start(a.dp);
					{
						TAlScore bestCell = std::numeric_limits<TAlScore>::min();
						{
							Ph ph(PH_DPFOUND);
							found = dp_found(d, s, a, false, *minsc, bestCell);
						}
						d.swmSeed.tallyGappedDp(readGaps, refGaps);
						s.prm.nExDps++;
						s.prm.nDpFail++;        // failed until proven successful
						s.prm.nExDpFails++;
						if(!found) {
							TAlScore& bl = anchor1 ? s.prm.bestLtMinscMate1 : s.prm.bestLtMinscMate2;
							if(bestCell > std::numeric_limits<TAlScore>::min() && bestCell > bl) bl = bestCell;
							continue;           // look for more anchor alignments
						}
					}
				}
				// aligner_sw_driver.cpp:1851-2353
				firstInner = true;
				foundConcordant = false;
				while(true) {
					if(state == FOUND_EE_) {
						if(!firstInner) break;
						res_kind = FOUND_EE_;
					} else if(state == FOUND_UNGAPPED_) {
						if(!firstInner) break;
						res_kind = FOUND_UNGAPPED_;
					} else {
						resGap_.reset();
						if(replay_done(d, a, false)) break;
						{
							Ph ph(PH_REPLAY);
							replay_next(d, s, a, false, *minsc, resGap_);
						}
						found = !resGap_.empty();
						if(!found) break;
						res_kind = FOUND_NONE_;
					}
					firstInner = false;
					{
						SwResult* res = res_ptr();
						Interval refival(tidx, 0, fw, tlen);
						if(gReportOverhangs && !refival.containsIgnoreOrient(res->alres.refival())) {
							res->alres.clipOutside(true, 0, tlen);
							if(res->alres.refExtent() == 0) continue;
						}
						if(!refival.overlapsIgnoreOrient(res->alres.refival())) continue;
						if(redA.overlap(res->alres)) continue;
						redA.add(res->alres);
						res->alres.setParams(seedmms, seedlen, seedival, *minsc);
						foundMate = false;
						off = res->alres.refoff();
					}
					if(msink->state().doneWithMate(!anchor1) && !msink->state().doneWithMate(anchor1))
						swMateImmediately = false;   // done with the opposite mate, not with the anchor
					if(found && swMateImmediately) {
						oleft = false;
						ofw = false;
						oll = olr = orl = orr = 0;
						foundMate = !oppFilt;
						ominsc_cur = *ominsc;
						oreadGaps = 0;
						orefGaps = 0;
						if(foundMate) {
							ominsc_cur = *ominsc;
							TAlScore ps;
							if(pair_floor(*this, msink, ps)) {
								TAlScore nc = ps - res_ptr()->alres.score().score();
								if(nc > ominsc_cur) ominsc_cur = nc;
							}
							oreadGaps = sc.maxReadGaps(ominsc_cur, ordlen);
							orefGaps = sc.maxRefGaps(ominsc_cur, ordlen);
							foundMate = pepol.otherMate(anchor1, fw, off, orows + oreadGaps, tlen,
							                            anchor1 ? rd.length() : ord.length(),
							                            anchor1 ? ord.length() : rd.length(), oleft, oll, olr, orl, orr, ofw);
						}
						if(foundMate) {
							DynProgFramer dpframe(!gReportOverhangs);
							foundMate = dpframe.frameFindMateRect(!oleft, oll, olr, orl, orr, orows, tlen, oreadGaps,
							                                      orefGaps, (size_t)onceil, R_maxhalf, orect);
						}
						if(foundMate) {
							oresGap_.reset();
							if(!need_dp(d, s, mate ^ 1, ofw, tidx, tlen, orect, ominsc_cur, false, false, a.cpu && res_kind == FOUND_NONE_, o)) {
								pc = X_AFTER_MDP;
								return EXTEND_BLOCKED;
							}
						after_mdp:
							o.start(o.dp);
							{
								TAlScore bestCell = std::numeric_limits<TAlScore>::min();
								foundMate = dp_found(d, s, o, true, ominsc_cur, bestCell);
								s.prm.nMateDps++;
								d.swmMate.tallyGappedDp(oreadGaps, orefGaps);
								if(!foundMate) {
									TAlScore& bl = anchor1 ? s.prm.bestLtMinscMate2 : s.prm.bestLtMinscMate1;
									if(bestCell > std::numeric_limits<TAlScore>::min() && bestCell > bl) bl = bestCell;
								}
							}
						}
						didAnchor = false;
						do {
							oresGap_.reset();
							if(foundMate && replay_done(d, o, true)) {
								foundMate = false;
							} else if(foundMate) {
								replay_next(d, s, o, true, ominsc_cur, oresGap_);
								foundMate = !oresGap_.empty();
							}
							SwResult* res = res_ptr();
							Interval refival(tidx, 0, fw, tlen);
							if(foundMate) {
								if(!redA.overlap(oresGap_.alres)) redA.add(oresGap_.alres);
								oresGap_.alres.setParams(seedmms, seedlen, seedival, *ominsc);
								if(gReportOverhangs && !refival.containsIgnoreOrient(oresGap_.alres.refival())) {
									oresGap_.alres.clipOutside(true, 0, tlen);
									foundMate = oresGap_.alres.refExtent() > 0;
								}
								if(foundMate && ((!gReportOverhangs && !refival.containsIgnoreOrient(oresGap_.alres.refival())) ||
								                 !refival.overlapsIgnoreOrient(oresGap_.alres.refival())))
									foundMate = false;
							}
							int pairCl = PE_ALS_DISCORD;
							if(foundMate) {
								const TRefOff off1 = anchor1 ? off : oresGap_.alres.refoff();
								const TRefOff off2 = anchor1 ? oresGap_.alres.refoff() : off;
								const size_t len1 = anchor1 ? res->alres.refExtent() : oresGap_.alres.refExtent();
								const size_t len2 = anchor1 ? oresGap_.alres.refExtent() : res->alres.refExtent();
								const bool fw1 = anchor1 ? res->alres.fw() : oresGap_.alres.fw();
								const bool fw2 = anchor1 ? oresGap_.alres.fw() : res->alres.fw();
								pairCl = pepol.peClassifyPair(off1, len1, fw1, off2, len2, fw2);
							}
							if(msink->state().doneConcordant()) foundMate = false;
							if(foundMate) {
								bool doneUnpaired = false;
								if(!anchor1 || !didAnchor) {
									if(anchor1) didAnchor = true;
									const AlnRes& r1 = anchor1 ? res->alres : oresGap_.alres;
									if(!redM1.overlap(r1)) {
										redM1.add(r1);
										if(msink->report(0, &r1, NULL)) doneUnpaired = true;
									}
								}
								if(anchor1 || !didAnchor) {
									if(!anchor1) didAnchor = true;
									const AlnRes& r2 = anchor1 ? oresGap_.alres : res->alres;
									if(!redM2.overlap(r2)) {
										redM2.add(r2);
										if(msink->report(0, NULL, &r2)) doneUnpaired = true;
									}
								}
								bool donePaired = false;
								if(pairCl != PE_ALS_DISCORD) {
									foundConcordant = true;
									if(msink->report(0, anchor1 ? &res->alres : &oresGap_.alres,
									                 anchor1 ? &oresGap_.alres : &res->alres)) {
										donePaired = true;
									} else {
										TAlScore ps;
										if(pair_floor(*this, msink, ps)) {
											TAlScore nc = ps - operfectScore;
											if(nc > *minsc) {
												*minsc = nc;
												if(*minsc > res->alres.score().score()) break;   // done with this anchor
											}
										}
									}
								}
								if(donePaired || doneUnpaired) return EXTEND_POLICY_FULFILLED;
								if(msink->state().doneWithMate(anchor1)) return EXTEND_POLICY_FULFILLED;
							} else if((mixed || discord) && !didAnchor) {
								didAnchor = true;
								if(!msink->state().doneUnpaired(anchor1)) {
									const AlnRes& r = res->alres;
									RedFlat& red = anchor1 ? redM1 : redM2;
									const AlnRes* r1 = anchor1 ? &res->alres : NULL;
									const AlnRes* r2 = anchor1 ? NULL : &res->alres;
									if(!red.overlap(r)) {
										red.add(r);
										if(msink->report(0, r1, r2)) return EXTEND_POLICY_FULFILLED;
									}
								}
								if(msink->state().doneWithMate(anchor1)) return EXTEND_POLICY_FULFILLED;
							}
						} while(!oresGap_.empty());
					} else if(found) {
						// an anchor alignment, no opposite-mate search (probably done with it)
						if(mixed || discord) {
							SwResult* res = res_ptr();
							if(!msink->state().doneUnpaired(anchor1)) {
								const AlnRes& r = res->alres;
								RedFlat& red = anchor1 ? redM1 : redM2;
								const AlnRes* r1 = anchor1 ? &res->alres : NULL;
								const AlnRes* r2 = anchor1 ? NULL : &res->alres;
								if(!red.overlap(r)) {
									red.add(r);
									if(msink->report(0, r1, r2)) return EXTEND_POLICY_FULFILLED;
								}
							}
							if(msink->state().doneWithMate(anchor1)) return EXTEND_POLICY_FULFILLED;
						}
					}
				}
				if(foundConcordant) {
					s.prm.nMateDpSuccs++;
					mateStreaks_[i] = 0;
					if(state == FOUND_UNGAPPED_) {
						s.prm.nExUgFails--;
						s.prm.nExUgSuccs++;
						s.prm.nUgLastSucc = s.prm.nExUgs - 1;
						if(s.prm.nUgFail > s.prm.nUgFailStreak) s.prm.nUgFailStreak = s.prm.nUgFail;
						s.prm.nUgFail = 0;
					} else if(state == FOUND_EE_) {
						s.prm.nExEeFails--;
						s.prm.nExEeSuccs++;
						s.prm.nEeLastSucc = s.prm.nExEes - 1;
						if(s.prm.nEeFail > s.prm.nEeFailStreak) s.prm.nEeFailStreak = s.prm.nEeFail;
						s.prm.nEeFail = 0;
					} else {
						s.prm.nExDpFails--;
						s.prm.nExDpSuccs++;
						s.prm.nDpLastSucc = s.prm.nExDps - 1;
						if(s.prm.nDpFail > s.prm.nDpFailStreak) s.prm.nDpFailStreak = s.prm.nDpFail;
						s.prm.nDpFail = 0;
					}
				} else {
					s.prm.nMateDpFails++;
					mateStreaks_[i]++;
				}
			}
		}
	}
	return EXTEND_EXHAUSTED_CANDIDATES;
}

#undef BT2GB_NELT_DEC
#undef BT2GB_EE_SETUP
#undef BT2GB_PRIO_SETUP
#undef BT2GB_NEXT_ELEMENT
#undef BT2GB_UNGAPPED

}  // namespace

// ---- the reference's SwDriver / GroupWalk2S pieces, served from the tables ------
extern "C" {
void bt2g_real__ZN8SwDriver6extendERK4ReadRK4EbwtPS4_jjjjbmmR14PerReadMetricsRmS9_(
	SwDriver*, const Read&, const Ebwt&, const Ebwt*, TIndexOffU, TIndexOffU, TIndexOffU, TIndexOffU, bool, size_t,
	size_t, PerReadMetrics&, size_t&, size_t&);
}

// SwDriver::extend (aligner_sw_driver.cpp:299-483) from the engine's results for
// this read (asked in the order prioritizeSATups calls it), else the CPU.
// (prioritizeSATups and eeSaTups are the reference's own definitions.)
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
	g_gw_inits.fetch_add(1, std::memory_order_relaxed);
	g_gw_elts.fetch_add(sa.size(), std::memory_order_relaxed);
	// the range's offset slots as the cache would hold them before any walk
	// (AlignmentCache::addOnTheFlyImpl only reserves them, bt2g_refspec.h)
	static_cast<bt2gref::TSliceAcc&>(sa.offs).fill(OFF_MASK);
	if(t_tab && t_tab->gw_on) t_tab->gw.push_back(GwRange{sa.topf, sa.size(), sa.offs, false});
}

template <>
bool GroupWalk2S<TSlice, 16>::advanceElement(TIndexOffU elt, const Ebwt& ebwtFw, const BitPairReference& ref,
                                             SARangeWithOffs<TSlice>& sa, GroupWalkState& gws, WalkResult& res,
                                             WalkMetrics& met, PerReadMetrics& prm) {
	(void)ref; (void)gws; (void)prm;
	g_gw_adv.fetch_add(1, std::memory_order_relaxed);
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

// ---- multiseedSearchWorker's per-read body (bt2_search.cpp:3266-4160) ----------
bool Driver::seeds_valid(const MateRes& m, bool fw, size_t i) const {
	if(i < 64) return ((fw ? m.valid_fw : m.valid_rc) >> i) & 1;
	const size_t k = (i - 64) * 2 + (fw ? 0 : 1);
	return k / 64 < m.valid_big.size() && ((m.valid_big[k / 64] >> (k % 64)) & 1);
}

void Driver::set_valid(MateRes& m, bool fw, size_t i) {
	if(i < 64) {
		(fw ? m.valid_fw : m.valid_rc) |= 1ull << i;
		return;
	}
	const size_t k = (i - 64) * 2 + (fw ? 0 : 1);
	if(m.valid_big.size() <= k / 64) m.valid_big.resize(k / 64 + 1, 0);
	m.valid_big[k / 64] |= 1ull << (k % 64);
}

// Per-read setup (bt2_search.cpp:3266-3451).
void Driver::setup_read(Slot& s) {
	s.prm.reset();
	s.prm.doFmString = false;
	if(R_sam_print_xt) gettimeofday(&s.prm.tv_beg, &s.prm.tz_beg);
	s.ca.nextRead();
	const bool paired = s.paired;
	const Read& ra = *s.rds[0];
	const Read& rb = *s.rds[1];
	s.rdlens[0] = ra.length();
	s.rdlens[1] = paired ? rb.length() : 0;
	s.msinkwrap.nextRead(s.msink, &ra, paired ? &rb : NULL, s.rdid, sc->qualitiesMatter());
	s.minsc[0] = s.minsc[1] = std::numeric_limits<TAlScore>::max();
	if(R_bwaSwLike) {
		float a = (float)sc->match(30);
		float T = R_bwaSwLikeT, c = R_bwaSwLikeC;
		s.minsc[0] = (TAlScore)max<float>(a * T, a * c * log(s.rdlens[0]));
		if(paired) s.minsc[1] = (TAlScore)max<float>(a * T, a * c * log(s.rdlens[1]));
	} else {
		s.minsc[0] = R_scoreMin.f<TAlScore>(s.rdlens[0]);
		if(paired) s.minsc[1] = R_scoreMin.f<TAlScore>(s.rdlens[1]);
		if(R_localAlign) {
			if(s.minsc[0] < 0) s.minsc[0] = 0;
			if(paired && s.minsc[1] < 0) s.minsc[1] = 0;
		} else {
			if(s.minsc[0] > 0) s.minsc[0] = 0;
			if(paired && s.minsc[1] > 0) s.minsc[1] = 0;
		}
	}
	size_t readns[2] = {0, 0};
	sc->nFilterPair(&ra.patFw, paired ? &rb.patFw : NULL, readns[0], readns[1], s.nfilt[0], s.nfilt[1]);
	s.scfilt[0] = sc->scoreFilter(s.minsc[0], s.rdlens[0]);
	s.scfilt[1] = sc->scoreFilter(s.minsc[1], s.rdlens[1]);
	s.lenfilt[0] = s.lenfilt[1] = true;
	if(s.rdlens[0] <= (size_t)R_multiseedMms || s.rdlens[0] < 2) s.lenfilt[0] = false;
	if((s.rdlens[1] <= (size_t)R_multiseedMms || s.rdlens[1] < 2) && paired) s.lenfilt[1] = false;
	if(s.rdlens[0] < 2) s.lenfilt[0] = false;
	if(s.rdlens[1] < 2 && paired) s.lenfilt[1] = false;
	s.qcfilt[0] = s.qcfilt[1] = true;
	if(R_qcFilter) {
		s.qcfilt[0] = (ra.filter != '0');
		s.qcfilt[1] = (rb.filter != '0');
	}
	for(int m = 0; m < 2; m++) s.filt[m] = s.nfilt[m] && s.scfilt[m] && s.lenfilt[m] && s.qcfilt[m];
	s.prm.nFilt += (s.filt[0] ? 0 : 1) + (s.filt[1] ? 0 : 1);
	s.sd.next_read();
	s.minedfw[0] = s.minedfw[1] = s.minedrc[0] = s.minedrc[1] = 0;
	s.nofw[0] = paired ? (gMate1fw ? gNofw : gNorc) : gNofw;
	s.norc[0] = paired ? (gMate1fw ? gNorc : gNofw) : gNorc;
	s.nofw[1] = paired ? (gMate2fw ? gNofw : gNorc) : gNofw;
	s.norc[1] = paired ? (gMate2fw ? gNorc : gNofw) : gNorc;
	s.nceil[0] = std::min(R_nCeil.f<int>((double)s.rdlens[0]), (int)s.rdlens[0]);
	s.nceil[1] = paired ? std::min(R_nCeil.f<int>((double)s.rdlens[1]), (int)s.rdlens[1]) : 0;
	s.exhaustive[0] = s.exhaustive[1] = false;
	s.matemap[0] = 0;
	s.matemap[1] = 1;
	const bool pairPostFilt = s.filt[0] && s.filt[1];
	if(pairPostFilt) s.rnd.init(ra.seed ^ rb.seed);
	else s.rnd.init(ra.seed);
	s.interval[0] = s.interval[1] = 0;
	for(int m = 0; m < (paired ? 2 : 1); m++) {
		s.interval[m] = R_msIval.f<int>((double)s.rdlens[m]);
		if(s.filt[0] && s.filt[1]) s.interval[m] = (int)(s.interval[m] * 1.2 + 0.5);   // boost for pairs
		s.interval[m] = std::max(s.interval[m], 1);
	}
	for(int m = 0; m < 2; m++) {
		s.streak[m] = R_maxDpStreak;
		s.mtStreak[m] = R_maxMateStreak;
		s.mxDp[m] = R_maxDp;
		s.mxUg[m] = R_maxUg;
		s.mxIter[m] = R_maxIters;
		if(R_allHits) {
			s.streak[m] = s.mtStreak[m] = s.mxDp[m] = s.mxUg[m] = s.mxIter[m] = std::numeric_limits<size_t>::max();
		} else if(R_khits > 1) {
			s.streak[m] += (R_khits - 1) * R_maxStreakIncr;
			s.mtStreak[m] += (R_khits - 1) * R_maxStreakIncr;
			s.mxDp[m] += (R_khits - 1) * R_maxItersIncr;
			s.mxUg[m] += (R_khits - 1) * R_maxItersIncr;
			s.mxIter[m] += (R_khits - 1) * R_maxItersIncr;
		}
	}
	if(s.filt[0] && s.filt[1]) {
		s.streak[0] = (size_t)ceil((double)s.streak[0] / 2.0);
		s.streak[1] = (size_t)ceil((double)s.streak[1] / 2.0);
	}
	s.prm.maxDPFails = s.streak[0];
	s.nrounds[0] = s.nrounds[1] = R_nSeedRounds;
	if(s.filt[0] && s.filt[1]) {
		s.nrounds[0] = (size_t)ceil((double)s.nrounds[0] / 2.0);
		s.nrounds[1] = (size_t)ceil((double)s.nrounds[1] / 2.0);
	}
	for(int m = 0; m < (paired ? 2 : 1); m++) {
		if(s.filt[m]) {
			s.shs[m].clear();
			s.shs[m].nextRead(*s.rds[m]);
		}
	}
	s.done[0] = !s.filt[0];
	s.done[1] = !s.filt[1];
	s.nelt[0] = s.nelt[1] = 0;
	for(int m = 0; m < 2; m++) {
		MateRes& x = s.mr[m];
		x.sd_ready = false;
		x.sweep_asked = false;
		x.mm_asked = false;
	}
	s.seedsTried = 0;
	for(int k = 0; k < 4; k++) s.seedsTriedMS[k] = s.nUniqueSeedsMS[k] = s.nRepeatSeedsMS[k] = s.seedHitTotMS[k] = 0;
	s.nUniqueSeeds = s.nRepeatSeeds = s.seedHitTot = 0;
	s.ndps = 0;
}

// instantiateSeeds (aligner_seed.cpp:498-587) for exact seeds: offsets,
// sequences and qualities into SeedResults; which seeds instantiate (an N
// disqualifies an exact seed: Constraint::canN, aligner_seed.h:88-92).
// Returns the number instantiated.
int Driver::instantiate(Slot& s, int mate, size_t offset) {
	const Read& rd = *s.rds[mate];
	MateRes& x = s.mr[mate];
	const int len = s.seeds[mate][0].len;
	const int per = s.interval[mate];
	int nseeds = 1;
	if((int)rd.length() - (int)offset > len) nseeds += ((int)rd.length() - (int)offset - len) / per;
	s.offIdx2off.clear();
	for(int i = 0; i < nseeds; i++) s.offIdx2off.push_back(per * i + (int)offset);
	SeedResults& sr = s.shs[mate];
	sr.reset(rd, s.offIdx2off, nseeds);
	x.valid_fw = x.valid_rc = 0;
	x.valid_big.clear();
	int ninst = 0, inst_fw = 0, inst_rc = 0;
	for(int fwi = 0; fwi < 2; fwi++) {
		const bool fw = fwi == 0;
		if((fw && s.nofw[mate]) || (!fw && s.norc[mate])) continue;
		for(int i = 0; i < nseeds; i++) {
			const int depth = i * per + (int)offset;
			const int sl = std::min<int>(len, (int)rd.length());
			// SeedAligner::instantiateSeq (aligner_seed.cpp:471-491): the seed's
			// bases as they align to the Watson strand (rc: complemented, reversed)
			// and its qualities, with the N test of the instantiation
			BTDnaString& sq = sr.seqs(fw)[i];
			BTString& sqq = sr.quals(fw)[i];
			sq.resize(sl);
			sqq.resize(sl);
			const char* pf = rd.patFw.buf();
			const char* qf = rd.qual.buf();
			bool ok = true;
			if(fw) {
				for(int k = 0; k < sl; k++) {
					const int c = pf[depth + k];
					sq.set(c, k);
					sqq.set(qf[depth + k], k);
					ok = ok && c < 4;
				}
			} else {
				for(int k = 0; k < sl; k++) {
					const int c = pf[depth + sl - k - 1];
					sq.set(c < 4 ? 3 - c : 4, k);
					sqq.set(qf[depth + sl - k - 1], k);
					ok = ok && c < 4;
				}
			}
			if(ok) {
				set_valid(x, fw, (size_t)i);
				ninst++;
				(fw ? inst_fw : inst_rc)++;
			} else {
				sdm.filteredseed++;
			}
		}
	}
	s.seedsTriedMS[mate * 2 + 0] = (size_t)inst_fw;
	s.seedsTriedMS[mate * 2 + 1] = (size_t)inst_rc;
	return ninst;
}

// searchAllSeeds' cache protocol and metrics (aligner_seed.cpp:597-718) over
// the engine's seed ranges: strand fw then rc, offsets ascending;
// SeedSearchCache::addOnTheFly for a hit (reportHit, aligner_seed.cpp:1576-1630),
// beginAlign / addAllCached / finishAlign, SeedResults::add.
void Driver::after_seeds(Slot& s, int mate) {
	SeedResults& sr = s.shs[mate];
	MateRes& x = s.mr[mate];
	const size_t nof = sr.numOffs();
	if((size_t)x.sd_ns != nof) {
		fprintf(stderr, "bt2g batch: seed offsets differ (engine %d, reference %zu)\n", x.sd_ns, nof);
		abort();
	}
	uint64_t possearches = 0, seedsearches = 0, ooms = 0;
	for(int fwi = 0; fwi < 2; fwi++) {
		const bool fw = fwi == 0;
		for(size_t i = 0; i < nof; i++) {
			if(!seeds_valid(x, fw, i)) continue;
			possearches++;
			seedsearches++;
			const BTDnaString& seq = sr.seqs(fw)[i];
			const uint32_t* q = &x.sd_out[((size_t)fwi * nof + i) * 4];
			// SeedSearchCache's protocol (aligner_seed.h:1461-1580) without its
			// per-seed vector: beginAlign; the range, if any, added while the
			// cache aligns (addAllCached: false when it does not); finishAlign
			QVal qv;
			const int ret = s.ca.beginAlign(seq, sr.quals(fw)[i], qv);
			if(ret == -1 || !s.ca.aligning()) {
				ooms++;
				continue;
			}
			if(q[1] > q[0] && !s.ca.addOnTheFly(seq, q[0], q[1], q[2], q[3])) {
				ooms++;
				continue;
			}
			qv = s.ca.finishAlign();
			if(qv.valid()) sr.add(qv, s.ca.current(), (uint32_t)i, fw);
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
	s.prm.nSdFmops += x.sd_ops;
	sdm.seedsearch += seedsearches;
	sdm.nrange += sr.numRanges();
	sdm.nelt += sr.numElts();
	sdm.possearch += possearches;
	sdm.ooms += ooms;
	sdm.bwops += x.sd_ops;
	x.sd_ready = false;
}

// A round's seed search, asked ahead: (round 0) with the exact sweep, its
// arguments being functions of the read and the server's options; (later
// rounds, pairs) both mates' searches in the round's one wait.  The round
// takes a result only when its own arguments are the same.
void Driver::prefetch_seeds(Slot& s, int mate) {
	if(R_seedSumm || R_nSeedRounds == 0 || R_multiseedMms != 0 || ebwtBw == NULL || !engine_read(s, mate)) return;
	MateRes& x = s.mr[mate];
	const int L = R_multiseedLen;
	const size_t off = s.round_off[mate];
	int nseeds = 1;
	if((int)s.rdlens[mate] - (int)off > L) nseeds += ((int)s.rdlens[mate] - (int)off - L) / s.interval[mate];
	if(x.sd_ready && x.sd_L == (uint32_t)L && x.sd_per == (uint32_t)s.interval[mate] && x.sd_off == (uint32_t)off &&
	   x.sd_nof == (uint32_t)nseeds)
		return;
	x.sd_L = (uint32_t)L;
	x.sd_per = (uint32_t)s.interval[mate];
	x.sd_off = (uint32_t)off;
	x.sd_nof = (uint32_t)nseeds;
	x.sd_ready = false;
	rq[K_SEEDS].push_back(Rq{&s, mate});
}

// Start one extendSeeds / extendSeedsPaired call for anchor `mate`
// (bt2_search.cpp:3505-3593, 3687-3775, 3963-4051).
void start_ext(Slot& s, int mate, int seedmms, int seedlen, int seedival) {
	SwDriverB& x = s.sd;
	x.pc = X_START;
	x.mate = mate;
	x.paired = s.paired;
	x.anchor1 = mate == 0;
	x.oppFilt = !s.filt[mate ^ 1];
	x.seedmms = seedmms;
	x.seedlen = seedlen;
	x.seedival = seedival;
	x.minsc = &s.minsc[mate];
	x.ominsc = &s.minsc[mate ^ 1];
	x.nceil = s.nceil[mate];
	x.onceil = s.nceil[mate ^ 1];
	x.nofw = s.nofw[mate];
	x.norc = s.norc[mate];
	x.maxIters = s.mxIter[mate];
	x.maxUg = s.mxUg[mate];
	x.maxDp = s.mxDp[mate];
	x.maxEeStreak = s.streak[mate];
	x.maxUgStreak = s.streak[mate];
	x.maxDpStreak = s.streak[mate];
	x.maxMateStreak = s.mtStreak[mate];
	x.swMateImmediately = true;
	x.exhaustive = &s.exhaustive[mate];
}

// extendSeeds' return code as the worker handles it (bt2_search.cpp:3601-3629).
void after_ext(Driver& d, Slot& s, int mate, int ret, bool perfect_check) {
	if(ret == EXTEND_EXHAUSTED_CANDIDATES) {
	} else if(ret == EXTEND_POLICY_FULFILLED) {
		if(s.msinkwrap.state().doneWithMate(mate == 0)) s.done[mate] = true;
		if(s.msinkwrap.state().doneWithMate(mate == 1)) s.done[mate ^ 1] = true;
	} else if(ret == EXTEND_PERFECT_SCORE) {
		s.done[mate] = true;
	} else if(ret == EXTEND_EXCEEDED_HARD_LIMIT) {
		s.done[mate] = true;
	} else if(ret == EXTEND_EXCEEDED_SOFT_LIMIT) {
	} else {
		fprintf(stderr, "Bad return value: %d\n", ret);
		throw 1;
	}
	if(perfect_check && !s.done[mate]) {
		const TAlScore perfectScore = d.sc->perfectScore(s.rdlens[mate]);
		if(s.minsc[mate] == perfectScore) s.done[mate] = true;
	}
}

// The offsets a rows request brought back (Svc::call_off), into the ranges'
// offset slots in the read's cache, where the reference's walks leave them.
void Driver::take_offsets(Slot& s) {
	for(size_t j = 0; j < s.off_vals.size(); j++) {
		const std::pair<size_t, size_t>& w = s.off_where[j];
		s.tab.gw[w.first].offs[w.second] = s.off_vals[j];
	}
	s.off_vals.clear();
	s.tab.gw.clear();
}

void Driver::step_read(Slot& s) {
	if(!s.off_vals.empty()) take_offsets(s);
	const bool paired = s.paired;
	const size_t nmates = paired ? 2 : 1;
	const size_t eePeEeltLimit = std::numeric_limits<size_t>::max();
	int ret = 0;
	size_t mate = 0;
	switch(s.pc) {
	case P_START: break;
	case P_AFTER_EXACT: goto after_exact;
	case P_EXT_EXACT: mate = s.matemap[s.matei]; goto ext_exact;
	case P_AFTER_1MM: goto after_1mm;
	case P_EXT_1MM: mate = s.matemap[s.matei]; goto ext_1mm;
	case P_AFTER_SEEDS: goto after_seeds_l;
	case P_EXT_SEEDS: mate = s.matemap[s.matei]; goto ext_seeds;
	default: abort();
	}
	{
		Ph ph(PH_SETUP);
		setup_read(s);
	}
	// exact end-to-end alignments (bt2_search.cpp:3453-3631)
	if(R_doExactUpFront) {
		{
			bool asked = false;
			for(size_t mi = 0; mi < nmates; mi++) {
				const size_t m = s.matemap[mi];
				if(!s.filt[m] || s.done[m] || s.msinkwrap.state().doneWithMate(m == 0)) continue;
				swmSeed.exatts++;
				if(engine_read(s, (int)m)) {
					rq[K_EXACT].push_back(Rq{&s, (int)m});
					s.mr[m].sweep_asked = true;
					{
						// the 1-mm search rides with the sweep when the engine takes it
						// (its gate is the sweep's result, bt2_search.cpp:3649-3650)
						MateRes& x = s.mr[m];
						x.pf_ok = false;
						x.pf_want = R_do1mmUpFront && !R_seedSumm && bsc_ok && s.minsc[m] >= std::numeric_limits<int32_t>::min() &&
						            s.minsc[m] <= std::numeric_limits<int32_t>::max() && R_localAlign == !sc->monotone &&
						            mm_prefetch_on();
						x.pf_minsc = (int32_t)s.minsc[m];
					}
					s.round_off[m] = 0;
					prefetch_seeds(s, (int)m);
					asked = true;
				} else {
					s.nelt[m] = al.exactSweep(*ebwtFw, *s.rds[m], *sc, s.nofw[m], s.norc[m], 2, s.minedfw[m], s.minedrc[m],
					                          true, s.shs[m], sdm);
					g_cpu[K_EXACT]++;
					const size_t bestmin = std::min(s.minedfw[m], s.minedrc[m]);
					if(bestmin == 0) sdm.bestmin0++;
					else if(bestmin == 1) sdm.bestmin1++;
					else sdm.bestmin2++;
				}
			}
			if(asked) {
				s.pc = P_AFTER_EXACT;
				return;
			}
		}
	after_exact:
		for(size_t m = 0; m < 2; m++) {
			MateRes& x = s.mr[m];
			if(!x.sweep_asked) continue;
			x.sweep_asked = false;
			const uint32_t* out = x.sweep;
			if(!s.nofw[m]) s.minedfw[m] = out[0];
			if(!s.norc[m]) s.minedrc[m] = out[1];
			sdm.bwops += out[6];
			size_t ne = 0;
			const int64_t score = (int64_t)s.rdlens[m] * sc->match();
			if(!s.nofw[m] && out[0] == 0 && out[3] > out[2]) {
				s.shs[m].addExactEeFw(out[2], out[3], NULL, NULL, true, score);
				ne += out[3] - out[2];
			}
			if(!s.norc[m] && out[1] == 0 && out[5] > out[4]) {
				s.shs[m].addExactEeRc(out[4], out[5], NULL, NULL, false, score);
				ne += out[5] - out[4];
			}
			s.nelt[m] = ne;
			const size_t bestmin = std::min(s.minedfw[m], s.minedrc[m]);
			if(bestmin == 0) sdm.bestmin0++;
			else if(bestmin == 1) sdm.bestmin1++;
			else sdm.bestmin2++;
		}
		s.matemap[0] = 0;
		s.matemap[1] = 1;
		if(s.nelt[0] > 0 && s.nelt[1] > 0 && s.nelt[0] > s.nelt[1]) {   // the mate with fewer exact hits first
			s.matemap[0] = 1;
			s.matemap[1] = 0;
		}
		for(s.matei = 0; s.matei < (R_seedSumm ? 0u : 2u); s.matei++) {
			mate = s.matemap[s.matei];
			if(s.nelt[mate] == 0 || s.nelt[mate] > eePeEeltLimit) {
				s.shs[mate].clearExactE2eHits();
				continue;
			}
			if(s.msinkwrap.state().doneWithMate(mate == 0)) {
				s.shs[mate].clearExactE2eHits();
				s.done[mate] = true;
				continue;
			}
			start_ext(s, (int)mate, -1, 0, 0);
		ext_exact:
			ret = ext(s);
			if(ret == EXTEND_BLOCKED) {
				s.pc = P_EXT_EXACT;
				return;
			}
			s.shs[mate].clearExactE2eHits();
			after_ext(*this, s, (int)mate, ret, true);
		}
	}
	// 1-mismatch end-to-end alignments (bt2_search.cpp:3633-3813)
	if(R_do1mmUpFront && !R_seedSumm) {
		{
			bool asked = false;
			for(size_t mi = 0; mi < nmates; mi++) {
				const size_t m = s.matemap[mi];
				if(!s.filt[m] || s.done[m] || s.nelt[m] > eePeEeltLimit) {
					s.shs[m].clear1mmE2eHits();
					s.nelt[m] = 0;
					continue;
				}
				s.nelt[m] = 0;
				s.yfw[m] = s.minedfw[m] <= 1 && !s.nofw[m];
				s.yrc[m] = s.minedrc[m] <= 1 && !s.norc[m];
				if(s.yfw[m] || s.yrc[m]) {
					swmSeed.mm1atts++;
					if(engine_read(s, (int)m) && bsc_ok && s.minsc[m] >= std::numeric_limits<int32_t>::min() &&
					   s.minsc[m] <= std::numeric_limits<int32_t>::max() && R_localAlign == !sc->monotone) {
						MateRes& x = s.mr[m];
						x.mm_nofw = s.yfw[m] ? 0 : 1;
						x.mm_norc = s.yrc[m] ? 0 : 1;
						x.mm_minsc = (int32_t)s.minsc[m];
						x.mm_asked = true;
						if(x.pf_ok && x.pf_nofw == x.mm_nofw && x.pf_norc == x.mm_norc && x.pf_minsc == x.mm_minsc) {
							x.pf_ok = false;               // (its hits are in x.mm already)
							g_mm_pf_used++;
						} else {
							rq[K_1MM].push_back(Rq{&s, (int)m});
							asked = true;
						}
					} else {
						al.oneMmSearch(ebwtFw, ebwtBw, *s.rds[m], *sc, s.minsc[m], !s.yfw[m], !s.yrc[m], R_localAlign, false,
						               true, s.shs[m], sdm);
						g_cpu[K_1MM]++;
						s.nelt[m] = s.shs[m].num1mmE2eHits();
					}
				}
			}
			if(asked) {
				s.pc = P_AFTER_1MM;
				return;
			}
		}
	after_1mm:
		for(size_t m = 0; m < 2; m++) {
			MateRes& x = s.mr[m];
			if(!x.mm_asked) continue;
			x.mm_asked = false;
			sdm.bwops += x.mm_ops;
			for(int32_t k = 0; k < x.mm_cnt; k++) {
				const bt2g_mm1& h = x.mm[k];
				Edit e((uint32_t)h.pos, h.chr, h.qchr, EDIT_TYPE_MM, false);
				s.shs[m].add1mmEe(h.top, h.bot, &e, NULL, h.fw != 0, h.score);
			}
			s.nelt[m] = s.shs[m].num1mmE2eHits();
		}
		s.matemap[0] = 0;
		s.matemap[1] = 1;
		if(s.nelt[0] > 0 && s.nelt[1] > 0 && s.nelt[0] > s.nelt[1]) {
			s.matemap[0] = 1;
			s.matemap[1] = 0;
		}
		for(s.matei = 0; s.matei < (R_seedSumm ? 0u : 2u); s.matei++) {
			mate = s.matemap[s.matei];
			if(s.nelt[mate] == 0 || s.nelt[mate] > eePeEeltLimit) continue;
			if(s.msinkwrap.state().doneWithMate(mate == 0)) {
				s.done[mate] = true;
				continue;
			}
			start_ext(s, (int)mate, -1, 0, 0);
		ext_1mm:
			ret = ext(s);
			if(ret == EXTEND_BLOCKED) {
				s.pc = P_EXT_1MM;
				return;
			}
			s.shs[mate].clear1mmE2eHits();
			after_ext(*this, s, (int)mate, ret, true);
		}
	}
	// seed rounds (bt2_search.cpp:3814-4090)
	s.seedlens[0] = s.seedlens[1] = R_multiseedLen;
	s.nrounds[0] = std::min<size_t>(s.nrounds[0], (size_t)s.interval[0]);
	s.nrounds[1] = std::min<size_t>(s.nrounds[1], (size_t)s.interval[1]);
	for(s.roundi = 0; s.roundi < R_nSeedRounds; s.roundi++) {
		s.ca.nextRead();
		s.shs[0].clearSeeds();
		s.shs[1].clearSeeds();
		{
			// which mates this round searches (until one stops it), and their engine
			// searches asked together
			bool asked = false;
			for(size_t mi = 0; mi < nmates; mi++) {
				const size_t m = s.matemap[mi];
				s.round_go[m] = false;
				if(s.done[m] || s.msinkwrap.state().doneWithMate(m == 0)) continue;
				if(s.roundi >= s.nrounds[m] || s.interval[m] <= (int)s.roundi) continue;
				s.round_off[m] = ((size_t)s.interval[m] * s.roundi) / s.nrounds[m];
				s.seeds[m].clear();
				Seed::mmSeeds(R_multiseedMms, s.seedlens[m], s.seeds[m], s.gc);
				if(s.round_off[m] > 0 && s.seeds[m][0].len + s.round_off[m] > s.rds[m]->length()) continue;
				s.round_go[m] = true;
				const size_t before = rq[K_SEEDS].size();
				prefetch_seeds(s, (int)m);
				asked = asked || rq[K_SEEDS].size() > before;
			}
			if(asked) {
				s.pc = P_AFTER_SEEDS;
				return;
			}
		}
	after_seeds_l:
		for(s.matei = 0; s.matei < nmates; s.matei++) {
			mate = s.matemap[s.matei];
			if(s.done[mate] || s.msinkwrap.state().doneWithMate(mate == 0)) {
				s.done[mate] = true;
				continue;
			}
			if(!s.round_go[mate]) continue;    // not this round (its count, its interval, or off the end)
			swmSeed.sdatts++;
			const Read& rd = *s.rds[mate];
			if(!engine_read(s, (int)mate) || R_multiseedMms != 0 || ebwtBw == NULL) {
				// the reference's own seed search on the host (instantiateSeeds +
				// searchAllSeeds, bt2_search.cpp:3873-3913)
				std::pair<int, int> instFw, instRc;
				std::pair<int, int> inst = al.instantiateSeeds(s.seeds[mate], s.round_off[mate], s.interval[mate], rd, *sc,
				                                               s.nofw[mate], s.norc[mate], s.ca, s.shs[mate], sdm, instFw,
				                                               instRc);
				if(inst.first + inst.second == 0) {
					s.done[mate] = true;
					break;
				}
				s.seedsTried += (inst.first + inst.second);
				s.seedsTriedMS[mate * 2 + 0] = instFw.first + instFw.second;
				s.seedsTriedMS[mate * 2 + 1] = instRc.first + instRc.second;
				al.searchAllSeeds(s.seeds[mate], ebwtFw, ebwtBw, rd, *sc, s.ca, s.shs[mate], sdm, s.prm);
				g_cpu[K_SEEDS]++;
			} else {
				int inst;
				{
					Ph ph(PH_INST);
					inst = instantiate(s, (int)mate, s.round_off[mate]);
				}
				if(inst == 0) {
					s.done[mate] = true;
					break;
				}
				s.seedsTried += (size_t)inst;
				const MateRes& x = s.mr[mate];
				if(!(x.sd_ready && x.sd_L == (uint32_t)s.seeds[mate][0].len && x.sd_per == (uint32_t)s.interval[mate] &&
				     x.sd_off == (uint32_t)s.round_off[mate] && x.sd_nof == (uint32_t)s.shs[mate].numOffs())) {
					fprintf(stderr, "bt2g batch: seed search of the round not asked\n");
					abort();
				}
				{
					Ph ph(PH_AFTER_SEEDS);
					after_seeds(s, (int)mate);
				}
			}
			if(s.shs[mate].empty()) {
				s.done[mate] = true;
				break;
			}
		}
		for(size_t m = 0; m < 2; m++) {
			if(!s.shs[m].empty()) {
				s.nUniqueSeeds += s.shs[m].numUniqueSeeds();
				s.nUniqueSeedsMS[m * 2 + 0] += s.shs[m].numUniqueSeedsStrand(true);
				s.nUniqueSeedsMS[m * 2 + 1] += s.shs[m].numUniqueSeedsStrand(false);
				s.nRepeatSeeds += s.shs[m].numRepeatSeeds();
				s.nRepeatSeedsMS[m * 2 + 0] += s.shs[m].numRepeatSeedsStrand(true);
				s.nRepeatSeedsMS[m * 2 + 1] += s.shs[m].numRepeatSeedsStrand(false);
				s.seedHitTot += s.shs[m].numElts();
				s.seedHitTotMS[m * 2 + 0] += s.shs[m].numEltsFw();
				s.seedHitTotMS[m * 2 + 1] += s.shs[m].numEltsRc();
			}
		}
		{
			double uniqFactor[2] = {0.0f, 0.0f};
			for(size_t m = 0; m < 2; m++) {
				if(!s.shs[m].empty()) {
					swmSeed.sdsucc++;
					uniqFactor[m] = s.shs[m].uniquenessFactor();
				}
			}
			s.matemap[0] = 0;
			s.matemap[1] = 1;
			if(!s.shs[0].empty() && !s.shs[1].empty() && uniqFactor[1] > uniqFactor[0]) {
				s.matemap[0] = 1;
				s.matemap[1] = 0;
			}
		}
		for(s.matei = 0; s.matei < nmates; s.matei++) {
			mate = s.matemap[s.matei];
			if(s.done[mate] || s.msinkwrap.state().doneWithMate(mate == 0)) {
				s.done[mate] = true;
				continue;
			}
			if(R_seedSumm) continue;
			if(s.shs[mate].empty()) continue;
			{
				Ph ph(PH_RANK);
				s.shs[mate].rankSeedHits(s.rnd, s.msinkwrap.allHits());
			}
			start_ext(s, (int)mate, R_multiseedMms, s.seedlens[mate], s.interval[mate]);
		ext_seeds:
			ret = ext(s);
			if(ret == EXTEND_BLOCKED) {
				s.pc = P_EXT_SEEDS;
				return;
			}
			after_ext(*this, s, (int)mate, ret, false);
		}
		for(size_t m = 0; m < 2; m++)
			if(!s.done[m] && s.shs[m].averageHitsPerSeed() < R_seedBoostThresh) s.done[m] = true;
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
		for(size_t m = 0; m < nmates; m++) {
			if(s.filt[m]) {
				size_t len = s.rdlens[m];
				if(!s.nofw[m] && !s.norc[m]) len *= 2;
				totnucs += len;
			}
		}
		s.prm.seedsPerNuc = totnucs > 0 ? ((float)s.seedsTried / totnucs) : -1;
		for(int k = 0; k < 4; k++) s.prm.seedsPerNucMS[k] = totnucs > 0 ? ((float)s.seedsTriedMS[k] / totnucs) : -1;
	}
	{
		Ph ph(PH_FINISH);
		s.msinkwrap.finishRead(&s.shs[0], &s.shs[1], s.exhaustive[0], s.exhaustive[1], s.nfilt[0], s.nfilt[1], s.scfilt[0],
		                       s.scfilt[1], s.lenfilt[0], s.lenfilt[1], s.qcfilt[0], s.qcfilt[1], s.rnd, rpm, s.prm, *sc,
		                       !R_seedSumm, R_seedSumm, R_scUnMapped, R_xeq);
	}
	s.pc = P_FINISH;
}

void Svc::run(std::vector<Rq>& v, std::vector<std::pair<Slot*, DpRes*>>& dp) {
	switch(kind) {
	case K_EXACT: call_exact(v); break;
	case K_1MM: call_1mm(v); break;
	case K_SEEDS: call_seeds(v); break;
	case K_EXT: call_ext(v); break;
	case K_OFF: call_off(v); break;
	case K_UG: call_ug(v); break;
	case K_DP: call_dp(dp); break;
	}
}

// A service thread: every driver's pending requests of its kind in one call.
void Svc::loop() {
	char nm[16];
	snprintf(nm, sizeof(nm), "bt2g-svc%d", kind);
	pthread_setname_np(pthread_self(), nm);
	bt2g_prof_thread(4 + kind);
	std::vector<Lane*> got;
	std::vector<Rq> v;
	std::vector<std::pair<Slot*, DpRes*>> dp;
	for(;;) {
		{
			std::unique_lock<std::mutex> lk(q->mu);
			q->cv.wait(lk, [this] { return !q->pending.empty(); });
			got.swap(q->pending);
		}
		v.clear();
		dp.clear();
		if(cu_masked && g_paired_seen.load(std::memory_order_relaxed)) {
			// (the DP service's CU share is a --local gain for unpaired
			// reads; with pairs -- mate searches -- it lost, r05ag: 107.9 -> 65.0 k
			// pairs/s.  At the first pair the server has seen, the worker's stream
			// goes back to every CU, unless $BT2G_DP_CU asked for the share)
			int rc = bt2g_set_cu_share(ctx, 0, 0);
			if(rc) die("bt2g_set_cu_share", rc);
			cu_masked = false;
		}
		const uint64_t t0 = now_us();
		for(Lane* l : got) {
			if(kind == K_DP) dp.insert(dp.end(), l->rq_dp.begin(), l->rq_dp.end());
			else v.insert(v.end(), l->rq[kind].begin(), l->rq[kind].end());
		}
		run(v, dp);
		g_svc_us[kind] += now_us() - t0;
		if(kprof_on()) {
			std::lock_guard<std::mutex> lk(st_mu);
			for(int k = 0; k < 16; k++) (void)bt2g_kernel_stats(ctx, k, &k_launch[k], &k_ms[k]);
		}
		for(Lane* l : got) l->d->svc_done(l);
		got.clear();
	}
}

void Driver::svc_done(Lane* l) {
	std::lock_guard<std::mutex> lk(out_mu);
	if(--l->outstanding == 0) out_cv.notify_one();
}

// The device's services, started by its first driver.
std::mutex g_svc_mu;
std::vector<std::array<Svc*, K_N>> g_svcs;

// "kernels": {kind: [[launches, ms] of ids 0..15 (kernels, then host phases)], work, items} summed over devices
int svc_stats(char* buf, size_t cap) {
	if(!kwork_on()) return 0;
	std::lock_guard<std::mutex> lk(g_svc_mu);
	int n = snprintf(buf, cap, ", \"kernels\": {");
	for(int k = 0; k < K_N; k++) {
		uint64_t L[16] = {}, W = 0, I = 0, KW[16] = {}, KI[16] = {};
		double M[16] = {};
		for(auto& dv : g_svcs) {
			if(!dv[k]) continue;
			for(Svc* v : dv[k]->workers) {
				std::lock_guard<std::mutex> l2(v->st_mu);
				for(int i = 0; i < 16; i++) {
					L[i] += v->k_launch[i];
					M[i] += v->k_ms[i];
					KW[i] += v->kwork[i].load();
					KI[i] += v->kitems[i].load();
				}
				W += v->work.load();
				I += v->items.load();
			}
		}
		n += snprintf(buf + n, cap - n, "%s\"%s\": {\"work\": %llu, \"items\": %llu, \"ids\": [", k ? ", " : "",
		              K_NAMES[k], (unsigned long long)W, (unsigned long long)I);
		// [launches, ms, algorithmic work, items] per kernel id
		for(int i = 0; i < 16; i++)
			n += snprintf(buf + n, cap - n, "%s[%llu, %.3f, %llu, %llu]", i ? ", " : "", (unsigned long long)L[i], M[i],
			              (unsigned long long)KW[i], (unsigned long long)KI[i]);
		n += snprintf(buf + n, cap - n, "]}");
	}
	n += snprintf(buf + n, cap - n, "}");
	return n;
}

// Hand lane l's requests to the services (services off: make the calls here,
// one kind after another, on the driver's own context).
void Driver::submit(Lane& l) {
	if(!services_on()) {
		static const int order[K_N] = {K_EXACT, K_SEEDS, K_1MM, K_EXT, K_OFF, K_UG, K_DP};
		for(int k : order) {
			own.kind = k;
			own.run(l.rq[k], l.rq_dp);
		}
		return;
	}
	int n = 0;
	for(int k = 0; k < K_N; k++) n += (k == K_DP ? !l.rq_dp.empty() : !l.rq[k].empty()) ? 1 : 0;
	if(!n) return;
	{
		std::lock_guard<std::mutex> lk(out_mu);
		l.outstanding = n;
	}
	for(int k = 0; k < K_N; k++) {
		if(k == K_DP ? l.rq_dp.empty() : l.rq[k].empty()) continue;
		Svc* v = svc[k];
		{
			std::lock_guard<std::mutex> lk(v->mu);
			v->pending.push_back(&l);
		}
		v->cv.notify_one();
	}
}

// Wait until the services have answered lane l's requests.
void Driver::wait(Lane& l) {
	{
		std::unique_lock<std::mutex> lk(out_mu);
		out_cv.wait(lk, [&l] { return l.outstanding == 0; });
	}
	for(int k = 0; k < K_N; k++) l.rq[k].clear();
	l.rq_dp.clear();
}

void Driver::feeder() {
	pthread_setname_np(pthread_self(), "bt2g-feed");
	bt2g_prof_thread(2);
	for(;;) {
		{
			std::unique_lock<std::mutex> lk(in_mu);
			// (buffers hold <= 16 reads, pat.cpp:2023): the slots fill up to max_slots --
			// not a few buffers per round, which held a driver's intake to ~64 reads a
			// round (r04c: ~250 reads in flight per driver against 2048 slots)
			room_cv.wait(lk, [this] { return active_a.load() + 16 * inbox.size() < max_slots; });
		}
		ReadElement re = R_factory->nextReadPair();      // blocks until a connection has reads
		Elem* e = elem_new(re);
		e->conn = &re.ps->msink();
		{
			std::lock_guard<std::mutex> lk(g_conn_mu);
			g_conns[e->conn].live++;
		}
		{
			std::lock_guard<std::mutex> lk(in_mu);
			inbox.push_back(e);
		}
		in_cv.notify_one();
	}
}

// One reference fewer for connection `c` (a buffer returned or a read
// finished); its held last buffer goes back when nothing else is left.
void conn_done(const void* c, long n) {
	Elem* ret = nullptr;
	{
		std::lock_guard<std::mutex> lk(g_conn_mu);
		auto it = g_conns.find(c);
		it->second.live -= n;
		if(it->second.last && it->second.live == 1) {
			ret = it->second.last;
			g_conns.erase(it);     // (before the connection may end and its AlnSink's address be reused)
		}
	}
	if(ret) {
		R_factory->returnUnready(ret->re);
		elem_free(ret);
	}
}

// The reads of one buffer, in the order the reference's worker takes them
// (bt2_search.cpp:3201-3211, 4174: the buffer is read to its end), copied into
// slots.
// $BT2G_READ_SWAP=0: copy the buffer's reads into the slot (Read::operator=)
bool read_swap_on() {
	static const bool on = [] { const char* e = getenv("BT2G_READ_SWAP"); return !(e && *e == '0'); }();
	return on;
}

// Exchange two Reads' members: every member of a Read (read.h:246-267) is a value
// or owns its heap buffer through a pointer (SStringExpandable), none points into
// the object itself, so exchanging the bytes exchanges the reads.
void swap_read(Read& a, Read& b) {
	alignas(Read) unsigned char t[sizeof(Read)];
	memcpy(t, (void*)&a, sizeof(Read));
	memcpy((void*)&a, (void*)&b, sizeof(Read));
	memcpy((void*)&b, t, sizeof(Read));
}

void Driver::admit(Elem* e) {
	PatternSourcePerThread* ps = e->re.ps;
	long n = 0;
	bool first = true;
	do {
		if(!first) e->re.nextReadPair();
		first = false;
		if(!e->re.readResult.first) continue;
		Read& ra = ps->read_a();
		if(ra.rdid < R_skipReads || ra.rdid >= R_qUpto) continue;
		Slot* s;
		if(freel.empty()) {
			bt2g_alloc_site_scope(1);
			all.emplace_back(new Slot(*rp, *mapq, (size_t)tid));
			bt2g_alloc_site_scope(0);
			g_slots++;
			g_slots_live++;
			s = all.back().get();
			s->idx = all.size() - 1;
		} else {
			s = freel.back();
			freel.pop_back();
		}
		s->paired = !ps->read_b().empty();
		if(s->paired && !g_paired_seen.load(std::memory_order_relaxed)) g_paired_seen.store(true);
		s->rdid = ra.rdid;
		if(read_swap_on()) {
			// the buffer's reads move into the slot and the slot's previous ones into
			// the buffer, which the connection's parser resets and refills
			// (PerThreadReadBuf::reset, pat.h) -- no copy of the ~8 strings a Read holds
			swap_read(s->rdbuf[0], ra);
			if(s->paired) swap_read(s->rdbuf[1], ps->read_b());
			else s->rdbuf[1].reset();
		} else {
			const long long m1 = bt2g_alloc_thread_net();
			s->rdbuf[0] = ra;
			s->rdbuf[1] = ps->read_b();
			s->mem += bt2g_alloc_thread_net() - m1;
		}
		s->msink = &ps->msink();
		s->conn = e->conn;
		s->pc = P_START;
		s->nsteps = 0;
		n++;
		active++;
		cur->run.push_back(s);
	} while(ps->nextReadPairReady());
	// this buffer is held; the one held before goes back (a connection cannot end
	// while one of its buffers is held, whether or not the input has ended --
	// the last batch is not always marked, pat.cpp:161-192)
	const void* conn = e->conn;
	Elem* prev;
	{
		std::lock_guard<std::mutex> lk(g_conn_mu);
		Conn& c = g_conns[conn];
		c.live += n;
		prev = c.last;
		c.last = e;
	}
	if(prev) {
		R_factory->returnUnready(prev->re);
		elem_free(prev);
		conn_done(conn, 1);
	} else {
		conn_done(conn, 0);                   // (returned now if none of its reads is in flight)
	}
}

void Driver::release(Slot* s) {
	g_steps += s->nsteps;
	{
		int b = 0;
		while(b < 15 && (2u << b) <= s->nsteps) b++;
		g_steps_hist[b]++;
	}
	active--;
	{
		const long long kib = s->mem >> 10;
		int b = 0;
		while(b < 15 && (2ll << b) <= kib) b++;
		g_slot_mem_hist[b]++;
	}
	const void* conn = s->conn;
	s->conn = nullptr;
	pool_trim(s->scCurrent.pool());
	pool_trim(s->sd.ee_pool());
	if(s->mem > slot_max) {
		// rebuilt: its memory goes back to this thread's allocator cache, where the
		// next slot (or the next heavy read) takes it
		const size_t i = s->idx;
		if(i + 1 != all.size()) {
			all[i].swap(all.back());
			all[i]->idx = i;
		}
		all.pop_back();
		g_slots_rebuilt++;
		g_slots_live--;
	} else {
		freel.push_back(s);
	}
	if(((++g_reads) & 0xffff) == 0) write_stats();
	conn_done(conn, 1);
}

void Driver::run_loop() {
	open_bases();
	const size_t ndev = g_bases.size();
	if(!services_on()) {
		// (with the services a driver makes no engine call: no context, so that its
		// stream takes none of the device's hardware queues)
		int rc = bt2g_open_shared(g_bases[(size_t)tid % ndev], &ctx);
		if(rc) die("bt2g_open_shared", rc);
	}
	sc = R_sc;
	ebwtFw = R_ebwtFw;
	ebwtBw = R_ebwtBw;
	ref = R_refs;
	bsc_ok = to_scoring(*sc, bsc);
	own.ctx = ctx;
	own.bsc = &bsc;
	if(services_on()) {
		const size_t dev = (size_t)tid % ndev;
		std::lock_guard<std::mutex> lk(g_svc_mu);
		if(g_svcs.size() < ndev) g_svcs.resize(ndev, std::array<Svc*, K_N>{});
		if(!g_svcs[dev][0]) {
			static bt2g_scoring s_bsc;              // (the same scoring for every driver)
			s_bsc = bsc;
			const int nw = std::max(1, (int)env_or("BT2G_SVC_WORKERS", 2));
			// (DP calls are the longest, ~3-6 ms: with three workers the DP service was
			// saturated and the drivers queued for it -- r04q 112-129 k reads/s, r04r
			// 190-214 k with six)
			const int nd = std::max(1, (int)env_or("BT2G_DP_WORKERS", 6));
			for(int k = 0; k < K_N; k++) {
				Svc* owner = nullptr;
				// (the standalone 1-mm and extend kinds are nearly never asked -- the sweep's
				// and the seed call carry them -- so one worker each: every context is a
				// stream the runtime maps onto one of its GPU_MAX_HW_QUEUES)
				const int nk = k == K_DP ? nd : (k == K_1MM || k == K_EXT) ? 1 : nw;
				for(int w = 0; w < nk; w++) {
					Svc* v = new Svc();             // lives as long as the server
					v->kind = k;
					v->bsc = &s_bsc;
					int rc2 = bt2g_open_shared(g_bases[dev], &v->ctx);
					if(rc2) die("bt2g_open_shared", rc2);
					if(kprof_on()) (void)bt2g_set_profiling(v->ctx, 1);
					// $BT2G_SVC_PRIO=1: the FM services' streams (exact sweep, seeds,
					// offsets, ungapped: latency-bound dependent gathers) at the
					// device's highest priority, the DP service's at the default
					if(k != K_DP && env_or("BT2G_SVC_PRIO", 0) == 1) {
						int rc3 = bt2g_set_priority(v->ctx, 1);
						if(rc3) die("bt2g_set_priority", rc3);
					}
					// $BT2G_DP_CU="num/den" (default 7/8 with --local, else every CU;
					// "0/0": every CU): the DP service's streams on num of every den CUs,
					// the rest left to the FM services' short launches.  r05ae, --local:
					// its one-walker backtrace launches (~10 ms) had filled the device and
					// the one-mm family waited for CUs, 5.2 ms per launch -> 1.7 ms, 71.4 k
					// -> 88.2 k aligned reads/s (3/4: 85.4 k); r05af, end-to-end: 202.2 k
					// -> 205.3 k (3/4: 199.6 k), within the box's spread; r05ag, paired:
					// 107.9 k -> 65.0 k pairs/s (the DP call's span 2.0 -> 4.3 ms)
					if(k == K_DP) {
						static const std::pair<unsigned, unsigned> share = [] {
							unsigned a = R_localAlign ? 7 : 0, b = R_localAlign ? 8 : 0;
							if(const char* e = getenv("BT2G_DP_CU"))
								if(sscanf(e, "%u/%u", &a, &b) != 2) a = b = 0;
							return std::make_pair(a, b);
						}();
						if(share.second) {
							int rc3 = bt2g_set_cu_share(v->ctx, share.first, share.second);
							if(rc3) die("bt2g_set_cu_share", rc3);
							v->cu_masked = share.first < share.second && !getenv("BT2G_DP_CU");
						}
					}
					if(!owner) owner = v;
					v->q = owner;
					owner->workers.push_back(v);
				}
				g_svcs[dev][k] = owner;
				for(Svc* v : owner->workers) std::thread(&Svc::loop, v).detach();
			}
		}
		for(int k = 0; k < K_N; k++) svc[k] = g_svcs[dev][k];
	}
	rp.reset(new ReportingParams(R_allHits ? std::numeric_limits<THitInt>::max() : R_khits, R_mhits, 0, R_msample,
	                             gReportDiscordant, gReportMixed));
	mapq.reset(new_mapq(R_mapqv, R_scoreMin, *sc));
	// the worker's paired-end policy (bt2_search.cpp:3148-3169)
	int pepolFlag;
	if(gMate1fw && gMate2fw) pepolFlag = PE_POLICY_FF;
	else if(gMate1fw && !gMate2fw) pepolFlag = PE_POLICY_FR;
	else if(!gMate1fw && gMate2fw) pepolFlag = PE_POLICY_RF;
	else pepolFlag = PE_POLICY_RR;
	pepol.reset(new PairedEndPolicy(pepolFlag, gMaxInsert, gMinInsert, R_localAlign, gFlippedMatesOK, gDovetailMatesOK,
	                                gContainMatesOK, gOlapMatesOK, gExpandToFrag));
	// (r05c, hg38-like genome, 16 drivers: 2 048 slots per driver 203 k reads/s at
	// 98 GB of host memory after 7 passes, 1 024 192 k at 57 GB after 4, 640 171 k
	// at 43 GB: a slot holds ~1-2 MB of the reference's per-read objects)
	max_slots = env_or("BT2G_BATCH_SLOTS", 1024);
	// (r05a: at 1 MB, 18 % of the reads had their slot rebuilt -- a slot's objects
	// grow to ~0.5-2 MB on hg38-like reads -- and the drivers' CPU per read doubled)
	slot_max = (long long)env_or("BT2G_SLOT_MAX_KB", 4096) << 10;
	// (r04aa, one box: 16 -> 200 k reads/s, 8 -> 228 k, 4 -> 219 k: past 8 the
	// speculative DPs cost the drivers and the DP service more than the rounds
	// they save)
	spec_k = env_or("BT2G_SPEC_DPS", 8);
	{
		char nm[16];
		snprintf(nm, sizeof(nm), "bt2g-drv%d", tid);
		pthread_setname_np(pthread_self(), nm);
		bt2g_prof_thread(1);
	}
	// $BT2G_DRV_NICE=n: the driver threads at nice n (the engine services and the
	// connections' threads keep 0): a service thread that wakes for a call's
	// result then preempts a stepping driver instead of queueing behind it on
	// the job's CPU quota
	if(const size_t nv = env_or("BT2G_DRV_NICE", 0)) (void)setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), (int)nv);
	if(exit_clean()) {
		static std::once_flag once;
		std::call_once(once, [] { std::thread(term_watch).detach(); });
	}
	std::thread(&Driver::feeder, this).detach();
	// (r04u: two lanes 144 k reads/s against 217 k with one -- half-size lanes
	// doubled the services' calls when each driver made its own.  Round 6, the
	// services merging every driver's requests into one call per kind: two
	// lanes 272.6 / 289.0 / 287.4 k against 259.5 / 261.2 / 251.1 k, one lease,
	// r06j; r06h 280.3 / 272.9 k against 240.4 / 256.1 k -- the default.  --local,
	// whose rounds wait on a ~13 ms DP call: 102.8 / 102.2 k against 104.9 /
	// 105.7 k with one lane, r06l -- one lane there)
	const int nlanes =
	    (int)std::min<long>(2, std::max<long>(1, env_or("BT2G_LANES", R_localAlign ? 1 : 2)));
	for(Lane& l : lanes) l.d = this;
	for(int li = 0;;) {
		Lane& L = lanes[li];
		cur = &L;
		rq = L.rq;
		rq_dp = &L.rq_dp;
		got.clear();
		{
			std::unique_lock<std::mutex> lk(in_mu);
			if(active == 0 && inbox.empty()) {
				const uint64_t ti = now_us();
				in_cv.wait(lk, [this] { return !inbox.empty(); });
				g_idle_us += now_us() - ti;
			}
			got.swap(inbox);
			// (the feeder counts the taken buffers' reads as in flight until they are
			// admitted: it had seen an empty inbox and a stale count meanwhile, and
			// the slots overshot max_slots -- r04af: 45 727 slots for 16 x 2 048)
			active_a.store(active + 16 * got.size());
		}
		{
			Ph ph(PH_ADMIT);
			for(Elem* e : got) admit(e);
		}
		if(phases_on() && !g_tsc0.load()) {
			uint64_t z = 0;
			if(g_tsc0.compare_exchange_strong(z, __builtin_ia32_rdtsc())) g_us0 = now_us();
		}
		active_a.store(active);
		if(!got.empty()) room_cv.notify_one();
		const uint64_t t0 = now_us();
		g_inflight += L.run.size();
		bt2g_prof_role(3);
		for(size_t k = 0; k < L.run.size(); k++) {
			Slot* s = L.run[k];
			s->nsteps++;
			const long long m0 = bt2g_alloc_thread_net();
			{
				Ph ph(PH_STEP);
				step_read(*s);
			}
			s->mem += bt2g_alloc_thread_net() - m0;
			if(s->pc == P_FINISH) {
				Ph ph(PH_RELEASE);
				release(s);
			} else {
				L.next.push_back(s);
			}
		}
		L.run.clear();
		active_a.store(active);
		room_cv.notify_one();
		const uint64_t t1 = now_us();
		bt2g_prof_role(1);
		ph_flush();
		submit(L);
		// the other lane's requests went out a step ago: their answers are what this
		// driver waits for while L's are served (one lane: L's own)
		li = (li + 1) % nlanes;
		Lane& M = lanes[li];
		wait(M);
		M.run.swap(M.next);
		const uint64_t t2 = now_us();
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
