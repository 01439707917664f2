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
// server was started with) on device $BT2G_DEVICE (default 0); with
// $BT2G_DEVICES="0,1,..." every listed device holds a replica of the index and
// the seams' dispatchers of all devices drain the same request queues.
//
// Batching across worker threads: each seam call becomes a request that the
// calling worker thread blocks on; one dispatcher thread drains the pending
// requests of a seam (grouped by their batch-wide arguments) into ONE bt2g_*
// call and wakes the workers.  The reference's per-read control flow stays
// exactly as written -- every read still runs in its own worker thread in
// program order -- so running the server with many workers (-p 256 ... 1024)
// turns the reference's one-read-at-a-time schedule into GPU batches of
// hundreds of reads/DPs without changing any decision.  BT2G_BATCH=0 serves
// every call synchronously instead.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <signal.h>
#include <unistd.h>
#include <fcntl.h>
#include <semaphore.h>
#include <atomic>
#include <chrono>
#include <pthread.h>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>
#include <limits>
#include <memory>
#include <unordered_map>
#include <algorithm>

#include "aligner_seed.h"
#include "aligner_cache.h"
#include "aligner_sw.h"
#include "read.h"
#include "scoring.h"
#include "aligner_sw_driver.h"
#include "bt2g.h"
#include "bt2g_fibers.h"
#include "bt2g_gw_spec.h"
#include "bt2g_refspec.h"

extern "C" void bt2g_prof_thread(int role);   // bt2g_prof.cpp: CPU samples of this thread ($BT2G_SAMPLE)

namespace {

std::mutex g_mu;
bt2g_ctx* g_ctx = nullptr;

enum { ST_EXACT, ST_1MM, ST_SEEDS, ST_UG, ST_DP, ST_EXT, ST_OFF, ST_N };
const char* const ST_NAMES[ST_N] = {"exact_sweep", "one_mm", "seed_search", "ungapped", "sw_dp", "extend",
                                    "get_offset"};
std::atomic<uint64_t> g_gpu[ST_N], g_cpu[ST_N], g_batches[ST_N];
std::atomic<uint64_t> g_call_us[ST_N], g_wait_us[ST_N];   // engine time per seam; request round trips
// of a round trip: from submit until a dispatcher takes the request (queue: the
// carrier's round, the batch window, earlier batches), and from the request's
// completion until its fiber runs again (resume: the carrier's ready queue)
std::atomic<uint64_t> g_queue_us[ST_N], g_resume_us[ST_N];
// speculative DP prefetch: group requests, DPs prefetched, align() calls served
// by them, and (BT2G_SPEC_VERIFY) served ones that differed from align()'s own
std::atomic<uint64_t> g_spec_dps{0}, g_spec_hits{0}, g_spec_groups{0}, g_spec_verify_bad{0};
// seed-phase prefetch: 1-mm searches / seed searches run with the exact sweep,
// those the seams took, and (BT2G_SEEDPF_VERIFY) taken ones that differed
std::atomic<uint64_t> g_pf[6];
// $BT2G_ADAPTER_PROF=1: kernel time per engine kernel id (bt2g_kernel_stats), all dispatchers
const int NKERN = 8;
const char* const KERN_NAMES[NKERN] = {"exact_sweep", "seed_search", "one_mm", "get_offset", "sw_align",
                                       "sw_backtrace", "ungapped", "frame"};
std::atomic<uint64_t> g_kern_n[NKERN], g_kern_us[NKERN];

uint64_t now_us() {
	return (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
		std::chrono::steady_clock::now().time_since_epoch()).count();
}
char g_stats_path[4096];

void write_stats() {
	if(!g_stats_path[0]) return;
	char buf[4096];
	int n = 0;
	n += snprintf(buf + n, sizeof(buf) - n, "{");
	for(int i = 0; i < ST_N; i++)
		n += snprintf(buf + n, sizeof(buf) - n, "%s\"%s\": [%llu, %llu, %llu, %.1f, %.1f]", i ? ", " : "",
		              ST_NAMES[i], (unsigned long long)g_gpu[i].load(), (unsigned long long)g_cpu[i].load(),
		              (unsigned long long)g_batches[i].load(), g_call_us[i].load() / 1000.0,
		              g_wait_us[i].load() / 1000.0);
	n += snprintf(buf + n, sizeof(buf) - n, ", \"queue_ms\": [");
	for(int i = 0; i < ST_N; i++)
		n += snprintf(buf + n, sizeof(buf) - n, "%s%.1f", i ? ", " : "", g_queue_us[i].load() / 1000.0);
	n += snprintf(buf + n, sizeof(buf) - n, "], \"resume_ms\": [");
	for(int i = 0; i < ST_N; i++)
		n += snprintf(buf + n, sizeof(buf) - n, "%s%.1f", i ? ", " : "", g_resume_us[i].load() / 1000.0);
	n += snprintf(buf + n, sizeof(buf) - n, "]");
	n += snprintf(buf + n, sizeof(buf) - n, ", \"spec\": [%llu, %llu, %llu, %llu]",
	              (unsigned long long)g_spec_groups.load(), (unsigned long long)g_spec_dps.load(),
	              (unsigned long long)g_spec_hits.load(), (unsigned long long)g_spec_verify_bad.load());
	n += snprintf(buf + n, sizeof(buf) - n, ", \"pf\": [%llu, %llu, %llu, %llu, %llu, %llu]",
	              (unsigned long long)g_pf[0].load(), (unsigned long long)g_pf[1].load(),
	              (unsigned long long)g_pf[2].load(), (unsigned long long)g_pf[3].load(),
	              (unsigned long long)g_pf[4].load(), (unsigned long long)g_pf[5].load());
	n += snprintf(buf + n, sizeof(buf) - n, ", \"kernels\": {");
	for(int i = 0; i < NKERN; i++)
		n += snprintf(buf + n, sizeof(buf) - n, "%s\"%s\": [%llu, %.1f]", i ? ", " : "", KERN_NAMES[i],
		              (unsigned long long)g_kern_n[i].load(), g_kern_us[i].load() / 1000.0);
	n += snprintf(buf + n, sizeof(buf) - n, "}}\n");
	int fd = open(g_stats_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
	if(fd >= 0) {
		ssize_t w = write(fd, buf, (size_t)n);
		(void)w;
		close(fd);
	}
}

extern "C" void bt2g_alloc_stats_dump();   // bt2g_alloc.cpp ($BT2G_ALLOC_STATS)

void on_term(int) {
	write_stats();
	bt2g_alloc_stats_dump();
	bt2gf::mutex_prof_dump();
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

// The HIP runtime's settings, from a static initializer: before main, so before
// any thread exists (setenv is not safe against a concurrent getenv).
struct EnvInit {
	EnvInit() {
		// dispatcher threads sleep in their stream waits: the server's workers need the
		// cores (the runtime's blocking wait still spins: r03d, 21 % of the CPU)
		setenv("BT2G_SYNC", "poll", 0);
		// one HIP hardware queue per stream (a context per seam dispatcher, ~10
		// streams): with HIP's default of 4 -- also what the GPU box exports -- a
		// 0.05 ms seed-search kernel waits behind other seams' DP kernels on a shared
		// in-order queue (r03p at 3.1 Gbp: 29.4k -> 43.6k reads/s with 16 queues).
		// $BT2G_HW_QUEUES overrides, clamped to the runtime's 1..32.
		const char* hq = getenv("BT2G_HW_QUEUES");
		int q = hq && atoi(hq) > 0 ? atoi(hq) : 16;
		if(q > 32) q = 32;
		char buf[16];
		snprintf(buf, sizeof(buf), "%d", q);
		setenv("GPU_MAX_HW_QUEUES", buf, 1);
	}
} g_env_init;

// $BT2G_ADAPTER_STATS: where the call counts go (written on SIGTERM too).
void init_env() {
	static std::once_flag once;
	std::call_once(once, [] {
		const char* sp = getenv("BT2G_ADAPTER_STATS");
		if(sp) {
			strncpy(g_stats_path, sp, sizeof(g_stats_path) - 1);
			signal(SIGTERM, on_term);
		}
		if(!getenv("BT2G_INDEX")) {
			fprintf(stderr, "bt2g adapter: BT2G_INDEX is not set\n");
			throw 1;
		}
	});
}

// The devices the dispatchers use: $BT2G_DEVICES (comma-separated, e.g.
// "0,1,2,3"; default $BT2G_DEVICE, else 0), one full index replica each
// (reads are independent, no exchange).  The first is g_ctx.
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

// Index replicas of the devices after the first (opened with the dispatchers).
std::vector<bt2g_ctx*> g_replicas;

// Opened lazily under g_mu.
bt2g_ctx* ctx() {
	if(g_ctx) return g_ctx;
	const char* base = getenv("BT2G_INDEX");
	if(!base) {
		fprintf(stderr, "bt2g adapter: BT2G_INDEX is not set\n");
		throw 1;
	}
	init_env();
	int rc = bt2g_open(base, devices()[0], &g_ctx);
	if(rc) die("bt2g_open", rc);
	return g_ctx;
}

// The batching dispatcher threads each own a context on one replica
// (bt2g_open_shared: own HIP stream and scratch), so the seams' batches run
// concurrently on the GPUs; the synchronous path uses the base context under g_mu.
thread_local bt2g_ctx* t_ctx = nullptr;
bt2g_ctx* cur_ctx() { return t_ctx ? t_ctx : ctx(); }

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

// A read as one row of codes (0..4) and Phred+33 qualities, inline: requests
// live on the caller's (fiber's) stack and allocate nothing.
struct Row {
	uint32_t len = 0;
	uint8_t codes[BT2G_MAX_READ_LEN];
	uint8_t quals[BT2G_MAX_READ_LEN];
	void set(const BTDnaString& s, const BTString& q) {
		len = (uint32_t)std::min<size_t>(s.length(), BT2G_MAX_READ_LEN);
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

// Outputs owned by the requester: up to N inline, a heap vector beyond.  The
// dispatcher writes them; keeping them inline means no block allocated by a
// dispatcher thread is freed by a carrier thread (glibc arena locks: 30 % of
// the host CPU in r03a).
template <typename T, size_t N>
struct Out {
	T inl[N];
	std::vector<T> big;
	size_t n = 0;
	void assign(const T* p, size_t k) {
		n = k;
		T* d = inl;
		if(k > N) {
			big.assign(p, p + k);
			return;
		}
		if(k) memcpy(d, p, k * sizeof(T));
	}
	const T* data() const { return n > N ? big.data() : inl; }
	size_t size() const { return n; }
	const T& operator[](size_t i) const { return data()[i]; }
};

// ---- requests and the dispatcher ---------------------------------------------
struct Req {
	int kind;
	uint64_t key;        // batch-wide arguments: requests with equal keys share one call
	int rc = 0;
	char err[256] = {0}; // bt2g_last_error() of the thread that ran the call
	void* fiber = nullptr;   // the waiting fiber (bt2g_fibers.cpp), else an OS thread on sem
	uint64_t t_sub = 0, t_take = 0, t_done = 0;   // submit, taken by a dispatcher, completed (us)
	std::atomic<int>* group = nullptr;   // submit_group: requests still to complete (the last wakes)
	sem_t sem;
	Req(int k, uint64_t ky) : kind(k), key(ky) {}
};

struct MmReq;
struct ExactReq : Req {      // bt2g_exact_sweep
	Row r;
	uint32_t mine_max;
	int nofw, norc;
	uint32_t out[8];
	MmReq* mm = nullptr;         // seed-phase prefetch: the gated 1-mm search to run after the sweep
	ExactReq(uint32_t mm, int f, int c) : Req(ST_EXACT, ((uint64_t)mm << 2) | (uint64_t)(f << 1) | (uint64_t)c),
	                                      mine_max(mm), nofw(f), norc(c) {}
};

struct MmReq : Req {         // bt2g_one_mm
	Row r;
	int32_t minsc;
	int nofw, norc;
	bt2g_scoring sc;
	Out<bt2g_mm1, 32> hits;
	int32_t cnt = 0;
	uint32_t ops = 0;
	bool pf_ran = false;         // (prefetch) the exact sweep's dispatcher ran it
	MmReq(int f, int c, const bt2g_scoring& s)
		: Req(ST_1MM, (uint64_t)(f << 1) | (uint64_t)c | ((uint64_t)s.local << 2)), nofw(f), norc(c), sc(s) {}
};

struct SeedReq : Req {       // bt2g_seed_search
	Row r;
	uint32_t seedlen, per, off, nof;
	Out<uint32_t, 2 * 32 * 4> out;    // [strand][seed offset][topf, botf, topb, botb]
	int32_t ns = 0;
	uint32_t ops = 0;
	SeedReq(uint32_t L, uint32_t p, uint32_t o, uint32_t n)
		: Req(ST_SEEDS, ((uint64_t)L << 48) | ((uint64_t)p << 24) | (uint64_t)o), seedlen(L), per(p), off(o), nof(n) {}
};

struct UgReq : Req {         // bt2g_ungapped
	Row r;
	bt2g_ug_problem p;
	bt2g_scoring sc;
	int ohang;
	bt2g_ug_result o;
	Out<bt2g_edit, 64> ed;
	UgReq(const bt2g_scoring& s, int oh) : Req(ST_UG, (uint64_t)oh | ((uint64_t)s.local << 1)), sc(s), ohang(oh) {}
};

struct DpState;

struct DpReq : Req {         // bt2g_sw_align_bt
	Row r;
	bt2g_sw_problem p;
	bt2g_sw_rect rect;
	std::vector<uint8_t> win;
	bt2g_scoring sc;
	int enable8;
	uint32_t cap, maxaln, maxedit;
	bt2g_sw_result o;
	DpState* st;                 // the SwAligner's state: receives candidates, fates, alignments, edits
	int32_t naln = 0;
	bool cpu = false;            // more candidates than the engine takes (> 8192): the CPU path
	// reads longer than 1024 bases batch apart (another fill; a batch is padded to its longest read)
	DpReq(const bt2g_scoring& s, int e8, bool lng, DpState* state)
		: Req(ST_DP, (uint64_t)e8 | ((uint64_t)s.local << 1) | ((uint64_t)lng << 2)), sc(s), enable8(e8), st(state) {}
};

// Per-SwAligner state between align() and the nextAlignment() calls (one per
// SwAligner of each worker; its vectors keep their capacity read after read).
struct DpState {
	bool gpu = false;          // served by the engine (else the reference's CPU path)
	bool u8 = false;           // u8 fill succeeded (RNG re-seed rule, aligner_sw.cpp:877 vs 932)
	std::vector<bt2g_sw_cand> cands;   // the sorted candidates
	std::vector<int8_t> fates; // engine's DpBtCandidate::fate per candidate
	std::vector<bt2g_sw_aln> alns;
	std::vector<bt2g_edit> edits;   // of every alignment, back to back
	uint32_t maxedit = 0;
	int32_t naln = 0;
	uint32_t next = 0;         // next engine alignment to hand out
	size_t next_edit = 0;      // its first edit
	// the problem as sent to the engine (for $BT2G_ADAPTER_DUMP on a mismatch)
	Row row;
	bt2g_sw_problem prob;
	bt2g_sw_rect rect;
	std::vector<uint8_t> win;
	int enable8 = 1;
};

struct ExtReq : Req {         // bt2g_extend: every seed-hit range of one read
	Row r;
	std::vector<bt2g_ext_in> in;       // (.read is set by the dispatcher)
	Out<bt2g_ext_out, 64> out;
	ExtReq() : Req(ST_EXT, 0) {}
};

struct OffReq : Req {         // bt2g_get_offset: the SA rows one read's walks resolve
	Row r;                        // (unused: no read data)
	std::vector<uint32_t> rows;
	Out<uint32_t, 128> offs;
	OffReq() : Req(ST_OFF, 0) { r.len = 0; }
};

// Rows of a batch as one [n][stride] array (stride = longest read); one per
// dispatcher thread, reused call after call.
struct Pack {
	std::vector<uint8_t> codes, quals;
	std::vector<uint32_t> lens;
	uint32_t stride = 1;
	template <typename R>
	void build(const std::vector<R*>& v) {
		stride = 1;
		for(R* q : v) stride = std::max(stride, q->r.len);
		codes.resize(v.size() * (size_t)stride);
		quals.resize(v.size() * (size_t)stride);
		lens.resize(v.size());
		for(size_t i = 0; i < v.size(); i++) {
			const uint32_t L = v[i]->r.len;
			lens[i] = L;
			uint8_t* c = &codes[i * stride];
			uint8_t* q = &quals[i * stride];
			memcpy(c, v[i]->r.codes, L);
			memcpy(q, v[i]->r.quals, L);
			if(L < stride) {
				memset(c + L, 4, stride - L);
				memset(q + L, 'I', stride - L);
			}
		}
	}
};

int run_mm(const std::vector<MmReq*>& v, uint32_t cap);
void enqueue_1mm(const std::vector<MmReq*>& v);   // onto the 1-mm seam's queue (Dispatcher below)

int run_exact(const std::vector<ExactReq*>& v) {
	thread_local Pack pk;
	thread_local std::vector<uint32_t> out;
	pk.build(v);
	out.resize(8 * v.size());
	int rc = bt2g_exact_sweep(cur_ctx(), pk.codes.data(), pk.stride, pk.lens.data(), (uint32_t)v.size(), v[0]->mine_max,
	                          v[0]->nofw, v[0]->norc, out.data());
	if(rc) return rc;
	for(size_t i = 0; i < v.size(); i++) memcpy(v[i]->out, &out[8 * i], sizeof(v[i]->out));
	// seed-phase prefetch: the 1-mm search the worker asks next, gated as
	// bt2_search.cpp:3640-3667 gates it (a strand whose sweep found <= 1 edit;
	// reads with exact hits too: most are not done after extending them, stub
	// run at 20 Mbp: 25 k of 30 k reads asked), goes to the 1-mm seam's queue
	// in the same round trip: the request's group (the worker's wait) grows by
	// one before the sweep's request completes.  (Run in this dispatcher's own
	// call instead it saturated the sweep's dispatcher, r03x / r03y.)
	std::vector<MmReq*> mm;
	for(ExactReq* q : v) {
		if(!q->mm || !q->group) continue;
		const bool yfw = !q->nofw && q->out[0] <= 1, yrc = !q->norc && q->out[1] <= 1;
		if(!yfw && !yrc) continue;
		MmReq* m = q->mm;
		m->nofw = yfw ? 0 : 1;
		m->norc = yrc ? 0 : 1;
		m->key = (uint64_t)(m->nofw << 1) | (uint64_t)m->norc | ((uint64_t)m->sc.local << 2);
		m->fiber = q->fiber;
		m->group = q->group;
		m->pf_ran = true;
		m->rc = 0;
		m->t_sub = now_us();
		q->group->fetch_add(1);
		mm.push_back(m);
	}
	if(!mm.empty()) {
		g_pf[0] += mm.size();
		enqueue_1mm(mm);
	}
	return BT2G_OK;
}

int run_mm(const std::vector<MmReq*>& v, uint32_t cap) {
	struct B {
		Pack pk;
		std::vector<int32_t> ms, cnt;
		std::vector<uint32_t> ops;
		std::vector<bt2g_mm1> h;
	};
	thread_local B b;
	b.pk.build(v);
	const size_t n = v.size();
	b.ms.resize(n);
	b.cnt.resize(n);
	b.ops.resize(n);
	b.h.resize(n * cap);
	for(size_t i = 0; i < n; i++) b.ms[i] = v[i]->minsc;
	int rc = bt2g_one_mm(cur_ctx(), b.pk.codes.data(), b.pk.quals.data(), b.pk.stride, b.pk.lens.data(), (uint32_t)n,
	                     b.ms.data(), &v[0]->sc, v[0]->nofw, v[0]->norc, cap, b.h.data(), b.cnt.data(), b.ops.data(),
	                     nullptr);
	if(rc && rc != BT2G_ERR_OVERFLOW) return rc;
	std::vector<std::pair<MmReq*, uint32_t>> again;    // more hits than the batch slots: alone, after
	for(size_t i = 0; i < n; i++) {
		if(b.cnt[i] > (int32_t)cap) {
			again.emplace_back(v[i], (uint32_t)b.cnt[i]);
			continue;
		}
		v[i]->cnt = b.cnt[i];
		v[i]->ops = b.ops[i];
		v[i]->hits.assign(&b.h[i * cap], (size_t)b.cnt[i]);
	}
	for(auto& qa : again) {
		std::vector<MmReq*> one{qa.first};
		if((rc = run_mm(one, qa.second))) return rc;
	}
	return BT2G_OK;
}

int run_seeds(const std::vector<SeedReq*>& v) {
	struct B {
		Pack pk;
		std::vector<uint32_t> out, ops;
		std::vector<int32_t> ns;
		std::vector<uint32_t> tmp;
	};
	thread_local B b;
	b.pk.build(v);
	const size_t n = v.size();
	uint32_t maxs = 1;
	for(SeedReq* q : v) maxs = std::max(maxs, q->nof);
	b.out.resize(n * 2 * maxs * 4);
	b.ops.resize(n);
	b.ns.resize(n);
	int rc = bt2g_seed_search(cur_ctx(), b.pk.codes.data(), b.pk.stride, b.pk.lens.data(), (uint32_t)n, v[0]->seedlen,
	                          v[0]->per, v[0]->off, maxs, b.out.data(), b.ns.data(), b.ops.data(), nullptr);
	if(rc) return rc;
	for(size_t i = 0; i < n; i++) {
		SeedReq* q = v[i];
		q->ns = b.ns[i];
		q->ops = b.ops[i];
		b.tmp.assign(2 * (size_t)q->nof * 4, 0);
		for(int f = 0; f < 2; f++)
			for(uint32_t k = 0; k < q->nof && k < maxs; k++)
				memcpy(&b.tmp[((size_t)f * q->nof + k) * 4], &b.out[((i * 2 + f) * maxs + k) * 4], 16);
		q->out.assign(b.tmp.data(), b.tmp.size());
	}
	return BT2G_OK;
}

int run_ug(const std::vector<UgReq*>& v) {
	struct B {
		Pack pk;
		std::vector<bt2g_ug_problem> P;
		std::vector<bt2g_ug_result> R;
		std::vector<bt2g_edit> E;
	};
	thread_local B b;
	b.pk.build(v);
	const size_t n = v.size();
	const uint32_t maxedit = b.pk.stride + 1;
	b.P.resize(n);
	b.R.resize(n);
	b.E.resize(n * maxedit);
	for(size_t i = 0; i < n; i++) {
		b.P[i] = v[i]->p;
		b.P[i].read = (uint32_t)i;
	}
	int rc = bt2g_ungapped(cur_ctx(), b.pk.codes.data(), b.pk.quals.data(), b.pk.stride, b.pk.lens.data(), b.P.data(),
	                       (uint32_t)n, &v[0]->sc, v[0]->ohang, maxedit, b.R.data(), b.E.data());
	if(rc) return rc;
	for(size_t i = 0; i < n; i++) {
		v[i]->o = b.R[i];
		const int32_t ne = b.R[i].ret == 1 ? std::min<int32_t>(std::max<int32_t>(b.R[i].nedit, 0), (int32_t)maxedit) : 0;
		v[i]->ed.assign(&b.E[i * maxedit], (size_t)ne);
	}
	return BT2G_OK;
}

// Fill + gather + the nextAlignment loop for every DP of the batch
// (bt2g_sw_align_bt_packed: only the candidates, fates and edits the problems
// produced come back).  A DP whose candidate list outgrew `cap`, or that may
// have more than `maxaln` alignments, runs again alone with room for all of them.
struct DpBufs {      // per dispatcher thread, grown as needed, never shrunk
	Pack pk;
	std::vector<bt2g_sw_problem> P;
	std::vector<bt2g_sw_rect> RC;
	std::vector<uint8_t> W;
	std::vector<bt2g_sw_result> R;
	std::vector<int32_t> NA;
	std::vector<bt2g_sw_aln> A;
	std::unique_ptr<bt2g_sw_cand[]> C;
	std::unique_ptr<int8_t[]> F;
	std::unique_ptr<bt2g_edit[]> E;
	size_t ncap = 0, necap = 0;
};

int run_dp(const std::vector<DpReq*>& v, uint32_t cap = 0, uint32_t maxaln = 8) {
	thread_local DpBufs b;
	Pack& pk = b.pk;
	pk.build(v);
	const size_t n = v.size();
	if(cap == 0) cap = v[0]->sc.local ? 2048 : 512;
	const uint32_t maxedit = 2 * pk.stride + 8;
	b.P.resize(n);
	b.RC.resize(n);
	b.W.clear();
	for(size_t i = 0; i < n; i++) {
		b.P[i] = v[i]->p;
		b.P[i].read = (uint32_t)i;
		if(v[i]->p.win_off >= 0) {     // the caller's window (align(): initRef's); else the resident reference
			b.P[i].win_off = (int64_t)b.W.size();
			b.W.insert(b.W.end(), v[i]->win.begin(), v[i]->win.end());
		}
		b.RC[i] = v[i]->rect;
	}
	b.R.resize(n);
	b.NA.resize(n);
	b.A.resize(n * maxaln);
	// packed outputs: worst-case capacity, only the used prefix is ever touched
	if(b.ncap < n * (size_t)cap) {
		b.ncap = n * (size_t)cap;
		b.C.reset(new bt2g_sw_cand[b.ncap]);
		b.F.reset(new int8_t[b.ncap]);
	}
	if(b.necap < n * (size_t)maxaln * maxedit) {
		b.necap = n * (size_t)maxaln * maxedit;
		b.E.reset(new bt2g_edit[b.necap]);
	}
	uint64_t tot[3] = {0, 0, 0};
	int rc = bt2g_sw_align_bt_packed(cur_ctx(), pk.codes.data(), pk.quals.data(), pk.stride, pk.lens.data(), b.P.data(),
	                                 (uint32_t)n, b.W.data(), b.W.size(), b.RC.data(), &v[0]->sc, v[0]->enable8, cap,
	                                 b.R.data(), maxaln, maxedit, b.NA.data(), b.A.data(), b.C.get(), b.F.get(),
	                                 b.E.get(), tot);
	if(rc && rc != BT2G_ERR_OVERFLOW) return rc;
	std::vector<std::pair<DpReq*, uint32_t>> again;      // (their own calls below reuse b)
	size_t oc = 0, oe = 0;
	for(size_t i = 0; i < n; i++) {
		DpReq* q = v[i];
		const bt2g_sw_result& r = b.R[i];
		const uint32_t nc = (uint32_t)std::min<int64_t>(std::max<int32_t>(r.ncand, 0), cap);
		const uint32_t na = (uint32_t)std::min<int64_t>(std::max<int32_t>(b.NA[i], 0), maxaln);
		uint32_t ne = 0;
		for(uint32_t k = 0; k < na; k++)
			ne += (uint32_t)std::min<int64_t>(std::max<int32_t>(b.A[i * maxaln + k].nedit, 0), maxedit);
		const size_t c0 = oc, e0 = oe;
		oc += nc;
		oe += ne;
		if(r.ncand > 8192) {         // beyond the engine's candidate capacity
			q->cpu = true;
			continue;
		}
		if(r.ncand > (int32_t)cap || (b.NA[i] == (int32_t)maxaln && r.ncand > (int32_t)maxaln)) {
			again.emplace_back(q, (uint32_t)r.ncand);
			continue;
		}
		q->o = r;
		q->naln = b.NA[i];
		q->cap = cap;
		q->maxaln = maxaln;
		q->maxedit = maxedit;
		DpState* st = q->st;
		st->cands.assign(b.C.get() + c0, b.C.get() + c0 + nc);
		st->fates.assign(b.F.get() + c0, b.F.get() + c0 + nc);
		st->alns.assign(b.A.begin() + i * maxaln, b.A.begin() + i * maxaln + na);
		st->edits.assign(b.E.get() + e0, b.E.get() + e0 + ne);
	}
	if(oc != tot[0] || oe != tot[2]) {
		fprintf(stderr, "bt2g adapter: packed DP outputs %llu/%llu, expected %zu/%zu\n", (unsigned long long)tot[0],
		        (unsigned long long)tot[2], oc, oe);
		return BT2G_ERR_FORMAT;
	}
	for(auto& qa : again) {
		std::vector<DpReq*> one{qa.first};
		if((rc = run_dp(one, std::max<uint32_t>(cap, qa.second), std::max<uint32_t>(maxaln, qa.second)))) return rc;
	}
	return BT2G_OK;
}

int run_ext(const std::vector<ExtReq*>& v) {
	struct B {
		Pack pk;
		std::vector<bt2g_ext_in> in;
		std::vector<bt2g_ext_out> out;
	};
	thread_local B b;
	b.pk.build(v);
	b.in.clear();
	for(size_t i = 0; i < v.size(); i++)
		for(const bt2g_ext_in& q : v[i]->in) {
			b.in.push_back(q);
			b.in.back().read = (uint32_t)i;
		}
	b.out.resize(b.in.size());
	int rc = bt2g_extend(cur_ctx(), b.pk.codes.data(), b.pk.stride, b.pk.lens.data(), (uint32_t)v.size(), b.in.data(),
	                     (uint32_t)b.in.size(), b.out.data());
	if(rc) return rc;
	size_t k = 0;
	for(ExtReq* q : v) {
		q->out.assign(&b.out[k], q->in.size());
		k += q->in.size();
	}
	return BT2G_OK;
}

int run_off(const std::vector<OffReq*>& v) {
	struct B {
		std::vector<uint32_t> rows, offs;
	};
	thread_local B b;
	b.rows.clear();
	for(OffReq* q : v) b.rows.insert(b.rows.end(), q->rows.begin(), q->rows.end());
	b.offs.resize(b.rows.size());
	int rc = bt2g_get_offset(cur_ctx(), b.rows.data(), (uint32_t)b.rows.size(), b.offs.data(), nullptr);
	if(rc) return rc;
	size_t k = 0;
	for(OffReq* q : v) {
		q->offs.assign(&b.offs[k], q->rows.size());
		k += q->rows.size();
	}
	return BT2G_OK;
}

int run_group(int kind, const std::vector<Req*>& g) {
	switch(kind) {
	case ST_EXACT: { std::vector<ExactReq*> v; for(Req* r : g) v.push_back(static_cast<ExactReq*>(r)); return run_exact(v); }
	case ST_1MM:   { std::vector<MmReq*> v;    for(Req* r : g) v.push_back(static_cast<MmReq*>(r));    return run_mm(v, 16); }
	case ST_SEEDS: { std::vector<SeedReq*> v;  for(Req* r : g) v.push_back(static_cast<SeedReq*>(r));  return run_seeds(v); }
	case ST_UG:    { std::vector<UgReq*> v;    for(Req* r : g) v.push_back(static_cast<UgReq*>(r));    return run_ug(v); }
	case ST_EXT:   { std::vector<ExtReq*> v;   for(Req* r : g) v.push_back(static_cast<ExtReq*>(r));   return run_ext(v); }
	case ST_OFF:   { std::vector<OffReq*> v;   for(Req* r : g) v.push_back(static_cast<OffReq*>(r));   return run_off(v); }
	default:       { std::vector<DpReq*> v;    for(Req* r : g) v.push_back(static_cast<DpReq*>(r));    return run_dp(v); }
	}
}

const size_t MAX_BATCH = 8192;
// requests that make a batch worth launching at once ($BT2G_BATCH_TARGET), and
// the longest wait for them after the first arrives ($BT2G_BATCH_WINDOW_US)
size_t env_or(const char* name, size_t dflt) {
	const char* e = getenv(name);
	return e && atol(e) > 0 ? (size_t)atol(e) : dflt;
}
// (fiber workers hand requests over a carrier round at a time, in bursts: a
// shorter window, a larger target)
const size_t BATCH_TARGET = env_or("BT2G_BATCH_TARGET", bt2gf::enabled() ? 1024 : 256);
const int BATCH_WINDOW_US = (int)env_or("BT2G_BATCH_WINDOW_US", bt2gf::enabled() ? 200 : 300);

bool seedpf_enabled();

class Dispatcher {
public:
	// Serve one request: queued for its seam's dispatcher thread (batching on)
	// or run at once under the shared context's lock.
	void submit(Req* r) {
		const uint64_t t0 = now_us();
		r->t_sub = t0;
		if(void* f = bt2gf::self()) {
			// a fiber (bt2g_fibers.cpp): the carrier hands the request over with the
			// rest of its round (flush below) and resumes the fiber when it is done
			r->fiber = f;
			bt2gf::block_on(r);
		} else if(!batching()) {
			std::lock_guard<std::mutex> lk(g_mu);
			r->rc = run_group(r->kind, std::vector<Req*>{r});
			if(r->rc) strncpy(r->err, bt2g_last_error(), sizeof(r->err) - 1);
			g_batches[r->kind]++;
		} else {
			sem_init(&r->sem, 0, 0);
			Q& q = q_[r->kind];
			{
				std::lock_guard<std::mutex> lk(q.mu);
				q.v.push_back(r);
			}
			q.cv.notify_one();
			while(sem_wait(&r->sem) != 0) {}
			sem_destroy(&r->sem);
		}
		const uint64_t t1 = now_us();
		g_wait_us[r->kind] += t1 - t0;
		if(r->t_take) g_queue_us[r->kind] += r->t_take - t0;
		if(r->t_done) g_resume_us[r->kind] += t1 - r->t_done;
		if(r->rc) {
			fprintf(stderr, "bt2g adapter: %s failed (%d): %s\n", ST_NAMES[r->kind], r->rc, r->err);
			throw 1;
		}
	}

	// Several requests of one worker at once (a fiber waits once, for all).
	void submit_group(Req* const* v, size_t n) {
		if(n == 0) return;
		void* f = bt2gf::self();
		if(!f) {
			for(size_t i = 0; i < n; i++) submit(v[i]);
			return;
		}
		std::atomic<int> left((int)n);
		const uint64_t t0 = now_us();
		for(size_t i = 0; i < n; i++) {
			v[i]->fiber = f;
			v[i]->group = &left;
			v[i]->t_sub = t0;
		}
		bt2gf::block_on_many(reinterpret_cast<void* const*>(v), n);
		const uint64_t t1 = now_us();
		for(size_t i = 0; i < n; i++) {
			Req* r = v[i];
			r->group = nullptr;
			g_wait_us[r->kind] += t1 - t0;
			if(r->t_take) g_queue_us[r->kind] += r->t_take - t0;
			if(r->t_done) g_resume_us[r->kind] += t1 - r->t_done;
			if(r->rc) {
				fprintf(stderr, "bt2g adapter: %s failed (%d): %s\n", ST_NAMES[r->kind], r->rc, r->err);
				throw 1;
			}
		}
	}

	void start() { (void)batching(); }

	// A carrier's round of fiber requests (bt2gf::set_flush): one lock per seam.
	static void flush(void* const* reqs, size_t n) {
		Dispatcher& d = instance();
		for(int k = 0; k < ST_N; k++) {
			bool any = false;
			for(size_t i = 0; i < n && !any; i++) any = static_cast<Req*>(reqs[i])->kind == k;
			if(!any) continue;
			Q& q = d.q_[k];
			{
				std::lock_guard<std::mutex> lk(q.mu);
				for(size_t i = 0; i < n; i++)
					if(static_cast<Req*>(reqs[i])->kind == k) q.v.push_back(static_cast<Req*>(reqs[i]));
			}
			q.cv.notify_one();
		}
	}
	static Dispatcher& instance();

	// requests a dispatcher hands on to another seam (their waiters' groups
	// already count them)
	void enqueue(int kind, Req* const* reqs, size_t n) {
		Q& q = q_[kind];
		{
			std::lock_guard<std::mutex> lk(q.mu);
			q.v.insert(q.v.end(), reqs, reqs + n);
		}
		q.cv.notify_one();
	}

private:
	struct Q {
		std::mutex mu;
		std::condition_variable cv;
		std::vector<Req*> v;
	};

	bool batching() {
		std::call_once(once_, [this] {
			const char* b = getenv("BT2G_BATCH");
			on_ = !(b && b[0] == '0');
			if(!on_ && bt2gf::enabled()) {
				fprintf(stderr, "bt2g adapter: fibers need batching (BT2G_BATCH=0 with BT2G_FIBERS=1)\n");
				throw 1;
			}
			if(on_) {
				init_env();
				{
					std::lock_guard<std::mutex> lk(g_mu);
					ctx();                          // the base context, before any dispatcher
				}
				// one index replica per further device, loaded concurrently
				const std::vector<int> devs = devices();
				std::vector<bt2g_ctx*> bases{g_ctx};
				g_replicas.assign(devs.size() - 1, nullptr);
				{
					std::vector<std::thread> ld;
					std::vector<int> rcs(devs.size(), 0);
					for(size_t i = 1; i < devs.size(); i++)
						ld.emplace_back([&, i] { rcs[i] = bt2g_open(getenv("BT2G_INDEX"), devs[i], &g_replicas[i - 1]); });
					for(std::thread& t : ld) t.join();
					for(size_t i = 1; i < devs.size(); i++) {
						if(rcs[i]) die("bt2g_open (replica)", rcs[i]);
						bases.push_back(g_replicas[i - 1]);
					}
				}
				// dispatchers per seam and device: $BT2G_SEAM_THREADS (default 1; the DP
				// seam, whose batches take longest, twice that), or per seam
				// $BT2G_SEAM_THREADS_<seam> (e.g. BT2G_SEAM_THREADS_one_mm=2); all of a
				// seam's dispatchers drain the one queue, so the devices share its load.
				// (r03i at 3.1 Gbp: 2 per seam 25.2k reads/s, 1 per seam 28.6k -- the
				// streams' kernels slow each other more than they overlap; with 16 HW
				// queues the DP seam gains from 4: r03q 40.7k -> 43.2k, r03t 54.8k)
				const char* t = getenv("BT2G_SEAM_THREADS");
				const int per = std::max(1, t ? atoi(t) : 1);
				for(bt2g_ctx* b : bases)
					for(int k = 0; k < ST_N; k++) {
						char nm[64];
						snprintf(nm, sizeof(nm), "BT2G_SEAM_THREADS_%s", ST_NAMES[k]);
						const char* tk = getenv(nm);
						// (the exact sweep's dispatcher also runs the prefetched 1-mm searches:
						// two of them, r03x: one was saturated, 3.9 ms per call)
						const int nk = tk && atoi(tk) > 0 ? atoi(tk)
						                                  : (k == ST_DP ? 4 * per : k == ST_EXACT && seedpf_enabled() ? 2 * per : per);
						for(int i = 0; i < nk; i++) std::thread(&Dispatcher::loop, this, k, b).detach();
					}
			}
		});
		return on_;
	}

	// Dispatcher threads of a seam share its queue: each drains it into batches,
	// grouped by the batch-wide arguments (arrival order kept within a group), on
	// its own context.
	void loop(int kind, bt2g_ctx* base) {
		bt2g_prof_thread(2);
		{
			char nm[16];
			snprintf(nm, sizeof(nm), "bt2g-%.10s", ST_NAMES[kind]);
			pthread_setname_np(pthread_self(), nm);
		}
		int rc0 = bt2g_open_shared(base, &t_ctx);
		if(rc0) {
			fprintf(stderr, "bt2g adapter: bt2g_open_shared (%s dispatcher) failed (%d): %s\n", ST_NAMES[kind], rc0,
			        bt2g_last_error());
			t_ctx = nullptr;                 // fall back to the shared context under g_mu
		}
		const char* pf = getenv("BT2G_ADAPTER_PROF");
		const bool prof = t_ctx && pf && pf[0] == '1';
		if(prof) bt2g_set_profiling(t_ctx, 1);
		uint64_t seen_n[NKERN] = {0};
		double seen_ms[NKERN] = {0};
		Q& q = q_[kind];
		std::vector<Req*> take;
		std::vector<void*> wake;
		for(;;) {
			{
				std::unique_lock<std::mutex> lk(q.mu);
				q.cv.wait(lk, [&q] { return !q.v.empty(); });
				// a short window for the batch to fill: every call costs a few copies and a
				// stream sync, which a batch of one or two requests does not amortise
				q.cv.wait_for(lk, std::chrono::microseconds(BATCH_WINDOW_US),
				              [&q] { return q.v.size() >= BATCH_TARGET; });
				const size_t m = std::min(q.v.size(), MAX_BATCH);
				take.assign(q.v.begin(), q.v.begin() + m);
				q.v.erase(q.v.begin(), q.v.begin() + m);
			}
			const uint64_t tk = now_us();
			for(Req* r : take) r->t_take = tk;
			std::vector<bool> done(take.size(), false);
			for(size_t i = 0; i < take.size(); i++) {
				if(done[i]) continue;
				std::vector<Req*> g;
				for(size_t j = i; j < take.size(); j++)
					if(!done[j] && take[j]->key == take[i]->key) { g.push_back(take[j]); done[j] = true; }
				int rc;
				const uint64_t t0 = now_us();
				if(t_ctx) {
					rc = run_group(kind, g);
				} else {
					std::lock_guard<std::mutex> lk(g_mu);
					rc = run_group(kind, g);
				}
				g_call_us[kind] += now_us() - t0;
				for(int k = 0; prof && k < NKERN; k++) {
					uint64_t ln = 0;
					double ms = 0;
					if(bt2g_kernel_stats(t_ctx, k, &ln, &ms) == BT2G_OK && ln > seen_n[k]) {
						g_kern_n[k] += ln - seen_n[k];
						g_kern_us[k] += (uint64_t)((ms - seen_ms[k]) * 1000.0);
						seen_n[k] = ln;
						seen_ms[k] = ms;
					}
				}
				g_batches[kind]++;
				wake.clear();
				const uint64_t td = now_us();
				for(Req* r : g) {
					r->t_done = td;
					r->rc = rc;
					if(rc) snprintf(r->err, sizeof(r->err), "%s (batch of %zu)", bt2g_last_error(), g.size());
					// (a request's last access here: the decrement that completes a group
					// lets its fiber resume and release the requests)
					if(r->fiber) {
						if(!r->group || r->group->fetch_sub(1) == 1) wake.push_back(r->fiber);
					} else {
						sem_post(&r->sem);
					}
				}
				if(!wake.empty()) bt2gf::wake_many(wake.data(), wake.size());
			}
		}
	}

	std::once_flag once_;
	bool on_ = false;
	Q q_[ST_N];
};

Dispatcher g_disp;
Dispatcher& Dispatcher::instance() { return g_disp; }
void enqueue_1mm(const std::vector<MmReq*>& v) {
	g_disp.enqueue(ST_1MM, reinterpret_cast<Req* const*>(v.data()), v.size());
}

// fibers (bt2g_fibers.cpp): their requests reach the dispatchers a carrier round
// at a time; the context and dispatchers start before the first fiber runs
struct FiberHooks {
	FiberHooks() {
		bt2gf::set_flush(&Dispatcher::flush);
		bt2gf::set_init([] { g_disp.start(); });
	}
} g_fiber_hooks;

// ---- seed-phase prefetch -------------------------------------------------------
// A read's seed phase is three round trips one after another: exactSweep,
// then (no exact hit, <= 1 edit on a strand) oneMmSearch, then the first seed
// round's searchAllSeeds (bt2_search.cpp:3450-3906) -- nearly every read that
// is not done after its exact hits reaches the seed round.  Their arguments
// are functions of the read length and the server's fixed options
// (scoreMin, the seed interval and length: bt2_search.cpp:3287-3400), which
// the seams learn from their own calls.  So with the exact sweep the binding
// also asks for the read's round-0 seed search (in parallel, on the seed
// dispatcher) and, in the sweep's own dispatcher call right after the sweep,
// the gated 1-mm search.  A seam takes a prefetched result only when its
// request is the identical one (same read, same arguments: checked), else
// asks the engine as before -- nothing the reference decides changes.
// $BT2G_SEEDPF=0 turns it off; BT2G_SEEDPF_VERIFY=1 re-runs every taken
// result as an ordinary request and counts differences.
bool seedpf_enabled() {
	static const bool on = [] {
		const char* e = getenv("BT2G_SEEDPF");
		return !(e && e[0] == '0') && bt2gf::enabled();
	}();
	return on;
}
bool seedpf_verify() {
	static const bool on = getenv("BT2G_SEEDPF_VERIFY") != nullptr;
	return on;
}

// learned per read length (the latest value seen; a prediction is only ever
// used after the seam has checked it)
struct Learned {
	std::atomic<uint8_t> st[BT2G_MAX_READ_LEN + 1];
	std::atomic<int64_t> v[BT2G_MAX_READ_LEN + 1];
	Learned() {
		for(auto& x : st) x.store(0);
		for(auto& x : v) x.store(0);
	}
	void learn(size_t len, int64_t val) {
		if(len > BT2G_MAX_READ_LEN) return;
		if(st[len].load(std::memory_order_relaxed) == 1 && v[len].load(std::memory_order_relaxed) == val) return;
		v[len].store(val, std::memory_order_relaxed);
		st[len].store(1, std::memory_order_release);
	}
	bool get(size_t len, int64_t& val) const {
		if(len > BT2G_MAX_READ_LEN || st[len].load(std::memory_order_acquire) != 1) return false;
		val = v[len].load(std::memory_order_relaxed);
		return true;
	}
};
Learned g_mm_minsc;            // oneMmSearch's minsc
Learned g_sd_par;              // round 0's (seed length << 40 | interval << 20 | offsets)
std::mutex g_pf_mu;
std::atomic<int> g_pf_sc_st{0};   // the 1-mm scoring: 0 unknown, 1 known, 2 varies
bt2g_scoring g_pf_sc;
void learn_scoring(const bt2g_scoring& sc) {
	const int st = g_pf_sc_st.load(std::memory_order_acquire);
	if(st == 2) return;
	if(st == 1) {
		if(memcmp(&sc, &g_pf_sc, sizeof(sc)) != 0) g_pf_sc_st.store(2, std::memory_order_release);   // (not one scheme)
		return;
	}
	std::lock_guard<std::mutex> lk(g_pf_mu);
	if(g_pf_sc_st.load() == 0) {
		g_pf_sc = sc;
		g_pf_sc_st.store(1, std::memory_order_release);
	}
}

// One prefetched read (per fiber: two, for a pair's mates).
struct SeedPf {
	bool live = false;
	uint32_t len = 0;
	uint8_t codes[BT2G_MAX_READ_LEN], quals[BT2G_MAX_READ_LEN];
	std::unique_ptr<MmReq> mm;
	std::unique_ptr<SeedReq> sd;
	bool mm_ok = false, sd_ok = false;
	bool same(const Read& rd) const {
		if(!live || rd.length() != len) return false;
		for(uint32_t i = 0; i < len; i++)
			if(codes[i] != (uint8_t)rd.patFw[i] || quals[i] != (uint8_t)rd.qual[i]) return false;
		return true;
	}
};
struct SeedPfState {
	SeedPf slot[2];
	unsigned next = 0;
	SeedPf* find(const Read& rd) {
		for(SeedPf& x : slot)
			if(x.same(rd)) return &x;
		return nullptr;
	}
};
SeedPfState& seed_pf();      // per fiber (DrvState below)

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


// One engine/reference disagreement as a JSON line in $BT2G_ADAPTER_DUMP:
// everything needed to replay the DP through the oracle and the reference.
void dump_dp(const DpState& st, const std::vector<DpBtCandidate>& cands, size_t cural, int64_t minsc_now,
             const char* why) {
	const char* path = getenv("BT2G_ADAPTER_DUMP");
	if(!path) return;
	static std::mutex mu;
	std::lock_guard<std::mutex> lk(mu);
	FILE* f = fopen(path, "a");
	if(!f) return;
	fprintf(f, "{\"why\": \"%s\", \"cural\": %zu, \"minsc_now\": %lld, \"fw\": %d, \"ncol\": %u, \"minsc\": %d, "
	           "\"rect\": [%d, %d, %d], \"enable8\": %d, \"read\": \"", why, cural, (long long)minsc_now,
	        st.prob.fw, st.prob.ncol, st.prob.minsc, st.rect.triml, st.rect.corel, st.rect.corer, st.enable8);
	for(uint32_t i = 0; i < st.row.len; i++) fputc("ACGTN"[st.row.codes[i] > 4 ? 4 : st.row.codes[i]], f);
	fprintf(f, "\", \"qual\": \"");
	for(uint32_t i = 0; i < st.row.len; i++) fputc(st.row.quals[i] == '"' || st.row.quals[i] == '\\' ? 'I' : st.row.quals[i], f);
	fprintf(f, "\", \"win\": [");
	for(size_t i = 0; i < st.win.size(); i++) fprintf(f, "%s%d", i ? ", " : "", st.win[i]);
	fprintf(f, "], \"cands\": [");
	for(size_t i = 0; i < cands.size(); i++)
		fprintf(f, "%s[%zu, %zu, %lld, %d]", i ? ", " : "", (size_t)cands[i].row, (size_t)cands[i].col,
		        (long long)cands[i].score, i < st.fates.size() ? st.fates[i] : -9);
	fprintf(f, "], \"alns\": [");
	for(int32_t k = 0; k < st.naln; k++)
		fprintf(f, "%s[%d, %d, %d, %d]", k ? ", " : "", st.alns[k].cand, st.alns[k].score, st.alns[k].off,
		        st.alns[k].nedit);
	fprintf(f, "]}\n");
	fclose(f);
}

// one entry per SwAligner of the worker (sw and osw, bt2_search.cpp:3130); a
// carrier thread holds those of all its fibers
thread_local std::unordered_map<const void*, DpState*> t_dp;

DpState& dp_state(const void* sw) {
	DpState*& p = t_dp[sw];
	if(!p) p = new DpState();
	return *p;
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
	ExactReq q((uint32_t)mineMax, nofw ? 1 : 0, norc ? 1 : 0);
	q.r.set(read.patFw, read.qual);
	SeedPf* pf = nullptr;
	if(seedpf_enabled() && bt2gf::self() && q.r.len == len) {
		SeedPfState& ps = seed_pf();
		pf = ps.find(read);
		if(!pf) pf = &ps.slot[ps.next++ & 1u];
		pf->live = true;
		pf->len = (uint32_t)len;
		memcpy(pf->codes, q.r.codes, len);
		memcpy(pf->quals, q.r.quals, len);
		pf->mm_ok = pf->sd_ok = false;
	}
	Req* extra = nullptr;
	if(pf) {
		int64_t minsc = 0, par = 0;
		if(g_pf_sc_st.load(std::memory_order_acquire) == 1 && g_mm_minsc.get(len, minsc)) {
			if(!pf->mm) pf->mm.reset(new MmReq(0, 0, g_pf_sc));
			MmReq* m = pf->mm.get();
			m->sc = g_pf_sc;
			m->r = q.r;
			m->minsc = (int32_t)minsc;
			m->pf_ran = false;
			m->rc = 0;
			q.mm = m;
		}
		if(g_sd_par.get(len, par)) {
			const uint32_t L = (uint32_t)(par >> 40), per = (uint32_t)((par >> 20) & 0xfffff), nof = (uint32_t)(par & 0xfffff);
			if(!pf->sd) pf->sd.reset(new SeedReq(L, per, 0, nof));
			SeedReq* sq = pf->sd.get();
			*sq = SeedReq(L, per, 0, nof);          // (fresh request state; the Row is copied below)
			sq->r = q.r;
			extra = sq;
		}
	}
	if(extra) {
		Req* g2[2] = {&q, extra};
		g_disp.submit_group(g2, 2);
		pf->sd_ok = true;
		g_pf[1]++;
	} else if(q.mm) {
		Req* g1[1] = {&q};
		g_disp.submit_group(g1, 1);    // (a group: the dispatcher may add the 1-mm request to it)
	} else {
		g_disp.submit(&q);
	}
	if(pf && q.mm) pf->mm_ok = q.mm->pf_ran && q.mm->rc == 0;
	const uint32_t* out = q.out;
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
	MmReq q(nofw ? 1 : 0, norc ? 1 : 0, bs);
	const MmReq* src = &q;
	if(seedpf_enabled() && bt2gf::self()) {
		learn_scoring(bs);
		g_mm_minsc.learn(len, minsc);
		SeedPf* pf = seed_pf().find(read);
		if(pf && pf->mm_ok) {
			pf->mm_ok = false;
			const MmReq* m = pf->mm.get();
			if(m->minsc == (int32_t)minsc && m->nofw == q.nofw && m->norc == q.norc &&
			   memcmp(&m->sc, &bs, sizeof(bs)) == 0) {
				src = m;
				g_pf[2]++;
			}
		}
	}
	if(src == &q || seedpf_verify()) {
		q.r.set(read.patFw, read.qual);
		q.minsc = (int32_t)minsc;
		g_disp.submit(&q);
		if(src != &q && (src->cnt != q.cnt || src->ops != q.ops || src->hits.size() != q.hits.size() ||
		                 memcmp(src->hits.data(), q.hits.data(), sizeof(bt2g_mm1) * q.hits.size()) != 0))
			g_pf[4]++;
	}
	const auto& h = src->hits;
	const int32_t cnt = src->cnt;
	const uint32_t ops = src->ops;
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
	SeedReq q((uint32_t)seeds[0].len, per, off, (uint32_t)nof);
	const SeedReq* src = &q;
	if(seedpf_enabled() && bt2gf::self()) {
		if(off == 0) g_sd_par.learn(len, ((int64_t)seeds[0].len << 40) | ((int64_t)per << 20) | (int64_t)nof);
		SeedPf* pf = seed_pf().find(read);
		if(pf && pf->sd_ok) {
			pf->sd_ok = false;
			const SeedReq* sq = pf->sd.get();
			if(sq->seedlen == (uint32_t)seeds[0].len && sq->per == per && sq->off == off && sq->nof == (uint32_t)nof) {
				src = sq;
				g_pf[3]++;
			}
		}
	}
	if(src == &q || seedpf_verify()) {
		q.r.set(read.patFw, read.qual);
		g_disp.submit(&q);
		if(src != &q && (src->ns != q.ns || src->ops != q.ops || src->out.size() != q.out.size() ||
		                 memcmp(src->out.data(), q.out.data(), sizeof(uint32_t) * q.out.size()) != 0))
			g_pf[5]++;
	}
	const auto& out = src->out;
	const int32_t ns = src->ns;
	const uint32_t ops = src->ops;
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
	UgReq q(bs, ohang ? 1 : 0);
	q.r.set_fw_of(rd, qu, fw);
	memset(&q.p, 0, sizeof(q.p));
	q.p.fw = fw ? 1 : 0;
	q.p.off = coord.off();
	q.p.refidx = (uint32_t)coord.ref();
	q.p.minsc = (int32_t)minsc;
	g_disp.submit(&q);
	const bt2g_ug_result& o = q.o;
	const auto& ed = q.ed;
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

// the speculative DP prefetch (below): align()'s DP among those it ran
namespace {
struct SpecEntry;
SpecEntry* spec_find(const DpReq& q, int64_t refl);
void spec_use(DpReq& q, SpecEntry* e);
void spec_check(const DpReq& q, SpecEntry* e);
bool spec_verify();
}  // namespace

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
	DpReq q(bs, (enable8_ && !readSse16_) ? 1 : 0, rdlen > 1024, &st);
	q.r.set(*rdfw_, *qufw_);
	bt2g_sw_problem& p = q.p;
	memset(&p, 0, sizeof(p));
	p.fw = fw_ ? 1 : 0;
	p.refidx = (uint32_t)refidx_;
	p.ncol = (uint32_t)ncol;
	p.minsc = (int32_t)minsc_;
	q.rect.triml = (int32_t)rect_->triml;
	q.rect.corel = (int32_t)rect_->corel;
	q.rect.corer = (int32_t)rect_->corer;
	q.rect.pad = 0;
	SpecEntry* se = spec_find(q, rect_->refl);
	if(se && !spec_verify()) {
		spec_use(q, se);
	} else {
		q.win.assign((const uint8_t*)rf_ + rfi_, (const uint8_t*)rf_ + rfi_ + ncol + 1);
		g_disp.submit(&q);
		if(se) spec_check(q, se);
	}
	if(q.cpu) return false;      // served = false: the reference's align() runs
	const bt2g_sw_result& o = q.o;
	static const bool dump = getenv("BT2G_ADAPTER_DUMP") != nullptr;
	if(dump) {
		st.row = q.r;
		st.prob = q.p;
		st.rect = q.rect;
		st.win = q.win;
		st.enable8 = q.enable8;
	}
	st.naln = q.naln;
	const std::vector<bt2g_sw_cand>& cands = st.cands;   // (written by run_dp)
	const uint32_t maxedit = q.maxedit;
	if(st.naln < 0) {
		fprintf(stderr, "bt2g adapter: sw_align_bt status %d\n", st.naln);
		throw 1;
	}
	served = true;
	count(ST_DP, true);
	st.gpu = true;
	st.maxedit = maxedit;
	st.next = 0;
	st.next_edit = 0;
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
			std::vector<DpBtCandidate> cv(btncand_.size());
			for(size_t i = 0; i < btncand_.size(); i++) cv[i] = btncand_[i];
			dump_dp(st, cv, cural_, minsc, "no fate");
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
			std::vector<DpBtCandidate> cv(btncand_.size());
			for(size_t i = 0; i < btncand_.size(); i++) cv[i] = btncand_[i];
			dump_dp(st, cv, cural_, minsc, "too few alignments");
			throw 1;
		}
		const bt2g_sw_aln& a = st.alns[st.next];
		if(a.cand != (int32_t)cural_ || a.nedit > (int32_t)st.maxedit) {
			fprintf(stderr, "bt2g adapter: alignment %u is candidate %d, expected %zu\n", st.next, a.cand, cural_);
			std::vector<DpBtCandidate> cv(btncand_.size());
			for(size_t i = 0; i < btncand_.size(); i++) cv[i] = btncand_[i];
			dump_dp(st, cv, cural_, minsc, "alignment order");
			throw 1;
		}
		const bt2g_edit* ed = st.edits.data() + st.next_edit;
		st.next_edit += (size_t)a.nedit;
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

// ---- SwDriver: seed-hit extension and SA-row resolution ----------------------
//
// prioritizeSATups (aligner_sw_driver.cpp:490-738) extends every seed-hit range
// with SwDriver::extend (299-483, LF walks left in the forward index and right
// in the mirror index), and both it and eeSaTups (66-290) hand the ranges they
// choose to GroupWalk2S, whose advanceElement (group_walk.h:1161-1216) walks LF
// until an SA sample to resolve a row's text offset.  On the reference's host
// these walks are cache misses into a 3 GB index.  Here:
//   * before the reference's prioritizeSATups runs, every range it will look at
//     (SeedResults::hitsByRank + AlignmentCacheIface::queryQval, in its own
//     order) is extended on the GPU in one request (bt2g_extend); the
//     reference's extend calls then read those results (extend below);
//   * GroupWalk2S::init only records the range (the explicit specialisations
//     declared by bt2g_gw_spec.h); when prioritizeSATups / eeSaTups return,
//     every unresolved row of the ranges they set up is resolved on the GPU in
//     one request (bt2g_get_offset == Ebwt::getOffset, bt2_idx.cpp:150-171) and
//     written into the range's offset list in the alignment cache, where the
//     reference's walk leaves it too; advanceElement reads it (or, for a row
//     that could not be batched, calls Ebwt::getOffset on the CPU).
// Results are the reference's; the walk metrics (WalkMetrics, per-read LF op
// counts of the walks) are not reproduced -- they reach no SAM field unless
// --read-times / --metrics are given.
extern "C" {
void bt2g_real__ZN8SwDriver16prioritizeSATupsERK4ReadR11SeedResultsRK4EbwtPS6_RK16BitPairReferenceimbbbmR19AlignmentCacheIfaceR12RandomSourceR11WalkMetricsR14PerReadMetricsRmb(
	SwDriver*, const Read&, SeedResults&, const Ebwt&, const Ebwt*, const BitPairReference&, int, size_t, bool, bool, bool,
	size_t, AlignmentCacheIface&, RandomSource&, WalkMetrics&, PerReadMetrics&, size_t&, bool);
bool bt2g_real__ZN8SwDriver8eeSaTupsERK4ReadR11SeedResultsRK4EbwtRK16BitPairReferenceR12RandomSourceR11WalkMetricsR9SwMetricsRmmb(
	SwDriver*, const Read&, SeedResults&, const Ebwt&, const BitPairReference&, RandomSource&, WalkMetrics&, SwMetrics&,
	size_t&, size_t, bool);
void bt2g_real__ZN8SwDriver6extendERK4ReadRK4EbwtPS4_jjjjbmmR14PerReadMetricsRmS9_(
	SwDriver*, const Read&, const Ebwt&, const Ebwt*, TIndexOffU, TIndexOffU, TIndexOffU, TIndexOffU, bool, size_t,
	size_t, PerReadMetrics&, size_t&, size_t&);
}

namespace {

bool drv_engine() {
	static const bool on = [] {
		const char* e = getenv("BT2G_DRIVER_SEAMS");
		return !(e && e[0] == '0');
	}();
	return on;
}

// extend() results of the read being prioritised (valid during one
// prioritizeSATups call on this thread: filled after the request's fiber
// switch, and no switch happens inside the reference's prioritizeSATups)
struct ExtTable {
	bool on = false;
	std::vector<bt2g_ext_in> keys;
	std::vector<bt2g_ext_out> vals;
};


// ranges handed to GroupWalk2S::init during one prioritizeSATups / eeSaTups call
struct GwRange {
	TIndexOffU topf;
	size_t size;
	TSlice offs;
};
struct GwTable {
	bool on = false;
	std::vector<GwRange> ranges;
};
// per worker (fiber): a fiber may be suspended inside the reference's
// prioritizeSATups (a contended lock yields, bt2g_fibers.cpp), and the other
// fibers of its carrier must not see its tables
const size_t SPEC_MAX = 32;

struct SpecEntry {
	int32_t fw, minsc, enable8;
	uint32_t refidx, ncol;
	int64_t refl;
	bt2g_sw_rect rect;
	bool ready = false, used = false;
	bt2g_sw_result o;
	int32_t naln = 0;
	uint32_t cap = 0, maxaln = 0, maxedit = 0;
	bool cpu = false;
	DpState st;
};

struct SpecCtx {
	bool on = false;               // inside an unpaired extendSeeds call
	const Read* rd = nullptr;
	const Scoring* sc = nullptr;
	TAlScore minsc = 0;
	int nceil = 0;
	size_t maxhalf = 0, cminlen = 0;
	bool doUngapped = false, enable8 = true;
	std::vector<SpecEntry*> entries;   // this extendSeeds call's prefetched DPs
	std::vector<SpecEntry*> spare;
	void clear() {
		for(SpecEntry* e : entries) spare.push_back(e);
		entries.clear();
	}
};
struct DrvState {
	ExtTable ext;
	GwTable gw;
	SpecCtx spec;
	SeedPfState pf;
};
DrvState& drv() {
	void** slot = bt2gf::local();
	if(!slot) {
		thread_local DrvState t;
		return t;
	}
	if(!*slot) *slot = new DrvState();
	return *static_cast<DrvState*>(*slot);
}

SeedPfState& seed_pf() { return drv().pf; }

// ---- speculative DP prefetch --------------------------------------------------
// SwDriver::extendSeeds (aligner_sw_driver.cpp:756-1297) resolves one seed-hit
// element at a time and, for each new diagonal, frames a rectangle and runs a
// DP (initRef + align) -- one engine round trip per DP, 5.5 per read at
// 3.1 Gbp (r03l), each waiting on a whole batch.  But once prioritizeSATups
// has chosen the ranges and their rows are resolved, every DP the loop can
// request at the current minimum score is known up to the loop's random visit
// order: for each element, joinedToTextOff + frameSeedExtensionRect with the
// loop's own arguments (aligner_sw_driver.cpp:935-1105).  So right there the
// binding frames them all (distinct diagonals, at most SPEC_MAX) and runs them
// in one group request; align() then takes its DP's result from here when the
// problem is the same one (same strand, reference, rectangle, minimum score,
// u8 choice; the read is fixed for the extendSeeds call), else asks the
// engine as before.  The prefetched problems read the reference from HBM
// (the engine's resident copy) where align()'s own request carries initRef's
// window: the same bytes (rectangle trimming at reference ends, Ns outside
// them, masks 1 << code; pinned at full size by bench.py's parity sample, and
// here by BT2G_SPEC_VERIFY=1, which runs every hit again as a normal request
// and counts differences).  Nothing the reference decides changes: align()
// returns what the engine computes for that problem either way.
SpecCtx& spec() {
	DrvState& d = drv();
	return d.spec;
}

bool spec_enabled() {
	static const bool on = [] {
		// off by default: r03n at 3.1 Gbp, 2048 workers: 12.8k reads/s with it, 24.5k
		// without -- 4.3M DPs prefetched for 1.48M align() calls served, and the DP
		// dispatchers were already saturated ($BT2G_SPEC=1 turns it on)
		const char* e = getenv("BT2G_SPEC");
		return e && e[0] == '1' && bt2gf::enabled();
	}();
	return on;
}
bool spec_verify() {
	static const bool on = getenv("BT2G_SPEC_VERIFY") != nullptr;
	return on;
}

// SwDriver's ranges (protected members; no added members: same layout)
struct SwDriverAcc : public SwDriver {
	const EList<SATupleAndPos, 16>& sp() const { return satpos_; }
};

void spec_prefetch(const SwDriver* sd, const Ebwt& ebwtFw) {
	SpecCtx& x = spec();
	x.clear();
	const Read& rd = *x.rd;
	const size_t rdlen = rd.length();
	bt2g_scoring bs;
	if(rdlen == 0 || rdlen > BT2G_MAX_READ_LEN || rdlen >= x.cminlen || !to_scoring(*x.sc, bs) ||
	   x.minsc < std::numeric_limits<int32_t>::min() || x.minsc > std::numeric_limits<int32_t>::max())
		return;
	const Scoring& sc = *x.sc;
	const int readGaps = sc.maxReadGaps(x.minsc, rdlen), refGaps = sc.maxRefGaps(x.minsc, rdlen);
	if(x.doUngapped && readGaps == 0 && refGaps == 0) return;   // the loop's ungapped path, no DP
	DynProgFramer dpframe(!gReportOverhangs);
	const EList<SATupleAndPos, 16>& sp = static_cast<const SwDriverAcc*>(sd)->sp();
	struct Diag { uint32_t tidx; int64_t refoff; bool fw; };
	std::vector<Diag> seen;
	std::vector<DpReq*> reqs;
	std::vector<std::unique_ptr<DpReq>> own;
	for(size_t i = 0; i < sp.size() && x.entries.size() < SPEC_MAX; i++) {
		const SATuple& sat = sp[i].sat;
		const bool fw = sp[i].pos.fw;
		uint32_t rdoff = sp[i].pos.rdoff;
		const uint32_t seedhitlen = sp[i].pos.seedlen;
		if(!fw) rdoff = (uint32_t)(rdlen - rdoff - seedhitlen);
		for(size_t elt = 0; elt < sat.size() && x.entries.size() < SPEC_MAX; elt++) {
			const TIndexOffU off = sat.offs[elt];
			if(off == OFF_MASK) continue;
			TIndexOffU tidx = 0, toff = 0, tlen = 0;
			bool straddled = false;
			ebwtFw.joinedToTextOff(sat.key.len, off, tidx, toff, tlen, false, straddled);
			if(tidx == OFF_MASK) continue;
			const int64_t refoff = (int64_t)toff - rdoff;
			bool dup = false;
			for(const Diag& d : seen) dup = dup || (d.tidx == tidx && d.refoff == refoff && d.fw == fw);
			if(dup) continue;
			seen.push_back(Diag{tidx, refoff, fw});
			DPRect rect;
			if(!dpframe.frameSeedExtensionRect(refoff, rdlen, tlen, readGaps, refGaps, (size_t)x.nceil, x.maxhalf, rect))
				continue;
			SpecEntry* e;
			if(!x.spare.empty()) {
				e = x.spare.back();
				x.spare.pop_back();
			} else {
				e = new SpecEntry();
			}
			e->fw = fw ? 1 : 0;
			e->minsc = (int32_t)x.minsc;
			e->enable8 = x.enable8 ? 1 : 0;
			e->refidx = (uint32_t)tidx;
			e->ncol = (uint32_t)(rect.refr + 1 - rect.refl);
			e->refl = rect.refl;
			e->rect.triml = (int32_t)rect.triml;
			e->rect.corel = (int32_t)rect.corel;
			e->rect.corer = (int32_t)rect.corer;
			e->rect.pad = 0;
			e->ready = e->used = false;
			x.entries.push_back(e);
			DpReq* q = new DpReq(bs, e->enable8, rdlen > 1024, &e->st);
			own.emplace_back(q);
			q->r.set(rd.patFw, rd.qual);
			memset(&q->p, 0, sizeof(q->p));
			q->p.fw = e->fw;
			q->p.refidx = e->refidx;
			q->p.ncol = e->ncol;
			q->p.minsc = e->minsc;
			q->p.refl = e->refl;
			q->p.win_off = -1;          // the engine's resident reference
			q->rect = e->rect;
			reqs.push_back(q);
		}
	}
	if(reqs.empty()) return;
	g_disp.submit_group(reinterpret_cast<Req* const*>(reqs.data()), reqs.size());
	g_spec_groups++;
	g_spec_dps += reqs.size();
	for(size_t k = 0; k < reqs.size(); k++) {
		SpecEntry* e = x.entries[k];
		const DpReq* q = reqs[k];
		e->o = q->o;
		e->naln = q->naln;
		e->cap = q->cap;
		e->maxaln = q->maxaln;
		e->maxedit = q->maxedit;
		e->cpu = q->cpu;
		e->ready = true;
	}
}

}  // namespace

namespace {

// align()'s DP among the prefetched ones (nullptr: not prefetched)
SpecEntry* spec_find(const DpReq& q, int64_t refl) {
	if(!spec_enabled() || !bt2gf::self()) return nullptr;
	SpecCtx& x = spec();
	if(!x.on) return nullptr;
	for(SpecEntry* e : x.entries)
		if(e->ready && !e->used && !e->cpu && e->fw == q.p.fw && e->refidx == q.p.refidx && e->ncol == q.p.ncol &&
		   e->minsc == q.p.minsc && e->enable8 == q.enable8 && e->refl == refl && e->rect.triml == q.rect.triml &&
		   e->rect.corel == q.rect.corel && e->rect.corer == q.rect.corer)
			return e;
	return nullptr;
}

// its outputs moved into q and q's DpState, as run_dp leaves them
void spec_use(DpReq& q, SpecEntry* e) {
	e->used = true;
	g_spec_hits++;
	q.o = e->o;
	q.naln = e->naln;
	q.cap = e->cap;
	q.maxaln = e->maxaln;
	q.maxedit = e->maxedit;
	q.cpu = false;
	DpState& st = *q.st;
	st.cands.swap(e->st.cands);
	st.fates.swap(e->st.fates);
	st.alns.swap(e->st.alns);
	st.edits.swap(e->st.edits);
}

// BT2G_SPEC_VERIFY: the prefetched answer against align()'s own request
void spec_check(const DpReq& q, SpecEntry* e) {
	e->used = true;
	g_spec_hits++;
	const DpState& st = *q.st;
	auto same = [](const void* a, const void* b, size_t n) { return n == 0 || memcmp(a, b, n) == 0; };
	const bool ok = same(&e->o, &q.o, sizeof(q.o)) && e->naln == q.naln && e->st.cands.size() == st.cands.size() &&
	                same(e->st.cands.data(), st.cands.data(), sizeof(bt2g_sw_cand) * st.cands.size()) &&
	                e->st.fates == st.fates && e->st.alns.size() == st.alns.size() &&
	                same(e->st.alns.data(), st.alns.data(), sizeof(bt2g_sw_aln) * st.alns.size()) &&
	                e->st.edits.size() == st.edits.size() &&
	                same(e->st.edits.data(), st.edits.data(), sizeof(bt2g_edit) * st.edits.size());
	if(!ok) g_spec_verify_bad++;
}


const size_t MAX_ROWS = 8192;    // rows per read per request (the rest: CPU getOffset)

void resolve_rows(const Ebwt& ebwtFw) {
	drv().gw.on = false;
	if(drv().gw.ranges.empty()) return;
	// the ranges leave the table before the request below yields
	std::vector<GwRange> ranges;
	ranges.swap(drv().gw.ranges);
	OffReq q;
	std::vector<std::pair<size_t, size_t>> where;    // (range, element) of each row
	for(size_t r = 0; r < ranges.size(); r++) {
		GwRange& x = ranges[r];
		for(size_t j = 0; j < x.size && q.rows.size() < MAX_ROWS; j++)
			if(x.offs[j] == OFF_MASK) {
				q.rows.push_back((uint32_t)(x.topf + j));
				where.emplace_back(r, j);
			}
	}
	if(!q.rows.empty()) {
		g_disp.submit(&q);
		count(ST_OFF, true);
		for(size_t k = 0; k < where.size(); k++) ranges[where[k].first].offs[where[k].second] = q.offs[k];
	}
	(void)ebwtFw;
}

}  // namespace

template <>
void GroupWalk2S<TSlice, 16>::init(const Ebwt& ebwtFw, const BitPairReference& ref, SARangeWithOffs<TSlice>& sa,
                                   RandomSource& rnd, WalkMetrics& met) {
	(void)ebwtFw; (void)ref; (void)rnd; (void)met;
	reset();
	elt_ += sa.size();
	// the range's offset slots as the cache would hold them before any walk
	// (AlignmentCache::addOnTheFlyImpl above only reserves them); rows resolved
	// earlier in this read are resolved again, to the same offsets
	static_cast<bt2gref::TSliceAcc&>(sa.offs).fill(OFF_MASK);
	if(drv().gw.on) drv().gw.ranges.push_back(GwRange{sa.topf, sa.size(), sa.offs});
}

template <>
bool GroupWalk2S<TSlice, 16>::advanceElement(TIndexOffU elt, const Ebwt& ebwtFw, const BitPairReference& ref,
                                             SARangeWithOffs<TSlice>& sa, GroupWalkState& gws, WalkResult& res,
                                             WalkMetrics& met, PerReadMetrics& prm) {
	(void)ref; (void)gws; (void)prm;
	if(sa.offs[elt] == OFF_MASK) {       // not batched: the reference's getOffset on the CPU
		sa.offs[elt] = ebwtFw.getOffset(sa.topf + elt);
		count(ST_OFF, false);
	}
	met.reports++;
	res.init(0, false, 0, elt, sa.topf + elt, (TIndexOffU)sa.len, sa.offs[elt]);
	rep_++;
	return true;
}

void SwDriver::prioritizeSATups(const Read& read, SeedResults& sh, const Ebwt& ebwtFw, const Ebwt* ebwtBw,
                                const BitPairReference& ref, int seedmms, size_t maxelt, bool doExtend, bool lensq,
                                bool szsq, size_t nsm, AlignmentCacheIface& ca, RandomSource& rnd, WalkMetrics& wlm,
                                PerReadMetrics& prm, size_t& nelt_out, bool all) {
	const bool eng = drv_engine();
	drv().ext.on = false;
	if(eng && doExtend && ebwtBw != NULL && read.length() > 0 && read.length() <= BT2G_MAX_READ_LEN) {
		// every range the loop at aligner_sw_driver.cpp:519-604 visits, in its order
		ExtReq q;
		q.r.set(read.patFw, read.qual);
		EList<SATuple, 16> sat;
		const size_t nonz = sh.nonzeroOffsets();
		for(size_t i = 0; i < nonz; i++) {
			bool fw = true;
			uint32_t offidx = 0, rdoff = 0, seedlen = 0;
			QVal qv = sh.hitsByRank(i, offidx, rdoff, fw, seedlen);
			size_t nr = 0, ne = 0;
			sat.clear();
			ca.queryQval(qv, sat, nr, ne);
			for(size_t j = 0; j < sat.size(); j++) {
				const TIndexOffU sz = (TIndexOffU)sat[j].size();
				bt2g_ext_in x;
				x.read = 0;
				x.fw = fw ? 1 : 0;
				x.off = rdoff;
				x.len = seedlen;
				x.topf = sat[j].topf;
				x.botf = sat[j].topf + sz;
				x.topb = sat[j].topb;
				x.botb = sat[j].topb + sz;
				if(sz > 0 && rdoff + seedlen <= read.length()) q.in.push_back(x);
			}
		}
		if(!q.in.empty()) {
			g_disp.submit(&q);
			count(ST_EXT, true);
			drv().ext.keys.assign(q.in.begin(), q.in.end());
			drv().ext.vals.assign(q.out.data(), q.out.data() + q.out.size());
			drv().ext.on = true;
		}
	}
	drv().gw.ranges.clear();
	drv().gw.on = eng;
	bt2g_real__ZN8SwDriver16prioritizeSATupsERK4ReadR11SeedResultsRK4EbwtPS6_RK16BitPairReferenceimbbbmR19AlignmentCacheIfaceR12RandomSourceR11WalkMetricsR14PerReadMetricsRmb(
		this, read, sh, ebwtFw, ebwtBw, ref, seedmms, maxelt, doExtend, lensq, szsq, nsm, ca, rnd, wlm, prm, nelt_out, all);
	drv().ext.on = false;
	resolve_rows(ebwtFw);
	if(spec_enabled() && spec().on) spec_prefetch(this, ebwtFw);
}

bool SwDriver::eeSaTups(const Read& rd, SeedResults& sh, const Ebwt& ebwt, const BitPairReference& ref,
                        RandomSource& rnd, WalkMetrics& wlm, SwMetrics& swmSeed, size_t& nelt_out, size_t maxelt,
                        bool all) {
	drv().gw.ranges.clear();
	drv().gw.on = drv_engine();
	bool ret = bt2g_real__ZN8SwDriver8eeSaTupsERK4ReadR11SeedResultsRK4EbwtRK16BitPairReferenceR12RandomSourceR11WalkMetricsR9SwMetricsRmmb(
		this, rd, sh, ebwt, ref, rnd, wlm, swmSeed, nelt_out, maxelt, all);
	resolve_rows(ebwt);
	return ret;
}

void SwDriver::extend(const Read& rd, const Ebwt& ebwtFw, const Ebwt* ebwtBw, TIndexOffU topf, TIndexOffU botf,
                      TIndexOffU topb, TIndexOffU botb, bool fw, size_t off, size_t len, PerReadMetrics& prm,
                      size_t& nlex, size_t& nrex) {
	if(drv().ext.on) {
		const std::vector<bt2g_ext_in>& K = drv().ext.keys;
		for(size_t i = 0; i < K.size(); i++) {
			const bt2g_ext_in& k = K[i];
			if(k.topf == topf && k.botf == botf && k.topb == topb && k.botb == botb && (k.fw != 0) == fw && k.off == off &&
			   k.len == len) {
				nlex += drv().ext.vals[i].nlex;
				nrex += drv().ext.vals[i].nrex;
				prm.nSdFmops += drv().ext.vals[i].fmops;
				return;
			}
		}
	}
	count(ST_EXT, false);
	bt2g_real__ZN8SwDriver6extendERK4ReadRK4EbwtPS4_jjjjbmmR14PerReadMetricsRmS9_(
		this, rd, ebwtFw, ebwtBw, topf, botf, topb, botb, fw, off, len, prm, nlex, nrex);
}

// ---- AlignmentCache::addOnTheFlyImpl (aligner_cache.cpp:55-104): bt2g_refspec.h

// ---- SwDriver::extendSeeds (aligner_sw_driver.cpp:756-1297) -------------------
// The unpaired extension loop, unchanged; the binding only records the
// arguments its DPs are framed with, for the speculative prefetch above.
extern "C" int __real__ZN8SwDriver11extendSeedsER4ReadbR11SeedResultsRK4EbwtPS5_RK16BitPairReferenceR9SwAlignerRK7ScoringiiiRlimbmmmmmbbmmbiR19AlignmentCacheIfaceR12RandomSourceR11WalkMetricsR9SwMetricsR14PerReadMetricsP11AlnSinkWrapbRb(
	SwDriver*, Read&, bool, SeedResults&, const Ebwt&, const Ebwt*, const BitPairReference&, SwAligner&, const Scoring&,
	int, int, int, TAlScore&, int, size_t, bool, size_t, size_t, size_t, size_t, size_t, bool, bool, size_t, size_t, bool,
	int, AlignmentCacheIface&, RandomSource&, WalkMetrics&, SwMetrics&, PerReadMetrics&, AlnSinkWrap*, bool, bool&);

extern "C" int __wrap__ZN8SwDriver11extendSeedsER4ReadbR11SeedResultsRK4EbwtPS5_RK16BitPairReferenceR9SwAlignerRK7ScoringiiiRlimbmmmmmbbmmbiR19AlignmentCacheIfaceR12RandomSourceR11WalkMetricsR9SwMetricsR14PerReadMetricsP11AlnSinkWrapbRb(
	SwDriver* self, Read& rd, bool mate1, SeedResults& sh, const Ebwt& ebwtFw, const Ebwt* ebwtBw,
	const BitPairReference& ref, SwAligner& swa, const Scoring& sc, int seedmms, int seedlen, int seedival,
	TAlScore& minsc, int nceil, size_t maxhalf, bool doUngapped, size_t maxIters, size_t maxUg, size_t maxDp,
	size_t maxUgStreak, size_t maxDpStreak, bool doExtend, bool enable8, size_t cminlen, size_t cpow2, bool doTri,
	int tighten, AlignmentCacheIface& ca, RandomSource& rnd, WalkMetrics& wlm, SwMetrics& swmSeed,
	PerReadMetrics& prm, AlnSinkWrap* msink, bool reportImmediately, bool& exhaustive) {
	const bool sp = spec_enabled() && bt2gf::self() != nullptr;
	if(sp) {
		SpecCtx& x = spec();
		x.clear();
		x.on = true;
		x.rd = &rd;
		x.sc = &sc;
		x.minsc = minsc;          // (the loop may tighten it later: those DPs miss)
		x.nceil = nceil;
		x.maxhalf = maxhalf;
		x.cminlen = cminlen;
		x.doUngapped = doUngapped;
		x.enable8 = enable8;
	}
	int ret;
	try {
		ret = __real__ZN8SwDriver11extendSeedsER4ReadbR11SeedResultsRK4EbwtPS5_RK16BitPairReferenceR9SwAlignerRK7ScoringiiiRlimbmmmmmbbmmbiR19AlignmentCacheIfaceR12RandomSourceR11WalkMetricsR9SwMetricsR14PerReadMetricsP11AlnSinkWrapbRb(
			self, rd, mate1, sh, ebwtFw, ebwtBw, ref, swa, sc, seedmms, seedlen, seedival, minsc, nceil, maxhalf,
			doUngapped, maxIters, maxUg, maxDp, maxUgStreak, maxDpStreak, doExtend, enable8, cminlen, cpow2, doTri,
			tighten, ca, rnd, wlm, swmSeed, prm, msink, reportImmediately, exhaustive);
	} catch(...) {
		if(sp) {
			spec().on = false;
			spec().clear();
		}
		throw;
	}
	if(sp) {
		spec().on = false;
		spec().clear();
	}
	return ret;
}
