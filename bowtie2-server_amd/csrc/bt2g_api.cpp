// bt2g_api.cpp -- host side of the C ABI (include/bt2g.h).
//
// Owns the HBM-resident index (one replica per GPU), turns the
// batch calls into kernel launches on a HIP stream, and provides the
// host-pointer convenience wrappers.  No exception crosses the ABI; errors are
// status codes plus a thread-local message (bt2g_last_error).
#include <atomic>
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <sys/prctl.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <time.h>

#include <algorithm>
#include <cstdarg>
#include <cstdlib>
#include <fstream>
#include <mutex>
#include <string>
#include <unordered_map>
#include <chrono>
#include <vector>

#include "bt2g_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
	char buf[512];
	va_list ap;
	va_start(ap, fmt);
	vsnprintf(buf, sizeof(buf), fmt, ap);
	va_end(ap);
	g_err = buf;
	return code;
}

#define HIPCHK(x)                                                                          \
	do {                                                                                   \
		hipError_t e_ = (x);                                                               \
		if(e_ != hipSuccess) return fail(BT2G_ERR_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
	} while(0)

struct DevBuf {
	void* p = nullptr;
	size_t n = 0;
};

}  // namespace

struct bt2g_ctx {
	int device = 0;
	hipStream_t stream = nullptr;
	DevEbwt fw{}, bw{};
	std::vector<void*> owned;           // device allocations of the index
	uint8_t* ref_codes = nullptr;
	uint64_t* ref_starts = nullptr;
	uint32_t nref = 0;
	uint64_t num_sides = 0;
	uint64_t hbm_bytes = 0;
	// contexts opened on this one's index (bt2g_open_shared) and still open; the
	// index owner cannot close before them.  `base`: the owner of a shared context
	std::atomic<int> shares{0};
	bt2g_ctx* base = nullptr;
	// profiling
	bool prof = false;
	struct Pending { int kid; hipEvent_t a, b; };
	std::vector<Pending> pending;
	std::vector<hipEvent_t> evpool;
	uint64_t launches[16] = {0};      // 0-7: kernels (HIP events); 8-15: host phases of a call
	double total_ms[16] = {0};
	// persistent SW scratch (bt2g_reserve_sw): no allocation / sync per call
	uint32_t sw_max_prob = 0, sw_max_cols = 0;
	uint32_t* sw_lists = nullptr;
	uint32_t* sw_counts = nullptr;
	uint32_t* sw_bnd = nullptr;
	// persistent backtrace scratch (bt2g_reserve_sw_bt)
	uint32_t bt_max_prob = 0, bt_max_stride = 0, bt_max_cols = 0;
	int bt_hbytes = 0;
	uint8_t* bt_plane = nullptr;
	uint32_t* bt_marks = nullptr;
	// the 1-mm search's second stream (the BWT' direction) and its fork/join events
	hipStream_t aux = nullptr;
	int prio = 0;                       // stream priority (bt2g_set_priority); 0 = default
	bool cu_masked = false;             // the stream is CU-masked (bt2g_set_cu_share)
	hipEvent_t mm_ev[4] = {nullptr, nullptr, nullptr, nullptr};
	// host-wrapper scratch (Arena): one device block reused call after call
	uint8_t* arena = nullptr;
	size_t arena_cap = 0, arena_used = 0, arena_need = 0;
	int arena_depth = 0;
	std::vector<void*> arena_spill;
	struct GuardRec { void* p; size_t n; int line; };
	std::vector<GuardRec> arena_guards;
	// pinned host staging for the wrappers' copies (same growth rule as the arena)
	uint8_t* pin = nullptr;
	size_t pin_cap = 0, pin_used = 0, pin_need = 0;
	// device mirror of `pin` (same size and offsets): a call's inputs are staged
	// in `pin` and reach the device in one copy, its outputs come back in one
	uint8_t* pin_dev = nullptr;
	// the device's view of `pin` itself (hipHostGetDevicePointer): kernels write
	// small variable-size outputs straight into host memory
	uint8_t* pin_dview = nullptr;
	// $BT2G_SYNC=poll: host waits query an event and sleep between queries
	hipEvent_t poll_ev = nullptr;
	// the ranks' communicator (bt2g_comm_init): an RCCL ncclComm_t
	void* comm = nullptr;
};

namespace {

// How a host thread waits for its stream.  $BT2G_SYNC=poll: record an event and
// query it, sleeping $BT2G_POLL_US (default 20) between queries -- no CPU burnt
// in the runtime's wait loop, which a process with a CPU quota and many busy
// threads (the drop-in server) cannot spare; otherwise hipStreamSynchronize.
bool poll_sync() {
	static const bool on = [] {
		const char* e = getenv("BT2G_SYNC");
		return e && !strcmp(e, "poll");
	}();
	return on;
}

hipError_t stream_wait(bt2g_ctx* c, hipStream_t st) {
	if(!poll_sync()) return hipStreamSynchronize(st);
	static const long us = [] {
		const char* e = getenv("BT2G_POLL_US");
		return e && atol(e) > 0 ? atol(e) : 20L;
	}();
	// (the thread's timer slack, 50 us by default, would stretch every 20-us sleep
	// to ~70 us: 1 us for a thread that waits here)
	static thread_local bool slack = (prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0), true);
	(void)slack;
	hipError_t e;
	if(!c->poll_ev && (e = hipEventCreateWithFlags(&c->poll_ev, hipEventDisableTiming)) != hipSuccess) return e;
	if((e = hipEventRecord(c->poll_ev, st)) != hipSuccess) return e;
	for(;;) {
		e = hipEventQuery(c->poll_ev);
		if(e != hipErrorNotReady) return e;
		timespec ts{0, us * 1000L};
		nanosleep(&ts, nullptr);
	}
}

// Device scratch.  Inside a host-pointer wrapper (Arena below) blocks come from
// the context's arena: the wrappers synchronise before they return, so the
// arena is simply rewound for the next call, and no allocator is shared by the
// threads that drive their own contexts.  The device-pointer calls (which a
// caller may enqueue on any stream, without waiting) take stream-ordered blocks
// from the device's memory pool.
//
// With BT2G_GUARD=1 (a debugging mode) every block gets a 4 KiB tail of 0xA5
// bytes that is checked when the block is released: a kernel writing past the
// end of its buffer is reported with the source line that allocated it.
const size_t GUARD_BYTES = 4096;

bool guard_on() {
	static const bool on = [] {
		const char* g = getenv("BT2G_GUARD");
		return g && g[0] == '1';
	}();
	return on;
}

struct GuardInfo {
	size_t n;
	int line;
};
std::mutex g_guard_mu;
std::unordered_map<void*, GuardInfo> g_guard;

// compare a guard tail (after the stream it was used on has drained)
bool guard_check(void* p, size_t n, int line) {
	std::vector<uint8_t> tail(GUARD_BYTES);
	if(hipMemcpy(tail.data(), (char*)p + n, GUARD_BYTES, hipMemcpyDeviceToHost) != hipSuccess) return false;
	for(size_t i = 0; i < GUARD_BYTES; i++)
		if(tail[i] != 0xA5) {
			fprintf(stderr, "bt2g guard: block of %zu bytes from bt2g_api.cpp:%d overwritten at +%zu\n", n, line,
			        n + i);
			return false;
		}
	return true;
}

hipError_t amalloc(bt2g_ctx* c, void** p, size_t n, hipStream_t st, int line = __builtin_LINE()) {
	const size_t g = guard_on() ? GUARD_BYTES : 0;
	hipError_t e;
	if(c->arena_depth > 0) {
		const size_t need = (n + g + 255) & ~(size_t)255;
		if(c->arena_used + need <= c->arena_cap) {
			*p = c->arena + c->arena_used;
			c->arena_used += need;
			c->arena_need = std::max(c->arena_need, c->arena_used);
		} else {
			// too small for this call: a block of its own now, a bigger arena next call
			c->arena_need = std::max(c->arena_need, c->arena_used + need);
			if((e = hipMalloc(p, n + g)) != hipSuccess) return e;
			c->arena_spill.push_back(*p);
		}
		if(g) {
			if((e = hipMemsetAsync((char*)*p + n, 0xA5, g, st)) != hipSuccess) return e;
			c->arena_guards.push_back(bt2g_ctx::GuardRec{*p, n, line});
		}
		return hipSuccess;
	}
	if((e = hipMallocAsync(p, n + g, st)) != hipSuccess) return e;
	if(g) {
		if((e = hipMemsetAsync((char*)*p + n, 0xA5, g, st)) != hipSuccess) return e;
		std::lock_guard<std::mutex> lk(g_guard_mu);
		g_guard[*p] = GuardInfo{n, line};
	}
	return hipSuccess;
}

hipError_t afree(bt2g_ctx* c, void* p, hipStream_t st) {
	if(c->arena_depth > 0) return hipSuccess;    // released when the wrapper's Arena ends
	if(guard_on() && p) {
		GuardInfo gi{0, 0};
		{
			std::lock_guard<std::mutex> lk(g_guard_mu);
			auto it = g_guard.find(p);
			if(it != g_guard.end()) {
				gi = it->second;
				g_guard.erase(it);
			}
		}
		if(gi.line) {
			hipError_t e = hipStreamSynchronize(st);
			if(e != hipSuccess) return e;
			guard_check(p, gi.n, gi.line);
		}
	}
	return hipFreeAsync(p, st);
}

// Scope of one host-pointer wrapper call on context c (not re-entrant across
// threads: a context is driven by one thread at a time).
struct Arena {
	bt2g_ctx* c;
	hipStream_t st;
	explicit Arena(bt2g_ctx* cx) : c(cx), st(cx->stream) {
		if(c->arena_depth++ > 0) return;
		c->arena_used = 0;
		if(c->arena_need > c->arena_cap) {
			// nothing of an earlier call is in flight: it synchronised before returning
			if(c->arena) (void)hipFree(c->arena);
			c->arena = nullptr;
			// (doubling: a regrowth frees and re-allocates -- hipFree waits for the device --
		// so a context that meets bigger and bigger calls regrows a few times, not at each)
		size_t cap = std::max<size_t>(c->arena_need * 2, (size_t)64 << 20);
			if(hipMalloc((void**)&c->arena, cap) == hipSuccess) {
				c->arena_cap = cap;
			} else {
				c->arena = nullptr;
				c->arena_cap = 0;
			}
		}
		c->pin_used = 0;
		if(c->pin_need > c->pin_cap) {
			if(c->pin) (void)hipHostFree(c->pin);
			if(c->pin_dev) (void)hipFree(c->pin_dev);
			c->pin = nullptr;
			c->pin_dev = nullptr;
			size_t cap = std::max<size_t>(c->pin_need * 2, (size_t)16 << 20);
			if(hipHostMalloc((void**)&c->pin, cap, hipHostMallocDefault) == hipSuccess &&
			   hipMalloc((void**)&c->pin_dev, cap) == hipSuccess &&
			   hipHostGetDevicePointer((void**)&c->pin_dview, c->pin, 0) == hipSuccess) {
				c->pin_cap = cap;
			} else {
				if(c->pin) (void)hipHostFree(c->pin);
				if(c->pin_dev) (void)hipFree(c->pin_dev);
				c->pin = nullptr;
				c->pin_dev = nullptr;
				c->pin_dview = nullptr;
				c->pin_cap = 0;
			}
		}
	}
	// pinned staging of `n` bytes for this call (nullptr: copy through pageable memory)
	uint8_t* pinned(size_t n) {
		const size_t need = (n + 63) & ~(size_t)63;
		c->pin_need = std::max(c->pin_need, c->pin_used + need);
		if(c->pin_used + need > c->pin_cap) return nullptr;
		uint8_t* p = c->pin + c->pin_used;
		c->pin_used += need;
		return p;
	}
	~Arena() {
		if(--c->arena_depth > 0) return;
		(void)stream_wait(c, st);   // an early error return may leave work in flight
		for(auto& g : c->arena_guards) guard_check(g.p, g.n, g.line);
		c->arena_guards.clear();
		for(void* p : c->arena_spill) (void)hipFree(p);
		c->arena_spill.clear();
		c->arena_used = 0;
		c->pin_used = 0;
	}
};

int dalloc(bt2g_ctx* c, void** p, size_t n) {
	if(n == 0) n = 16;
	hipError_t e = hipMalloc(p, n);
	if(e != hipSuccess) return fail(BT2G_ERR_NOMEM, "hipMalloc(%zu): %s", n, hipGetErrorString(e));
	c->owned.push_back(*p);
	c->hbm_bytes += n;
	return BT2G_OK;
}

template <typename T>
int upload(bt2g_ctx* c, T** dst, const T* src, size_t count) {
	int rc = dalloc(c, (void**)dst, count * sizeof(T));
	if(rc) return rc;
	if(count) HIPCHK(hipMemcpy(*dst, src, count * sizeof(T), hipMemcpyHostToDevice));
	return BT2G_OK;
}

// the backtrace reads the reference through aligned 16-B windows: `pad` zero
// bytes after the end keep the last window in bounds
int upload_padded(bt2g_ctx* c, uint8_t** dst, const uint8_t* src, size_t count, size_t pad) {
	int rc = dalloc(c, (void**)dst, count + pad);
	if(rc) return rc;
	if(count) HIPCHK(hipMemcpy(*dst, src, count, hipMemcpyHostToDevice));
	HIPCHK(hipMemset(*dst + count, 0, pad));
	return BT2G_OK;
}

hipEvent_t get_event(bt2g_ctx* c) {
	if(!c->evpool.empty()) {
		hipEvent_t e = c->evpool.back();
		c->evpool.pop_back();
		return e;
	}
	hipEvent_t e;
	if(hipEventCreate(&e) != hipSuccess) return nullptr;
	return e;
}

struct ProfScope {
	bt2g_ctx* c;
	int kid;
	hipStream_t st;
	hipEvent_t a = nullptr;
	ProfScope(bt2g_ctx* c_, int kid_, hipStream_t st_) : c(c_), kid(kid_), st(st_) {
		if(c->prof) {
			a = get_event(c);
			if(a) (void)hipEventRecord(a, st);
		}
	}
	~ProfScope() {
		if(c->prof && a) {
			hipEvent_t b = get_event(c);
			if(b) {
				(void)hipEventRecord(b, st);
				c->pending.push_back({kid, a, b});
			}
		}
	}
};

void drain_prof(bt2g_ctx* c) {
	for(auto& p : c->pending) {
		float ms = 0.f;
		(void)hipEventSynchronize(p.b);
		if(hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
			c->launches[p.kid]++;
			c->total_ms[p.kid] += ms;
		}
		c->evpool.push_back(p.a);
		c->evpool.push_back(p.b);
	}
	c->pending.clear();
}

// The context's second stream (the 1-mm search's BWT' direction) with its
// fork/join events, and the event the poll wait records: made when the context
// is opened (or its stream remade), on the opening thread -- round 6: they had
// been made lazily by whichever service thread first needed them, after a
// profiler's tool init; the r04ag/r05aa/r05h SIGSEGVs inside the profiler's HSA
// intercept came from such threads' first launches.  Without the aux stream
// (creation failed) the directions run in turn.
bool mm_merged() {
	const char* e = getenv("BT2G_MM_MERGED");
	return !(e && *e == '0');
}

void make_aux(bt2g_ctx* c, bool need) {
	// (only for the two-stream 1-mm search, $BT2G_MM_MERGED=0: a stream made is a
	// stream the runtime maps onto one of its few hardware queues, used or not)
	if(!c->aux && need) {
		bool ok = hipStreamCreateWithPriority(&c->aux, hipStreamNonBlocking, c->prio) == hipSuccess;
		for(int i = 0; ok && i < 4; i++) ok = hipEventCreateWithFlags(&c->mm_ev[i], hipEventDisableTiming) == hipSuccess;
		if(!ok) {
			for(hipEvent_t& e : c->mm_ev)
				if(e) { (void)hipEventDestroy(e); e = nullptr; }
			if(c->aux) (void)hipStreamDestroy(c->aux);
			c->aux = nullptr;
		}
	}
	if(!c->poll_ev) (void)hipEventCreateWithFlags(&c->poll_ev, hipEventDisableTiming);
}

// NULL is the null (legacy default) stream, as everywhere in HIP; the host
// wrappers below pass the context stream explicitly.
hipStream_t pick(bt2g_ctx*, void* s) { return (hipStream_t)s; }

// --- .bt2 reading (bt2_io.cpp:39-616; reference.cpp:100-235) ---------------
bool read_file(const std::string& path, std::vector<uint8_t>& out) {
	std::ifstream f(path, std::ios::binary);
	if(!f) return false;
	f.seekg(0, std::ios::end);
	size_t n = (size_t)f.tellg();
	f.seekg(0, std::ios::beg);
	out.resize(n);
	if(n) f.read((char*)out.data(), (std::streamsize)n);
	return (bool)f;
}

struct HostEbwt {
	uint32_t len = 0, zoff = 0, line_rate = 0, off_rate = 0, ftab_chars = 0;
	std::vector<uint32_t> fchr, ftab, eftab, offs, rstarts;
	std::vector<uint8_t> sides;
};

int parse_ebwt(const std::string& p1, const std::string& p2, HostEbwt& e) {
	std::vector<uint8_t> d;
	if(!read_file(p1, d)) return fail(BT2G_ERR_IO, "cannot read %s", p1.c_str());
	size_t p = 0;
	auto u32 = [&](uint32_t& v) -> bool {
		if(p + 4 > d.size()) return false;
		memcpy(&v, d.data() + p, 4);
		p += 4;
		return true;
	};
	uint32_t one, lps, flags, npat, nfrag;
	if(!u32(one) || one != 1) return fail(BT2G_ERR_FORMAT, "%s: bad endianness word", p1.c_str());
	if(!u32(e.len) || !u32(e.line_rate) || !u32(lps) || !u32(e.off_rate) || !u32(e.ftab_chars) || !u32(flags))
		return fail(BT2G_ERR_FORMAT, "%s: short header", p1.c_str());
	if(e.line_rate != 6) return fail(BT2G_ERR_FORMAT, "%s: lineRate %u unsupported (64-B sides)", p1.c_str(), e.line_rate);
	if(!u32(npat)) return fail(BT2G_ERR_FORMAT, "%s: short", p1.c_str());
	p += 4ull * npat;
	if(!u32(nfrag)) return fail(BT2G_ERR_FORMAT, "%s: short", p1.c_str());
	e.rstarts.resize(3ull * nfrag);
	if(p + 12ull * nfrag > d.size()) return fail(BT2G_ERR_FORMAT, "%s: short rstarts", p1.c_str());
	memcpy(e.rstarts.data(), d.data() + p, 12ull * nfrag);
	p += 12ull * nfrag;
	uint64_t bwt_sz = e.len / 4 + 1, side_bwt_sz = 48;
	uint64_t nsides = (bwt_sz + side_bwt_sz - 1) / side_bwt_sz;
	if(p + nsides * 64 > d.size()) return fail(BT2G_ERR_FORMAT, "%s: short ebwt", p1.c_str());
	e.sides.assign(d.begin() + p, d.begin() + p + nsides * 64);
	p += nsides * 64;
	if(!u32(e.zoff)) return fail(BT2G_ERR_FORMAT, "%s: short", p1.c_str());
	e.fchr.resize(5);
	for(int i = 0; i < 5; i++) if(!u32(e.fchr[i])) return fail(BT2G_ERR_FORMAT, "%s: short fchr", p1.c_str());
	uint64_t flen = (1ull << (2 * e.ftab_chars)) + 1;
	e.ftab.resize(flen);
	e.eftab.resize(2ull * e.ftab_chars);
	if(p + 4 * (flen + e.eftab.size()) > d.size()) return fail(BT2G_ERR_FORMAT, "%s: short ftab", p1.c_str());
	memcpy(e.ftab.data(), d.data() + p, 4 * flen);
	p += 4 * flen;
	memcpy(e.eftab.data(), d.data() + p, 4 * e.eftab.size());
	if(!p2.empty()) {
		std::vector<uint8_t> d2;
		if(!read_file(p2, d2)) return fail(BT2G_ERR_IO, "cannot read %s", p2.c_str());
		if(d2.size() < 4) return fail(BT2G_ERR_FORMAT, "%s: short", p2.c_str());
		e.offs.resize((d2.size() - 4) / 4);
		memcpy(e.offs.data(), d2.data() + 4, e.offs.size() * 4);
	}
	return BT2G_OK;
}

int parse_ref(const std::string& base, std::vector<uint8_t>& codes, std::vector<uint64_t>& starts) {
	std::vector<uint8_t> d3, d4;
	if(!read_file(base + ".3.bt2", d3)) return fail(BT2G_ERR_IO, "cannot read %s.3.bt2", base.c_str());
	if(!read_file(base + ".4.bt2", d4)) return fail(BT2G_ERR_IO, "cannot read %s.4.bt2", base.c_str());
	if(d3.size() < 8) return fail(BT2G_ERR_FORMAT, ".3.bt2 short");
	uint32_t one, nrec;
	memcpy(&one, d3.data(), 4);
	memcpy(&nrec, d3.data() + 4, 4);
	if(one != 1) return fail(BT2G_ERR_FORMAT, ".3.bt2 endianness");
	uint64_t jo = 0;
	for(uint32_t i = 0; i < nrec; i++) {
		size_t q = 8 + 9ull * i;
		if(q + 9 > d3.size()) return fail(BT2G_ERR_FORMAT, ".3.bt2 short");
		uint32_t off, len;
		memcpy(&off, d3.data() + q, 4);
		memcpy(&len, d3.data() + q + 4, 4);
		bool first = d3[q + 8] != 0;
		if(first) starts.push_back(codes.size());
		codes.insert(codes.end(), off, (uint8_t)4);
		for(uint32_t k = 0; k < len; k++, jo++) {
			if((jo >> 2) >= d4.size()) return fail(BT2G_ERR_FORMAT, ".4.bt2 short");
			codes.push_back((d4[jo >> 2] >> ((jo & 3) * 2)) & 3);
		}
	}
	starts.push_back(codes.size());
	return BT2G_OK;
}

int make_dev_ebwt(bt2g_ctx* c, const bt2g_ebwt_mem& m, bool fw, DevEbwt& d) {
	int rc;
	uint8_t* sides;
	uint32_t *ftab, *eftab, *offs = nullptr;
	if((rc = upload(c, &sides, m.sides, m.sides_bytes))) return rc;
	if((rc = upload(c, &ftab, m.ftab, (size_t)(1ull << (2 * m.ftab_chars)) + 1))) return rc;
	if((rc = upload(c, &eftab, m.eftab, (size_t)2 * m.ftab_chars))) return rc;
	if(m.offs && m.offs_len) {
		if((rc = upload(c, &offs, m.offs, (size_t)m.offs_len))) return rc;
	}
	d.sides = sides; d.ftab = ftab; d.eftab = eftab; d.offs = offs;
	d.len = m.len; d.zoff = m.zoff; d.ftab_chars = m.ftab_chars; d.off_rate = m.off_rate; d.fw = fw ? 1 : 0;
	uint32_t side = m.zoff / 192u, co = m.zoff % 192u;
	d.zbyte = side * 64u + (co >> 2);
	d.zbp = (int32_t)(co & 3);
	for(int i = 0; i < 5; i++) d.fchr[i] = m.fchr[i];
	if(fw) c->num_sides = m.sides_bytes / 64;
	return BT2G_OK;
}

}  // namespace

extern "C" {

const char* bt2g_last_error(void) { return g_err.c_str(); }

int bt2g_open_mem(const bt2g_index_mem* m, int device, bt2g_ctx** out) {
	if(!m || !out) return fail(BT2G_ERR_ARG, "null argument");
	if(m->fw.line_rate != 6 || m->bw.line_rate != 6) return fail(BT2G_ERR_FORMAT, "lineRate must be 6");
	int ndev = 0;
	HIPCHK(hipGetDeviceCount(&ndev));
	if(device < 0 || device >= ndev) return fail(BT2G_ERR_ARG, "device %d of %d", device, ndev);
	HIPCHK(hipSetDevice(device));
	// $BT2G_SYNC: how a host thread waits for the device (blocking | yield | spin);
	// a process with many threads driving contexts wants its cores back (blocking)
	if(const char* sy = getenv("BT2G_SYNC")) {
		unsigned fl = !strcmp(sy, "blocking") ? hipDeviceScheduleBlockingSync
		            : !strcmp(sy, "yield")    ? hipDeviceScheduleYield
		            : !strcmp(sy, "spin")     ? hipDeviceScheduleSpin
		                                      : hipDeviceScheduleAuto;
		(void)hipSetDeviceFlags(fl);
	}
	// the device's stream-ordered pool keeps what the _dev calls free
	// (hipMallocAsync scratch): with the default release threshold of 0 every
	// synchronisation may hand it back to the driver and the next call maps it
	// again ($BT2G_POOL_KEEP=1 keeps it; opt-in until measured on the paired step)
	{
		const char* pk = getenv("BT2G_POOL_KEEP");
		hipMemPool_t pool;
		if(pk && pk[0] == '1' && hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
			uint64_t keep = UINT64_MAX;
			(void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
		}
	}
	// the workgroup walk's LDS opt-in on this device, before the context has a
	// stream (sw_backtrace_wg.hip)
	sw_bt_wg_lds_init(device);
	sw_bt_lds_init(device);
	bt2g_ctx* c = new bt2g_ctx();
	c->device = device;
	int rc;
	if(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
		delete c;
		return fail(BT2G_ERR_HIP, "hipStreamCreate failed");
	}
	if((rc = make_dev_ebwt(c, m->fw, true, c->fw)) || (rc = make_dev_ebwt(c, m->bw, false, c->bw)) ||
	   (rc = upload_padded(c, &c->ref_codes, m->ref_codes, (size_t)m->ref_starts[m->nref], 64)) ||
	   (rc = upload(c, &c->ref_starts, m->ref_starts, (size_t)m->nref + 1))) {
		bt2g_close(c);
		return rc;
	}
	c->nref = m->nref;
	make_aux(c, !mm_merged());
	*out = c;
	return BT2G_OK;
}

int bt2g_set_priority(bt2g_ctx* c, int high) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	HIPCHK(hipSetDevice(c->device));
	int least = 0, greatest = 0;
	HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
	const int p = high ? greatest : 0;
	if(p == c->prio) return BT2G_OK;
	if(c->cu_masked) return fail(BT2G_ERR_ARG, "bt2g_set_priority on a context with a CU share (bt2g_set_cu_share)");
	hipStream_t s = nullptr;
	HIPCHK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, p));
	if(c->stream) {
		(void)hipStreamSynchronize(c->stream);
		drain_prof(c);
		(void)hipStreamDestroy(c->stream);
	}
	c->stream = s;
	if(c->aux) {                        // made again, at the new priority
		(void)hipStreamSynchronize(c->aux);
		(void)hipStreamDestroy(c->aux);
		c->aux = nullptr;
		for(hipEvent_t& e : c->mm_ev)
			if(e) { (void)hipEventDestroy(e); e = nullptr; }
	}
	c->prio = p;
	make_aux(c, !mm_merged());
	return BT2G_OK;
}

int bt2g_set_cu_share(bt2g_ctx* c, uint32_t num, uint32_t den) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	HIPCHK(hipSetDevice(c->device));
	int ncu = 0;
	HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device));
	hipStream_t s = nullptr;
	if(den == 0 || num >= den) {
		HIPCHK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, c->prio));
	} else {
		if(c->prio) return fail(BT2G_ERR_ARG, "bt2g_set_cu_share on a context with a priority (bt2g_set_priority)");
		std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
		int kept = 0;
		for(int i = 0; i < ncu; i++)
			if((uint32_t)i % den < num) {
				mask[(size_t)i / 32] |= 1u << (i % 32);
				kept++;
			}
		if(kept == 0) return fail(BT2G_ERR_ARG, "CU share %u/%u keeps no CU", num, den);
		HIPCHK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
	}
	if(c->stream) {
		(void)hipStreamSynchronize(c->stream);
		drain_prof(c);
		(void)hipStreamDestroy(c->stream);
	}
	c->stream = s;
	c->cu_masked = den != 0 && num < den;
	return BT2G_OK;
}

int bt2g_open_shared(bt2g_ctx* base, bt2g_ctx** out) {
	if(!base || !out) return fail(BT2G_ERR_ARG, "null argument");
	HIPCHK(hipSetDevice(base->device));
	bt2g_ctx* c = new bt2g_ctx();
	c->device = base->device;
	if(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
		delete c;
		return fail(BT2G_ERR_HIP, "hipStreamCreate failed");
	}
	// the index stays owned by `base` (c->owned is empty)
	c->fw = base->fw;
	c->bw = base->bw;
	c->ref_codes = base->ref_codes;
	c->ref_starts = base->ref_starts;
	c->nref = base->nref;
	c->num_sides = base->num_sides;
	c->hbm_bytes = base->hbm_bytes;
	c->base = base;
	base->shares++;
	make_aux(c, !mm_merged());
	*out = c;
	return BT2G_OK;
}

int bt2g_open(const char* index_base, int device, bt2g_ctx** out) {
	if(!index_base || !out) return fail(BT2G_ERR_ARG, "null argument");
	std::string b(index_base);
	HostEbwt F, B;
	int rc;
	if((rc = parse_ebwt(b + ".1.bt2", b + ".2.bt2", F))) return rc;
	if((rc = parse_ebwt(b + ".rev.1.bt2", "", B))) return rc;
	std::vector<uint8_t> codes;
	std::vector<uint64_t> starts;
	if((rc = parse_ref(b, codes, starts))) return rc;
	auto mem = [](HostEbwt& e) {
		bt2g_ebwt_mem m{};
		m.len = e.len; m.zoff = e.zoff; m.ftab_chars = e.ftab_chars; m.off_rate = e.off_rate;
		m.line_rate = e.line_rate; m.fchr = e.fchr.data(); m.sides = e.sides.data();
		m.sides_bytes = e.sides.size(); m.ftab = e.ftab.data(); m.eftab = e.eftab.data();
		m.offs = e.offs.empty() ? nullptr : e.offs.data(); m.offs_len = e.offs.size();
		m.rstarts = e.rstarts.data(); m.nfrag = (uint32_t)(e.rstarts.size() / 3);
		return m;
	};
	bt2g_index_mem m{};
	m.fw = mem(F);
	m.bw = mem(B);
	m.ref_codes = codes.data();
	m.ref_starts = starts.data();
	m.nref = (uint32_t)(starts.size() - 1);
	return bt2g_open_mem(&m, device, out);
}

static int rccl_destroy(void* comm);   // (multi-GPU section below)

int bt2g_close(bt2g_ctx* c) {
	if(!c) return BT2G_OK;
	if(c->shares.load() > 0)
		return fail(BT2G_ERR_ARG, "%d shared context(s) still use this index: close them first", c->shares.load());
	if(c->base) c->base->shares--;
	(void)hipSetDevice(c->device);
	if(c->stream) (void)hipStreamSynchronize(c->stream);
	drain_prof(c);
	for(hipEvent_t e : c->evpool) (void)hipEventDestroy(e);
	for(void* p : c->owned) (void)hipFree(p);
	if(c->sw_lists) { (void)hipFree(c->sw_lists); (void)hipFree(c->sw_counts); (void)hipFree(c->sw_bnd); }
	if(c->bt_plane) { (void)hipFree(c->bt_plane); (void)hipFree(c->bt_marks); }
	if(c->arena) (void)hipFree(c->arena);
	if(c->pin) (void)hipHostFree(c->pin);
	if(c->pin_dev) (void)hipFree(c->pin_dev);
	for(hipEvent_t& e : c->mm_ev)
		if(e) (void)hipEventDestroy(e);
	if(c->aux) (void)hipStreamDestroy(c->aux);
	if(c->poll_ev) (void)hipEventDestroy(c->poll_ev);
	if(c->comm) (void)rccl_destroy(c->comm);
	if(c->stream) (void)hipStreamDestroy(c->stream);
	delete c;
	return BT2G_OK;
}

int bt2g_info(bt2g_ctx* c, uint64_t* out, int n) {
	if(!c || !out) return fail(BT2G_ERR_ARG, "null argument");
	uint64_t v[13] = {c->fw.len, c->fw.zoff, c->bw.zoff, c->fw.fchr[0], c->fw.fchr[1], c->fw.fchr[2],
	                  c->fw.fchr[3], c->fw.fchr[4], c->fw.ftab_chars, c->fw.off_rate, c->num_sides, c->nref,
	                  c->hbm_bytes};
	for(int i = 0; i < n && i < 13; i++) out[i] = v[i];
	return BT2G_OK;
}

int bt2g_set_profiling(bt2g_ctx* c, int on) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	c->prof = on != 0;
	// the events of the first calls made here, on the calling thread (a service
	// thread then only takes them from the pool: see make_aux)
	HIPCHK(hipSetDevice(c->device));
	while(on && c->evpool.size() < 64) {
		hipEvent_t e;
		if(hipEventCreate(&e) != hipSuccess) break;
		c->evpool.push_back(e);
	}
	return BT2G_OK;
}

int bt2g_kernel_stats(bt2g_ctx* c, int k, uint64_t* launches, double* total_ms) {
	if(!c || k < 0 || k >= 16) return fail(BT2G_ERR_ARG, "bad kernel id");
	drain_prof(c);
	if(launches) *launches = c->launches[k];
	if(total_ms) *total_ms = c->total_ms[k];
	return BT2G_OK;
}

int bt2g_reset_stats(bt2g_ctx* c) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	drain_prof(c);
	memset(c->launches, 0, sizeof(c->launches));
	memset(c->total_ms, 0, sizeof(c->total_ms));
	return BT2G_OK;
}

// ---------------------------------------------------------------- FM engine
static int check_reads(uint32_t stride, uint32_t n) {
	if(stride == 0 || stride > BT2G_MAX_READ_LEN) return fail(BT2G_ERR_ARG, "stride %u out of range", stride);
	(void)n;
	return BT2G_OK;
}

int bt2g_exact_sweep_dev(bt2g_ctx* c, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t n,
                         uint32_t mine_max, int nofw, int norc, uint32_t* out, void* stream) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	if(int rc = check_reads(stride, n)) return rc;
	if(n == 0) return BT2G_OK;
	hipStream_t st = pick(c, stream);
	{
		ProfScope ps(c, 0, st);
		launch_exact_sweep(c->fw, reads, stride, lens, n, mine_max, nofw, norc, out, st);
	}
	HIPCHK(hipGetLastError());
	return BT2G_OK;
}

int bt2g_seed_search_dev(bt2g_ctx* c, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t n,
                         uint32_t seedlen, uint32_t interval, uint32_t offset, uint32_t maxseeds, uint32_t* out,
                         int32_t* nseeds, uint32_t* bwops, uint32_t* loads, void* stream) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	if(int rc = check_reads(stride, n)) return rc;
	if(seedlen == 0 || interval == 0 || maxseeds == 0) return fail(BT2G_ERR_ARG, "bad seed policy");
	if(n == 0) return BT2G_OK;
	hipStream_t st = pick(c, stream);
	HIPCHK(hipMemsetAsync(bwops, 0, sizeof(uint32_t) * n, st));
	if(loads) HIPCHK(hipMemsetAsync(loads, 0, sizeof(uint32_t) * n, st));
	{
		ProfScope ps(c, 1, st);
		launch_seed_search(c->fw, c->bw, reads, stride, lens, n, seedlen, interval, offset, maxseeds, out, nseeds,
		                   bwops, loads, st);
	}
	HIPCHK(hipGetLastError());
	return BT2G_OK;
}

namespace {
struct OneMmScratch {
	bt2g_mm1* slots = nullptr;
	int32_t* slot_counts = nullptr;
	int32_t* ovf = nullptr;        // ovf[0] overflow flag, ovf[1..4] item counts / queue heads
	uint32_t* items = nullptr;
	uint4* near_state = nullptr;
	uint32_t* near_dep = nullptr;
	MmBranch* brq = nullptr;
	uint32_t* fb_items = nullptr;
	uint4* fb_st4 = nullptr;
	uint32_t* fb_sdep = nullptr;
	uint32_t* slot_flag = nullptr;
};
}  // namespace

static int one_mm_impl(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                       const uint32_t* lens, uint32_t n, const int32_t* minsc, const bt2g_scoring* sc, int nofw,
                       int norc, const uint32_t* gate, uint32_t cap, bt2g_mm1* hits, int32_t* counts,
                       uint32_t* bwops, uint32_t* loads, void* stream, bool sync_overflow) {
	if(!c || !sc) return fail(BT2G_ERR_ARG, "null argument");
	if(int rc = check_reads(stride, n)) return rc;
	if(cap == 0) return fail(BT2G_ERR_ARG, "cap must be > 0");
	if(n == 0) return BT2G_OK;
	hipStream_t st = pick(c, stream);
	if(!c->aux && !mm_merged()) make_aux(c, true);     // (the variable changed after the context opened)
	OneMmScratch s;
	HIPCHK(amalloc(c, (void**)&s.slots, sizeof(bt2g_mm1) * (size_t)n * 4 * cap, st));
	HIPCHK(amalloc(c, (void**)&s.slot_counts, sizeof(int32_t) * (size_t)n * 4, st));
	HIPCHK(amalloc(c, (void**)&s.ovf, sizeof(int32_t) * 16, st));
	HIPCHK(amalloc(c, (void**)&s.items, sizeof(uint32_t) * (size_t)n * 4, st));
	HIPCHK(amalloc(c, (void**)&s.near_state, sizeof(uint4) * (size_t)n * 4, st));
	HIPCHK(amalloc(c, (void**)&s.near_dep, sizeof(uint32_t) * (size_t)n * 4, st));
	// far-half branches queued for the branch kernel (16 per read: an item that
	// meets a full queue is redone whole by the in-place state machine)
	// ($BT2G_MM_BRQ_CAP: a smaller queue, for the tests of the overflow paths)
	uint32_t brq_cap = n * 16 + 1024;
	if(const char* e = getenv("BT2G_MM_BRQ_CAP"))
		if(atol(e) > 0 && (uint32_t)atol(e) < brq_cap) brq_cap = (uint32_t)atol(e);
	HIPCHK(amalloc(c, (void**)&s.brq, sizeof(MmBranch) * (size_t)brq_cap, st));
	HIPCHK(amalloc(c, (void**)&s.fb_items, sizeof(uint32_t) * (size_t)n * 4, st));
	HIPCHK(amalloc(c, (void**)&s.fb_st4, sizeof(uint4) * (size_t)n * 4, st));
	HIPCHK(amalloc(c, (void**)&s.fb_sdep, sizeof(uint32_t) * (size_t)n * 4, st));
	HIPCHK(amalloc(c, (void**)&s.slot_flag, sizeof(uint32_t) * (size_t)n * 4, st));
	HIPCHK(hipMemsetAsync(s.ovf, 0, sizeof(int32_t) * 16, st));
	// (bwops, loads and the slot flags are zeroed by k_one_mm_items, the first kernel)
	{
		ProfScope ps(c, 2, st);
		launch_one_mm(c->fw, c->bw, reads, quals, stride, lens, n, minsc, *sc, nofw, norc, gate, cap, s.items,
		              (uint32_t*)s.ovf + 1, s.near_state, s.near_dep, s.slots, s.slot_counts, hits, counts, bwops,
		              loads, s.ovf, s.brq, brq_cap, s.fb_items, s.fb_st4, s.fb_sdep, s.slot_flag, st, c->aux, c->aux ? c->mm_ev : nullptr);
	}
	HIPCHK(hipGetLastError());
	int32_t ovf = 0;
	if(sync_overflow) HIPCHK(hipMemcpyAsync(&ovf, s.ovf, sizeof(int32_t), hipMemcpyDeviceToHost, st));
	HIPCHK(afree(c, s.slots, st));
	HIPCHK(afree(c, s.slot_counts, st));
	HIPCHK(afree(c, s.ovf, st));
	HIPCHK(afree(c, s.items, st));
	HIPCHK(afree(c, s.near_state, st));
	HIPCHK(afree(c, s.near_dep, st));
	HIPCHK(afree(c, s.brq, st));
	HIPCHK(afree(c, s.fb_items, st));
	HIPCHK(afree(c, s.fb_st4, st));
	HIPCHK(afree(c, s.fb_sdep, st));
	HIPCHK(afree(c, s.slot_flag, st));
	if(sync_overflow) {
		HIPCHK(stream_wait(c, st));
		if(ovf) return fail(BT2G_ERR_OVERFLOW, "one-mismatch hits exceed cap %u", cap);
	}
	return BT2G_OK;
}

int bt2g_one_mm_dev(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride, const uint32_t* lens,
                    uint32_t n, const int32_t* minsc, const bt2g_scoring* sc, int nofw, int norc, uint32_t cap,
                    bt2g_mm1* hits, int32_t* counts, uint32_t* bwops, uint32_t* loads, void* stream) {
	return one_mm_impl(c, reads, quals, stride, lens, n, minsc, sc, nofw, norc, nullptr, cap, hits, counts, bwops,
	                   loads, stream, true);
}

int bt2g_one_mm_gated_dev(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                          const uint32_t* lens, uint32_t n, const int32_t* minsc, const bt2g_scoring* sc,
                          const uint32_t* sweep, uint32_t cap, bt2g_mm1* hits, int32_t* counts, uint32_t* bwops,
                          uint32_t* loads, void* stream) {
	if(!sweep) return fail(BT2G_ERR_ARG, "null sweep");
	return one_mm_impl(c, reads, quals, stride, lens, n, minsc, sc, 0, 0, sweep, cap, hits, counts, bwops, loads,
	                   stream, false);
}

int bt2g_get_offset_dev(bt2g_ctx* c, const uint32_t* rows, uint32_t n, uint32_t* offs, uint32_t* loads,
                        void* stream) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	if(!c->fw.offs) return fail(BT2G_ERR_ARG, "SA sample not loaded");
	if(n == 0) return BT2G_OK;
	hipStream_t st = pick(c, stream);
	{
		ProfScope ps(c, 3, st);
		launch_get_offset(c->fw, rows, n, offs, loads, st);
	}
	HIPCHK(hipGetLastError());
	return BT2G_OK;
}

int bt2g_extend_dev(bt2g_ctx* c, const uint8_t* reads, uint32_t stride, const uint32_t* lens, const bt2g_ext_in* in,
                    uint32_t n, bt2g_ext_out* out, void* stream) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	if(int rc = check_reads(stride, n)) return rc;
	if(n == 0) return BT2G_OK;
	hipStream_t st = pick(c, stream);
	{
		ProfScope ps(c, 12, st);
		launch_extend(c->fw, c->bw, c->bw.sides != nullptr, reads, stride, lens, in, n, out, st);
	}
	HIPCHK(hipGetLastError());
	return BT2G_OK;
}

// ---------------------------------------------------------------- SW engine
// The packed two-problems-per-lane fill covers end-to-end scoring without a
// match bonus and local scoring whose profile bytes (match + penalty) fit a
// byte and whose scores cannot saturate i16, without matrix dumps; anything
// else runs the one-problem-per-lane fills.
static bool sw_packed_ok(const bt2g_scoring& sc, const SwConst& C, const int16_t* mat, uint32_t stride) {
	if(mat || sc.gapbar < 1 || C.npen < 1 || C.npen > 255) return false;
	for(int q = 0; q <= 40; q++)
		if(C.mmpen[q] < 1 || C.mmpen[q] > 255) return false;   // non-zero profile marks a real row
	if(C.rdgo < 0 || C.rdge < 0 || C.rfgo < 0 || C.rfge < 0) return false;
	if(!sc.local) return sc.match == 0;
	if(C.match < 1 || C.match + C.npen > 255 || (uint64_t)stride * (uint64_t)C.match >= 32767u) return false;
	for(int q = 0; q <= 40; q++)
		if(C.match + C.mmpen[q] > 255) return false;
	return true;
}

// the systolic fill's LDS holds (64/S) groups of selector (and local) words
static bool sw_use_packed(const bt2g_scoring& sc, const SwConst& C, const int16_t* mat, uint32_t stride,
                          uint32_t maxcol) {
	const uint32_t S = (stride + 15u) / 16u;
	if(S > 128u) return false;                     // one problem pair's rows across two waves at most
	const uint64_t lds = (uint64_t)(S > 64u ? 1u : 64u / S) * sw_packed_group_words(maxcol, sc.local != 0) * 4u;
	return sw_packed_ok(sc, C, mat, stride) && lds <= 65536u;
}

// Fill + gather + candidate sort.  plane != NULL (systolic path only): also
// write the score plane for the backtrace.  maxcol_hint: widest problem when
// the caller already knows it (0: read the problems back).
static int sw_align_impl(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                         const uint32_t* lens, const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* windows,
                         const bt2g_scoring* sc, int enable8, uint32_t cap, bt2g_sw_result* res, bt2g_sw_cand* cands,
                         int16_t* mat, const uint64_t* mat_off, uint8_t* plane, uint64_t hslot, int hbytes,
                         uint32_t maxcol_hint, hipStream_t st) {
	SwConst C;
	sw_fill_consts(*sc, C);
	// problem lists per fill variant + boundary scratch
	uint32_t *lists, *counts, *bnd;
	size_t nblk = (nprob + 63) / 64;
	uint32_t maxcol = maxcol_hint;
	const bool reserved = nprob <= c->sw_max_prob && c->sw_lists && (maxcol == 0 || maxcol <= c->sw_max_cols);
	if(reserved) {
		// the reserved boundary scratch is sw_max_cols wide; a caller's width hint
		// (the backtrace's score-plane pitch) stays the launch width, since the
		// plane was laid out with it
		lists = c->sw_lists; counts = c->sw_counts; bnd = c->sw_bnd;
		if(maxcol == 0) maxcol = c->sw_max_cols;
	} else {
		if(maxcol == 0) {
			// widest problem decides the boundary buffer width (problems live on the device)
			std::vector<bt2g_sw_problem> hp(nprob);
			HIPCHK(hipMemcpyAsync(hp.data(), probs, sizeof(bt2g_sw_problem) * nprob, hipMemcpyDeviceToHost, st));
			HIPCHK(stream_wait(c, st));
			for(auto& p : hp) maxcol = p.ncol > maxcol ? p.ncol : maxcol;
		}
		HIPCHK(amalloc(c, (void**)&lists, sizeof(uint32_t) * (size_t)nprob * 3, st));
		HIPCHK(amalloc(c, (void**)&counts, sizeof(uint32_t) * 8, st));
		HIPCHK(amalloc(c, (void**)&bnd, sizeof(uint32_t) * nblk * (size_t)maxcol * 64 * 2, st));
	}
	HIPCHK(hipMemsetAsync(counts, 0, sizeof(uint32_t) * 8, st));
	uint32_t* list8 = lists;
	uint32_t* list16 = lists + nprob;
	uint32_t* satl = lists + 2 * (size_t)nprob;
	{
		ProfScope ps(c, 4, st);
		if(sw_use_packed(*sc, C, mat, stride, maxcol)) {
			launch_sw_packed(sc->local != 0, probs, nprob, reads, quals, stride, lens, windows, c->ref_codes,
			                 c->ref_starts, C, enable8, cap, maxcol, res, cands, plane, hslot, hbytes, st);
		} else {
		const PlaneOut po{plane, hslot, sw_plane_pitch(maxcol)};   // u16 score plane (hslot from sw_plane_slot(.., 2))
		launch_sw_partition(probs, nprob, sc->local, enable8, list8, counts + 0, list16, counts + 1, st);
		int v8 = sc->local ? 2 : 0, v16 = sc->local ? 3 : 1;
		launch_sw_fill(v8, probs, nprob, list8, counts + 0, reads, quals, stride, lens, windows, c->ref_codes,
		               c->ref_starts, C, cap, bnd, maxcol, res, cands, mat, mat_off, satl, counts + 2, po, st);
		launch_sw_fill(v16, probs, nprob, list16, counts + 1, reads, quals, stride, lens, windows, c->ref_codes,
		               c->ref_starts, C, cap, bnd, maxcol, res, cands, mat, mat_off, satl, counts + 3, po, st);
		if(sc->local) {
			// local u8 saturated -> i16 (aligner_sw.cpp:587-605)
			launch_sw_fill(3, probs, nprob, satl, counts + 2, reads, quals, stride, lens, windows, c->ref_codes,
			               c->ref_starts, C, cap, bnd, maxcol, res, cands, mat, mat_off, satl, counts + 3, po, st);
		}
		}
	}
	{
		ProfScope ps(c, 11, st);            // (kernel-stats id 11: the candidate sort)
		launch_sort_cands(res, cands, nprob, cap, list8, counts + 4, st);   // list8 is free again
	}
	HIPCHK(hipGetLastError());
	if(!reserved) {
		HIPCHK(afree(c, lists, st));
		HIPCHK(afree(c, counts, st));
		HIPCHK(afree(c, bnd, st));
	}
	return BT2G_OK;
}

static int sw_args_ok(const bt2g_scoring* sc, uint32_t cap) {
	if(!sc) return fail(BT2G_ERR_ARG, "null argument");
	if(cap == 0 || cap > 8192) return fail(BT2G_ERR_ARG, "cap out of range (1..8192)");
	if(sc->local && sc->match <= 0) return fail(BT2G_ERR_ARG, "local mode needs a match bonus");
	return BT2G_OK;
}

int bt2g_sw_align_dev(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                      const uint32_t* lens, const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* windows,
                      const bt2g_scoring* sc, int enable8, uint32_t cap, bt2g_sw_result* res, bt2g_sw_cand* cands,
                      int16_t* mat, const uint64_t* mat_off, void* stream) {
	if(!c) return fail(BT2G_ERR_ARG, "null argument");
	if(int rc = sw_args_ok(sc, cap)) return rc;
	if(int rc = check_reads(stride, nprob)) return rc;
	if(nprob == 0) return BT2G_OK;
	return sw_align_impl(c, reads, quals, stride, lens, probs, nprob, windows, sc, enable8, cap, res, cands, mat,
	                     mat_off, nullptr, 0, 0, 0, pick(c, stream));
}

}  // extern "C"

// What a host caller knows about its problems without reading them back from
// the device: widest window, longest read, whether every minsc fits the u8 fill.
struct SwHint {
	uint32_t maxcol, maxrow;
	bool all8;
};

static SwHint sw_hint(const bt2g_sw_problem* probs, uint32_t nprob, const uint32_t* lens, int enable8) {
	SwHint h{0, 0, enable8 != 0};
	for(uint32_t i = 0; i < nprob; i++) {
		h.maxcol = probs[i].ncol > h.maxcol ? probs[i].ncol : h.maxcol;
		const uint32_t L = lens[probs[i].read];
		h.maxrow = L > h.maxrow ? L : h.maxrow;
		h.all8 = h.all8 && probs[i].minsc >= -254;
	}
	return h;
}

// The widest DP (columns / rows) whose fill writes the walk's decision plane
// ($BT2G_DEC_RATIO, default 6: mate searches, ~150 x 700, included -- their
// walks then take the workgroup kernel; r04ad, paired through the batch server:
// 104.8 k pairs/s against 58.9 k with the H plane; wider ones keep the H plane)
static uint32_t dec_ratio() {
	static const uint32_t r = [] {
		const char* e = getenv("BT2G_DEC_RATIO");
		return e && atol(e) > 0 ? (uint32_t)atol(e) : 6u;
	}();
	return r;
}

static bool bt_hplane() {
	static const bool on = [] { const char* e = getenv("BT2G_BT_HPLANE"); return e && *e == '1'; }();
	return on;
}

static int sw_align_bt_impl(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                            const uint32_t* lens, const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* windows,
                            const bt2g_sw_rect* rects, const bt2g_scoring* sc, int enable8, uint32_t cap,
                            bt2g_sw_result* res, bt2g_sw_cand* cands, uint32_t maxaln, uint32_t maxedit,
                            int32_t* naln, bt2g_sw_aln* alns, bt2g_edit* edits, int8_t* fates, void* stream,
                            const SwHint* hint) {
	if(!c) return fail(BT2G_ERR_ARG, "null argument");
	if(int rc = sw_args_ok(sc, cap)) return rc;
	if(int rc = check_reads(stride, nprob)) return rc;
	if(maxaln == 0 || maxedit == 0 || !naln || !alns || !edits) return fail(BT2G_ERR_ARG, "bad backtrace outputs");
	if(nprob == 0) return BT2G_OK;
	hipStream_t st = pick(c, stream);
	SwConst C;
	sw_fill_consts(*sc, C);
	const uint32_t S16 = sw_packed_rows(stride);
	BtArgs a{};
	std::vector<void*> tmp;
	auto talloc = [&](void** p, size_t n) -> int {
		HIPCHK(amalloc(c, p, n ? n : 16, st));
		tmp.push_back(*p);
		return BT2G_OK;
	};
	int rc;
	bool packed;
	int hb;
	uint8_t* plane = nullptr;
	uint32_t maxcol = 0, maxrow = stride;
	const bool reserved = c->bt_plane && nprob <= c->bt_max_prob && stride <= c->bt_max_stride &&
	                      nprob <= c->sw_max_prob && c->sw_lists && c->bt_max_cols == c->sw_max_cols &&
	                      (sw_use_packed(*sc, C, nullptr, stride, c->bt_max_cols) || c->bt_hbytes == 2) &&
	                      (!sc->local || c->bt_hbytes == 2);    // local: u16 plane and dominance tiles
	if(reserved) {
		// the fill marks problems wider than the reservation (flag -3, not aligned)
		maxcol = c->bt_max_cols;
		maxrow = c->bt_max_stride;
		packed = sw_use_packed(*sc, C, nullptr, stride, maxcol);
		hb = packed ? c->bt_hbytes : 2;
		plane = c->bt_plane;
		a.marks = c->bt_marks;
	} else {
		bool all8 = enable8 != 0;
		if(hint) {
			maxcol = hint->maxcol;
			maxrow = hint->maxrow;
			all8 = hint->all8;
		} else {
			// problems and lengths live on the device: read them back (two syncs)
			std::vector<bt2g_sw_problem> hp(nprob);
			HIPCHK(hipMemcpyAsync(hp.data(), probs, sizeof(bt2g_sw_problem) * nprob, hipMemcpyDeviceToHost, st));
			uint32_t nreads = 0;
			HIPCHK(stream_wait(c, st));
			for(auto& p : hp) {
				maxcol = p.ncol > maxcol ? p.ncol : maxcol;
				nreads = p.read + 1 > nreads ? p.read + 1 : nreads;
				all8 = all8 && p.minsc >= -254;
			}
			std::vector<uint32_t> hl(nreads);
			HIPCHK(hipMemcpyAsync(hl.data(), lens, sizeof(uint32_t) * nreads, hipMemcpyDeviceToHost, st));
			HIPCHK(stream_wait(c, st));
			maxrow = 0;
			for(uint32_t i = 0; i < nreads; i++) maxrow = hl[i] > maxrow ? hl[i] : maxrow;
		}
		packed = sw_use_packed(*sc, C, nullptr, stride, maxcol);
		hb = packed && all8 && !sc->local ? 1 : 2;
		// end-to-end systolic fills, u8 and i16 alike (long reads: minsc < -254), write
		// the walk's decisions (kind 2, the u8 plane's layout)
		if(packed && !sc->local && !bt_hplane() && maxcol <= dec_ratio() * maxrow) hb = 1;
		if((rc = talloc((void**)&plane, (size_t)sw_plane_slot(stride, maxcol, hb) * nprob))) return rc;
	}
	// systolic fill: bottom-aligned rows, u8 (hb 1) or u16 plane with block masks;
	// one-problem-per-lane fills (local, other scorings): top-aligned u16 plane
	// end-to-end systolic fills: the fill writes the walk's decision per cell (kind
	// 2, 4 bits); BT2G_BT_HPLANE=1 keeps the H score plane (kind 0) for A/B runs
	// (wide DPs -- mate searches, 150 x 705 -- keep the H plane: the decision bits
	// cost fill work per cell, and their walks touch a small share of the cells)
	const bool dec = packed && !sc->local && !bt_hplane() && maxcol <= dec_ratio() * maxrow && (!reserved || hb == 1);
	const int kind = dec ? 2 : hb == 1 ? 0 : 1;
	a.plane = plane;
	a.slot = sw_plane_slot(stride, maxcol, hb);
	a.plane_top = !packed ? 1 : sc->local ? 2 : 0;
	if((rc = sw_align_impl(c, reads, quals, stride, lens, probs, nprob, windows, sc, enable8, cap, res, cands,
	                       nullptr, nullptr, plane, a.slot, kind == 2 ? 3 : hb, maxcol, st)))
		return rc;
	a.rwords = sw_bt_rcols(maxrow, maxcol);
	a.rrows = sw_bt_rrows(maxrow);
	a.mwords = sw_bt_tcols(maxcol);
	a.mrows = sw_bt_trows(maxrow);
	a.mslot = sw_bt_mslot(maxrow, maxcol, sc->local != 0);
	a.mdom = sc->local ? sw_bt_mdom(maxrow, maxcol) : 0u;
	if(!a.marks && (rc = talloc((void**)&a.marks, sizeof(uint32_t) * (a.mslot * nprob + 64u)))) return rc;
	// one DP per lane; BT2G_BT_QUEUE=1: lanes take DPs from a counter after this
	// call's marks (exact, but measured slower: 32.1 vs 22.9 ms per 1M DPs --
	// lanes at different phases make every wave iteration issue every path)
	static const bool bt_queue = [] { const char* e = getenv("BT2G_BT_QUEUE"); return e && *e == '1'; }();
	if(bt_queue) {
		a.queue = a.marks + a.mslot * nprob;
		HIPCHK(hipMemsetAsync(a.queue, 0, sizeof(uint32_t), st));
	}
	a.probs = probs; a.nprob = nprob; a.reads = reads; a.quals = quals; a.stride = stride; a.lens = lens;
	a.windows = windows; a.ref_codes = c->ref_codes; a.ref_starts = c->ref_starts; a.rects = rects;
	a.res = res; a.cands = cands; a.cap = cap; a.cstride = S16; a.pcols = sw_plane_pitch(maxcol);
#ifdef BT2G_SW_NOMASK
	a.use_mask = 0;   // timing experiments only
#else
	a.use_mask = packed && S16 <= 256u;
#endif
	a.C = C; a.local = sc->local; a.ncl_const = sc->ncl_const; a.ncl_lin = sc->ncl_lin;
	a.maxaln = maxaln; a.maxedit = maxedit; a.naln = naln; a.alns = alns; a.edits = edits; a.fates = fates;
	{
		ProfScope ps(c, 5, st);
		launch_sw_bt(kind, a, st);
	}
	HIPCHK(hipGetLastError());
	for(void* p : tmp) HIPCHK(afree(c, p, st));
	return BT2G_OK;
}

extern "C" {

int bt2g_sw_align_bt_dev(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                         const uint32_t* lens, const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* windows,
                         const bt2g_sw_rect* rects, const bt2g_scoring* sc, int enable8, uint32_t cap,
                         bt2g_sw_result* res, bt2g_sw_cand* cands, uint32_t maxaln, uint32_t maxedit,
                         int32_t* naln, bt2g_sw_aln* alns, bt2g_edit* edits, int8_t* fates, void* stream) {
	return sw_align_bt_impl(c, reads, quals, stride, lens, probs, nprob, windows, rects, sc, enable8, cap, res, cands,
	                        maxaln, maxedit, naln, alns, edits, fates, stream, nullptr);
}

int bt2g_ungapped_dev(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                      const uint32_t* lens, const bt2g_ug_problem* probs, uint32_t n, const bt2g_scoring* sc,
                      int ohang, uint32_t maxedit, bt2g_ug_result* res, bt2g_edit* edits, void* stream) {
	if(!c || !sc || !res || (!edits && maxedit)) return fail(BT2G_ERR_ARG, "null argument");
	if(int rc = check_reads(stride, n)) return rc;
	if(n == 0) return BT2G_OK;
	hipStream_t st = pick(c, stream);
	SwConst C;
	sw_fill_consts(*sc, C);
	{
		ProfScope ps(c, 6, st);
		launch_ungapped(probs, n, reads, quals, stride, lens, c->ref_codes, c->ref_starts, C, sc->local, sc->ncl_const,
		                sc->ncl_lin, ohang, maxedit, res, edits, st);
	}
	HIPCHK(hipGetLastError());
	return BT2G_OK;
}

int bt2g_frame_dev(bt2g_ctx* c, const bt2g_frame_in* in, uint32_t n, const uint32_t* lens, const bt2g_scoring* sc,
                   const bt2g_pe_policy* pe, int32_t maxhalf, int trim_to_ref, bt2g_sw_problem* probs,
                   bt2g_sw_rect* rects, int32_t* ok, void* stream) {
	if(!c || !sc || (n && (!in || !lens || !probs || !rects || !ok))) return fail(BT2G_ERR_ARG, "null argument");
	if(maxhalf < 0) return fail(BT2G_ERR_ARG, "maxhalf %d < 0", maxhalf);
	bt2g_pe_policy P{};
	P.policy = 3;
	P.maxfrag = 500;
	if(pe) {
		if(pe->policy < 1 || pe->policy > 4) return fail(BT2G_ERR_ARG, "no such PE policy %d", pe->policy);
		if(pe->maxfrag <= 0 || pe->minfrag < 0 || pe->maxfrag < pe->minfrag)
			return fail(BT2G_ERR_ARG, "bad fragment lengths [%d, %d]", pe->minfrag, pe->maxfrag);
		P = *pe;
	}
	if(n == 0) return BT2G_OK;
	hipStream_t st = pick(c, stream);
	FrameConst F;
	F.match = sc->match;
	F.rdgo = sc->rdg_const + sc->rdg_lin; F.rdge = sc->rdg_lin;
	F.rfgo = sc->rfg_const + sc->rfg_lin; F.rfge = sc->rfg_lin;
	F.maxhalf = maxhalf; F.trim_to_ref = trim_to_ref != 0;
	F.ncl_const = sc->ncl_const; F.ncl_lin = sc->ncl_lin;
	// every kind-1 input needs a policy: checked on the device would cost a
	// round trip, so a NULL policy is simply the defaults (--fr, -X 500)
	{
		ProfScope ps(c, 7, st);
		launch_frame(in, n, lens, c->ref_starts, F, P, probs, rects, ok, st);
	}
	HIPCHK(hipGetLastError());
	return BT2G_OK;
}

int bt2g_reserve_sw_bt(bt2g_ctx* c, uint32_t max_problems, uint32_t max_stride, uint32_t max_cols, int hbytes) {
	if(!c || max_problems == 0 || max_cols == 0 || max_stride == 0 || (hbytes != 1 && hbytes != 2))
		return fail(BT2G_ERR_ARG, "bad reservation");
	if(int rc = bt2g_reserve_sw(c, max_problems, max_cols)) return rc;
	// bt2g_reserve_sw synchronised the device: the old scratch is idle
	if(c->bt_plane) { (void)hipFree(c->bt_plane); (void)hipFree(c->bt_marks); }
	c->bt_plane = nullptr; c->bt_marks = nullptr;
	c->bt_max_prob = c->bt_max_stride = c->bt_max_cols = 0;
	c->bt_hbytes = 0;
	const uint64_t slot = sw_plane_slot(max_stride, max_cols, hbytes);
	uint8_t* plane = nullptr;
	uint32_t* marks = nullptr;
	hipError_t e = hipMalloc((void**)&plane, slot * max_problems);
	if(e == hipSuccess)
		e = hipMalloc((void**)&marks, sizeof(uint32_t) * (sw_bt_mslot(max_stride, max_cols, hbytes == 2) * max_problems + 64u));
	if(e != hipSuccess) {
		if(plane) (void)hipFree(plane);
		return fail(BT2G_ERR_NOMEM, "bt2g_reserve_sw_bt: %s", hipGetErrorString(e));
	}
	// commit only after every allocation succeeded
	c->bt_plane = plane;
	c->bt_marks = marks;
	c->bt_max_prob = max_problems;
	c->bt_max_stride = max_stride;
	c->bt_max_cols = max_cols;
	c->bt_hbytes = hbytes;
	return BT2G_OK;
}

int bt2g_reserve_sw(bt2g_ctx* c, uint32_t max_problems, uint32_t max_cols) {
	if(!c || max_problems == 0 || max_cols == 0) return fail(BT2G_ERR_ARG, "bad reservation");
	HIPCHK(hipSetDevice(c->device));
	HIPCHK(hipDeviceSynchronize());   // the old scratch may be in use on any stream
	if(c->sw_lists) { (void)hipFree(c->sw_lists); (void)hipFree(c->sw_counts); (void)hipFree(c->sw_bnd); }
	c->sw_lists = c->sw_counts = c->sw_bnd = nullptr;
	c->sw_max_prob = c->sw_max_cols = 0;
	size_t nblk = ((size_t)max_problems + 63) / 64;
	uint32_t *lists = nullptr, *counts = nullptr, *bnd = nullptr;
	hipError_t e = hipMalloc((void**)&lists, sizeof(uint32_t) * (size_t)max_problems * 3);
	if(e == hipSuccess) e = hipMalloc((void**)&counts, sizeof(uint32_t) * 8);
	if(e == hipSuccess) e = hipMalloc((void**)&bnd, sizeof(uint32_t) * nblk * (size_t)max_cols * 64 * 2);
	if(e != hipSuccess) {
		if(lists) (void)hipFree(lists);
		if(counts) (void)hipFree(counts);
		return fail(BT2G_ERR_NOMEM, "bt2g_reserve_sw: %s", hipGetErrorString(e));
	}
	c->sw_lists = lists;
	c->sw_counts = counts;
	c->sw_bnd = bnd;
	c->sw_max_prob = max_problems;
	c->sw_max_cols = max_cols;
	return BT2G_OK;
}

}  // extern "C"

// ------------------------------------------------------ host-pointer wrappers
namespace {
// Device copies of a host-flavour call's arrays.  Inputs are staged in the
// context's pinned block and placed at the same offsets of its device mirror,
// so that send() moves them all in ONE copy; outputs declared with out() get a
// slot in the same mirror, and finish() brings every one of them back in ONE
// copy.  Scratch (up() without host data) comes from the arena.  Everything on
// the context's stream, one stream synchronisation per finish(): no null-stream
// copy that would wait on the other contexts' work.  When the pinned block is
// too small (its first use, or a bigger call) the arrays are copied one by one
// and the block grows for the next call.
struct Tmp {
	Arena ar;
	bt2g_ctx* c;
	hipStream_t st;
	struct Out { void* h; const void* pin; size_t n; };
	std::vector<Out> outs;
	struct Late { void* h; const void* d; size_t n; };
	std::vector<Late> late;               // outputs outside the mirror (copied at finish)
	size_t sent = 0;                      // pinned bytes already on the device
	size_t in_hi = 0;                     // end of the highest staged input (outputs past it are not sent)
	size_t mo_lo = SIZE_MAX, mo_hi = 0;   // mirrored outputs still to bring back
	size_t map_lo = SIZE_MAX;             // lowest pinned offset a kernel writes directly
	bool pending = false;                 // staged inputs not yet sent
	explicit Tmp(bt2g_ctx* cx) : ar(cx), c(cx), st(cx->stream) {}
	template <typename T>
	int up(T** d, const T* h, size_t count) {
		const size_t bytes = count * sizeof(T);
		// (pinned() also records the size the block needs: it grows for the next call)
		if(uint8_t* pn = h && count ? ar.pinned(bytes) : nullptr) {
			memcpy(pn, h, bytes);
			*d = (T*)(c->pin_dev + (pn - c->pin));
			in_hi = std::max(in_hi, (size_t)(pn - c->pin) + bytes);
			pending = true;
			return BT2G_OK;
		}
		if(amalloc(c, (void**)d, bytes + 16, st) != hipSuccess)
			return fail(BT2G_ERR_NOMEM, "device scratch (%zu bytes)", bytes + 16);
		if(h && count && hipMemcpyAsync(*d, h, bytes, hipMemcpyHostToDevice, st) != hipSuccess)
			return fail(BT2G_ERR_HIP, "hipMemcpyAsync H2D");
		return BT2G_OK;
	}
	// the staged inputs to the device (before the first launch that reads them)
	int send() {
		// only the staged inputs: the out() slots and mapped() blocks after them are
		// written by the kernels (the whole used span was copied, up to
		// several MB of worst-case candidate / edit slots per DP batch)
		if(in_hi > sent) {
			HIPCHK(hipMemcpyAsync(c->pin_dev + sent, c->pin + sent, in_hi - sent, hipMemcpyHostToDevice, st));
			sent = in_hi;
		}
		pending = false;
		return BT2G_OK;
	}
	// a block of pinned host memory that kernels write directly (no copy back):
	// the device's pointer to it, *h the host's; nullptr when the block is too
	// small this call.  Called after the call's out()s.
	template <typename T>
	T* mapped(size_t count, T** h) {
		uint8_t* pn = ar.pinned(count * sizeof(T) + 16);
		if(!pn) return nullptr;
		map_lo = std::min(map_lo, (size_t)(pn - c->pin));
		*h = (T*)pn;
		return (T*)(c->pin_dview + (pn - c->pin));
	}
	// a device output that finish() copies to h (`count` elements)
	template <typename T>
	int out(T** d, T* h, size_t count) {
		const size_t bytes = count * sizeof(T);
		uint8_t* pn = bytes ? ar.pinned(bytes) : nullptr;
		if(!pn) {
			// no mirror slot (the block grows for the next call): arena output, copied
			// back by finish() after the work that writes it
			int rc = up(d, (const T*)nullptr, count);
			if(rc == BT2G_OK && bytes) late.push_back(Late{(void*)h, (const void*)*d, bytes});
			return rc;
		}
		*d = (T*)(c->pin_dev + (pn - c->pin));
		const size_t o = (size_t)(pn - c->pin);
		mo_lo = std::min(mo_lo, o);
		mo_hi = std::max(mo_hi, o + bytes);
		outs.push_back(Out{h, pn, bytes});
		return BT2G_OK;
	}
	// enqueue a result copy (valid after finish)
	template <typename T>
	int down(T* h, const T* d, size_t count) {
		const size_t bytes = count * sizeof(T);
		if(bytes == 0) return BT2G_OK;
		uint8_t* pn = ar.pinned(bytes);
		HIPCHK(hipMemcpyAsync(pn ? (void*)pn : (void*)h, d, bytes, hipMemcpyDeviceToHost, st));
		if(pn) outs.push_back(Out{h, pn, bytes});
		return BT2G_OK;
	}
	int finish() {
		if(pending) return fail(BT2G_ERR_ARG, "internal: inputs staged but never sent");
		// (the mirror's copy back must not cover host memory a kernel wrote)
		if(mo_hi > mo_lo && mo_hi > map_lo) return fail(BT2G_ERR_ARG, "internal: out() after mapped()");
		if(mo_hi > mo_lo) {
			HIPCHK(hipMemcpyAsync(c->pin + mo_lo, c->pin_dev + mo_lo, mo_hi - mo_lo, hipMemcpyDeviceToHost, st));
			mo_lo = SIZE_MAX;
			mo_hi = 0;
		}
		for(const Late& l : late) HIPCHK(hipMemcpyAsync(l.h, l.d, l.n, hipMemcpyDeviceToHost, st));
		late.clear();
		HIPCHK(stream_wait(c, st));
		for(const Out& o : outs) memcpy(o.h, o.pin, o.n);
		outs.clear();
		return BT2G_OK;
	}
};
}  // namespace

extern "C" {

int bt2g_exact_sweep(bt2g_ctx* c, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t n,
                     uint32_t mine_max, int nofw, int norc, uint32_t* out) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	HIPCHK(hipSetDevice(c->device));
	Tmp t(c);
	uint8_t* dr;
	uint32_t *dl, *dout;
	int rc;
	if((rc = t.up(&dr, reads, (size_t)n * stride)) || (rc = t.up(&dl, lens, n)) ||
	   (rc = t.out(&dout, out, (size_t)n * 8)) || (rc = t.send()))
		return rc;
	if((rc = bt2g_exact_sweep_dev(c, dr, stride, dl, n, mine_max, nofw, norc, dout, c->stream))) return rc;
	return t.finish();
}

int bt2g_seed_search(bt2g_ctx* c, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t n,
                     uint32_t seedlen, uint32_t interval, uint32_t offset, uint32_t maxseeds, uint32_t* out,
                     int32_t* nseeds, uint32_t* bwops, uint32_t* loads) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	HIPCHK(hipSetDevice(c->device));
	Tmp t(c);
	uint8_t* dr;
	uint32_t *dl, *dout, *dops, *dld = nullptr;
	int32_t* dns;
	int rc;
	size_t no = (size_t)n * 2 * maxseeds * 4;
	if((rc = t.up(&dr, reads, (size_t)n * stride)) || (rc = t.up(&dl, lens, n)) || (rc = t.out(&dout, out, no)) ||
	   (rc = t.out(&dns, nseeds, n)) || (rc = t.out(&dops, bwops, n)))
		return rc;
	if(loads && (rc = t.out(&dld, loads, n))) return rc;
	if((rc = t.send())) return rc;
	if((rc = bt2g_seed_search_dev(c, dr, stride, dl, n, seedlen, interval, offset, maxseeds, dout, dns, dops, dld,
	                              c->stream)))
		return rc;
	return t.finish();
}

int bt2g_seed_search_ext(bt2g_ctx* c, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t n,
                         uint32_t seedlen, uint32_t interval, uint32_t offset, uint32_t maxseeds, uint32_t* out,
                         int32_t* nseeds, uint32_t* bwops, uint32_t* loads, bt2g_ext_out* ext, uint32_t off_cap,
                         uint32_t* offs) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	if(offs && (!c->fw.offs || off_cap == 0)) return fail(BT2G_ERR_ARG, "offsets need the SA sample and off_cap > 0");
	HIPCHK(hipSetDevice(c->device));
	Tmp t(c);
	uint8_t* dr;
	uint32_t *dl, *dout, *dops, *dld = nullptr, *doffs = nullptr;
	bt2g_ext_out* dext = nullptr;
	int32_t* dns;
	int rc;
	const size_t nr = (size_t)n * 2 * maxseeds;
	if((rc = t.up(&dr, reads, (size_t)n * stride)) || (rc = t.up(&dl, lens, n)) || (rc = t.out(&dout, out, nr * 4)) ||
	   (rc = t.out(&dns, nseeds, n)) || (rc = t.out(&dops, bwops, n)))
		return rc;
	if(loads && (rc = t.out(&dld, loads, n))) return rc;
	if(ext && (rc = t.out(&dext, ext, nr))) return rc;
	if(offs && (rc = t.out(&doffs, offs, nr * off_cap))) return rc;
	if((rc = t.send())) return rc;
	if((rc = bt2g_seed_search_dev(c, dr, stride, dl, n, seedlen, interval, offset, maxseeds, dout, dns, dops, dld,
	                              c->stream)))
		return rc;
	// (kernel-stats ids: 12 the seed ranges' extension, 3 their rows' offsets)
	if(n && dext) {
		ProfScope ps(c, 12, c->stream);
		launch_seed_extend(c->fw, c->bw, c->bw.sides != nullptr, dr, stride, dl, n, seedlen, interval, offset, maxseeds,
		                   dout, dext, c->stream);
		HIPCHK(hipGetLastError());
	}
	if(n && doffs) {
		ProfScope ps(c, 3, c->stream);
		launch_seed_offsets(c->fw, dout, nr, off_cap, doffs, c->stream);
		HIPCHK(hipGetLastError());
	}
	return t.finish();
}

int bt2g_one_mm(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride, const uint32_t* lens,
                uint32_t n, const int32_t* minsc, const bt2g_scoring* sc, int nofw, int norc, uint32_t cap,
                bt2g_mm1* hits, int32_t* counts, uint32_t* bwops, uint32_t* loads) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	HIPCHK(hipSetDevice(c->device));
	Tmp t(c);
	uint8_t *dr, *dq;
	uint32_t *dl, *dops, *dld = nullptr;
	int32_t *dms, *dcnt;
	bt2g_mm1* dh;
	int rc;
	if((rc = t.up(&dr, reads, (size_t)n * stride)) || (rc = t.up(&dq, quals, (size_t)n * stride)) ||
	   (rc = t.up(&dl, lens, n)) || (rc = t.up(&dms, minsc, n)) || (rc = t.out(&dh, hits, (size_t)n * cap)) ||
	   (rc = t.out(&dcnt, counts, n)) || (rc = t.out(&dops, bwops, n)))
		return rc;
	if(loads && (rc = t.out(&dld, loads, n))) return rc;
	if((rc = t.send())) return rc;
	// (the overflow shows in the counts copied back: no sync of its own)
	if((rc = one_mm_impl(c, dr, dq, stride, dl, n, dms, sc, nofw, norc, nullptr, cap, dh, dcnt, dops, dld, c->stream,
	                     false)))
		return rc;
	if((rc = t.finish())) return rc;
	for(uint32_t i = 0; i < n; i++)
		if(counts[i] > (int32_t)cap) return fail(BT2G_ERR_OVERFLOW, "one-mismatch hits exceed cap %u", cap);
	return BT2G_OK;
}

int bt2g_exact_sweep_1mm(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                         const uint32_t* lens, uint32_t n, uint32_t mine_max, int nofw, int norc, int skip_exact,
                         const int32_t* minsc, const bt2g_scoring* sc, uint32_t cap, uint32_t* sweep,
                         bt2g_mm1* hits, int32_t* counts, uint32_t* bwops, uint32_t* mm_loads, uint32_t off_cap,
                         uint32_t* offs) {
	if(!c || !sc) return fail(BT2G_ERR_ARG, "null argument");
	if(offs && (!c->fw.offs || off_cap == 0)) return fail(BT2G_ERR_ARG, "offsets need the SA sample and off_cap > 0");
	HIPCHK(hipSetDevice(c->device));
	if(n == 0) return BT2G_OK;
	Tmp t(c);
	uint8_t *dr, *dq;
	uint32_t *dl, *dsw, *dops;
	int32_t *dms, *dcnt;
	bt2g_mm1* dh;
	int rc;
	if((rc = t.up(&dr, reads, (size_t)n * stride)) || (rc = t.up(&dq, quals, (size_t)n * stride)) ||
	   (rc = t.up(&dl, lens, n)) || (rc = t.up(&dms, minsc, n)) || (rc = t.out(&dsw, sweep, (size_t)n * 8)) ||
	   (rc = t.out(&dh, hits, (size_t)n * cap)) || (rc = t.out(&dcnt, counts, n)) || (rc = t.out(&dops, bwops, n)))
		return rc;
	uint32_t *doffs = nullptr, *dld = nullptr;
	if(offs && (rc = t.out(&doffs, offs, (size_t)n * (2u + cap) * off_cap))) return rc;
	if(mm_loads && (rc = t.out(&dld, mm_loads, n))) return rc;
	if((rc = t.send())) return rc;
	if((rc = bt2g_exact_sweep_dev(c, dr, stride, dl, n, mine_max, nofw, norc, dsw, c->stream))) return rc;
	// the gate reads the sweep on the device: no round trip between the two searches
	// (the items kernel reads the gate rule from bit 1 of nofw: MM_GATE_KEEP_EXACT)
	if((rc = one_mm_impl(c, dr, dq, stride, dl, n, dms, sc, (nofw ? 1 : 0) | (skip_exact ? 0 : MM_GATE_KEEP_EXACT),
	                     norc ? 1 : 0, dsw, cap, dh, dcnt, dops, dld, c->stream, false)))
		return rc;
	if(doffs) {
		{
			ProfScope ps(c, 3, c->stream);
			launch_range_offsets(c->fw, dsw, dh, dcnt, n, cap, off_cap, doffs, c->stream);
		}
		HIPCHK(hipGetLastError());
	}
	return t.finish();
}

int bt2g_extend(bt2g_ctx* c, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t nreads,
                const bt2g_ext_in* in, uint32_t n, bt2g_ext_out* out) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	HIPCHK(hipSetDevice(c->device));
	if(n == 0) return BT2G_OK;
	for(uint32_t i = 0; i < n; i++) {
		if(in[i].read >= nreads) return fail(BT2G_ERR_ARG, "range %u: read %u >= %u", i, in[i].read, nreads);
		const uint32_t L = lens[in[i].read];
		if(L > stride || in[i].off + in[i].len > L || in[i].botf <= in[i].topf || in[i].botb - in[i].topb != in[i].botf - in[i].topf)
			return fail(BT2G_ERR_ARG, "range %u: bad seed hit", i);
	}
	Tmp t(c);
	uint8_t* dr;
	uint32_t* dl;
	bt2g_ext_in* din;
	bt2g_ext_out* dout;
	int rc;
	if((rc = t.up(&dr, reads, (size_t)nreads * stride)) || (rc = t.up(&dl, lens, nreads)) || (rc = t.up(&din, in, n)) ||
	   (rc = t.out(&dout, out, n)) || (rc = t.send()))
		return rc;
	if((rc = bt2g_extend_dev(c, dr, stride, dl, din, n, dout, c->stream))) return rc;
	return t.finish();
}

int bt2g_get_offset(bt2g_ctx* c, const uint32_t* rows, uint32_t n, uint32_t* offs, uint32_t* loads) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	HIPCHK(hipSetDevice(c->device));
	Tmp t(c);
	uint32_t *drow, *doff, *dld = nullptr;
	int rc;
	if((rc = t.up(&drow, rows, n)) || (rc = t.out(&doff, offs, n))) return rc;
	if(loads && (rc = t.out(&dld, loads, n))) return rc;
	if((rc = t.send())) return rc;
	if((rc = bt2g_get_offset_dev(c, drow, n, doff, dld, c->stream))) return rc;
	return t.finish();
}

int bt2g_sw_align(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride, const uint32_t* lens,
                  const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* windows, uint64_t windows_len,
                  const bt2g_scoring* sc, int enable8, uint32_t cap, bt2g_sw_result* res, bt2g_sw_cand* cands,
                  int16_t* mat, const uint64_t* mat_off) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	HIPCHK(hipSetDevice(c->device));
	if(nprob == 0) return BT2G_OK;
	uint32_t nreads = 0;
	for(uint32_t i = 0; i < nprob; i++) nreads = probs[i].read + 1 > nreads ? probs[i].read + 1 : nreads;
	Tmp t(c);
	uint8_t *dr, *dq, *dw = nullptr;
	uint32_t* dl;
	bt2g_sw_problem* dp;
	bt2g_sw_result* dres;
	bt2g_sw_cand* dc;
	int16_t* dm = nullptr;
	uint64_t* dmo = nullptr;
	int rc;
	if((rc = t.up(&dr, reads, (size_t)nreads * stride)) || (rc = t.up(&dq, quals, (size_t)nreads * stride)) ||
	   (rc = t.up(&dl, lens, nreads)) || (rc = t.up(&dp, probs, nprob)) ||
	   (rc = t.up(&dres, (const bt2g_sw_result*)nullptr, nprob)) ||
	   (rc = t.up(&dc, (const bt2g_sw_cand*)nullptr, (size_t)nprob * cap)))
		return rc;
	if(windows && windows_len && (rc = t.up(&dw, windows, windows_len))) return rc;
	if(mat && (rc = t.up(&dmo, mat_off, nprob))) return rc;
	size_t matn = 0;
	if(mat) {
		for(uint32_t i = 0; i < nprob; i++) {
			size_t e = mat_off[i] + (size_t)lens[probs[i].read] * probs[i].ncol * 3;
			matn = e > matn ? e : matn;
		}
		if((rc = t.up(&dm, (const int16_t*)nullptr, matn))) return rc;
	}
	if((rc = t.send())) return rc;
	if((rc = bt2g_sw_align_dev(c, dr, dq, stride, dl, dp, nprob, dw, sc, enable8, cap, dres, dc, dm, dmo, c->stream)))
		return rc;
	if((rc = t.down(res, dres, nprob)) || (rc = t.down(cands, dc, (size_t)nprob * cap))) return rc;
	if(mat && (rc = t.down(mat, dm, matn))) return rc;
	if((rc = t.finish())) return rc;
	for(uint32_t i = 0; i < nprob; i++)
		if(res[i].ncand > (int32_t)cap) return fail(BT2G_ERR_OVERFLOW, "problem %u: %d candidates > cap %u", i,
		                                             res[i].ncand, cap);
	return BT2G_OK;
}

}  // extern "C"

extern "C" {

int bt2g_sw_align_bt(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                     const uint32_t* lens, const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* windows,
                     uint64_t windows_len, const bt2g_sw_rect* rects, const bt2g_scoring* sc, int enable8,
                     uint32_t cap, bt2g_sw_result* res, bt2g_sw_cand* cands, uint32_t maxaln, uint32_t maxedit,
                     int32_t* naln, bt2g_sw_aln* alns, bt2g_edit* edits, int8_t* fates) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	HIPCHK(hipSetDevice(c->device));
	if(nprob == 0) return BT2G_OK;
	uint32_t nreads = 0;
	for(uint32_t i = 0; i < nprob; i++) nreads = probs[i].read + 1 > nreads ? probs[i].read + 1 : nreads;
	Tmp t(c);
	uint8_t *dr, *dq, *dw = nullptr;
	uint32_t* dl;
	bt2g_sw_problem* dp;
	bt2g_sw_rect* drc = nullptr;
	bt2g_sw_result* dres;
	bt2g_sw_cand* dc;
	int32_t* dna;
	bt2g_sw_aln* dal;
	bt2g_edit* ded;
	int8_t* dft = nullptr;
	int rc;
	const size_t na = (size_t)nprob * maxaln;
	if((rc = t.up(&dr, reads, (size_t)nreads * stride)) || (rc = t.up(&dq, quals, (size_t)nreads * stride)) ||
	   (rc = t.up(&dl, lens, nreads)) || (rc = t.up(&dp, probs, nprob)) ||
	   (rc = t.up(&dres, (const bt2g_sw_result*)nullptr, nprob)) ||
	   (rc = t.up(&dc, (const bt2g_sw_cand*)nullptr, (size_t)nprob * cap)) ||
	   (rc = t.up(&dna, (const int32_t*)nullptr, nprob)) || (rc = t.up(&dal, (const bt2g_sw_aln*)nullptr, na)) ||
	   (rc = t.up(&ded, (const bt2g_edit*)nullptr, na * maxedit)))
		return rc;
	if(windows && windows_len && (rc = t.up(&dw, windows, windows_len))) return rc;
	if(rects && (rc = t.up(&drc, rects, nprob))) return rc;
	if(fates && (rc = t.up(&dft, (const int8_t*)nullptr, (size_t)nprob * cap))) return rc;
	if((rc = t.send())) return rc;
	const SwHint hint = sw_hint(probs, nprob, lens, enable8);
	if((rc = sw_align_bt_impl(c, dr, dq, stride, dl, dp, nprob, dw, drc, sc, enable8, cap, dres, dc, maxaln, maxedit,
	                          dna, dal, ded, dft, c->stream, &hint)))
		return rc;
	if((rc = t.down(res, dres, nprob)) || (rc = t.down(cands, dc, (size_t)nprob * cap)) ||
	   (rc = t.down(naln, dna, nprob)) || (rc = t.down(alns, dal, na)) || (rc = t.down(edits, ded, na * maxedit)))
		return rc;
	if(fates && (rc = t.down(fates, dft, (size_t)nprob * cap))) return rc;
	if((rc = t.finish())) return rc;
	for(uint32_t i = 0; i < nprob; i++)
		if(res[i].ncand > (int32_t)cap) return fail(BT2G_ERR_OVERFLOW, "problem %u: %d candidates > cap %u", i,
		                                             res[i].ncand, cap);
	return BT2G_OK;
}

int bt2g_sw_align_bt_packed(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                            const uint32_t* lens, const bt2g_sw_problem* probs, uint32_t nprob,
                            const uint8_t* windows, uint64_t windows_len, const bt2g_sw_rect* rects,
                            const bt2g_scoring* sc, int enable8, uint32_t cap, bt2g_sw_result* res, uint32_t maxaln,
                            uint32_t maxedit, int32_t* naln, bt2g_sw_aln* alns, bt2g_sw_cand* cands, int8_t* fates,
                            bt2g_edit* edits, uint64_t* totals) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	if(!totals) return fail(BT2G_ERR_ARG, "null totals");
	HIPCHK(hipSetDevice(c->device));
	totals[0] = totals[1] = totals[2] = 0;
	if(nprob == 0) return BT2G_OK;
	// (profiling: host phases as ids 8 staging, 9 enqueueing, 10 waiting + copying out)
	auto hnow = [] { return std::chrono::steady_clock::now(); };
	auto hadd = [c](int k, std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
		c->launches[k]++;
		c->total_ms[k] += std::chrono::duration<double, std::milli>(b - a).count();
	};
	const auto h0 = hnow();
	uint32_t nreads = 0;
	for(uint32_t i = 0; i < nprob; i++) nreads = probs[i].read + 1 > nreads ? probs[i].read + 1 : nreads;
	Tmp t(c);
	uint8_t *dr, *dq, *dw = nullptr;
	uint32_t *dl, *dcnt, *doff;
	bt2g_sw_problem* dp;
	bt2g_sw_rect* drc = nullptr;
	bt2g_sw_result* dres;
	bt2g_sw_cand *dc, *dpc;
	int32_t* dna;
	bt2g_sw_aln* dal;
	bt2g_edit *ded, *dpe;
	int8_t *dft = nullptr, *dpf = nullptr;
	int rc;
	const size_t na = (size_t)nprob * maxaln;
	uint32_t tot[3];
	if((rc = t.up(&dr, reads, (size_t)nreads * stride)) || (rc = t.up(&dq, quals, (size_t)nreads * stride)) ||
	   (rc = t.up(&dl, lens, nreads)) || (rc = t.up(&dp, probs, nprob)))
		return rc;
	if(windows && windows_len && (rc = t.up(&dw, windows, windows_len))) return rc;
	if(rects && (rc = t.up(&drc, rects, nprob))) return rc;
	if((rc = t.out(&dres, res, nprob)) || (rc = t.out(&dna, naln, nprob)) || (rc = t.out(&dal, alns, na)) ||
	   (rc = t.up(&dc, (const bt2g_sw_cand*)nullptr, (size_t)nprob * cap)) ||
	   (rc = t.up(&ded, (const bt2g_edit*)nullptr, na * maxedit)) ||
	   (rc = t.up(&dcnt, (const uint32_t*)nullptr, 3 * (size_t)nprob)) ||
	   (rc = t.up(&doff, (const uint32_t*)nullptr, 3 * (size_t)nprob + 3)))
		return rc;
	if(fates && (rc = t.up(&dft, (const int8_t*)nullptr, (size_t)nprob * cap))) return rc;
	// the packed outputs go straight to pinned host memory when it has room (one
	// synchronisation per call); else to the device, copied back once the
	// totals are known (two)
	bt2g_sw_cand* hpc = nullptr;
	int8_t* hpf = nullptr;
	bt2g_edit* hpe = nullptr;
	dpc = t.mapped((size_t)nprob * cap, &hpc);
	dpe = dpc ? t.mapped(na * maxedit, &hpe) : nullptr;
	dpf = dpe && fates ? t.mapped((size_t)nprob * cap, &hpf) : nullptr;
	const bool direct = dpc && dpe && (dpf || !fates);
	if(!direct) {
		if((rc = t.up(&dpc, (const bt2g_sw_cand*)nullptr, (size_t)nprob * cap)) ||
		   (rc = t.up(&dpe, (const bt2g_edit*)nullptr, na * maxedit)) ||
		   (fates && (rc = t.up(&dpf, (const int8_t*)nullptr, (size_t)nprob * cap))))
			return rc;
	}
	const SwHint hint = sw_hint(probs, nprob, lens, enable8);
	const auto h1 = hnow();
	{
		// (kernel-stats id 7: the call's whole span on the stream, copies included)
		ProfScope ps(c, 7, c->stream);
		if((rc = t.send())) return rc;
		if((rc = sw_align_bt_impl(c, dr, dq, stride, dl, dp, nprob, dw, drc, sc, enable8, cap, dres, dc, maxaln, maxedit,
		                          dna, dal, ded, dft, c->stream, &hint)))
			return rc;
		launch_sw_pack(dres, dna, dal, dc, dft, ded, nprob, cap, maxaln, maxedit, dcnt, doff, dpc, dpf, dpe, c->stream);
		HIPCHK(hipGetLastError());
		if((rc = t.down(tot, doff + 3 * (size_t)nprob, 3))) return rc;
	}
	const auto h2 = hnow();
	if((rc = t.finish())) return rc;
	if(direct) {
		memcpy(cands, hpc, sizeof(bt2g_sw_cand) * tot[0]);
		if(fates) memcpy(fates, hpf, tot[0]);
		memcpy(edits, hpe, sizeof(bt2g_edit) * tot[2]);
	} else {
		if((rc = t.down(cands, dpc, tot[0])) || (fates && (rc = t.down(fates, dpf, tot[0]))) ||
		   (rc = t.down(edits, dpe, tot[2])))
			return rc;
		if((rc = t.finish())) return rc;
	}
	totals[0] = tot[0];
	totals[1] = tot[1];
	totals[2] = tot[2];
	if(c->prof) {
		const auto h3 = hnow();
		hadd(8, h0, h1);
		hadd(9, h1, h2);
		hadd(10, h2, h3);
	}
	for(uint32_t i = 0; i < nprob; i++)
		if(res[i].ncand > (int32_t)cap) return fail(BT2G_ERR_OVERFLOW, "problem %u: %d candidates > cap %u", i,
		                                             res[i].ncand, cap);
	return BT2G_OK;
}

}  // extern "C"

extern "C" {

int bt2g_frame(bt2g_ctx* c, const bt2g_frame_in* in, uint32_t n, const uint32_t* lens, uint32_t nreads,
               const bt2g_scoring* sc, const bt2g_pe_policy* pe, int32_t maxhalf, int trim_to_ref,
               bt2g_sw_problem* probs, bt2g_sw_rect* rects, int32_t* ok) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	HIPCHK(hipSetDevice(c->device));
	if(n == 0) return BT2G_OK;
	for(uint32_t i = 0; i < n; i++) {
		if(in[i].read >= nreads) return fail(BT2G_ERR_ARG, "input %u: read %u >= %u", i, in[i].read, nreads);
		if(in[i].refidx >= c->nref) return fail(BT2G_ERR_ARG, "input %u: reference %u >= %u", i, in[i].refidx, c->nref);
		if(in[i].kind == 1 && !pe) return fail(BT2G_ERR_ARG, "input %u: mate search without a PE policy", i);
	}
	Tmp t(c);
	bt2g_frame_in* din;
	uint32_t* dl;
	bt2g_sw_problem* dp;
	bt2g_sw_rect* dr;
	int32_t* dok;
	int rc;
	if((rc = t.up(&din, in, n)) || (rc = t.up(&dl, lens, nreads)) || (rc = t.out(&dp, probs, n)) ||
	   (rc = t.out(&dr, rects, n)) || (rc = t.out(&dok, ok, n)) || (rc = t.send()))
		return rc;
	if((rc = bt2g_frame_dev(c, din, n, dl, sc, pe, maxhalf, trim_to_ref, dp, dr, dok, c->stream))) return rc;
	return t.finish();
}

int bt2g_ungapped(bt2g_ctx* c, const uint8_t* reads, const uint8_t* quals, uint32_t stride, const uint32_t* lens,
                  const bt2g_ug_problem* probs, uint32_t n, const bt2g_scoring* sc, int ohang, uint32_t maxedit,
                  bt2g_ug_result* res, bt2g_edit* edits) {
	if(!c) return fail(BT2G_ERR_ARG, "null ctx");
	HIPCHK(hipSetDevice(c->device));
	if(n == 0) return BT2G_OK;
	uint32_t nreads = 0;
	for(uint32_t i = 0; i < n; i++) nreads = probs[i].read + 1 > nreads ? probs[i].read + 1 : nreads;
	Tmp t(c);
	uint8_t *dr, *dq;
	uint32_t* dl;
	bt2g_ug_problem* dp;
	bt2g_ug_result* dres;
	bt2g_edit* ded;
	int rc;
	if((rc = t.up(&dr, reads, (size_t)nreads * stride)) || (rc = t.up(&dq, quals, (size_t)nreads * stride)) ||
	   (rc = t.up(&dl, lens, nreads)) || (rc = t.up(&dp, probs, n)) || (rc = t.out(&dres, res, n)) ||
	   (rc = t.out(&ded, edits, (size_t)n * maxedit)) || (rc = t.send()))
		return rc;
	if((rc = bt2g_ungapped_dev(c, dr, dq, stride, dl, dp, n, sc, ohang, maxedit, dres, ded, c->stream))) return rc;
	return t.finish();
}

}  // extern "C"

// ------------------------------------------------------------- multi-GPU
// RCCL entry points, resolved from librccl.so.1 on first use (no link-time
// dependency for the single-GPU path).  Signatures as rccl.h declares them.
namespace {
struct Rccl {
	bool ok = false;
	int (*get_unique_id)(void* id) = nullptr;
	void* init_rank = nullptr;
	int (*all_reduce)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;
	int (*destroy)(void*) = nullptr;
	const char* (*err)(int) = nullptr;
};
struct Id128 { char b[BT2G_COMM_ID_BYTES]; };
const int NCCL_UINT64 = 5, NCCL_SUM = 0;     // ncclUint64, ncclSum (rccl.h)

Rccl& rccl() {
	static Rccl r = [] {
		Rccl x;
		void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
		if(!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
		if(!h) return x;
		x.get_unique_id = (int (*)(void*))dlsym(h, "ncclGetUniqueId");
		x.init_rank = dlsym(h, "ncclCommInitRank");
		x.all_reduce = (int (*)(const void*, void*, size_t, int, int, void*, hipStream_t))dlsym(h, "ncclAllReduce");
		x.destroy = (int (*)(void*))dlsym(h, "ncclCommDestroy");
		x.err = (const char* (*)(int))dlsym(h, "ncclGetErrorString");
		x.ok = x.get_unique_id && x.init_rank && x.all_reduce && x.destroy && x.err;
		return x;
	}();
	return r;
}
}  // namespace

static int rccl_destroy(void* comm) {
	Rccl& r = rccl();
	return r.ok ? r.destroy(comm) : 0;
}

extern "C" {

int bt2g_comm_unique_id(uint8_t* id) {
	if(!id) return fail(BT2G_ERR_ARG, "null id");
	Rccl& r = rccl();
	if(!r.ok) return fail(BT2G_ERR_HIP, "RCCL (librccl.so.1) not available");
	if(int e = r.get_unique_id(id)) return fail(BT2G_ERR_HIP, "ncclGetUniqueId: %s", r.err(e));
	return BT2G_OK;
}

int bt2g_comm_init(bt2g_ctx* c, int nranks, int rank, const uint8_t* id) {
	if(!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(BT2G_ERR_ARG, "bad communicator arguments");
	Rccl& r = rccl();
	if(!r.ok) return fail(BT2G_ERR_HIP, "RCCL (librccl.so.1) not available");
	if(c->comm) return fail(BT2G_ERR_ARG, "context already has a communicator");
	HIPCHK(hipSetDevice(c->device));
	Id128 uid;
	memcpy(uid.b, id, BT2G_COMM_ID_BYTES);
	auto init = (int (*)(void**, int, Id128, int))r.init_rank;
	if(int e = init(&c->comm, nranks, uid, rank)) {
		c->comm = nullptr;
		return fail(BT2G_ERR_HIP, "ncclCommInitRank: %s", r.err(e));
	}
	return BT2G_OK;
}

int bt2g_allreduce_counts(bt2g_ctx* c, uint64_t* counts, uint32_t k) {
	if(!c || (!counts && k)) return fail(BT2G_ERR_ARG, "null argument");
	if(!c->comm) return fail(BT2G_ERR_ARG, "no communicator (bt2g_comm_init)");
	if(k == 0) return BT2G_OK;
	HIPCHK(hipSetDevice(c->device));
	Rccl& r = rccl();
	uint64_t* d = nullptr;
	HIPCHK(hipMalloc((void**)&d, sizeof(uint64_t) * k));
	int rc = BT2G_OK;
	if(hipMemcpyAsync(d, counts, sizeof(uint64_t) * k, hipMemcpyHostToDevice, c->stream) != hipSuccess) {
		rc = fail(BT2G_ERR_HIP, "hipMemcpyAsync H2D");
	} else if(int e = r.all_reduce(d, d, k, NCCL_UINT64, NCCL_SUM, c->comm, c->stream)) {
		rc = fail(BT2G_ERR_HIP, "ncclAllReduce: %s", r.err(e));
	} else if(hipMemcpyAsync(counts, d, sizeof(uint64_t) * k, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
	          stream_wait(c, c->stream) != hipSuccess) {
		rc = fail(BT2G_ERR_HIP, "all-reduce result copy");
	}
	(void)hipFree(d);
	return rc;
}

}  // extern "C"
