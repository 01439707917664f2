// integration/bt2g_fibers.cpp -- the reference's search workers as user-mode
// fibers: the drop-in's batch-first schedule.
//
// The reference runs one OS thread per search worker (`-p N` workers spawned
// by multiseedSearch, bt2_search.cpp:4913-4925), each aligning one read at a
// time (multiseedSearchWorker, bt2_search.cpp:3050-4197).  With the engines
// under it, every seam call (exactSweep, oneMmSearch, searchAllSeeds,
// ungappedAlign, SwAligner::align) becomes a batched GPU call, so the worker
// waits at each seam; as OS threads that is a futex sleep and a wake with cold
// caches per seam call -- ~0.7 ms of host CPU per read in round 2, 4x the
// stock server's whole alignment.
//
// Here every worker the reference spawns becomes a fiber: its own stack, run
// by one of a few carrier threads (one per core).  A seam call queues its
// request in the carrier's outbox and switches back to the carrier, which runs
// the next runnable fiber; once every runnable fiber has had its turn the
// outbox goes to the seam dispatchers in one hand-off, and fibers whose
// requests completed come back through the carrier's inbox.  The reference's
// per-read control flow is untouched (each worker still runs its own reads in
// program order, with its own RNG, SeedResults, SwDriver and AlnSinkWrap), so
// the SAM is the reference's; what changes is that thousands of reads are in
// flight on a handful of OS threads and a seam round trip costs a user-mode
// context switch instead of a sleep/wake pair.
//
// Interception (integration/Makefile, -Wl,--wrap):
//   std::thread::_M_start_thread  the worker spawn (the reference's
//                                 std::thread(multiseedSearchWorker, tps) at
//                                 bt2_search.cpp:4921): a thread whose state
//                                 is a void(*)(void*) call becomes a fiber;
//                                 every other thread (listener, connection
//                                 threads, pat.h:2104,2163) is created as usual
//   std::thread::detach           of a fiber's handle: nothing to detach
//   nanosleep                     the SLEEP(10) after each spawn
//                                 (bt2_search.cpp:4924): skipped for fibers
//   std::condition_variable::wait a fiber waiting for reads
//   + notify_one / notify_all     (LockedQueueCV::pop, pat.h:1996-2002) must
//                                 not block its carrier: it registers on the
//                                 condition variable, releases the lock and
//                                 yields; a notify on that variable hands it
//                                 back to its carrier, and it returns (the
//                                 caller's predicate loop re-checks, as after
//                                 any wake-up)
//
// $BT2G_FIBERS=0 keeps OS threads; $BT2G_CARRIERS sets the carrier count
// (default: the CPUs this process may use); $BT2G_FIBER_STACK the stack size
// in KiB (default 256; the worker's frame is 21 KiB, -fstack-usage).
#include "bt2g_fibers.h"

#include <errno.h>
#include <malloc.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <typeinfo>
#include <unordered_map>
#include <vector>

// ---- context switch (x86-64 System V) -----------------------------------------
// bt2gf_switch(save, to): push the callee-saved registers, the MXCSR and the
// x87 control word, store the stack pointer at *save, load `to` and pop the
// same frame from it.  A new fiber's stack is laid out as such a frame whose
// return address is bt2gf_entry, which calls r13(r12).
extern "C" void bt2gf_switch(void** save, void* to);
extern "C" void bt2gf_entry();
asm(R"(
	.text
	.globl bt2gf_switch
	.type bt2gf_switch,@function
bt2gf_switch:
	pushq %rbp
	pushq %rbx
	pushq %r12
	pushq %r13
	pushq %r14
	pushq %r15
	subq $8, %rsp
	stmxcsr (%rsp)
	fnstcw 4(%rsp)
	movq %rsp, (%rdi)
	movq %rsi, %rsp
	ldmxcsr (%rsp)
	fldcw 4(%rsp)
	addq $8, %rsp
	popq %r15
	popq %r14
	popq %r13
	popq %r12
	popq %rbx
	popq %rbp
	ret
	.size bt2gf_switch,.-bt2gf_switch

	.globl bt2gf_entry
	.type bt2gf_entry,@function
bt2gf_entry:
	movq %r12, %rdi
	callq *%r13
	ud2
	.size bt2gf_entry,.-bt2gf_entry
)");

namespace bt2gf {
namespace {

// READY: runnable; BLOCKED: its request is with the dispatchers, or it waits on a
// condition variable -- wake_many brings it back either way; PARKED: a timed
// sleep, polled by its carrier; DONE: the work returned
enum State { READY, BLOCKED, PARKED, DONE };

struct Carrier;

struct Fiber {
	void* sp = nullptr;              // saved stack pointer while suspended
	void* stack = nullptr;
	size_t stack_bytes = 0;
	std::thread::_State* work = nullptr;
	Carrier* home = nullptr;
	State state = READY;
	uint64_t wake_at_ns = 0;          // PARKED by nanosleep: not before this time
	const void* cv = nullptr;         // the condition variable it waits on
	void* user = nullptr;             // bt2gf::local()
	// on a carrier's inbox (set by wake_many, cleared when the carrier takes it):
	// a second wake-up before that is a scheduler bug -- checked, it would run the
	// fiber twice
	std::atomic<bool> queued{false};
};

uint64_t now_ns() {
	timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

const bool g_dbg = getenv("BT2G_FIBER_DEBUG") != nullptr;
#define FDBG(...) do { if(g_dbg) fprintf(stderr, __VA_ARGS__); } while(0)

FlushFn g_flush = nullptr;
InitFn g_init = nullptr;

struct Carrier {
	std::thread th;
	void* sched_sp = nullptr;        // the scheduler's context while a fiber runs
	Fiber* cur = nullptr;
	std::vector<Fiber*> ready, round, parked;
	std::vector<void*> outbox;
	// fibers handed to this carrier: new ones and those whose requests completed
	std::mutex mu;
	std::condition_variable cv;
	std::vector<Fiber*> inbox;
	bool sleeping = false;

	void run();
	void flush() {
		if(outbox.empty()) return;
		FDBG("carrier %p: flush %zu\n", (void*)this, outbox.size());
		g_flush(outbox.data(), outbox.size());
		outbox.clear();
	}
};

}  // namespace
}  // namespace bt2gf
extern "C" int __real_pthread_mutex_lock(pthread_mutex_t* m);
namespace bt2gf {
namespace {

// The scheduler's own mutexes (a carrier's inbox lock, the condition-variable
// tables, the carrier list) are taken with the real pthread_mutex_lock: never
// through the fiber-yielding wrapper below.  A fiber that yielded while in the
// middle of scheduler code would let another fiber of its carrier run the same
// code on the same thread-local state (r03w: a fiber suspended at a contended
// carrier lock inside wake_many, another fiber's wake_many reallocated the
// thread-local grouping vector, the first resumed on a dangling reference and
// the server died -- "once in ~6 runs" with the unlock-time baton, which called
// wake_many from fibers at every unlock; the lock-time baton had the same
// window, less often).
struct RealGuard {
	pthread_mutex_t* m;
	explicit RealGuard(std::mutex& mu) : m(mu.native_handle()) { __real_pthread_mutex_lock(m); }
	~RealGuard() { pthread_mutex_unlock(m); }
	RealGuard(const RealGuard&) = delete;
	RealGuard& operator=(const RealGuard&) = delete;
};

// BT2GF_R03W (test builds only, tests/test_fibers.py): the round-3 scheduler
// -- the scheduler's mutexes through the yielding wrapper and wake_many's
// grouping list thread-local -- so that the stress test can show the race.
#ifdef BT2GF_R03W
typedef std::lock_guard<std::mutex> SchedGuard;
#else
typedef RealGuard SchedGuard;
#endif

thread_local Carrier* t_carrier = nullptr;   // set on carrier threads only
thread_local int t_skip_sleep = 0;            // spawns whose SLEEP(10) is skipped

std::mutex g_mu;                              // carriers, fiber handles
// fibers waiting on each condition variable (woken by its notify_one/_all)
std::mutex g_cv_mu;
std::unordered_map<const void*, std::vector<Fiber*>> g_cv_waiters;
// fibers a notify_all released but did not wake yet: each woken fiber wakes
// the next once it holds the lock again (the "baton"), so they re-take the
// mutex one after another instead of all at once -- every one still returns
// from its wait, as notify_all requires.  (The reference's ready queue of
// reads notifies all its waiters per pushed element, pat.h:1981-1985: with
// thousands of idle workers that herd was 4.2M contended lock attempts per
// 400k reads at --reads-per-batch 1, r03r.)
std::unordered_map<const void*, std::deque<Fiber*>> g_cv_baton;
std::vector<Carrier*> g_carriers;
size_t g_next_carrier = 0;
// fibers' std::thread ids: tagged in the top 16 bits (a pthread_t is a user-space
// address, below 2^47)
const uintptr_t FIBER_HANDLE_TAG = 0xF1BE;
uintptr_t g_next_handle = 0;

size_t stack_bytes() {
	static const size_t sz = [] {
		const char* e = getenv("BT2G_FIBER_STACK");
		size_t kb = e ? (size_t)atol(e) : 256;
		if(kb < 64) kb = 64;
		return kb << 10;
	}();
	return sz;
}

// CPUs this process may use: the affinity mask, capped by a cgroup v2 CPU
// quota (the GPU box gives a 16-CPU quota over a 256-CPU affinity mask)
size_t usable_cpus() {
	size_t n = 0;
	cpu_set_t set;
	if(sched_getaffinity(0, sizeof(set), &set) == 0) n = (size_t)CPU_COUNT(&set);
	if(n == 0) {
		long m = sysconf(_SC_NPROCESSORS_ONLN);
		n = m > 0 ? (size_t)m : 1;
	}
	if(FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
		char q[64] = {0};
		unsigned long period = 0;
		if(fscanf(f, "%63s %lu", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
			const size_t cap = (size_t)((strtoul(q, nullptr, 10) + period - 1) / period);
			if(cap > 0 && cap < n) n = cap;
		}
		fclose(f);
	}
	return n;
}

// a carrier's outbox goes to the dispatchers when it holds $BT2G_FLUSH_N
// requests or its oldest waited $BT2G_FLUSH_US (defaults 64, 100 us)
size_t flush_n() {
	static const size_t n = [] {
		const char* e = getenv("BT2G_FLUSH_N");
		return e && atol(e) > 0 ? (size_t)atol(e) : (size_t)64;
	}();
	return n;
}
uint64_t flush_ns() {
	static const uint64_t ns = [] {
		const char* e = getenv("BT2G_FLUSH_US");
		return (e && atol(e) > 0 ? (uint64_t)atol(e) : (uint64_t)100) * 1000ull;
	}();
	return ns;
}

size_t n_carriers() {
	const char* e = getenv("BT2G_CARRIERS");
	if(e && atoi(e) > 0) return (size_t)atoi(e);
	return usable_cpus();
}

[[noreturn]] void fiber_main(Fiber* f);

void switch_to(Carrier* c, Fiber* f) {
	c->cur = f;
	f->state = READY;
	bt2gf_switch(&c->sched_sp, f->sp);
	c->cur = nullptr;
}

// Back to the carrier's scheduler, leaving the fiber in state `st`.
void suspend(Fiber* f, State st) {
	f->state = st;
	bt2gf_switch(&f->sp, f->home->sched_sp);
}

void fiber_main(Fiber* f) {
	f->work->_M_run();
	delete f->work;
	f->work = nullptr;
	suspend(f, DONE);
	abort();   // a finished fiber is never resumed
}

}  // namespace
}  // namespace bt2gf
extern "C" void bt2g_prof_thread(int role);
namespace bt2gf {
namespace {

void Carrier::run() {
	t_carrier = this;
	bt2g_prof_thread(1);
	char nm[16];
	snprintf(nm, sizeof(nm), "bt2g-carrier");
	pthread_setname_np(pthread_self(), nm);
	uint64_t last_poll = 0;
	for(;;) {
		{
			RealGuard lk(mu);
			if(!inbox.empty()) {
				for(Fiber* f : inbox) f->queued.store(false, std::memory_order_relaxed);
				ready.insert(ready.end(), inbox.begin(), inbox.end());
				inbox.clear();
			}
		}
		if(!parked.empty()) {
			// timed sleeps: re-run them when due (checked when nothing else is
			// runnable, and at least every 100 us)
			const uint64_t t = now_ns();
			if(ready.empty() || t - last_poll > 100000) {
				last_poll = t;
				size_t k = 0;
				for(Fiber* f : parked) {
					if(f->wake_at_ns && f->wake_at_ns > t) parked[k++] = f;
					else ready.push_back(f);
				}
				parked.resize(k);
			}
		}
		if(ready.empty()) {
			flush();
			std::unique_lock<std::mutex> lk(mu);
			sleeping = true;
			if(parked.empty()) cv.wait(lk, [this] { return !inbox.empty(); });
			else cv.wait_for(lk, std::chrono::microseconds(100), [this] { return !inbox.empty(); });
			sleeping = false;
			continue;
		}
		round.swap(ready);
		uint64_t t_flush = now_ns();
		for(Fiber* f : round) {
			FDBG("carrier %p: run fiber %p\n", (void*)this, (void*)f);
			// requests leave during the round, not only at its end: a long round
			// (hundreds of fibers) would otherwise hold the first ones' requests
			// back for its whole length
			if(!outbox.empty()) {
				const uint64_t t = now_ns();
				if(outbox.size() >= flush_n() || t - t_flush >= flush_ns()) {
					flush();
					t_flush = t;
				}
			}
			switch_to(this, f);
			FDBG("carrier %p: fiber %p -> state %d\n", (void*)this, (void*)f, (int)f->state);
			switch(f->state) {
			case READY: ready.push_back(f); break;
			case PARKED: parked.push_back(f); break;
			case BLOCKED: break;        // its request is in the outbox; wake_many brings it back
			case DONE:
				munmap(f->stack, f->stack_bytes);
				delete f;
				break;
			}
		}
		round.clear();
		flush();
	}
}

Carrier* pick_carrier() {
	// under g_mu
	if(g_carriers.empty()) {
		const size_t n = n_carriers();
		for(size_t i = 0; i < n; i++) g_carriers.push_back(new Carrier());
		for(Carrier* c : g_carriers) c->th = std::thread(&Carrier::run, c);
		for(Carrier* c : g_carriers) c->th.detach();
	}
	Carrier* c = g_carriers[g_next_carrier % g_carriers.size()];
	g_next_carrier++;
	return c;
}

Fiber* make_fiber(std::thread::_State* work) {
	Fiber* f = new Fiber();
	f->work = work;
	const size_t page = (size_t)sysconf(_SC_PAGESIZE);
	f->stack_bytes = stack_bytes() + page;
	void* mem = mmap(nullptr, f->stack_bytes, PROT_READ | PROT_WRITE,
	                 MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE | MAP_STACK, -1, 0);
	if(mem == MAP_FAILED) {
		fprintf(stderr, "bt2g fibers: cannot map a %zu-byte stack: %s\n", f->stack_bytes, strerror(errno));
		abort();
	}
	mprotect(mem, page, PROT_NONE);   // guard page: an overflow faults instead of corrupting
	f->stack = mem;
	// initial frame popped by bt2gf_switch: [mxcsr|fpucw][r15][r14][r13][r12][rbx][rbp][ret];
	// after its ret rsp == top (16-aligned), as before a call: bt2gf_entry's call is aligned
	uintptr_t top = ((uintptr_t)mem + f->stack_bytes) & ~(uintptr_t)15;
	uint64_t* sp = (uint64_t*)top;
	*--sp = (uint64_t)(uintptr_t)&bt2gf_entry;   // ret
	*--sp = 0;                                   // rbp
	*--sp = 0;                                   // rbx
	*--sp = (uint64_t)(uintptr_t)f;              // r12: argument
	*--sp = (uint64_t)(uintptr_t)&fiber_main;    // r13: function
	*--sp = 0;                                   // r14
	*--sp = 0;                                   // r15
	uint32_t csr[2] = {0x1f80u, 0x037fu};        // default MXCSR, x87 control word
	__asm__ volatile("stmxcsr %0" : "=m"(csr[0]));
	__asm__ volatile("fnstcw %0" : "=m"(csr[1]));
	--sp;
	memcpy(sp, csr, 8);
	f->sp = sp;
	return f;
}

Fiber* cur_fiber() { return t_carrier ? t_carrier->cur : nullptr; }

// Allocator settings for thousands of workers on a few threads: no heap
// trimming and no mmap for blocks below 4 MB (the dispatchers' batch buffers
// and the workers' per-read lists otherwise cycle pages through mprotect /
// madvise and page faults).
struct MallocTuning {
	MallocTuning() {
		if(!enabled()) return;
		mallopt(M_MMAP_THRESHOLD, 4 << 20);   // (the workers' 20 MB cache pools: mmap, untouched)
		mallopt(M_TRIM_THRESHOLD, 1 << 30);
		mallopt(M_TOP_PAD, 16 << 20);
	}
} g_malloc_tuning;

}  // namespace

void* self() { return cur_fiber(); }

void** local() {
	Fiber* f = cur_fiber();
	return f ? &f->user : nullptr;
}

bool enabled() {
	static const bool on = [] {
		const char* e = getenv("BT2G_FIBERS");
		return !(e && e[0] == '0');
	}();
	return on;
}

size_t count() {
	RealGuard lk(g_mu);
	return (size_t)g_next_handle;
}

void set_flush(FlushFn fn) { g_flush = fn; }
void set_init(InitFn fn) { g_init = fn; }

void block_on(void* req) {
	Fiber* f = cur_fiber();
	f->home->outbox.push_back(req);
	suspend(f, BLOCKED);
}

void block_on_many(void* const* reqs, size_t n) {
	Fiber* f = cur_fiber();
	f->home->outbox.insert(f->home->outbox.end(), reqs, reqs + n);
	suspend(f, BLOCKED);
}

void wake_many(void* const* fibers, size_t n) {
	// grouped per carrier: one lock (and at most one wake-up) per carrier.  (On
	// the caller's stack: a thread-local list is shared by every fiber of the
	// carrier, see RealGuard.)
#ifdef BT2GF_R03W
	thread_local std::vector<std::pair<Carrier*, std::vector<Fiber*>>> groups;
#else
	std::vector<std::pair<Carrier*, std::vector<Fiber*>>> groups;
#endif
	for(size_t i = 0; i < n; i++) {
		Fiber* f = static_cast<Fiber*>(fibers[i]);
		if(f->queued.exchange(true, std::memory_order_relaxed)) {
			fprintf(stderr, "bt2g fibers: fiber %p woken twice\n", (void*)f);
			abort();
		}
		size_t g = 0;
		while(g < groups.size() && groups[g].first != f->home) g++;
		if(g == groups.size()) groups.emplace_back(f->home, std::vector<Fiber*>());
		groups[g].second.push_back(f);
	}
	for(auto& g : groups) {
		if(g.second.empty()) continue;
		Carrier* c = g.first;
		bool notify;
		{
			SchedGuard lk(c->mu);
			c->inbox.insert(c->inbox.end(), g.second.begin(), g.second.end());
			notify = c->sleeping;
		}
		if(notify) c->cv.notify_one();
#ifdef BT2GF_R03W
		g.second.clear();
#endif
	}
}

}  // namespace bt2gf

// ---- interception ---------------------------------------------------------------
using namespace bt2gf;

extern "C" {

void __real__ZNSt6thread15_M_start_threadESt10unique_ptrINS_6_StateESt14default_deleteIS1_EEPFvvE(
	std::thread* self, std::unique_ptr<std::thread::_State> st, void (*dep)());
void __real__ZNSt6thread6detachEv(std::thread* self);
void __real__ZNSt18condition_variable4waitERSt11unique_lockISt5mutexE(std::condition_variable* cv,
                                                                      std::unique_lock<std::mutex>& lk);
int __real_nanosleep(const struct timespec* req, struct timespec* rem);

// std::thread's constructor: the search workers (a void(*)(void*) and its
// argument: std::thread(multiseedSearchWorker, (void*)&tps[i])) become fibers.
void __wrap__ZNSt6thread15_M_start_threadESt10unique_ptrINS_6_StateESt14default_deleteIS1_EEPFvvE(
	std::thread* self, std::unique_ptr<std::thread::_State> st, void (*dep)()) {
	static const char* const WORKER = "NSt6thread11_State_implINS_8_InvokerISt5tupleIJPFvPvES3_EEEEEE";
	FDBG("start_thread: %s\n", st ? typeid(*st).name() : "null");
	if(!enabled() || !st || strcmp(typeid(*st).name(), WORKER) != 0) {
		__real__ZNSt6thread15_M_start_threadESt10unique_ptrINS_6_StateESt14default_deleteIS1_EEPFvvE(
			self, std::move(st), dep);
		return;
	}
	static std::once_flag once;
	std::call_once(once, [] {
		if(g_init) g_init();
		if(!g_flush) {
			fprintf(stderr, "bt2g fibers: no seam dispatcher registered\n");
			abort();
		}
	});
	Fiber* f = make_fiber(st.release());
	uintptr_t handle;
	Carrier* c;
	{
		RealGuard lk(g_mu);
		c = pick_carrier();
		f->home = c;
		handle = ((uintptr_t)FIBER_HANDLE_TAG << 48) | ++g_next_handle;
	}
	*reinterpret_cast<std::thread::native_handle_type*>(self) = (std::thread::native_handle_type)handle;
	t_skip_sleep++;
	void* one = f;
	wake_many(&one, 1);
}

void __wrap__ZNSt6thread6detachEv(std::thread* self) {
	const uintptr_t h = (uintptr_t) * reinterpret_cast<std::thread::native_handle_type*>(self);
	if((h >> 48) == FIBER_HANDLE_TAG) {      // a fiber's handle: nothing to detach
		*reinterpret_cast<std::thread::native_handle_type*>(self) = 0;
		return;
	}
	__real__ZNSt6thread6detachEv(self);
}

// a fiber woken from `cv` holds the lock again: the next fiber a notify_all released goes
static void pass_baton(const void* cv) {
	Fiber* w = nullptr;
	{
		SchedGuard g(g_cv_mu);
		auto it = g_cv_baton.find(cv);
		if(it == g_cv_baton.end() || it->second.empty()) return;
		w = it->second.front();
		it->second.pop_front();
	}
	void* one = w;
	wake_many(&one, 1);
}

void __wrap__ZNSt18condition_variable4waitERSt11unique_lockISt5mutexE(std::condition_variable* cv,
                                                                      std::unique_lock<std::mutex>& lk) {
	Fiber* f = cur_fiber();
	if(!f) {
		__real__ZNSt18condition_variable4waitERSt11unique_lockISt5mutexE(cv, lk);
		return;
	}
	// registered while the caller still holds the lock: a notifier that changes
	// the predicate's state under that lock cannot notify before we are on the list
	f->cv = cv;
	{
		SchedGuard g(g_cv_mu);
		g_cv_waiters[cv].push_back(f);
	}
	lk.unlock();
	suspend(f, BLOCKED);
	lk.lock();
	pass_baton(cv);
}

// notify: fibers waiting on `cv` go back to their carriers, then the OS threads
// (notify_all: the first now, the rest through the baton)
static void wake_cv_fibers(const void* cv, bool all) {
	Fiber* w = nullptr;
	{
		SchedGuard g(g_cv_mu);
		auto it = g_cv_waiters.find(cv);
		if(it == g_cv_waiters.end() || it->second.empty()) return;
		w = it->second.front();
		it->second.erase(it->second.begin());
		if(all && !it->second.empty()) {
			std::deque<Fiber*>& b = g_cv_baton[cv];
			b.insert(b.end(), it->second.begin(), it->second.end());
			it->second.clear();
		}
	}
	void* one = w;
	wake_many(&one, 1);
}

void __real__ZNSt18condition_variable10notify_allEv(std::condition_variable* cv);
void __real__ZNSt18condition_variable10notify_oneEv(std::condition_variable* cv);

void __wrap__ZNSt18condition_variable10notify_allEv(std::condition_variable* cv) {
	wake_cv_fibers(cv, true);
	__real__ZNSt18condition_variable10notify_allEv(cv);
}

void __wrap__ZNSt18condition_variable10notify_oneEv(std::condition_variable* cv) {
	wake_cv_fibers(cv, false);
	__real__ZNSt18condition_variable10notify_oneEv(cv);
}

// pthread_mutex_lock (std::mutex::lock of the reference's objects and the
// binding): a fiber must not block its carrier -- a contended lock would stop
// every other fiber of that carrier, and a condition-variable wake-up of many
// fibers (LockedQueueCV::push notifies all, pat.h:1981-1985) makes them all
// re-lock the queue's mutex at once.  A fiber tries the lock, spins briefly,
// then yields to its carrier and tries again on the carrier's next round.
int __real_pthread_mutex_lock(pthread_mutex_t* m);

int __wrap_pthread_mutex_lock(pthread_mutex_t* m) {
	Fiber* f = cur_fiber();
	if(!f) return __real_pthread_mutex_lock(m);
	for(int spin = 0;; spin++) {
		const int r = pthread_mutex_trylock(m);
		if(r != EBUSY) return r;
		if(spin == 0) bt2gf::mutex_prof_note(__builtin_return_address(0));
		if(spin < 4) {        // (64: trylock spinning 11 % of the carriers, r03p)
			__builtin_ia32_pause();
			continue;
		}
		suspend(f, READY);
	}
}

}  // extern "C"

// $BT2G_MUTEX_PROF: contended lock call sites (offsets into the executable, for
// addr2line) and how often a fiber found the lock taken there
extern "C" char __executable_start;
namespace bt2gf {
namespace {
struct MxSite {
	std::atomic<uintptr_t> pc{0};
	std::atomic<uint64_t> n{0};
};
MxSite g_mx[1024];
bool mx_on() {
	static const bool on = getenv("BT2G_MUTEX_PROF") != nullptr;
	return on;
}
}  // namespace
void mutex_prof_note(void* ra) {
	if(!mx_on()) return;
	const uintptr_t pc = (uintptr_t)ra;
	for(size_t i = (pc >> 4) % 1024, k = 0; k < 1024; k++, i = (i + 1) % 1024) {
		uintptr_t cur = g_mx[i].pc.load(std::memory_order_relaxed);
		if(cur == 0 && g_mx[i].pc.compare_exchange_strong(cur, pc)) cur = pc;
		if(cur == pc) {
			g_mx[i].n.fetch_add(1, std::memory_order_relaxed);
			return;
		}
	}
}
void mutex_prof_dump() {
	const char* path = getenv("BT2G_MUTEX_PROF");
	if(!path) return;
	FILE* f = fopen(path, "w");
	if(!f) return;
	for(MxSite& x : g_mx)
		if(x.pc.load()) fprintf(f, "0x%lx %llu\n", (unsigned long)(x.pc.load() - (uintptr_t)&__executable_start),
		                        (unsigned long long)x.n.load());
	fclose(f);
}
}  // namespace bt2gf

extern "C" {

int __wrap_nanosleep(const struct timespec* req, struct timespec* rem) {
	if(t_skip_sleep > 0) {          // the spawn loop's SLEEP(10) after a fiber was created
		t_skip_sleep--;
		return 0;
	}
	Fiber* f = cur_fiber();
	if(!f || !req) return __real_nanosleep(req, rem);
	f->wake_at_ns = now_ns() + (uint64_t)req->tv_sec * 1000000000ull + (uint64_t)req->tv_nsec;
	suspend(f, PARKED);
	f->wake_at_ns = 0;
	if(rem) rem->tv_sec = rem->tv_nsec = 0;
	return 0;
}

}  // extern "C"
