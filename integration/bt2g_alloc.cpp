// integration/bt2g_alloc.cpp -- the drop-in's operator new / delete: per-thread
// caches of freed blocks by size class.
//
// The reference allocates with new / new[] (EList, SStringExpandable, the
// per-connection read buffers PatternSourceServiceFactory::align creates and
// destroys, pat.cpp:2030-2075).  Under fibers the server holds thousands of
// workers on a few carrier threads, and the per-connection buffers are built
// on the connection's thread, grown on the carriers (PatternSourcePerThread::
// finalize) and freed on the connection's thread again.  glibc's arenas take
// that badly: frees into another thread's arena contend for its lock, and a
// heap that empties completely is unmapped (heap_trim ignores
// M_TRIM_THRESHOLD for that case) and re-created later one mprotect per
// allocation that does not fit -- r03k at 3.1 Gbp: mprotect 19 %, malloc
// internals 7 % of the carriers' CPU.
//
// Replacing the global operator new / delete (the standard's replaceable
// allocation functions: the executable's definitions serve every object and
// library of the process) with size-class caches removes both: a freed block
// goes to the freeing thread's cache, blocks beyond a cache's cap move to a
// shared depot in batches (one lock per batch), and a thread that finds its
// cache empty takes a batch from the depot before it asks malloc.  Memory is
// never returned to the system -- the server's working set is stable once the
// first connections have run.  Blocks up to 64 MiB are cached too (power-of-two
// classes): freed big blocks (the alignment caches' pools, grown ELists) had
// gone back to glibc, which trimmed the heap and grew it again one mprotect per
// allocation (r03p at 3.1 Gbp: mprotect 14 % of the carriers' CPU, all of it
// under this allocator's malloc calls).  Larger blocks go to malloc / free
// directly.  $BT2G_ALLOC=0 keeps glibc's allocator.
#include <dlfcn.h>
#include <errno.h>
#include <execinfo.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sched.h>
#include <sys/mman.h>
#include <malloc.h>

#include <atomic>
#include <new>
#include <string>

namespace {

const int NCLASS = 23;                  // 16 B .. 64 MiB
const size_t MAXSZ = (size_t)16 << (NCLASS - 1);
const size_t HDR = 16;                  // keeps the default new alignment (16)
const uint32_t MAGIC_CACHED = 0xB72C0DE5u, MAGIC_MALLOC = 0xB72C0DE6u;
const int BATCH = 32;                   // blocks moved to / from the depot at once

struct Hdr {
	uint32_t magic;
	uint32_t cls;
	uint64_t pad;
};
static_assert(sizeof(Hdr) == HDR, "header size");

struct Node {
	Node* next;
};

inline int cls_of(size_t n) {
	// the smallest c with 16 << c >= n
	return n <= 16 ? 0 : 60 - __builtin_clzll((unsigned long long)(n - 1));
}
inline size_t size_of(int c) { return (size_t)16 << c; }
// blocks a thread keeps per class before half go to the depot (~4 MiB per class
// up to 256 KiB blocks, at least 64 of them; ~16 MiB and at least 2 beyond)
inline int cap_of(int c) {
	if(size_of(c) > ((size_t)256 << 10)) {
		const size_t v = ((size_t)16 << 20) / size_of(c);
		return v < 2 ? 2 : (int)v;
	}
	const size_t v = ((size_t)4 << 20) / size_of(c);
	return v < 64 ? 64 : (v > 4096 ? 4096 : (int)v);
}

bool enabled() {
	static const bool on = [] {
		const char* e = getenv("BT2G_ALLOC");
		return !(e && e[0] == '0');
	}();
	return on;
}

// a spin lock: held for a few list operations, and never yields (the drop-in
// wraps pthread_mutex_lock to yield a fiber; an allocation must not)
struct Spin {
	std::atomic_flag f = ATOMIC_FLAG_INIT;
	void lock() {
		// (yields after a while: with more threads than cores the holder may be
		// descheduled -- r04f: 16 drivers + 7 engine services on a 16-CPU quota)
		for(int k = 0; f.test_and_set(std::memory_order_acquire); k++) {
			if(k < 64) __builtin_ia32_pause();
			else sched_yield();
		}
	}
	void unlock() { f.clear(std::memory_order_release); }
};
struct Guard {
	Spin& s;
	explicit Guard(Spin& x) : s(x) { s.lock(); }
	~Guard() { s.unlock(); }
};

struct Depot {
	Spin mu[NCLASS];
	Node* head[NCLASS] = {};
	size_t n[NCLASS] = {};
};
Depot& depot() {
	static Depot* d = new (malloc(sizeof(Depot))) Depot();   // never destroyed (used until exit)
	return *d;
}

thread_local bool t_dead = false;       // the thread's cache is gone (thread exit)

struct Cache {
	Node* head[NCLASS] = {};
	int n[NCLASS] = {};
	~Cache() {
		// a thread that ends (the server makes one per connection) leaves its blocks
		// to the others; frees by later thread-exit destructors go to the depot
		t_dead = true;
		for(int c = 0; c < NCLASS; c++) {
			if(!head[c]) continue;
			Node* tail = head[c];
			while(tail->next) tail = tail->next;
			Depot& d = depot();
			Guard lk(d.mu[c]);
			tail->next = d.head[c];
			d.head[c] = head[c];
			d.n[c] += (size_t)n[c];
			head[c] = nullptr;
			n[c] = 0;
		}
	}
};
thread_local Cache t_cache;

// $BT2G_ALLOC_STATS=<path>: blocks taken from malloc per class (fresh), from
// the depot, and big ones; written by bt2g_alloc_stats_dump (at SIGTERM)
std::atomic<uint64_t> g_fresh[NCLASS + 1], g_refill[NCLASS], g_topot[NCLASS], g_big[48];
bool stats_on() {
	static const bool on = getenv("BT2G_ALLOC_STATS") != nullptr;
	return on;
}

// A class's new blocks come from 1 MiB slabs (one malloc for many blocks;
// blocks of 64 KiB and up one at a time): the rest of a slab goes to the
// calling thread's cache.  Blocks are never returned, so slabs never are.
const size_t SLAB = (size_t)1 << 20;

// Blocks of 1 MiB and up come from one reserved, never-committed address range
// (MAP_NORESERVE; pages are backed when first touched): a malloc'd block that
// big is a mapping of its own, and the batch driver's slots each hold one
// (the reference's 20 MB alignment cache pool, ds.h Pool, mostly untouched) --
// tens of thousands of slots would pass the kernel's limit on mappings
// (vm.max_map_count, 65 530).  $BT2G_ARENA_GB sizes the range (default
// 8192); when it cannot be reserved, or is used up, malloc as before.
// The small classes' 1 MiB slabs come from a second such range, with
// transparent huge pages asked for (MADV_HUGEPAGE: a slab's blocks are all
// initialised at once, 256 page faults a slab otherwise -- and a slab from
// malloc was an mmap of its own: r04f, 45 k mappings and half the drivers'
// CPU in the allocator while their slots were first filled).  The big blocks'
// range keeps small pages: the 20 MB pools are mostly never touched.
struct Range {
	char* base = nullptr;
	size_t cap = 0;
	std::atomic<size_t> used{0};
	Range(size_t gb, bool huge) {
		cap = gb << 30;
		if(!cap) return;
		void* m = mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
		if(m == MAP_FAILED) return;
		base = (char*)m;
		// (the big blocks' range asks for small pages outright: with transparent huge
		// pages "always" a slot's 20 MB pool, of which a read touches a few 16 KB
		// pages, would be backed 2 MB at a time)
		(void)madvise(base, cap, huge ? MADV_HUGEPAGE : MADV_NOHUGEPAGE);
	}
	char* take(size_t bytes) {
		if(!base) return nullptr;
		bytes = (bytes + 4095) & ~(size_t)4095;
		const size_t o = used.fetch_add(bytes, std::memory_order_relaxed);
		if(o + bytes > cap) return nullptr;
		return base + o;
	}
};

size_t arena_gb() {
	const char* e = getenv("BT2G_ARENA_GB");
	const long gb = e ? atol(e) : 8192;
	return gb > 0 ? (size_t)gb : 0;
}

char* arena_take(size_t bytes) {
	static Range* r = new (malloc(sizeof(Range))) Range(arena_gb(), false);
	return r->take(bytes);
}

char* slab_take(size_t bytes) {
	// ($BT2G_SLAB_HUGE=0: small pages.  On the CPU stand-in the drivers spent 29 %
	// of their samples in a slab's first touch with huge pages and 15 % without, but
	// on the GPU box the drivers' CPU rose from 29.8 s to 45.7 s without them, r04w
	// vs r04y: huge pages by default)
	static const bool huge = [] { const char* e = getenv("BT2G_SLAB_HUGE"); return !(e && *e == '0'); }();
	static Range* r = new (malloc(sizeof(Range))) Range(arena_gb() ? 1024 : 0, huge);
	return r->take(bytes);
}

thread_local size_t t_fresh = 0;        // bytes of the slab the last allocation took ($BT2G_ALLOC_SITES=fresh)
// bytes this thread allocated minus bytes it freed (block sizes incl. headers):
// the batch driver charges a read slot with the difference across its steps, and
// rebuilds slots whose reference objects grew big (bt2g_alloc_thread_net)
thread_local long long t_net = 0;

void* fresh(int c) {
	if(stats_on()) g_fresh[c].fetch_add(1, std::memory_order_relaxed);
	t_fresh = size_of(c) < ((size_t)64 << 10) ? SLAB : HDR + size_of(c);
	const size_t bsz = HDR + size_of(c);
	const size_t nb = size_of(c) < ((size_t)64 << 10) && !t_dead ? SLAB / bsz : 1;
	// (64 KiB - 1 MiB blocks one at a time from the slab range too: from malloc they
	// grew glibc's heaps, mprotect on ~10 % of the drivers' samples in r04r)
	char* p = size_of(c) >= ((size_t)1 << 20) ? arena_take(bsz) : slab_take(bsz * nb);
	if(!p) p = (char*)malloc(bsz * nb);
	if(!p) return nullptr;
	for(size_t i = 0; i < nb; i++) {
		Hdr* h = (Hdr*)(p + i * bsz);
		h->magic = MAGIC_CACHED;
		h->cls = (uint32_t)c;
	}
	// blocks 1..nb-1 to this thread's cache (it was empty: the caller found no block)
	Cache& tc = t_cache;
	for(size_t i = nb; i-- > 1;) {
		Node* b = (Node*)(p + i * bsz + HDR);
		b->next = tc.head[c];
		tc.head[c] = b;
		tc.n[c]++;
	}
	return p + HDR;
}

void* alloc(size_t n) {
	if(n == 0) n = 1;
	if(!enabled() || n > MAXSZ) {
		if(stats_on()) {
			g_fresh[NCLASS].fetch_add(1, std::memory_order_relaxed);
			int b = 0;
			while(b < 47 && ((size_t)1 << b) < n) b++;
			if(g_big[b].fetch_add(1, std::memory_order_relaxed) == 0 && b >= 30 && getenv("BT2G_ALLOC_TRACE")) {
				void* bt[24];
				const int k = backtrace(bt, 24);
				fprintf(stderr, "bt2g alloc: %zu bytes\n", n);
				backtrace_symbols_fd(bt, k, 2);
			}
		}
		void* p = malloc(HDR + n);
		if(!p) return nullptr;
		((Hdr*)p)->magic = MAGIC_MALLOC;
		// (the bytes release() will count back: malloc's usable size, not HDR + n)
		t_net += (long long)malloc_usable_size(p);
		return (char*)p + HDR;
	}
	const int c = cls_of(n);
	t_net += (long long)(HDR + size_of(c));
	if(!t_dead) {
		Cache& tc = t_cache;
		if(!tc.head[c]) {
			// refill from the depot (one lock for a batch)
			Depot& d = depot();
			Guard lk(d.mu[c]);
			const int nb = BATCH < cap_of(c) ? BATCH : cap_of(c);
			if(stats_on()) g_refill[c].fetch_add(1, std::memory_order_relaxed);
			for(int i = 0; i < nb && d.head[c]; i++) {
				Node* b = d.head[c];
				d.head[c] = b->next;
				d.n[c]--;
				b->next = tc.head[c];
				tc.head[c] = b;
				tc.n[c]++;
			}
		}
		if(Node* b = tc.head[c]) {
			tc.head[c] = b->next;
			tc.n[c]--;
			// the next block of the class, whose link the next allocation reads: a
			// cold line otherwise (a block freed long ago; r05s: the link load was
			// ~60 % of the allocator's samples)
			if(tc.head[c]) __builtin_prefetch(tc.head[c], 1, 3);
			return b;
		}
	}
	return fresh(c);
}

bool xtrace_on();
void xcheck(void* p);
bool live_on();
}  // namespace
void live_untag(void* p);
namespace {

void release(void* p) {
	if(!p) return;
	if(xtrace_on()) xcheck(p);
	if(live_on()) live_untag(p);
	Hdr* h = (Hdr*)((char*)p - HDR);
	if(h->magic == MAGIC_MALLOC) {
		t_net -= (long long)malloc_usable_size(h);
		free(h);
		return;
	}
	if(h->magic != MAGIC_CACHED || h->cls >= (uint32_t)NCLASS) abort();   // not ours: a heap corruption
	const int c = (int)h->cls;
	t_net -= (long long)(HDR + size_of(c));
	Node* b = (Node*)p;
	if(t_dead) {
		Depot& d = depot();
		Guard lk(d.mu[c]);
		b->next = d.head[c];
		d.head[c] = b;
		d.n[c]++;
		return;
	}
	Cache& tc = t_cache;
	b->next = tc.head[c];
	tc.head[c] = b;
	if(++tc.n[c] > cap_of(c)) {
		// half of the cache to the depot
		const int k = tc.n[c] / 2;
		if(stats_on()) g_topot[c].fetch_add((uint64_t)k, std::memory_order_relaxed);
		Node* first = tc.head[c];
		Node* last = first;
		for(int i = 1; i < k; i++) last = last->next;
		tc.head[c] = last->next;
		tc.n[c] -= k;
		Depot& d = depot();
		Guard lk(d.mu[c]);
		last->next = d.head[c];
		d.head[c] = first;
		d.n[c] += (size_t)k;
	}
}

}  // namespace

// $BT2G_ALLOC_XTRACE=1 (diagnostics): every block remembers its allocating
// thread and call site (the header's spare word); a block freed by another
// thread counts its call site -- which code feeds the cross-thread flows that
// make the depot traffic.  Dumped with the stats (call sites as module + offset).
namespace {
bool xtrace_on() {
	static const bool on = getenv("BT2G_ALLOC_XTRACE") != nullptr;
	return on;
}
std::atomic<uint32_t> g_tid_next{1};
thread_local uint32_t t_tid = 0;
inline uint64_t my_tid() {
	if(!t_tid) t_tid = g_tid_next.fetch_add(1) & 0xffffu;
	return t_tid;
}
const size_t XSLOT = 1u << 14;
std::atomic<uint64_t> g_xpc[XSLOT];
std::atomic<uint64_t> g_xcnt[XSLOT];
inline void xtag(void* p, void* ra) {
	if(!p) return;
	Hdr* h = (Hdr*)((char*)p - HDR);
	h->pad = (my_tid() << 48) | ((uint64_t)(uintptr_t)ra & 0xffffffffffffull);
}
inline void xcheck(void* p) {
	Hdr* h = (Hdr*)((char*)p - HDR);
	const uint64_t t = h->pad >> 48;
	if(!t || t == my_tid()) return;
	const uint64_t pc = h->pad & 0xffffffffffffull;
	size_t k = (size_t)((pc * 0x9E3779B97F4A7C15ull) >> 50) & (XSLOT - 1);
	for(int probe = 0; probe < 64; probe++, k = (k + 1) & (XSLOT - 1)) {
		uint64_t cur = g_xpc[k].load(std::memory_order_relaxed);
		if(cur == pc) { g_xcnt[k].fetch_add(1, std::memory_order_relaxed); return; }
		if(cur == 0) {
			uint64_t z = 0;
			if(g_xpc[k].compare_exchange_strong(z, pc) || z == pc) { g_xcnt[k].fetch_add(1, std::memory_order_relaxed); return; }
		}
	}
}
// $BT2G_ALLOC_SITES=1 (diagnostics): bytes allocated inside a scope the caller
// marks (bt2g_alloc_site_scope: the batch driver's slot construction), by call
// site -- what makes a slot's footprint.  Dumped with the stats.
std::atomic<uint64_t> g_spc[XSLOT], g_scnt[XSLOT], g_sbytes[XSLOT];
thread_local int t_site_scope = 0;
bool sites_on() {
	static const bool on = getenv("BT2G_ALLOC_SITES") != nullptr;
	return on;
}
// $BT2G_ALLOC_SITES=fresh: only the allocations that took new memory (a slab,
// or a block of its own), counted with the bytes taken
bool sites_fresh() {
	static const bool on = [] { const char* e = getenv("BT2G_ALLOC_SITES"); return e && !strcmp(e, "fresh"); }();
	return on;
}
// $BT2G_ALLOC_SITES=all: every allocation, anywhere (which call sites allocate per read)
bool sites_all() {
	static const bool on = [] { const char* e = getenv("BT2G_ALLOC_SITES"); return e && !strcmp(e, "all"); }();
	return on;
}
// $BT2G_ALLOC_SITES_CLASS=<bytes>: also every allocation of that size class, anywhere
int sites_cls() {
	static const int c = [] {
		const char* e = getenv("BT2G_ALLOC_SITES_CLASS");
		return e && atol(e) > 0 ? cls_of((size_t)atol(e)) : -1;
	}();
	return c;
}
inline void site_count(void* ra, size_t n) {
	const uint64_t pc = (uint64_t)(uintptr_t)ra;
	size_t k = (size_t)((pc * 0x9E3779B97F4A7C15ull) >> 50) & (XSLOT - 1);
	for(int probe = 0; probe < 64; probe++, k = (k + 1) & (XSLOT - 1)) {
		uint64_t cur = g_spc[k].load(std::memory_order_relaxed);
		if(cur == 0) {
			uint64_t z = 0;
			if(!g_spc[k].compare_exchange_strong(z, pc) && z != pc) continue;
			cur = pc;
		}
		if(cur == pc) {
			g_scnt[k].fetch_add(1, std::memory_order_relaxed);
			g_sbytes[k].fetch_add(n, std::memory_order_relaxed);
			return;
		}
	}
}
}  // namespace

// $BT2G_ALLOC_LIVE=1 (diagnostics): bytes live by allocation site -- a block
// remembers its call site in the header's spare word and gives its bytes back to
// that site when freed; dumped with the stats ("live <module> <offset> <bytes>").
namespace {
bool live_on() {
	// (the live tag and $BT2G_ALLOC_XTRACE's tag share the header's spare word:
	// with both set, the live tag is off)
	static const bool on = [] {
		if(!getenv("BT2G_ALLOC_LIVE")) return false;
		if(xtrace_on()) {
			fprintf(stderr, "bt2g alloc: BT2G_ALLOC_LIVE ignored with BT2G_ALLOC_XTRACE (one header word)\n");
			return false;
		}
		return true;
	}();
	return on;
}
std::atomic<uint64_t> g_lpc[XSLOT];
std::atomic<long long> g_lbytes[XSLOT];
inline size_t live_slot(uint64_t pc) {
	size_t k = (size_t)((pc * 0x9E3779B97F4A7C15ull) >> 50) & (XSLOT - 1);
	for(int probe = 0; probe < 256; probe++, k = (k + 1) & (XSLOT - 1)) {
		uint64_t cur = g_lpc[k].load(std::memory_order_relaxed);
		if(cur == pc) return k;
		if(cur == 0) {
			uint64_t z = 0;
			if(g_lpc[k].compare_exchange_strong(z, pc) || z == pc) return k;
		}
	}
	return XSLOT;
}
inline void live_tag(void* p, void* ra) {
	if(!p) return;
	Hdr* h = (Hdr*)((char*)p - HDR);
	const size_t k = live_slot((uint64_t)(uintptr_t)ra);
	h->pad = k;
	if(k < XSLOT) {
		const long long n = h->magic == MAGIC_MALLOC ? (long long)malloc_usable_size(h) : (long long)(HDR + size_of((int)h->cls));
		g_lbytes[k].fetch_add(n, std::memory_order_relaxed);
	}
}
}  // namespace
void live_untag(void* p) {
	Hdr* h = (Hdr*)((char*)p - HDR);
	const size_t k = (size_t)h->pad;
	if(k >= XSLOT) return;
	const long long n = h->magic == MAGIC_MALLOC ? (long long)malloc_usable_size(h) : (long long)(HDR + size_of((int)h->cls));
	g_lbytes[k].fetch_sub(n, std::memory_order_relaxed);
}

extern "C" void bt2g_alloc_site_scope(int on) { t_site_scope += on ? 1 : -1; }

// Bytes the calling thread allocated minus those it freed (0 with $BT2G_ALLOC=0).
extern "C" long long bt2g_alloc_thread_net() { return enabled() ? t_net : 0; }

extern "C" void bt2g_alloc_stats_dump() {
	const char* path = getenv("BT2G_ALLOC_STATS");
	if(!path) return;
	FILE* f = fopen(path, "w");
	if(!f) return;
	for(int c = 0; c <= NCLASS; c++)
		fprintf(f, "%s %llu %llu %llu %llu\n", c < NCLASS ? std::to_string(size_of(c)).c_str() : "big",
		        (unsigned long long)g_fresh[c].load(), c < NCLASS ? (unsigned long long)g_refill[c].load() : 0ull,
		        c < NCLASS ? (unsigned long long)g_topot[c].load() : 0ull, c < NCLASS ? (unsigned long long)depot().n[c] : 0ull);
	for(int b = 0; b < 48; b++)
		if(g_big[b].load()) fprintf(f, "big<=2^%d %llu\n", b, (unsigned long long)g_big[b].load());
	if(xtrace_on())
		for(size_t k = 0; k < XSLOT; k++) {
			const uint64_t pc = g_xpc[k].load();
			if(!pc) continue;
			Dl_info di;
			if(dladdr((void*)(uintptr_t)pc, &di) && di.dli_fname)
				fprintf(f, "xfree %s %lx %llu\n", di.dli_fname, (unsigned long)(pc - (uint64_t)(uintptr_t)di.dli_fbase),
				        (unsigned long long)g_xcnt[k].load());
		}
	if(live_on())
		for(size_t k = 0; k < XSLOT; k++) {
			const uint64_t pc = g_lpc[k].load();
			if(!pc) continue;
			Dl_info di;
			if(dladdr((void*)(uintptr_t)pc, &di) && di.dli_fname)
				fprintf(f, "live %s %lx %lld\n", di.dli_fname, (unsigned long)(pc - (uint64_t)(uintptr_t)di.dli_fbase),
				        (long long)g_lbytes[k].load());
		}
	if(sites_on())
		for(size_t k = 0; k < XSLOT; k++) {
			const uint64_t pc = g_spc[k].load();
			if(!pc) continue;
			Dl_info di;
			if(dladdr((void*)(uintptr_t)pc, &di) && di.dli_fname)
				fprintf(f, "site %s %lx %llu %llu\n", di.dli_fname, (unsigned long)(pc - (uint64_t)(uintptr_t)di.dli_fbase),
				        (unsigned long long)g_scnt[k].load(), (unsigned long long)g_sbytes[k].load());
		}
	fclose(f);
}

void* operator new(size_t n) {
	void* p = alloc(n);
	if(!p) throw std::bad_alloc();
	if(xtrace_on()) xtag(p, __builtin_return_address(0));
	if(live_on()) live_tag(p, __builtin_return_address(0));
	if(sites_on()) {
		if(sites_fresh()) {
			if(t_fresh) site_count(__builtin_return_address(0), t_fresh);
		} else if(sites_all() || t_site_scope || (n <= MAXSZ && cls_of(n) == sites_cls())) {
			site_count(__builtin_return_address(0), n);
		}
		t_fresh = 0;
	}
	return p;
}
void* operator new[](size_t n) {
	void* p = alloc(n);
	if(!p) throw std::bad_alloc();
	if(xtrace_on()) xtag(p, __builtin_return_address(0));
	if(live_on()) live_tag(p, __builtin_return_address(0));
	if(sites_on()) {
		if(sites_fresh()) {
			if(t_fresh) site_count(__builtin_return_address(0), t_fresh);
		} else if(sites_all() || t_site_scope || (n <= MAXSZ && cls_of(n) == sites_cls())) {
			site_count(__builtin_return_address(0), n);
		}
		t_fresh = 0;
	}
	return p;
}
void* operator new(size_t n, const std::nothrow_t&) noexcept {
	void* p = alloc(n);
	if(live_on()) live_tag(p, __builtin_return_address(0));
	return p;
}
void* operator new[](size_t n, const std::nothrow_t&) noexcept {
	void* p = alloc(n);
	if(live_on()) live_tag(p, __builtin_return_address(0));
	return p;
}
void operator delete(void* p) noexcept { release(p); }
void operator delete[](void* p) noexcept { release(p); }
void operator delete(void* p, size_t) noexcept { release(p); }
void operator delete[](void* p, size_t) noexcept { release(p); }
void operator delete(void* p, const std::nothrow_t&) noexcept { release(p); }
void operator delete[](void* p, const std::nothrow_t&) noexcept { release(p); }
