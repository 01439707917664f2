// integration/bt2g_prof.cpp -- a flat CPU sampler for the drop-in server
// (diagnostics only; no effect unless $BT2G_SAMPLE names an output file).
//
// SIGPROF at 1 kHz of each registered thread's CPU time (carriers and seam
// dispatchers register, bt2g_prof_thread); each signal counts the interrupted
// instruction pointer in a lock-free table.  Every 2 s the table is written to
// $BT2G_SAMPLE as "<mapping path> <offset in mapping> <samples>" lines, which
// scripts/prof_symbolize.py turns into per-function totals with addr2line.
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <sys/uio.h>
#include <time.h>
#include <malloc.h>
#include <ucontext.h>
#include <unistd.h>

#include <atomic>
#include <string>
#include <thread>
#include <vector>

namespace {

const size_t NSLOT = 1u << 20;
std::atomic<uint64_t>* g_pc = nullptr;     // key: instruction pointer (0 = empty)
std::atomic<uint32_t>* g_cnt = nullptr;
// (pc, word at the stack pointer) pairs: for a sample inside a frameless leaf
// (a libc syscall wrapper) that word is its caller's return address
std::atomic<uint64_t>* g_pc2 = nullptr;
std::atomic<uint64_t>* g_ret2 = nullptr;
std::atomic<uint32_t>* g_cnt2 = nullptr;
std::atomic<uint64_t> g_lost{0};
// the executable's text: for a sample outside it (libc, the HIP runtime), the
// first stack word that points into it is recorded as the sample's "exe caller"
// (role 8 + role in the pair table) -- which of the server's functions led to
// a hot spot in a library (mprotect <- sysmalloc <- malloc <- ?)
uint64_t g_text_lo = 0, g_text_hi = 0;
thread_local uint64_t t_role = 0;           // 1 carrier, 2 dispatcher (folded into the pair table)

void count_pair(uint64_t pc, uint64_t ret) {
	size_t h = (size_t)(((pc ^ (ret * 0xC2B2AE3D27D4EB4Full)) * 0x9E3779B97F4A7C15ull) >> 44) & (NSLOT - 1);
	for(size_t probe = 0; probe < 64; probe++, h = (h + 1) & (NSLOT - 1)) {
		uint64_t k = g_pc2[h].load(std::memory_order_relaxed);
		if(k == pc && g_ret2[h].load(std::memory_order_relaxed) == ret) {
			g_cnt2[h].fetch_add(1, std::memory_order_relaxed);
			return;
		}
		if(k == 0) {
			uint64_t z = 0;
			if(g_pc2[h].compare_exchange_strong(z, pc)) {
				g_ret2[h].store(ret, std::memory_order_relaxed);
				g_cnt2[h].fetch_add(1, std::memory_order_relaxed);
				return;
			}
		}
	}
}

void on_prof(int, siginfo_t*, void* uc) {
	const uint64_t pc = (uint64_t)((ucontext_t*)uc)->uc_mcontext.gregs[REG_RIP];
	if(!pc) return;
	const uint64_t sp = (uint64_t)((ucontext_t*)uc)->uc_mcontext.gregs[REG_RSP];
	if(sp) count_pair(pc, *(const uint64_t*)sp ^ (t_role << 60));
	if(sp && g_text_hi && (pc < g_text_lo || pc >= g_text_hi)) {
		// the stack words above sp, read without faulting past the stack's end
		uint64_t w[256];
		iovec loc{w, sizeof(w)}, rem{(void*)sp, sizeof(w)};
		const ssize_t got = process_vm_readv(getpid(), &loc, 1, &rem, 1, 0);
		for(ssize_t i = 0; got > 0 && i < got / 8; i++)
			if(w[i] >= g_text_lo && w[i] < g_text_hi) {
				count_pair(pc, w[i] ^ ((t_role | 8) << 60));
				break;
			}
	}
	size_t h = (size_t)((pc * 0x9E3779B97F4A7C15ull) >> 44) & (NSLOT - 1);
	for(size_t probe = 0; probe < 64; probe++, h = (h + 1) & (NSLOT - 1)) {
		uint64_t k = g_pc[h].load(std::memory_order_relaxed);
		if(k == pc) {
			g_cnt[h].fetch_add(1, std::memory_order_relaxed);
			return;
		}
		if(k == 0) {
			uint64_t z = 0;
			if(g_pc[h].compare_exchange_strong(z, pc) || z == pc) {
				g_cnt[h].fetch_add(1, std::memory_order_relaxed);
				return;
			}
		}
	}
	g_lost.fetch_add(1, std::memory_order_relaxed);
}

struct Map {
	uint64_t lo, hi, off;
	std::string path;
};

void dump(const char* path) {
	std::vector<Map> maps;
	if(FILE* f = fopen("/proc/self/maps", "r")) {
		char line[4096];
		while(fgets(line, sizeof(line), f)) {
			unsigned long lo, hi, off;
			char perm[8], dev[16], p[3000] = {0};
			unsigned long ino;
			int n = sscanf(line, "%lx-%lx %7s %lx %15s %lu %2999s", &lo, &hi, perm, &off, dev, &ino, p);
			if(n >= 6 && perm[2] == 'x') maps.push_back(Map{lo, hi, off, n == 7 ? p : "?"});
		}
		fclose(f);
	}
	std::string tmp = std::string(path) + ".tmp";
	FILE* o = fopen(tmp.c_str(), "w");
	if(!o) return;
	fprintf(o, "# lost %llu\n", (unsigned long long)g_lost.load());
	auto where = [&](uint64_t a, char* buf, size_t n) {
		for(const Map& x : maps)
			if(a >= x.lo && a < x.hi) {
				snprintf(buf, n, "%s %lx", x.path.c_str(), (unsigned long)(a - x.lo + x.off));
				return;
			}
		snprintf(buf, n, "? %lx", (unsigned long)a);
	};
	for(size_t i = 0; i < NSLOT; i++) {
		uint64_t pc = g_pc2[i].load(std::memory_order_relaxed);
		if(!pc) continue;
		char a[4200], b[4200];
		where(pc, a, sizeof(a));
		const uint64_t rr = g_ret2[i].load(std::memory_order_relaxed);
		where(rr & ~(0xFull << 60), b, sizeof(b));
		fprintf(o, "#pair %s %s %u %llu\n", a, b, g_cnt2[i].load(std::memory_order_relaxed),
		        (unsigned long long)(rr >> 60));
	}
	for(size_t i = 0; i < NSLOT; i++) {
		uint64_t pc = g_pc[i].load(std::memory_order_relaxed);
		if(!pc) continue;
		uint32_t c = g_cnt[i].load(std::memory_order_relaxed);
		const Map* m = nullptr;
		for(const Map& x : maps)
			if(pc >= x.lo && pc < x.hi) { m = &x; break; }
		if(m) fprintf(o, "%s %lx %u\n", m->path.c_str(), (unsigned long)(pc - m->lo + m->off), c);
		else fprintf(o, "? %lx %u\n", (unsigned long)pc, c);
	}
	fclose(o);
	rename(tmp.c_str(), path);
}

// $BT2G_SAMPLE_ALL=1: one process-wide CPU-time timer (ITIMER_PROF) instead of
// per-thread ones -- every thread is sampled, the runtime's and the reference's
// connection threads included (role 0 unless registered)
bool sample_all() {
	static const bool on = [] { const char* e = getenv("BT2G_SAMPLE_ALL"); return e && *e == '1'; }();
	return on;
}

struct Sampler {
	Sampler() {
		const char* path = getenv("BT2G_SAMPLE");
		if(!path || !*path) return;
		g_pc = new std::atomic<uint64_t>[NSLOT]();
		g_cnt = new std::atomic<uint32_t>[NSLOT]();
		g_pc2 = new std::atomic<uint64_t>[NSLOT]();
		g_ret2 = new std::atomic<uint64_t>[NSLOT]();
		g_cnt2 = new std::atomic<uint32_t>[NSLOT]();
		struct sigaction sa;
		memset(&sa, 0, sizeof(sa));
		sa.sa_sigaction = on_prof;
		sa.sa_flags = SA_SIGINFO | SA_RESTART;
		sigaction(SIGPROF, &sa, nullptr);
		char exe[4096] = {0};
		if(readlink("/proc/self/exe", exe, sizeof(exe) - 1) > 0)
			if(FILE* f = fopen("/proc/self/maps", "r")) {
				char line[4096];
				while(fgets(line, sizeof(line), f)) {
					unsigned long lo, hi, off, ino;
					char perm[8], dev[16], pth[3000] = {0};
					if(sscanf(line, "%lx-%lx %7s %lx %15s %lu %2999s", &lo, &hi, perm, &off, dev, &ino, pth) == 7 &&
					   perm[2] == 'x' && !strcmp(pth, exe)) {
						g_text_lo = lo;
						g_text_hi = hi;
					}
				}
				fclose(f);
			}
		if(sample_all()) {
			itimerval it;
			it.it_interval.tv_sec = 0;
			it.it_interval.tv_usec = 1000;
			it.it_value = it.it_interval;
			setitimer(ITIMER_PROF, &it, nullptr);
		}
		std::string p(path);
		std::thread([p] {
			for(int k = 0;; k++) {
				sleep(2);
				dump(p.c_str());
				// the allocator's arenas over time (system bytes per heap)
				if(FILE* f = fopen((p + ".malloc").c_str(), "a")) {
					fprintf(f, "<!-- t=%d -->\n", 2 * (k + 1));
					malloc_info(0, f);
					fclose(f);
				}
			}
		}).detach();
	}
} g_sampler;

}  // namespace

// Sample the calling thread's CPU time (no-op unless $BT2G_SAMPLE is set).
extern "C" void bt2g_prof_thread(int role) {
	if(!g_pc) return;
	t_role = (uint64_t)role & 0xF;
	if(sample_all()) return;             // the process timer samples every thread
	sigevent sev;
	memset(&sev, 0, sizeof(sev));
	sev.sigev_notify = SIGEV_THREAD_ID;
	sev.sigev_signo = SIGPROF;
	sev._sigev_un._tid = (pid_t)syscall(SYS_gettid);
	timer_t t;
	if(timer_create(CLOCK_THREAD_CPUTIME_ID, &sev, &t) != 0) return;
	itimerspec it;
	it.it_interval.tv_sec = 0;
	it.it_interval.tv_nsec = 1000000;
	it.it_value = it.it_interval;
	timer_settime(t, 0, &it, nullptr);
}

// Change the calling thread's role tag (which phase its samples belong to).
extern "C" void bt2g_prof_role(int role) { t_role = (uint64_t)role & 0xF; }
