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
#include <time.h>
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
std::atomic<uint64_t> g_lost{0};

void on_prof(int, siginfo_t*, void* uc) {
	const uint64_t pc = (uint64_t)((ucontext_t*)uc)->uc_mcontext.gregs[REG_RIP];
	if(!pc) return;
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

struct Sampler {
	Sampler() {
		const char* path = getenv("BT2G_SAMPLE");
		if(!path || !*path) return;
		g_pc = new std::atomic<uint64_t>[NSLOT]();
		g_cnt = new std::atomic<uint32_t>[NSLOT]();
		struct sigaction sa;
		memset(&sa, 0, sizeof(sa));
		sa.sa_sigaction = on_prof;
		sa.sa_flags = SA_SIGINFO | SA_RESTART;
		sigaction(SIGPROF, &sa, nullptr);
		std::string p(path);
		std::thread([p] {
			for(;;) {
				sleep(2);
				dump(p.c_str());
			}
		}).detach();
	}
} g_sampler;

}  // namespace

// Sample the calling thread's CPU time (no-op unless $BT2G_SAMPLE is set).
extern "C" void bt2g_prof_thread() {
	if(!g_pc) return;
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
