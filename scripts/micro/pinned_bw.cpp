// Host memcpy bandwidth into / out of hipHostMalloc'd memory by flag (the
// engine wrappers stage inputs and read outputs through such a block).
//   hipcc -O2 scripts/micro/pinned_bw.cpp -o /tmp/pinned_bw && /tmp/pinned_bw
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

static double gbs(size_t bytes, std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
	return bytes / std::chrono::duration<double>(b - a).count() / 1e9;
}

int main() {
	const size_t n = 8u << 20;
	std::vector<char> src(n, 1), dst(n, 0);
	struct F { const char* name; unsigned flags; } fl[] = {
		{"default", hipHostMallocDefault},
		{"noncoherent", hipHostMallocNonCoherent},
		{"coherent", hipHostMallocCoherent},
		{"mapped|noncoherent", hipHostMallocMapped | hipHostMallocNonCoherent},
	};
	for(auto& f : fl) {
		char* p = nullptr;
		if(hipHostMalloc((void**)&p, n, f.flags) != hipSuccess) { printf("%s: alloc failed\n", f.name); continue; }
		memset(p, 0, n);
		double in = 0, out = 0;
		for(int r = 0; r < 5; r++) {
			auto t0 = std::chrono::steady_clock::now();
			memcpy(p, src.data(), n);
			auto t1 = std::chrono::steady_clock::now();
			memcpy(dst.data(), p, n);
			auto t2 = std::chrono::steady_clock::now();
			in = std::max(in, gbs(n, t0, t1));
			out = std::max(out, gbs(n, t1, t2));
		}
		printf("%-20s into %.2f GB/s  out of %.2f GB/s\n", f.name, in, out);
		(void)hipHostFree(p);
	}
	return 0;
}
