// Random 64-B gather rate from a table far larger than the Infinity Cache
// (the access pattern of an FM-index LF step), independent and dependent.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t hash(uint32_t x) {
	x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
	return x;
}
// INFL independent 64-B gathers in flight per lane, ITERS rounds
template <int INFL>
__global__ void __launch_bounds__(256) k_indep(const u32x4* __restrict__ t, uint32_t nside, uint32_t iters,
                                               uint32_t* out) {
	uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x, acc = 0;
	for(uint32_t it = 0; it < iters; it++) {
		u32x4 v[INFL][4];
#pragma unroll
		for(int k = 0; k < INFL; k++) {
			const uint32_t s = hash(gid * 977u + it * 131u + k) % nside;
#pragma unroll
			for(int q = 0; q < 4; q++) v[k][q] = t[(size_t)s * 4 + q];
		}
#pragma unroll
		for(int k = 0; k < INFL; k++) acc += v[k][0].x ^ v[k][1].y ^ v[k][2].z ^ v[k][3].w;
	}
	out[gid] = acc;
}
// dependent chain: next side index from the loaded data (pointer chase).  The
// lane id enters every step's address, and the table holds distinct words
// (k_fill): with a constant table the loaded words cancelled and every lane
// chased the same line, i.e. the "chain" rows measured a cache hit.
__global__ void __launch_bounds__(256) k_chain(const u32x4* __restrict__ t, uint32_t nside, uint32_t iters,
                                               uint32_t* out) {
	uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
	uint32_t s = hash(gid) % nside, acc = 0;
	for(uint32_t it = 0; it < iters; it++) {
		u32x4 a = t[(size_t)s * 4], b = t[(size_t)s * 4 + 1], c = t[(size_t)s * 4 + 2], d = t[(size_t)s * 4 + 3];
		acc += a.x ^ b.y ^ c.z ^ d.w;
		s = hash(acc ^ (gid * 0x9e3779b9u) ^ it) % nside;
	}
	out[gid] = acc;
}
// The same chain with the wave's 64 sides of a step loaded cooperatively and
// staged in LDS ("coalesced occ-table gathers with LDS-staged rank blocks"):
// in round k (0..3) lane i loads quarter i&3 of the side of lane 16k + i/4, so
// one dwordx4 instruction covers 16 whole 64-B lines (the per-lane form: 64
// lines, a quarter each, 4 instructions per side); the lanes then read their
// own side back from LDS.
__global__ void __launch_bounds__(256) k_chain_lds(const u32x4* __restrict__ t, uint32_t nside, uint32_t iters,
                                                   uint32_t* out) {
	__shared__ u32x4 st[4][64][4];                // [wave of the block][lane][quarter]
	const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
	uint32_t s = hash(gid) % nside, acc = 0;
	for(uint32_t it = 0; it < iters; it++) {
		u32x4 q[4];
#pragma unroll
		for(int k = 0; k < 4; k++) {
			const uint32_t owner = 16u * k + (lane >> 2);
			const uint32_t so = __shfl(s, owner);
			q[k] = t[(size_t)so * 4 + (lane & 3u)];
		}
#pragma unroll
		for(int k = 0; k < 4; k++) st[wv][16u * k + (lane >> 2)][lane & 3u] = q[k];
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		const u32x4 a = st[wv][lane][0], b = st[wv][lane][1], c = st[wv][lane][2], d = st[wv][lane][3];
		acc += a.x ^ b.y ^ c.z ^ d.w;
		__builtin_amdgcn_wave_barrier();
		s = hash(acc ^ (gid * 0x9e3779b9u) ^ it) % nside;
	}
	out[gid] = acc;
}
__global__ void k_fill(uint32_t* t, size_t n) {
	for(size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
		t[i] = hash((uint32_t)i * 2654435761u + 12345u);
}
int main() {
	const size_t bytes = 2ull << 30;   // 2 GiB table
	const uint32_t nside = (uint32_t)(bytes / 64);
	u32x4* t;
	uint32_t* o;
	(void)hipMalloc(&t, bytes);
	hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t*)t, bytes / 4);
	(void)hipDeviceSynchronize();
	(void)hipMalloc(&o, 64u << 20);
	hipEvent_t e0, e1;
	(void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
	auto run = [&](const char* name, auto launch, double gathers) {
		float best = 1e9f;
		for(int rep = 0; rep < 3; rep++) {
			(void)hipEventRecord(e0);
			launch();
			(void)hipEventRecord(e1);
			(void)hipEventSynchronize(e1);
			float ms;
			(void)hipEventElapsedTime(&ms, e0, e1);
			if(rep && ms < best) best = ms;
		}
		printf("%-34s %8.3f ms  %7.2f G gathers/s  %7.1f GB/s (64 B each)\n", name, best, gathers / best / 1e6,
		       gathers * 64 / best / 1e6);
	};
	// the latency of one dependent 64-B gather: few waves (one per workgroup), a
	// long chain -- what an LF walk over a small batch sees step by step
	for(uint32_t waves : {16u, 256u, 1024u}) {
		const uint32_t iters = 2000;
		float best = 1e9f;
		for(int rep = 0; rep < 3; rep++) {
			(void)hipEventRecord(e0);
			hipLaunchKernelGGL(k_chain, dim3(waves), dim3(64), 0, 0, t, nside, iters, o);
			(void)hipEventRecord(e1);
			(void)hipEventSynchronize(e1);
			float ms;
			(void)hipEventElapsedTime(&ms, e0, e1);
			if(rep && ms < best) best = ms;
		}
		printf("chain latency %5u waves x 64 lanes  %8.3f ms  %6.3f us per dependent step\n", waves, best,
		       best * 1e3 / iters);
	}
	for(int blocksPerCU : {4, 8, 16}) {
		const uint32_t blocks = 256 * blocksPerCU, iters = 64;
		const double g = (double)blocks * 256 * iters;
		char nm[64];
		snprintf(nm, sizeof nm, "indep x1  %2d blk/CU", blocksPerCU);
		run(nm, [&] { hipLaunchKernelGGL(k_indep<1>, dim3(blocks), dim3(256), 0, 0, t, nside, iters, o); }, g);
		snprintf(nm, sizeof nm, "indep x4  %2d blk/CU", blocksPerCU);
		run(nm, [&] { hipLaunchKernelGGL(k_indep<4>, dim3(blocks), dim3(256), 0, 0, t, nside, iters, o); }, g * 4);
		snprintf(nm, sizeof nm, "chain     %2d blk/CU", blocksPerCU);
		run(nm, [&] { hipLaunchKernelGGL(k_chain, dim3(blocks), dim3(256), 0, 0, t, nside, iters, o); }, g);
		snprintf(nm, sizeof nm, "chain LDS-staged %2d blk/CU", blocksPerCU);
		run(nm, [&] { hipLaunchKernelGGL(k_chain_lds, dim3(blocks), dim3(256), 0, 0, t, nside, iters, o); }, g);
	}
	return 0;
}
