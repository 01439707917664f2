// dev_util.h -- small device helpers shared by the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Exclusive prefix of v over the wave and the wave total (shuffles, no LDS).
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t& total) {
	const uint32_t lane = threadIdx.x & 63u;
	uint32_t x = v;
#pragma unroll
	for(int o = 1; o < 64; o <<= 1) {
		const uint32_t y = (uint32_t)__shfl_up((int)x, o);
		if(lane >= (uint32_t)o) x += y;
	}
	total = (uint32_t)__shfl((int)x, 63);
	return x - v;
}

// Each thread of the workgroup claims `count` consecutive slots from
// *counter, in thread order within the workgroup, with ONE global atomic per
// workgroup (a single queue word sustains only ~90 atomics/us chip-wide).
// Every thread of the block must call it (it synchronises the block).
template <int BLOCK>
__device__ __forceinline__ uint32_t block_alloc(uint32_t count, uint32_t* counter) {
	static_assert(BLOCK % 64 == 0 && BLOCK <= 1024, "block of whole waves");
	__shared__ uint32_t wave_off[BLOCK / 64];
	__shared__ uint32_t block_base;
	const uint32_t wid = threadIdx.x >> 6;
	uint32_t wtot;
	const uint32_t pre = wave_excl_scan(count, wtot);
	if((threadIdx.x & 63u) == 0) wave_off[wid] = wtot;
	__syncthreads();
	if(threadIdx.x == 0) {
		uint32_t acc = 0;
		for(int w = 0; w < BLOCK / 64; w++) {
			const uint32_t t = wave_off[w];
			wave_off[w] = acc;
			acc += t;
		}
		block_base = acc ? atomicAdd(counter, acc) : 0u;
	}
	__syncthreads();
	const uint32_t base = block_base + wave_off[wid] + pre;
	__syncthreads();   // the shared words may be reused by the next call
	return base;
}

// One slot of *counter for every lane active at this call site, with ONE
// atomic per wave (a lone queue word sustains only ~90 atomics/us chip-wide:
// per-lane atomics on it serialise a whole kernel).  Lanes of a wave that
// reach the call together get consecutive slots in lane order.
__device__ __forceinline__ uint32_t wave_alloc1(uint32_t* counter) {
	const uint64_t m = __ballot(1);
	const uint32_t lane = threadIdx.x & 63u;
	const int leader = __builtin_ctzll(m);
	uint32_t base = 0;
	if((int)lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
	base = (uint32_t)__shfl((int)base, leader);
	return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}
