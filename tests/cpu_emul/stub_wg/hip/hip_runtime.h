// tests/cpu_emul/stub_wg/hip/hip_runtime.h -- TEST INFRASTRUCTURE ONLY.
// The HIP names the workgroup backtrace kernel (sw_backtrace_wg.hip) uses, for
// tests/cpu_emul/wg_emul.cpp: a workgroup runs as 64 host threads (one per
// lane) with a barrier for __syncthreads and the cross-lane shuffles done
// through a shared exchange array, so the kernel's cooperative phases run as
// they would on a wave.  Not a HIP implementation; never linked into the product.
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>
#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __launch_bounds__(...)
struct dim3 { uint32_t x = 1, y = 1, z = 1; dim3(uint32_t a = 1, uint32_t b = 1, uint32_t c = 1) : x(a), y(b), z(c) {} };
struct uint4 { uint32_t x, y, z, w; };
struct uint3v { uint32_t x = 0, y = 0, z = 0; };
inline uint4 make_uint4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return uint4{a, b, c, d}; }
extern thread_local uint3v threadIdx, blockIdx;
typedef void* hipStream_t;
typedef void* hipEvent_t;
// (sw_bt_wg_lds_limit: the emulation keeps the 64 KiB default)
typedef int hipError_t;
enum { hipSuccess = 0 };
enum { hipDeviceAttributeSharedMemPerBlockOptin = 0 };
enum { hipFuncAttributeMaxDynamicSharedMemorySize = 0 };
inline hipError_t hipGetDevice(int* d) { *d = 0; return hipSuccess; }
inline hipError_t hipDeviceGetAttribute(int* v, int, int) { *v = 65536; return hipSuccess; }
inline hipError_t hipFuncSetAttribute(const void*, int, int) { return hipSuccess; }
inline hipError_t hipGetLastError() { return hipSuccess; }
struct int2 { int32_t x, y; };
struct uint2 { uint32_t x, y; };

// one workgroup's shared state
struct EmulGroup {
	uint32_t n = 0;
	std::atomic<uint32_t> arrived{0}, gen{0};
	std::vector<uint8_t> lds;
	int32_t xchg[64];
	void barrier() {
		// (spin with yields: far fewer futex round trips than a condition variable)
		const uint32_t g = gen.load(std::memory_order_acquire);
		if(arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == n) {
			arrived.store(0, std::memory_order_relaxed);
			gen.store(g + 1, std::memory_order_release);
		} else {
			while(gen.load(std::memory_order_acquire) == g) std::this_thread::yield();
		}
	}
};
extern thread_local EmulGroup* t_group;
inline void __syncthreads() { t_group->barrier(); }
inline int __shfl_xor(int v, int o, int w = 64) {
	(void)w;
	t_group->xchg[threadIdx.x] = v;
	t_group->barrier();
	const int r = t_group->xchg[threadIdx.x ^ (uint32_t)o];
	t_group->barrier();
	return r;
}
inline int __shfl_up(int v, int o, int w = 64) {
	(void)w;
	t_group->xchg[threadIdx.x] = v;
	t_group->barrier();
	const int r = threadIdx.x >= (uint32_t)o ? t_group->xchg[threadIdx.x - (uint32_t)o] : v;
	t_group->barrier();
	return r;
}
inline uint32_t atomicOr(uint32_t* a, uint32_t v) { return __atomic_fetch_or(a, v, __ATOMIC_SEQ_CST); }
#define HIP_DYNAMIC_SHARED(type, var) type* var = (type*)t_group->lds.data();

template <typename K, typename... A>
void emul_launch(K k, dim3 g, dim3 b, size_t sh, A... a) {
	for(uint32_t bx = 0; bx < g.x; bx++) {
		EmulGroup grp;
		grp.n = b.x;
		grp.lds.assign(sh + 16, 0xcd);           // garbage: the kernel must initialise what it reads
		std::vector<std::thread> th;
		for(uint32_t tx = 0; tx < b.x; tx++)
			th.emplace_back([&, bx, tx] {
				blockIdx.x = bx;
				threadIdx.x = tx;
				t_group = &grp;
				k(a...);
			});
		for(auto& t : th) t.join();
	}
}
#define hipLaunchKernelGGL(k, g, b, sh, st, ...) emul_launch(k, g, b, sh, __VA_ARGS__)
// (fm_device.h's quad FM step, never called here: a lane is its own quad)
#define __builtin_amdgcn_mov_dpp(x, ctrl, rm, bm, bc) (x)
