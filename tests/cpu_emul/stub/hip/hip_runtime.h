// tests/cpu_emul/stub/hip/hip_runtime.h -- TEST INFRASTRUCTURE ONLY.
// The few HIP names the backtrace kernel source uses, so that
// tests/cpu_emul/bt_emul.cpp can compile bowtie2-server_amd/csrc/sw_backtrace.hip
// unchanged with g++ and run its kernel body lane by lane on the CPU (to catch
// indexing faults before a GPU run).  Not a HIP implementation; never linked
// into the product.
#pragma once
#include <stdint.h>
#include <stddef.h>
#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __shared__ static
#define amdgpu_waves_per_eu(...) unused
struct dim3 { uint32_t x = 1, y = 1, z = 1; dim3(uint32_t a = 1, uint32_t b = 1, uint32_t c = 1) : x(a), y(b), z(c) {} };
struct uint4 { uint32_t x, y, z, w; };
struct int2 { int32_t x, y; };
struct uint2 { uint32_t x, y; };
inline uint2 make_uint2(uint32_t a, uint32_t b) { return uint2{a, b}; }
struct uint3v { uint32_t x = 0, y = 0, z = 0; };
inline uint4 make_uint4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return uint4{a, b, c, d}; }
inline int2 make_int2(int32_t a, int32_t b) { return int2{a, b}; }
extern thread_local uint3v threadIdx, blockIdx;
typedef void* hipStream_t;
typedef void* hipEvent_t;
typedef int hipError_t;
enum { hipSuccess = 0 };
enum { hipDeviceAttributeSharedMemPerBlockOptin = 0 };
enum { hipFuncAttributeMaxDynamicSharedMemorySize = 0 };
inline hipError_t hipGetDevice(int* d) { *d = 0; return hipSuccess; }
inline hipError_t hipDeviceGetAttribute(int* v, int, int) { *v = 65536; return hipSuccess; }
inline hipError_t hipFuncSetAttribute(const void*, int, int) { return hipSuccess; }
inline hipError_t hipGetLastError() { return hipSuccess; }
template <typename K, typename... A>
void emul_launch(K k, dim3 g, dim3 b, A... a) {
	for(uint32_t bx = 0; bx < g.x; bx++)
		for(uint32_t tx = 0; tx < b.x; tx++) {
			blockIdx.x = bx;
			threadIdx.x = tx;
			k(a...);
		}
}
#define hipLaunchKernelGGL(k, g, b, sh, st, ...) emul_launch(k, g, b, __VA_ARGS__)
// wave intrinsics for one lane at a time: the lane is its own wave
inline uint64_t __ballot(int pr) { return pr ? (1ull << threadIdx.x) : 0ull; }
inline int __ffsll(unsigned long long x) { return __builtin_ffsll((long long)x); }
inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
inline int __shfl(int v, int) { return v; }
inline uint32_t atomicAdd(uint32_t* a, uint32_t v) { const uint32_t o = *a; *a += v; return o; }
// (the LDS-resident variants need a whole workgroup: never launched here,
// bt_emul.cpp sets BT2G_BT_LDS_MAX=0; they only have to compile)
inline void __syncthreads() {}
#define HIP_DYNAMIC_SHARED(type, var) static type var[1];
// (fm_device.h's quad FM step, never called here: a lane is its own quad)
#define __builtin_amdgcn_mov_dpp(x, ctrl, rm, bm, bc) (x)
