// Issue rate of the integer VALU forms the SW cell can be written in (gfx950).
// Eight independent chains per lane, inline asm so nothing folds.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define N_ITERS 2048
#define BODY(INS)                                                                              \
	for(int it = 0; it < N_ITERS; it++) {                                                      \
		asm volatile(INS " %0, %0, %8\n" INS " %1, %1, %8\n" INS " %2, %2, %8\n" INS " %3, %3, %8\n" \
		             INS " %4, %4, %8\n" INS " %5, %5, %8\n" INS " %6, %6, %8\n" INS " %7, %7, %8\n" \
		             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
		             : "v"(b));                                                                 \
	}
#define BODY3(INS)                                                                             \
	for(int it = 0; it < N_ITERS; it++) {                                                      \
		asm volatile(INS " %0, %0, %8, %9\n" INS " %1, %1, %8, %9\n" INS " %2, %2, %8, %9\n" INS " %3, %3, %8, %9\n" \
		             INS " %4, %4, %8, %9\n" INS " %5, %5, %8, %9\n" INS " %6, %6, %8, %9\n" INS " %7, %7, %8, %9\n" \
		             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
		             : "v"(b), "v"(c));                                                         \
	}
#define KERNEL(NAME, STMT)                                                                     \
	__global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {               \
		uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, \
		         a6 = a0 * 17, a7 = a0 * 19;                                                     \
		uint32_t b = seed ^ 0x00050003u, c = 0x0c010c05u;                                        \
		(void)c;                                                                                 \
		STMT;                                                                                    \
		out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;       \
	}
KERNEL(k_pk_max_u16, BODY("v_pk_max_u16"))
KERNEL(k_pk_sub_u16, BODY("v_pk_sub_u16"))
KERNEL(k_pk_add_u16, BODY("v_pk_add_u16"))
KERNEL(k_pk_max_i16, BODY("v_pk_max_i16"))
KERNEL(k_max_u32, BODY("v_max_u32"))
KERNEL(k_add_u32, BODY("v_add_u32"))
KERNEL(k_sub_u32, BODY("v_sub_u32"))
KERNEL(k_max_u16, BODY("v_max_u16"))
KERNEL(k_and_b32, BODY("v_and_b32"))
KERNEL(k_perm_b32, BODY3("v_perm_b32"))
KERNEL(k_max3_u32, BODY3("v_max3_u32"))
KERNEL(k_bfe_u32, BODY3("v_bfe_u32"))
KERNEL(k_sub_u32_clamp, for(int it = 0; it < N_ITERS; it++) { asm volatile("v_sub_u32_e64 %0, %0, %8 clamp\nv_sub_u32_e64 %1, %1, %8 clamp\nv_sub_u32_e64 %2, %2, %8 clamp\nv_sub_u32_e64 %3, %3, %8 clamp\nv_sub_u32_e64 %4, %4, %8 clamp\nv_sub_u32_e64 %5, %5, %8 clamp\nv_sub_u32_e64 %6, %6, %8 clamp\nv_sub_u32_e64 %7, %7, %8 clamp\n" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b)); })
KERNEL(k_pk_sub_u16_clamp, for(int it = 0; it < N_ITERS; it++) { asm volatile("v_pk_sub_u16 %0, %0, %8 clamp\nv_pk_sub_u16 %1, %1, %8 clamp\nv_pk_sub_u16 %2, %2, %8 clamp\nv_pk_sub_u16 %3, %3, %8 clamp\nv_pk_sub_u16 %4, %4, %8 clamp\nv_pk_sub_u16 %5, %5, %8 clamp\nv_pk_sub_u16 %6, %6, %8 clamp\nv_pk_sub_u16 %7, %7, %8 clamp\n" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b)); })

typedef void (*KF)(uint32_t*, uint32_t);
int main() {
	uint32_t* d;
	const int blocks = 256 * 8 * 4, threads = 256;
	(void)hipMalloc(&d, sizeof(uint32_t) * blocks * threads);
	hipEvent_t e0, e1;
	(void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
	struct { const char* n; KF f; } ks[] = {
		{"v_pk_max_u16", k_pk_max_u16}, {"v_pk_sub_u16", k_pk_sub_u16}, {"v_pk_sub_u16 clamp", k_pk_sub_u16_clamp},
		{"v_pk_add_u16", k_pk_add_u16}, {"v_pk_max_i16", k_pk_max_i16}, {"v_max_u32", k_max_u32},
		{"v_add_u32", k_add_u32}, {"v_sub_u32", k_sub_u32}, {"v_sub_u32 clamp", k_sub_u32_clamp},
		{"v_max_u16", k_max_u16}, {"v_and_b32", k_and_b32}, {"v_perm_b32", k_perm_b32},
		{"v_max3_u32", k_max3_u32}, {"v_bfe_u32", k_bfe_u32}};
	for(auto& k : ks) {
		float best = 1e9f;
		for(int rep = 0; rep < 3; rep++) {
			(void)hipEventRecord(e0);
			hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 7u);
			(void)hipEventRecord(e1);
			(void)hipEventSynchronize(e1);
			float ms;
			(void)hipEventElapsedTime(&ms, e0, e1);
			if(rep && ms < best) best = ms;
		}
		double ops = (double)blocks * threads * N_ITERS * 8;
		printf("%-20s %8.3f ms  %8.1f G lane-ops/s\n", k.n, best, ops / best / 1e6);
	}
	return 0;
}
