// sw_pack.hip -- compacts the per-problem outputs of bt2g_sw_align_bt_dev for
// the host: the candidate lists, their fates and the edits of every
// alignment, each packed back to back in problem order, so a host caller
// copies what the problems produced instead of the capacity-sized slots
// (cap candidates and maxaln x maxedit edits per problem: ~26 KB per
// end-to-end DP, against ~0.3 KB used on average).
#include "bt2g_kernels.h"

namespace {

// per problem: {candidates, alignments, edits} actually produced
__global__ void k_pack_count(const bt2g_sw_result* __restrict__ res, const int32_t* __restrict__ naln,
                             const bt2g_sw_aln* __restrict__ alns, uint32_t n, uint32_t cap, uint32_t maxaln,
                             uint32_t maxedit, uint32_t* __restrict__ cnt) {
	const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
	if(p >= n) return;
	int32_t nc = res[p].ncand;
	nc = nc < 0 ? 0 : (nc > (int32_t)cap ? (int32_t)cap : nc);
	int32_t na = naln[p];
	na = na < 0 ? 0 : (na > (int32_t)maxaln ? (int32_t)maxaln : na);
	uint32_t ne = 0;
	for(int32_t k = 0; k < na; k++) {
		int32_t e = alns[(size_t)p * maxaln + k].nedit;
		ne += e < 0 ? 0u : (e > (int32_t)maxedit ? maxedit : (uint32_t)e);
	}
	cnt[3 * (size_t)p + 0] = (uint32_t)nc;
	cnt[3 * (size_t)p + 1] = (uint32_t)na;
	cnt[3 * (size_t)p + 2] = ne;
}

// exclusive scan of the three counts over all problems, one workgroup;
// off[3n .. 3n+2] = totals
__global__ void __launch_bounds__(1024) k_pack_scan(const uint32_t* __restrict__ cnt, uint32_t n,
                                                    uint32_t* __restrict__ off) {
	__shared__ uint32_t part[3][1024];
	const uint32_t t = threadIdx.x;
	const uint32_t per = (n + 1023u) / 1024u;
	const uint32_t lo = t * per, hi = min(n, lo + per);
	uint32_t s[3] = {0u, 0u, 0u};
	for(uint32_t p = lo; p < hi; p++)
		for(int k = 0; k < 3; k++) s[k] += cnt[3 * (size_t)p + k];
	for(int k = 0; k < 3; k++) part[k][t] = s[k];
	__syncthreads();
	// Hillis-Steele inclusive scan of the per-thread sums
	for(uint32_t d = 1; d < 1024u; d <<= 1) {
		uint32_t v[3];
		for(int k = 0; k < 3; k++) v[k] = t >= d ? part[k][t - d] : 0u;
		__syncthreads();
		for(int k = 0; k < 3; k++) part[k][t] += v[k];
		__syncthreads();
	}
	uint32_t run[3];
	for(int k = 0; k < 3; k++) run[k] = part[k][t] - s[k];
	for(uint32_t p = lo; p < hi; p++)
		for(int k = 0; k < 3; k++) {
			off[3 * (size_t)p + k] = run[k];
			run[k] += cnt[3 * (size_t)p + k];
		}
	if(t == 1023u)
		for(int k = 0; k < 3; k++) off[3 * (size_t)n + k] = part[k][1023];
}

// one wave per problem: its candidates (+ fates) and its alignments' edits
__global__ void k_pack_gather(const bt2g_sw_cand* __restrict__ cands, const int8_t* __restrict__ fates,
                              const bt2g_sw_aln* __restrict__ alns, const bt2g_edit* __restrict__ edits,
                              const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ off, uint32_t n,
                              uint32_t cap, uint32_t maxaln, uint32_t maxedit, bt2g_sw_cand* __restrict__ pc,
                              int8_t* __restrict__ pf, bt2g_edit* __restrict__ pe) {
	const uint32_t lane = threadIdx.x & 63u;
	const uint32_t p = blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u;
	if(p >= n) return;
	const uint32_t nc = cnt[3 * (size_t)p], na = cnt[3 * (size_t)p + 1];
	const uint32_t oc = off[3 * (size_t)p], oe0 = off[3 * (size_t)p + 2];
	for(uint32_t i = lane; i < nc; i += 64u) {
		pc[oc + i] = cands[(size_t)p * cap + i];
		if(fates) pf[oc + i] = fates[(size_t)p * cap + i];
	}
	uint32_t oe = oe0;
	for(uint32_t k = 0; k < na; k++) {
		int32_t e = alns[(size_t)p * maxaln + k].nedit;
		const uint32_t ne = e < 0 ? 0u : (e > (int32_t)maxedit ? maxedit : (uint32_t)e);
		const bt2g_edit* src = edits + ((size_t)p * maxaln + k) * maxedit;
		for(uint32_t i = lane; i < ne; i += 64u) pe[oe + i] = src[i];
		oe += ne;
	}
}

}  // namespace

void launch_sw_pack(const bt2g_sw_result* res, const int32_t* naln, const bt2g_sw_aln* alns,
                    const bt2g_sw_cand* cands, const int8_t* fates, const bt2g_edit* edits, uint32_t n, uint32_t cap,
                    uint32_t maxaln, uint32_t maxedit, uint32_t* cnt, uint32_t* off, bt2g_sw_cand* pc, int8_t* pf,
                    bt2g_edit* pe, hipStream_t st) {
	if(n == 0) return;
	hipLaunchKernelGGL(k_pack_count, dim3((n + 255u) / 256u), dim3(256), 0, st, res, naln, alns, n, cap, maxaln,
	                   maxedit, cnt);
	hipLaunchKernelGGL(k_pack_scan, dim3(1), dim3(1024), 0, st, cnt, n, off);
	hipLaunchKernelGGL(k_pack_gather, dim3((n + 3u) / 4u), dim3(256), 0, st, cands, fates, alns, edits, cnt, off, n,
	                   cap, maxaln, maxedit, pc, pf, pe);
}
