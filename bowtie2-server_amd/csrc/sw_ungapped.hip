// sw_ungapped.hip -- SwAligner::ungappedAlign (aligner_sw.cpp:286-494) for a
// batch of (read, strand, reference offset) problems: the seed-diagonal
// ungapped alignment SwDriver tries before framing a DP rectangle
// (aligner_sw_driver.cpp:1032-1073).
//
// One lane per problem; the read, its qualities and the reference diagonal are
// streamed through 16-byte register windows.  End-to-end: running score, stop
// as soon as it drops below minsc or the N count exceeds the ceiling (the
// score only falls); local: the reference's running maximum with a floor at 0,
// -1 when more than one disjoint solution reaches the maximum.  A second pass
// over [rowi, rowf] writes the mismatch edits in their final (5'->3',
// trimmed) positions.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "bt2g_kernels.h"

namespace {

__device__ __forceinline__ char ug_mask2dna(int code) { return "ACGTN"[code > 3 ? 4 : code]; }

struct Win16 {
	uint64_t a;
	uint4 w;
	// byte at p; [lo, hi) bounds the 16-B loads (single byte load outside)
	__device__ __forceinline__ int at(const uint8_t* p, const uint8_t* lo, const uint8_t* hi) {
		const uint64_t addr = (uint64_t)p, aa = addr & ~15ull;
		if(aa != a) {
			if(aa < (uint64_t)lo || aa + 16u > (uint64_t)hi) return *p;
			a = aa;
			w = *(const uint4*)(p - (addr & 15u));     // pointer provenance: global, not flat
		}
		const uint32_t di = (uint32_t)(addr >> 2) & 3u;
		const uint32_t d = di == 0 ? w.x : di == 1 ? w.y : di == 2 ? w.z : w.w;
		return (int)((d >> ((addr & 3u) * 8u)) & 0xffu);
	}
};

}  // namespace

__global__ void __launch_bounds__(64)
k_ungapped(const bt2g_ug_problem* __restrict__ probs, uint32_t n, const uint8_t* __restrict__ reads,
           const uint8_t* __restrict__ quals, uint32_t stride, const uint32_t* __restrict__ lens,
           const uint8_t* __restrict__ ref_codes, const uint64_t* __restrict__ ref_starts, SwConst C, int local,
           double ncl_const, double ncl_lin, int ohang, uint32_t maxedit, bt2g_ug_result* __restrict__ res,
           bt2g_edit* __restrict__ edits) {
	const uint32_t p = blockIdx.x * 64u + threadIdx.x;
	if(p >= n) return;
	const bt2g_ug_problem P = probs[p];
	const uint32_t len = lens[P.read];
	bt2g_ug_result out{};
	out.ret = 0;
	const bool fw = P.fw != 0;
	// Scoring::nCeil.f<int>(len) (simple_func.h:90-115)
	int32_t nceil;
	{
		double v = ncl_const + ncl_lin * (double)len;
		v = v < 0.0 ? 0.0 : v;
		nceil = v >= 2147483647.0 ? 2147483647 : (int32_t)v;
	}
	const uint64_t rs = ref_starts[P.refidx], reflen = ref_starts[P.refidx + 1] - rs;
	const int64_t rfi = P.off, rff = rfi + (int64_t)len;
	int64_t leftNs = 0, rightNs = 0;
	bool go = len > 0;
	if(rfi < 0) { if(!ohang) go = false; leftNs = -rfi; }
	if(rff > (int64_t)reflen) { if(!ohang) go = false; rightNs = rff - (int64_t)reflen; }
	if(go && leftNs + rightNs > nceil) go = false;
	if(!go) { res[p] = out; return; }
	const uint8_t* rd = reads + (size_t)P.read * stride;
	const uint8_t* qu = quals + (size_t)P.read * stride;
	const uint8_t* rf0 = ref_codes + rs;
	const uint8_t* rfhi = ref_codes + rs + reflen + 16u;   // bt2g_open pads the reference
	Win16 wr{~0ull, {}}, wq{~0ull, {}}, wf{~0ull, {}};
	auto rdc = [&](uint32_t i) -> int {
		const int c = wr.at(rd + (fw ? i : len - 1 - i), reads, rd + stride);
		return fw ? c : (c > 3 ? 4 : 3 - c);
	};
	auto qv = [&](uint32_t i) -> int {
		const int q = wq.at(qu + (fw ? i : len - 1 - i), quals, qu + stride) - 33;
		return q < 0 ? 0 : (q > 40 ? 40 : q);
	};
	auto rfc = [&](uint32_t i) -> int {   // reference code at rfi + i, 4 off the reference
		const int64_t o = rfi + (int64_t)i;
		if(o < 0 || o >= (int64_t)reflen) return 4;
		const int c = wf.at(rf0 + o, ref_codes, rfhi);
		return c > 3 ? 4 : c;
	};
	// Scoring::score(rdc, 1 << rf, q, ns) (scoring.h:258-269)
	int32_t score = 0, ns = 0;
	uint32_t rowi = 0, rowf = len - 1;
	auto sc1 = [&](int r, int f, int q) -> int32_t {
		if(r > 3 || f > 3) { ns++; return -C.npen; }
		return r == f ? C.match : -C.mmpen[q];
	};
	if(!local) {
		for(uint32_t i = 0; i < len; i++) {
			score += sc1(rdc(i), rfc(i), qv(i));
			if(score < P.minsc || ns > nceil) { res[p] = out; return; }
		}
	} else {
		int32_t scoreMax = 0;
		uint32_t lastfloor = 0, sols = 0;
		rowi = 0xffffffffu;
		for(uint32_t i = 0; i < len; i++) {
			score += sc1(rdc(i), rfc(i), qv(i));
			if(score >= P.minsc && score >= scoreMax) {
				scoreMax = score;
				rowf = i;
				if(rowi != lastfloor) { rowi = lastfloor; sols++; }
			}
			if(score <= 0) { score = 0; lastfloor = i + 1; }
		}
		if(ns > nceil || scoreMax < P.minsc) { res[p] = out; return; }
		if(sols > 1) { out.ret = -1; res[p] = out; return; }
		score = scoreMax;
	}
	// edits: mismatches and Ns in [rowi, rowf], counted first (the Crick order is reversed)
	uint32_t ned = 0;
	int32_t refns = 0;
	for(uint32_t i = rowi; i <= rowf; i++) {
		const int f = rfc(i);
		if(f > 3 || rdc(i) != f) { ned++; refns += f > 3; }
	}
	const uint32_t trimEnd = len - 1 - rowf, sz = len - rowi - trimEnd;
	bt2g_edit* ed = edits + (size_t)p * maxedit;
	uint32_t k = 0;
	for(uint32_t i = rowi; i <= rowf; i++) {
		const int f = rfc(i), r = rdc(i);
		if(f > 3 || r != f) {
			const uint32_t slot = fw ? k : ned - 1 - k;
			const uint32_t pos = fw ? i - rowi : sz - (i - rowi) - 1;
			if(slot < maxedit) ed[slot] = bt2g_edit{pos, 3, (uint8_t)ug_mask2dna(f), (uint8_t)"ACGTN"[r], 0};
			k++;
		}
	}
	out.ret = 1;
	out.score = score;
	out.refoff = rfi + (int64_t)rowi;
	out.ns = ns;
	out.refns = refns;
	out.nedit = (int32_t)ned;
	out.trim5p = (int32_t)(fw ? rowi : trimEnd);
	out.trim3p = (int32_t)(fw ? trimEnd : rowi);
	res[p] = out;
}

void launch_ungapped(const bt2g_ug_problem* probs, uint32_t n, const uint8_t* reads, const uint8_t* quals,
                     uint32_t stride, const uint32_t* lens, const uint8_t* ref_codes, const uint64_t* ref_starts,
                     const SwConst& C, int local, double ncl_const, double ncl_lin, int ohang, uint32_t maxedit,
                     bt2g_ug_result* res, bt2g_edit* edits, hipStream_t st) {
	if(n == 0) return;
	hipLaunchKernelGGL(k_ungapped, dim3((n + 63u) / 64u), dim3(64), 0, st, probs, n, reads, quals, stride, lens,
	                   ref_codes, ref_starts, C, local, ncl_const, ncl_lin, ohang, maxedit, res, edits);
}
