// frame.hip -- DP rectangle framing (row A14) on the device: the seed-extension
// rectangle of DynProgFramer::frameSeedExtensionRect (dp_framer.cpp:81-129)
// and the mate-search rectangle of PairedEndPolicy::otherMate (pe.cpp:161-352)
// + DynProgFramer::frameFindMateRect (dp_framer.h:155-197,
// dp_framer.cpp:177-383), with the gap budgets of Scoring::maxReadGaps /
// maxRefGaps (scoring.cpp:42-98).
//
// One thread per rectangle; pure integer arithmetic written with the
// reference's own operand types (size_t / int64_t mixes included), so that
// even out-of-range inputs (a minsc above the perfect score gives a gap
// budget of -1, i.e. SIZE_MAX once it meets size_t) wrap exactly as the
// reference's do.  The output is a bt2g_sw_problem (the DP's reference window
// [rect.refl, rect.refr]) plus the DPRect fields the backtrace reads.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "bt2g_kernels.h"

namespace {

// Scoring::maxReadGaps (scoring.cpp:42-66): matches turned into read gaps
// until the perfect score drops below minsc
__device__ __forceinline__ int max_read_gaps(const FrameConst& F, int64_t minsc, size_t rdlen) {
	int64_t sc = (int64_t)(rdlen * (size_t)F.match);
	bool first = true;
	int num = 0;
	while(sc >= minsc) {
		sc -= first ? F.rdgo : F.rdge;
		first = false;
		num++;
	}
	return num - 1;
}

// Scoring::maxRefGaps (scoring.cpp:73-98): each reference gap also loses a match
__device__ __forceinline__ int max_ref_gaps(const FrameConst& F, int64_t minsc, size_t rdlen) {
	int64_t sc = (int64_t)(rdlen * (size_t)F.match);
	bool first = true;
	int num = 0;
	while(sc >= minsc) {
		sc -= F.match;
		sc -= first ? F.rfgo : F.rfge;
		first = false;
		num++;
	}
	return num - 1;
}

struct Rect {
	int64_t refl, refr;
	size_t triml, trimr, maxgap, corel, corer;
};

// the trimming common to every framer: columns past the reference ends beyond
// the N budget are cut (dp_framer.cpp:104-118, 226-236, 339-349)
__device__ __forceinline__ void trim_rect(Rect& R, int64_t refl, int64_t refr, int64_t reflen, int64_t maxns,
                                          size_t rdlen, bool trim_to_ref) {
	size_t triml = 0, trimr = 0;
	if(trim_to_ref) maxns = 0;
	else if(maxns == (int64_t)rdlen) maxns--;
	if(refr >= reflen + maxns) trimr = (size_t)(refr - (reflen + maxns - 1));
	if(refl < -maxns) triml = (size_t)(-refl) - (size_t)maxns;
	R.refl = refl + (int64_t)triml;
	R.refr = refr - (int64_t)trimr;
	R.triml = triml;
	R.trimr = trimr;
}

// DynProgFramer::frameSeedExtensionRect (dp_framer.cpp:81-129)
__device__ bool frame_seed_ext(int64_t off, size_t rdlen, int64_t reflen, size_t maxrdgap, size_t maxrfgap,
                               int64_t maxns, size_t maxhalf, bool trim_to_ref, Rect& R) {
	size_t maxgap = maxrdgap > maxrfgap ? maxrdgap : maxrfgap;
	maxgap = maxgap < maxhalf ? maxgap : maxhalf;
	const int64_t refl = off - 2 * maxgap;
	const int64_t refr = off + (rdlen - 1) + 2 * maxgap;
	trim_rect(R, refl, refr, reflen, maxns, rdlen, trim_to_ref);
	R.maxgap = maxgap;
	R.corel = maxgap;
	R.corer = R.corel + 2 * maxgap;
	return !(R.refr < R.refl);   // DPRect::entirelyTrimmed (dp_framer.h:100-105)
}

// DynProgFramer::frameFindMateAnchorLeftRect / AnchorRightRect
// (dp_framer.cpp:177-289, 291-383): the rectangle spans the diagonals on which
// the opposite mate may end (anchor left) or start (anchor right), padded by
// max(maxgap, maxhalf) on both sides; those diagonals are the core ones
__device__ bool frame_mate(bool anchor_left, int64_t ll, int64_t lr, int64_t rl, int64_t rr, size_t rdlen,
                           int64_t reflen, size_t maxrdgap, size_t maxrfgap, int64_t maxns, size_t maxhalf,
                           bool trim_to_ref, Rect& R) {
	size_t maxgap = maxrdgap > maxrfgap ? maxrdgap : maxrfgap;
	maxgap = maxgap > maxhalf ? maxgap : maxhalf;
	const int64_t pad_left = maxgap, pad_right = maxgap;
	int64_t st_left, en_right;
	if(anchor_left) {
		st_left = rl - (rdlen - 1);
		en_right = rr;
	} else {
		st_left = ll;
		en_right = lr + (rdlen - 1);
	}
	const int64_t refl = st_left - pad_left;
	const int64_t refr = en_right + pad_right;
	trim_rect(R, refl, refr, reflen, maxns, rdlen, trim_to_ref);
	const size_t width = (size_t)(refr - refl + 1);
	R.maxgap = maxgap;
	R.corel = maxgap;
	R.corer = width - maxgap - 1;
	return !(R.refr < R.refl);
}

// pePolicyMateDir (pe.h:130-164)
__device__ __forceinline__ void mate_dir(int policy, bool is1, bool fw, bool& left, bool& mfw) {
	switch(policy) {
	case 1: left = is1 != fw; mfw = fw; break;      // PE_POLICY_FF
	case 2: left = is1 == fw; mfw = fw; break;      // PE_POLICY_RR
	case 3: left = !fw; mfw = !fw; break;           // PE_POLICY_FR
	default: left = fw; mfw = !fw; break;           // PE_POLICY_RF
	}
}

// PairedEndPolicy::otherMate (pe.cpp:161-352): where the opposite mate's
// leftmost (oll..olr) and rightmost (orl..orr) reference characters may fall
__device__ bool other_mate(const bt2g_pe_policy& P, bool is1, bool fw, int64_t off, int64_t maxalcols,
                           size_t len1, size_t len2, bool& oleft, int64_t& oll, int64_t& olr, int64_t& orl,
                           int64_t& orr, bool& ofw) {
	mate_dir(P.policy, is1, fw, oleft, ofw);
	const size_t alen = is1 ? len1 : len2;
	size_t maxfrag = (size_t)P.maxfrag, minfrag = (size_t)P.minfrag;
	if(minfrag < 1) minfrag = 1;
	if(len1 > maxfrag && P.expand) maxfrag = len1;
	if(len2 > maxfrag && P.expand) maxfrag = len2;
	if(!P.expand && (len1 > maxfrag || len2 > maxfrag)) return false;
	if(oleft) {
		oll = off + alen - maxfrag;
		olr = off + alen - minfrag;
		orl = oll;
		orr = off + maxfrag - 1;
		if(!P.olap) {
			orr = orr < off - 1 ? orr : off - 1;
			if(orr < olr) olr = orr;
		} else if(!P.dovetail) {
			const int64_t lim = off + alen - 1;
			orr = orr < lim ? orr : lim;
		} else if(!P.flip && maxalcols != -1) {
			const int64_t lim = off + alen - 1 + (maxalcols - 1);
			orr = orr < lim ? orr : lim;
		}
	} else {
		orr = off + (maxfrag - 1);
		orl = off + (minfrag - 1);
		oll = off + alen - maxfrag;
		olr = orr;
		if(!P.olap) {
			const int64_t lim = off + alen;
			oll = oll > lim ? oll : lim;
			if(oll > orl) orl = oll;
		} else if(!P.dovetail) {
			oll = oll > off ? oll : off;
		} else if(!P.flip && maxalcols != -1) {
			const int64_t lim = off - maxalcols + 1;
			oll = oll > lim ? oll : lim;
		}
	}
	return true;
}

__global__ void __launch_bounds__(256)
k_frame_rect(const bt2g_frame_in* __restrict__ in, uint32_t n, const uint32_t* __restrict__ lens,
        const uint64_t* __restrict__ ref_starts, FrameConst F, bt2g_pe_policy P, bt2g_sw_problem* __restrict__ probs,
        bt2g_sw_rect* __restrict__ rects, int32_t* __restrict__ ok) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= n) return;
	const bt2g_frame_in x = in[i];
	const size_t rdlen = lens[x.read];
	const int64_t tlen = (int64_t)(ref_starts[x.refidx + 1] - ref_starts[x.refidx]);
	// nceil = min(nCeil.f<int>(len), len) (bt2_search.cpp multiseedSearchWorker;
	// simple_func.h:90-115: linear, floor 0)
	double v = F.ncl_const + F.ncl_lin * (double)rdlen;
	v = v < 0.0 ? 0.0 : v;
	int nceil = v >= 2147483647.0 ? 2147483647 : (int)v;
	nceil = nceil < (int)rdlen ? nceil : (int)rdlen;
	const int rdgaps = max_read_gaps(F, x.minsc, rdlen), rfgaps = max_ref_gaps(F, x.minsc, rdlen);
	Rect R{};
	bool found, fw = x.fw != 0;
	if(x.kind == 0) {
		found = frame_seed_ext(x.off, rdlen, tlen, (size_t)rdgaps, (size_t)rfgaps, (int64_t)(size_t)nceil,
		                       (size_t)F.maxhalf, F.trim_to_ref != 0, R);
	} else {
		bool oleft = false, ofw = false;
		int64_t oll = 0, olr = 0, orl = 0, orr = 0;
		const size_t alen = x.alen;
		found = other_mate(P, x.anchor1 != 0, fw, x.off, (int64_t)rdlen + rdgaps, x.anchor1 ? alen : rdlen,
		                   x.anchor1 ? rdlen : alen, oleft, oll, olr, orl, orr, ofw);
		if(found)
			found = frame_mate(!oleft, oll, olr, orl, orr, rdlen, tlen, (size_t)rdgaps, (size_t)rfgaps,
			                   (int64_t)(size_t)nceil, (size_t)F.maxhalf, F.trim_to_ref != 0, R);
		fw = ofw;
	}
	ok[i] = found ? 1 : 0;
	bt2g_sw_problem p{};
	p.read = x.read;
	p.fw = fw ? 1 : 0;
	p.refl = R.refl;
	p.win_off = -1;
	p.refidx = x.refidx;
	p.ncol = found ? (uint32_t)(R.refr - R.refl + 1) : 0u;
	p.minsc = x.minsc;
	probs[i] = p;
	rects[i] = bt2g_sw_rect{(int32_t)R.triml, (int32_t)R.corel, (int32_t)R.corer, 0};
}

}  // namespace

void launch_frame(const bt2g_frame_in* in, uint32_t n, const uint32_t* lens, const uint64_t* ref_starts,
                  const FrameConst& F, const bt2g_pe_policy& P, bt2g_sw_problem* probs, bt2g_sw_rect* rects,
                  int32_t* ok, hipStream_t st) {
	if(n == 0) return;
	hipLaunchKernelGGL(k_frame_rect, dim3((n + 255u) / 256u), dim3(256), 0, st, in, n, lens, ref_starts, F, P, probs,
	                   rects, ok);
}
