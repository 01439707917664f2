// fm_one_mm.hip -- SeedAligner::oneMmSearch (aligner_seed.cpp:973-1323) with
// rep1mm=true, repex=false.
//
// A work item is one (read, strand, index direction) the reference would run
// (k_one_mm_items applies the exact-sweep gate of bt2_search.cpp:3640-3667 and
// the "at most one N" rule and splits the items by index direction, so each
// launch walks one index with wave-uniform parameters).  Each lane runs a
// small state machine over its item -- near half exact, far half with one
// mismatch, one branch walk per alternative base -- performing exactly one LF
// operation (one or two 64-B side gathers) per loop iteration, so lanes in
// different phases still issue their gathers together.  A far-half
// alternative that survives its mismatch step is not walked in place: it goes
// to a global branch queue (k_one_mm_branch walks every queued branch in its
// own lane), so an item in a high-copy repeat -- thousands of LF steps of
// branch walks one after another in the reference -- no longer holds its wave
// for the whole kernel (hg38-like genome: p50 161 but max 16 379 LF ops per
// read).  Each candidate carries its discovery number; hits land in per-item
// slots in completion order and k_one_mm_compact restores the reference's
// order and concatenates the four slots of a read in its loop order
// (fw/BWT, fw/BWT', rc/BWT, rc/BWT').
#include "fm_device.h"
#include "bt2g_kernels.h"
#include "dev_util.h"


namespace {

__device__ __forceinline__ int mmpen_q(const MmParams& p, int q) {
	int ii = q < 40 ? q : 40;
	float frac = (float)ii / 40.0f;
	return p.mmp_min + (int)(frac * (float)(p.mmp_max - p.mmp_min));
}

enum : int { ST_IDLE = 0, ST_FAR, ST_ALT, ST_BR, ST_DONE };

// Local mode: the alignment with its one mismatch at depth `dep` is valid iff
// the running scores from either end stay positive (aligner_seed.cpp:1166-1290
// scans both ends of the read).  Every other position matches (+match), so
// only the mismatch's own step can take a sum to <= 0: an O(1) test for the
// O(len) scan, which had made the local 1-mm search 4.5x the end-to-end one.
__device__ __forceinline__ bool local_ok(uint32_t dep, uint32_t len, int64_t matchsc, int pen) {
	return (int64_t)dep * matchsc + pen > 0 && (int64_t)(len - 1u - dep) * matchsc + pen > 0;
}

// register-array access by a data-dependent index without going through scratch
__device__ __forceinline__ uint32_t at4(const uint32_t a[4], int i) {
	uint32_t x0 = a[0], x1 = a[1], x2 = a[2], x3 = a[3];
	asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));   // the compiler would index a stack copy
	return i == 0 ? x0 : i == 1 ? x1 : i == 2 ? x2 : x3;
}
__device__ __forceinline__ void set4(uint32_t a[4], int i, uint32_t v) {
#pragma unroll
	for(int k = 0; k < 4; k++) a[k] = i == k ? v : a[k];
}

}  // namespace

// Work lists: item = read << 3 | fwi << 2 | ebwtfwi << 1 | (read has an N);
// items[0..2n) for the BWT, items[2n..4n) for BWT'; nitems[0], nitems[2] their lengths.
__global__ void __launch_bounds__(256)
k_one_mm_items(const uint8_t* __restrict__ reads, uint32_t stride, const uint32_t* __restrict__ lens, uint32_t n,
               const uint32_t* __restrict__ gate, int nofw, int norc, uint32_t* __restrict__ items,
               uint32_t* __restrict__ nitems, int32_t* __restrict__ slot_counts, uint32_t* __restrict__ ops,
               uint32_t* __restrict__ loads, uint32_t* __restrict__ slot_flag) {
	// one wave of 64 reads: their rows are contiguous, so the Ns are counted
	// from coalesced dword loads (N = code 4: bit 2 of a byte) into per-read
	// LDS counters
	__shared__ uint32_t ncount_s[256], lens_s[256];
	const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t lane = threadIdx.x & 63u;
	const uint32_t r0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63u);   // this wave's first read
	const uint32_t nr = r0 >= n ? 0u : (n - r0 < 64u ? n - r0 : 64u);
	uint32_t* ncount = ncount_s + (threadIdx.x & ~63u);
	uint32_t* lenS = lens_s + (threadIdx.x & ~63u);
	ncount[lane] = 0;
	lenS[lane] = r < n ? lens[r] : 0u;
	__syncthreads();
	{
		const uint8_t* src = reads + (size_t)r0 * stride;
		const uint32_t bytes = nr * stride;
		const uint32_t head = (uint32_t)((4u - ((uintptr_t)src & 3u)) & 3u);   // bytes before a dword boundary
		// byte o of the wave's rows is an N of read o/stride iff inside its length
		auto add_byte = [&](uint32_t o, uint32_t code) {
			const uint32_t rr = o / stride;
			if(code > 3 && o - rr * stride < lenS[rr]) atomicAdd(&ncount[rr], 1u);
		};
		if(lane < head && lane < bytes) add_byte(lane, src[lane]);
		const uint32_t* src32 = reinterpret_cast<const uint32_t*>(src + head);
		const uint32_t nw = bytes > head ? (bytes - head) / 4u : 0u;
		for(uint32_t w = lane; w < nw; w += 64u) {
			const uint32_t v = src32[w];
			if(!(v & 0x04040404u)) continue;
			const uint32_t o = head + 4u * w, rr = o / stride;
			if(rr == (o + 3) / stride && o + 3 - rr * stride < lenS[rr]) {
				atomicAdd(&ncount[rr], (uint32_t)__popc(v & 0x04040404u));
			} else {
				for(uint32_t k = 0; k < 4; k++) add_byte(o + k, (v >> (8 * k)) & 0xffu);
			}
		}
		for(uint32_t o = head + 4u * nw + lane; o < bytes; o += 64u) add_byte(o, src[o]);
	}
	__syncthreads();
	uint32_t runmask = 0, ns = 0;
	if(r < n) {
		ns = ncount[lane];
		const bool nofw1 = (nofw & 1) != 0, keep_exact = (nofw & MM_GATE_KEEP_EXACT) != 0;
		bool nofw_r = nofw1, norc_r = norc, gated_off = false;
		if(gate) {
			// bt2_search.cpp:3476-3506, 3640-3667: skipped when an exact end-to-end hit
			// exists (bestmin == 0; not with MM_GATE_KEEP_EXACT); otherwise nofw =
			// !(mineFw <= 1), norc = !(mineRc <= 1)
			const uint32_t mfw = gate[(size_t)r * 8 + 0], mrc = gate[(size_t)r * 8 + 1];
			const uint32_t bestmin = mfw < mrc ? mfw : mrc;
			const bool yfw = mfw <= 1 && !nofw1, yrc = mrc <= 1 && !norc;
			gated_off = (bestmin == 0 && !keep_exact) || !(yfw || yrc);
			nofw_r = !yfw;
			norc_r = !yrc;
		}
		for(int d = 0; d < 4; d++) {
			const bool fw = (d >> 1) == 0;
			if(!gated_off && ns <= 1 && !((fw && nofw_r) || (!fw && norc_r))) runmask |= 1u << d;
			slot_counts[(size_t)r * 4 + d] = 0;
			slot_flag[(size_t)r * 4 + d] = 0;
		}
		// the read's FM-op and side-load counters, accumulated by the walks after
		// this kernel (were three memsets of the call's stream)
		ops[r] = 0;
		if(loads) loads[r] = 0;
	}
	// two lists by index direction (BWT: d even, BWT': d odd) so that each
	// search launch reads one index with wave-uniform parameters
	for(uint32_t li = 0; li < 2; li++) {
		const uint32_t want = ((runmask >> li) & 1u) + ((runmask >> (li + 2)) & 1u);
		uint32_t pos = block_alloc<256>(want, &nitems[2 * li]);
		for(uint32_t d = li; d < 4; d += 2)
			if((runmask >> d) & 1u) items[(size_t)li * 2 * n + pos++] = (r << 3) | (d << 1) | (ns ? 1u : 0u);
	}
}

// Near half (aligner_seed.cpp:1003-1110): ftab jump and exact bidirectional
// steps over the half of the read nearest the index's starting end.  One lane
// per item, lean state (it is most of the LF work and runs at high occupancy);
// the surviving range (+ mirror) and depth go to the far-half kernel.
template <bool EBWTFW>
__device__ __forceinline__ void one_mm_near_body(const uint32_t blk_, DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, uint32_t stride,
              const uint32_t* __restrict__ lens, const uint32_t* __restrict__ items,
              const uint32_t* __restrict__ nitems_p, uint4* __restrict__ st4, uint32_t* __restrict__ sdep,
              uint32_t* __restrict__ ops_out, uint32_t* __restrict__ loads_out) {
	walk_prio();
	const uint32_t qi = blk_ * blockDim.x + threadIdx.x;
	if(qi >= *nitems_p) return;
	const DevEbwt& E = EBWTFW ? F : B;
	const DevEbwt& Ep = EBWTFW ? B : F;
	const uint32_t item = items[qi];
	const uint32_t r = item >> 3;
	const bool fw = ((item >> 2) & 1u) == 0;
	const uint32_t len = lens[r];
	// seq = fw ? (ebwtfw ? patFw : patFwRev) : (ebwtfw ? patRc : patRcRev)
	const SeqView seq{reads + (size_t)r * stride, len, fw ? !EBWTFW : EBWTFW, !fw};
	const uint32_t nea = EBWTFW ? (len >> 1) : (len >> 1) + (len & 1);
	const uint32_t flen = E.ftab_chars;
	uint32_t top = 0, bot = 0, topp = 0, botp = 0, dep = 0, ops = 0, loads = 0;
	bool alive = len != 0;
	if(item & 1u)                               // the read has an N: none may be in the near half
		for(uint32_t d = 0; alive && d < nea; d++)
			if(seq[len - d - 1] > 3) alive = false;
	if(alive) {
		if(flen > 1 && flen <= nea) {
			// ftabSeqToInt(seq, len-flen, rev=!ebwtfw) (bt2_idx.h:1383-1390)
			uint32_t fi = 0, fip = 0;
			for(uint32_t i = 0; i < flen; i++) {
				fi = (fi << 2) | (uint32_t)seq[len - flen + i];
				fip = (fip << 2) | (uint32_t)seq[len - 1 - i];
			}
			top = ftab_hi(E, fi); bot = ftab_lo(E, fi + 1);
			topp = ftab_hi(Ep, fip); botp = ftab_lo(Ep, fip + 1);
			dep = flen;
		} else {
			const int c = seq[len - 1];
			top = topp = fchr_at(E, c);
			bot = botp = fchr_at(E, c + 1);
			dep = 1;
		}
		alive = bot != top;
	}
	SeqWin sw{seq, ReadWin{seq.p, seq.p + stride}};
	while(alive && dep < nea) {
		const int c = sw[len - dep - 1];
		ops++;
		if(bot - top > 1) {
			uint32_t t[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0}, tp[4], bp[4];
			tp[0] = topp;
			loads += bi_step(E, top, bot, topp, t, b, tp, bp);
			const uint32_t nt = at4(t, c), nb = at4(b, c);
			if(nb <= nt) { alive = false; break; }
			top = nt; bot = nb; topp = at4(tp, c); botp = at4(bp, c);
		} else {
			SideData s1;
			load_side(E, top / 192u, s1);
			loads++;
			if(side_rowL(s1, top % 192u) != c || top == E.zoff) { alive = false; break; }
			top = occ1(E, s1, top, c);
			bot = top + 1;
		}
		dep++;
	}
	st4[qi] = alive ? make_uint4(top, bot, topp, botp) : make_uint4(0, 0, 0, 0);
	sdep[qi] = dep | (alive ? 0x80000000u : 0u);
	if(ops) atomicAdd(&ops_out[r], ops);
	if(ops && loads_out) atomicAdd(&loads_out[r], loads);
}

template <bool EBWTFW>
__global__ void __launch_bounds__(256)
k_one_mm_near(DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, uint32_t stride,
              const uint32_t* __restrict__ lens, const uint32_t* __restrict__ items,
              const uint32_t* __restrict__ nitems_p, uint4* __restrict__ st4, uint32_t* __restrict__ sdep,
              uint32_t* __restrict__ ops_out, uint32_t* __restrict__ loads_out) {
	one_mm_near_body<EBWTFW>(blockIdx.x, F, B, reads, stride, lens, items, nitems_p, st4, sdep, ops_out, loads_out);
}

#ifndef BT2G_MM_WAVES
#define BT2G_MM_WAVES 3
#endif
template <bool EBWTFW>
__device__ __forceinline__ void one_mm_q_body(const uint32_t blk_, uint32_t (*alt_s)[256], DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, const uint8_t* __restrict__ quals,
           uint32_t stride, const uint32_t* __restrict__ lens, const int32_t* __restrict__ minscs, MmParams P,
           double ncl_const, double ncl_lin, const uint32_t* __restrict__ items,
           const uint32_t* __restrict__ nitems_p, const uint4* __restrict__ st4,
           const uint32_t* __restrict__ sdep, uint32_t cap, bt2g_mm1* __restrict__ slots, int32_t* __restrict__ slot_counts, uint32_t* __restrict__ ops_out,
           uint32_t* __restrict__ loads_out, MmBranch* __restrict__ brq, uint32_t* __restrict__ brq_n,
           uint32_t brq_cap) {
	walk_prio();
	const uint32_t nitems = *nitems_p;
	const int64_t matchsc = (int64_t)((float)P.match + 0.5f);

	// per-lane item state
	int st = ST_IDLE;
	uint32_t r = 0, len = 0, slot = 0, dep = 0, depm = 0;
	constexpr bool ebwtfw = EBWTFW;
	const DevEbwt& E = EBWTFW ? F : B;          // the index walked (uniform)
	bool fw = true, hasn = false;
	int nceil = 0;
	int64_t minsc = 0;
	const uint8_t* rd = reads;
	const uint8_t* qd = quals;
	SeqView seq{reads, 0, false, false};
	bool qrev = false;
	uint32_t top = 0, bot = 0, topp = 0, botp = 0;            // main range (+ mirror)
	// the far step's four ranges (+ mirrors) live in LDS: read only when
	// alternatives are enumerated, they would otherwise pin 16 registers
	const uint32_t tid = threadIdx.x;
#define T_(i) alt_s[(i)][tid]
#define B_(i) alt_s[4 + (i)][tid]
#define TP_(i) alt_s[8 + (i)][tid]
#define BP_(i) alt_s[12 + (i)][tid]
	int rdc = 0, quc = 0, clo = 0, chi = 3, j = 0;
	bool match = true;
	uint32_t topm = 0, botm = 0, topmp = 0, botmp = 0;        // branch range (+ mirror)
	int32_t nh = 0;
	uint32_t dseq = 0, bseq = 0;                // discovery numbers: next, and the in-place branch's
	uint32_t ops = 0, loads = 0;
#pragma unroll
	for(int i = 0; i < 16; i++) alt_s[i][tid] = 0;
	bool exhausted = false;

	for(;;) {
		// ---- transitions that need no side gather (bounded per iteration)
		for(int pass = 0; pass < 8; pass++) {
			if(st == ST_ALT) {
				// alternatives clo..chi at depth dep (aligner_seed.cpp:1166-1290)
				bool started = false;
				if(!hasn || rdc > 3) {
					for(; j <= chi; j++) {
						if(j == rdc || B_(j) == T_(j)) continue;
						depm = dep + 1;
						topm = T_(j); botm = B_(j); topmp = TP_(j); botmp = BP_(j);
						// the hit this alternative would report (aligner_seed.cpp:1166-1290)
						uint32_t off5p = dep;
						if(fw == ebwtfw) off5p = len - off5p - 1;
						int64_t score = (int64_t)(len - 1) * matchsc;
						const int pen = rdc > 3 ? -P.npen : -mmpen_q(P, quc - 33);
						score += pen;
						bool valid = true;
						if(P.local) valid = local_ok(dep, len, matchsc, pen);
						valid = valid && score >= minsc;
						const uint32_t myseq = dseq++;
						if(depm < len) {
							// hand the walk to the branch kernel; walk in place when the queue is full
							const uint32_t q = wave_alloc1(brq_n);
							if(q < brq_cap) {
								MmBranch b;
								b.rng = make_uint4(topm, botm, topmp, botmp);
								b.slot = slot;
								b.seq = myseq;
								b.meta = depm | ((uint32_t)j << 16) | ((uint32_t)rdc << 20) | ((valid ? 1u : 0u) << 24) |
								         ((ebwtfw ? 1u : 0u) << 25);
								b.score = (int32_t)score;
								b.off5p = (int32_t)off5p;
								b.pad[0] = b.pad[1] = b.pad[2] = 0;
								brq[q] = b;
								continue;
							}
							bseq = myseq;
							started = true;
							break;
						}
						// branch complete at the last base: report (no further LF step)
						if(valid) {
							if((uint32_t)nh < cap)
								slots[(size_t)slot * cap + nh] = bt2g_mm1{ebwtfw ? topm : topmp, ebwtfw ? botm : botmp,
								                                          fw ? 1 : 0, (int32_t)score, (int32_t)off5p,
								                                          j, rdc, (int32_t)myseq};
							nh++;
						}
					}
				}
				if(started) {
					st = ST_BR;
				} else if(bot > top && match && dep != len - 1) {
					dep++;
					st = ST_FAR;
				} else {
					st = ST_DONE;
				}
			}
			if(st == ST_DONE) {
				slot_counts[slot] = nh;
				if(ops) atomicAdd(&ops_out[r], ops);
				if(ops && loads_out) atomicAdd(&loads_out[r], loads);
				st = ST_IDLE;
			}
			// one item per lane (a refilling work queue measured slower: at ~700k
			// items there is no tail to fill, and the queue costs registers)
			if(exhausted) break;
			exhausted = true;
			const uint32_t qi = blk_ * blockDim.x + threadIdx.x;
			if(qi >= nitems) continue;
			// ---- item initialisation (aligner_seed.cpp:1003-1100)
			const uint32_t item = items[qi];
			r = item >> 3;
			const uint32_t fwi = (item >> 2) & 1u, ebi = (item >> 1) & 1u;
			hasn = item & 1u;
			fw = fwi == 0;
			slot = r * 4 + fwi * 2 + ebi;
			len = lens[r];
			rd = reads + (size_t)r * stride;
			qd = quals + (size_t)r * stride;
			minsc = minscs[r];
			nceil = (int)(ncl_const + ncl_lin * (double)len);
			if(nceil < 0) nceil = 0;
			nh = 0;
			dseq = 0;
			ops = loads = 0;
			// seq = fw ? (ebwtfw ? patFw : patFwRev) : (ebwtfw ? patRc : patRcRev)
			seq = SeqView{rd, len, fw ? !ebwtfw : ebwtfw, !fw};
			qrev = fw ? !ebwtfw : ebwtfw;
			// resume after the near half (k_one_mm_near)
			const uint32_t sd = sdep[qi];
			const uint4 q4 = st4[qi];
			top = q4.x; bot = q4.y; topp = q4.z; botp = q4.w;
			dep = sd & 0x7fffffffu;
			st = (sd >> 31) ? ST_FAR : ST_DONE;
		}
		const uint64_t busy = __ballot(st != ST_IDLE);
		if(busy == 0 && exhausted) break;
		if(st == ST_FAR && dep >= len) st = ST_DONE;   // far half empty: no step
		if(st == ST_FAR) {
			rdc = seq[len - dep - 1];
			quc = qd[qrev ? dep : len - dep - 1];
			if(rdc > 3 && nceil == 0) st = ST_DONE;
			else if(bot - top <= 1 && top == E.zoff) st = ST_DONE;   // mapLF1 hit '$'
		}
		if(!(st == ST_FAR || st == ST_BR)) continue;

		// ---- one LF operation (bt2_idx.h mapBiLFEx / mapLF1)
		const bool br = st == ST_BR;
		const uint32_t qT = br ? topm : top, qB = br ? botm : bot, qP = br ? topmp : topp;
		uint32_t ot[4], ob[4], otp[4], obp[4];
		ops++;
		const bool multi = qB - qT > 1;
		int rowl = 0;
		uint32_t lf1 = 0;
		if(multi) {
#pragma unroll
			for(int i = 0; i < 4; i++) ot[i] = ob[i] = 0;
			otp[0] = qP;
			loads += bi_step(E, qT, qB, qP, ot, ob, otp, obp);
		} else {
			SideData s1;
			load_side(E, qT / 192u, s1);
			loads++;
			rowl = side_rowL(s1, qT % 192u);
			lf1 = occ1(E, s1, qT, rowl);
		}

		if(st == ST_FAR) {
			clo = 0; chi = 3; match = true;
			if(multi) {
#pragma unroll
				for(int i = 0; i < 4; i++) { T_(i) = ot[i]; B_(i) = ob[i]; TP_(i) = otp[i]; BP_(i) = obp[i]; }
				match = rdc < 4;
				if(rdc < 4) { top = at4(ot, rdc); bot = at4(ob, rdc); topp = at4(otp, rdc); botp = at4(obp, rdc); }
			} else {
				// only alternative clo is visited (clo..chi with chi = clo)
				clo = rowl;
				top = lf1;
				match = clo == rdc;
				bot = top + 1;
				T_(clo) = top;
				B_(clo) = bot;
				BP_(clo) = botp;
				TP_(clo) = topp;
				chi = clo;
			}
			j = clo;
			st = ST_ALT;
		} else {   // ST_BR
			const int c = seq[len - depm - 1];
			bool dead;
			if(multi) {
				topm = at4(ot, c); botm = at4(ob, c); topmp = at4(otp, c); botmp = at4(obp, c);
				dead = botm <= topm;
			} else {
				dead = rowl != c || qT == E.zoff;
				if(!dead) { topm = lf1; botm = topm + 1; }
			}
			if(dead) { j++; st = ST_ALT; continue; }
			depm++;
			if(depm == len) {
				uint32_t off5p = dep;
				if(fw == ebwtfw) off5p = len - off5p - 1;
				int64_t score = (int64_t)(len - 1) * matchsc;
				const int pen = rdc > 3 ? -P.npen : -mmpen_q(P, quc - 33);
				score += pen;
				bool valid = true;
				if(P.local) valid = local_ok(dep, len, matchsc, pen);
				if(valid && score >= minsc) {
					if((uint32_t)nh < cap)
						slots[(size_t)slot * cap + nh] = bt2g_mm1{ebwtfw ? topm : topmp, ebwtfw ? botm : botmp,
						                                          fw ? 1 : 0, (int32_t)score, (int32_t)off5p, j, rdc,
						                                          (int32_t)bseq};
					nh++;
				}
				j++;
				st = ST_ALT;
			}
		}
	}
}

template <bool EBWTFW>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BT2G_MM_WAVES)))
k_one_mm_q(DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, const uint8_t* __restrict__ quals,
           uint32_t stride, const uint32_t* __restrict__ lens, const int32_t* __restrict__ minscs, MmParams P,
           double ncl_const, double ncl_lin, const uint32_t* __restrict__ items,
           const uint32_t* __restrict__ nitems_p, const uint4* __restrict__ st4,
           const uint32_t* __restrict__ sdep, uint32_t cap, bt2g_mm1* __restrict__ slots, int32_t* __restrict__ slot_counts, uint32_t* __restrict__ ops_out,
           uint32_t* __restrict__ loads_out, MmBranch* __restrict__ brq, uint32_t* __restrict__ brq_n,
           uint32_t brq_cap) {
	__shared__ uint32_t alt_s[16][256];
	one_mm_q_body<EBWTFW>(blockIdx.x, alt_s, F, B, reads, quals, stride, lens, minscs, P, ncl_const, ncl_lin, items, nitems_p, st4, sdep, cap, slots, slot_counts, ops_out, loads_out, brq, brq_n, brq_cap);
}

// Far half, lean form (aligner_seed.cpp:1110-1315): the main path's LF steps
// with the read's base at every far depth, and for each non-empty alternative
// base the hit it would make -- queued for k_one_mm_branch when the walk has
// bases left, reported at once when the mismatch is the last base.  No branch
// is walked here, so the loop is as lean as the near half's (the state
// machine k_one_mm_q, which also walks branches in place, only runs for the
// rare items that meet a full queue: they are handed over whole, and their
// queued branches are dropped by the branch kernel via slot_flag).
#ifdef BT2G_MM_PROF
// profiling build: per far-kernel wave, first start / last end (wall_clock64)
// and the largest per-lane LF-step count, [EBWTFW ? 0 : 65536] + wave index
__device__ unsigned long long g_mm_t0[2u << 16], g_mm_t1[2u << 16];
__device__ unsigned int g_mm_steps[2u << 16];
extern "C" int bt2g_mm_prof_waves(unsigned long long* t0, unsigned long long* t1, unsigned int* steps) {
	if(hipMemcpyFromSymbol(t0, HIP_SYMBOL(g_mm_t0), sizeof(unsigned long long) * (2u << 16)) != hipSuccess) return -1;
	if(hipMemcpyFromSymbol(t1, HIP_SYMBOL(g_mm_t1), sizeof(unsigned long long) * (2u << 16)) != hipSuccess) return -1;
	if(hipMemcpyFromSymbol(steps, HIP_SYMBOL(g_mm_steps), sizeof(unsigned int) * (2u << 16)) != hipSuccess) return -1;
	static unsigned long long z[2u << 16];
	static unsigned int zs[2u << 16];
	(void)hipMemcpyToSymbol(HIP_SYMBOL(g_mm_t0), z, sizeof(z));
	(void)hipMemcpyToSymbol(HIP_SYMBOL(g_mm_t1), z, sizeof(z));
	(void)hipMemcpyToSymbol(HIP_SYMBOL(g_mm_steps), zs, sizeof(zs));
	return 0;
}
#endif
#ifndef MM_BRBUF
#define MM_BRBUF 160             // staged far-half branches per wave (48 B each, LDS)
#endif
#ifndef BT2G_MM_FAR_WAVES
#define BT2G_MM_FAR_WAVES 3      // 4 and 5 spill (84 / 152 B per lane)
#endif
template <bool EBWTFW>
__device__ __forceinline__ void one_mm_far_body(const uint32_t blk_, MmBranch (*s_br)[MM_BRBUF], uint32_t* s_brn, DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, const uint8_t* __restrict__ quals,
             uint32_t stride, const uint32_t* __restrict__ lens, const int32_t* __restrict__ minscs, MmParams P,
             double ncl_const, double ncl_lin, const uint32_t* __restrict__ items,
             const uint32_t* __restrict__ nitems_p, const uint4* __restrict__ st4, const uint32_t* __restrict__ sdep,
             uint32_t cap, bt2g_mm1* __restrict__ slots, int32_t* __restrict__ slot_counts,
             uint32_t* __restrict__ ops_out, uint32_t* __restrict__ loads_out, MmBranch* __restrict__ brq,
             uint32_t* __restrict__ brq_n, uint32_t brq_cap, uint32_t* __restrict__ fb_items,
             uint4* __restrict__ fb_st4, uint32_t* __restrict__ fb_sdep, uint32_t* __restrict__ fb_n,
             uint32_t* __restrict__ slot_flag) {
	walk_prio();
	const uint32_t qi = blk_ * blockDim.x + threadIdx.x;
	// Far-half branches are staged in LDS per wave and go to the global queue in
	// one allocation and a coalesced copy when the wave is done: a global atomic
	// (whose return the store waits for) and a store inside the LF loop made
	// every later side load of the wave wait behind them (vmcnt is in order) --
	// ~13 us per LF step with most waves pushing at some step.
	const uint32_t wv = threadIdx.x >> 6;
	if((threadIdx.x & 63u) == 0) s_brn[wv] = 0;
	if(qi >= *nitems_p) return;
#ifdef BT2G_MM_PROF
	const uint32_t wslot = (EBWTFW ? 0u : 65536u) + ((qi >> 6) & 0xffffu);
	if((qi & 63u) == 0) g_mm_t0[wslot] = wall_clock64();
	uint32_t prof_ops = 0;
	struct Flush {
		uint32_t w;
		uint32_t* ops;
		__device__ ~Flush() {
			atomicMax(&g_mm_t1[w], (unsigned long long)wall_clock64());
			atomicMax(&g_mm_steps[w], *ops);
		}
	} flush_{wslot, &prof_ops};
#endif
	constexpr bool ebwtfw = EBWTFW;
	const DevEbwt& E = EBWTFW ? F : B;
	const uint32_t item = items[qi];
	const uint32_t r = item >> 3;
	const uint32_t fwi = (item >> 2) & 1u, ebi = (item >> 1) & 1u;
	const bool hasn = item & 1u;
	const bool fw = fwi == 0;
	const uint32_t slot = r * 4 + fwi * 2 + ebi;
	const uint32_t sd = sdep[qi];
	if(!(sd >> 31)) { slot_counts[slot] = 0; return; }           // the near half died
	const uint32_t len = lens[r];
	const uint8_t* qd = quals + (size_t)r * stride;
	const int64_t minsc = minscs[r];
	int nceil = (int)(ncl_const + ncl_lin * (double)len);
	if(nceil < 0) nceil = 0;
	const int64_t matchsc = (int64_t)((float)P.match + 0.5f);
	// seq = fw ? (ebwtfw ? patFw : patFwRev) : (ebwtfw ? patRc : patRcRev)
	const SeqView sv{reads + (size_t)r * stride, len, fw ? !ebwtfw : ebwtfw, !fw};
	SeqWin seq{sv, ReadWin{sv.p, sv.p + stride}};
	const bool qrev = fw ? !ebwtfw : ebwtfw;
	const uint4 q4 = st4[qi];
	uint32_t top = q4.x, bot = q4.y, topp = q4.z, botp = q4.w;
	uint32_t dep = sd & 0x7fffffffu;
	int32_t nh = 0;
	uint32_t dseq = 0, ops = 0, loads = 0;
	bool handed = false;
	while(dep < len) {
		const int rdc = seq[len - dep - 1];
		const int quc = qd[qrev ? dep : len - dep - 1];
		if(rdc > 3 && nceil == 0) break;
		if(bot - top <= 1 && top == E.zoff) break;                // mapLF1 would hit '$'
		ops++;
#ifdef BT2G_MM_PROF
		prof_ops = ops;
#endif
		uint32_t ot[4], ob[4];
		int clo = 0, chi = 3;
		bool match;
		const bool single = bot - top <= 1;
		if(!single) {
			loads += bi_step_tb(E, top, bot, ot, ob);
			match = rdc < 4;
		} else {
			SideData s1;
			load_side(E, top / 192u, s1);
			loads++;
			const int rowl = side_rowL(s1, top % 192u);
			const uint32_t lf1 = occ1(E, s1, top, rowl);
#pragma unroll
			for(int i = 0; i < 4; i++) { ot[i] = lf1; ob[i] = lf1 + 1; }
			clo = chi = rowl;
			match = rowl == rdc;
		}
		// mirror range of character j (mapBiLFEx's prefix sums; a single row keeps its mirror)
		auto mirror = [&](int jj, uint32_t& mt, uint32_t& mb) {
			if(single) { mt = topp; mb = botp; return; }
			uint32_t acc = topp;
#pragma unroll
			for(int i = 0; i < 3; i++) acc += i < jj ? ob[i] - ot[i] : 0u;
			mt = acc;
			mb = acc + (at4(ob, jj) - at4(ot, jj));
		};
		// alternatives clo..chi at this depth (aligner_seed.cpp:1166-1290); with an N in
		// the read only the N itself may be the mismatch
		if(!hasn || rdc > 3) {
#pragma unroll 1
			for(int j = clo; j <= chi; j++) {
				if(j == rdc || at4(ob, j) == at4(ot, j)) continue;
				const uint32_t depm = dep + 1;
				uint32_t off5p = dep;
				if(fw == ebwtfw) off5p = len - off5p - 1;
				int64_t score = (int64_t)(len - 1) * matchsc;
				const int pen = rdc > 3 ? -P.npen : -mmpen_q(P, quc - 33);
				score += pen;
				bool valid = true;
				if(P.local) valid = local_ok(dep, len, matchsc, pen);
				valid = valid && score >= minsc;
				const uint32_t myseq = dseq++;
				uint32_t tpm, bpm;
				mirror(j, tpm, bpm);
				const uint32_t tm = at4(ot, j), bm = at4(ob, j);
				if(depm < len) {
					// MmBranch as three 16-B words; pad[0] = the item (for a queue
					// overflow at the flush)
					const uint32_t meta = depm | ((uint32_t)j << 16) | ((uint32_t)rdc << 20) | ((valid ? 1u : 0u) << 24) |
					                      ((ebwtfw ? 1u : 0u) << 25);
					const uint4 w0 = make_uint4(tm, bm, tpm, bpm);
					const uint4 w1 = make_uint4(slot, myseq, meta, (uint32_t)(int32_t)score);
					const uint4 w2 = make_uint4((uint32_t)(int32_t)off5p, qi, 0u, 0u);
					const uint32_t k = atomicAdd(&s_brn[wv], 1u);
					if(k < MM_BRBUF) {
						uint4* dst = (uint4*)&s_br[wv][k];
						dst[0] = w0; dst[1] = w1; dst[2] = w2;
					} else {
						// the wave's LDS buffer is full: straight to the global queue
						const uint32_t q = atomicAdd(brq_n, 1u);
						if(q >= brq_cap) { handed = true; break; }
						uint4* dst = (uint4*)&brq[q];
						dst[0] = w0; dst[1] = w1; dst[2] = w2;
					}
				} else if(valid) {                       // the mismatch is the last base
					if((uint32_t)nh < cap)
						slots[(size_t)slot * cap + nh] = bt2g_mm1{ebwtfw ? tm : tpm, ebwtfw ? bm : bpm, fw ? 1 : 0,
						                                          (int32_t)score, (int32_t)off5p, j, rdc,
						                                          (int32_t)myseq};
					nh++;
				}
			}
		}
		if(handed) break;
		if(match) {
			uint32_t mt, mb;
			mirror(rdc, mt, mb);
			top = at4(ot, rdc); bot = at4(ob, rdc); topp = mt; botp = mb;
		}
		if(!(bot > top && match && dep != len - 1)) break;
		dep++;
	}
	// a lane that met the full queue claims its item before the flush, so the
	// flush skips the item's staged entries (their slot flag is set) and the
	// item reaches the state machine's list exactly once (below)
	const bool claimed = handed && atomicExch(&slot_flag[slot], 1u) == 0u;
	// flush the wave's staged branches (every lane still running is here)
	bool overflow = false;
	{
		const uint32_t n = s_brn[wv] < MM_BRBUF ? s_brn[wv] : MM_BRBUF;
		if(n) {
			const uint64_t act = __ballot(1);
			const uint32_t me = threadIdx.x & 63u, lead = (uint32_t)__ffsll((long long)act) - 1u;
			uint32_t qb = 0;
			if(me == lead) qb = atomicAdd(brq_n, n);
			qb = (uint32_t)__shfl((int)qb, (int)lead);
			const uint32_t rank = (uint32_t)__popcll(act & ((1ull << me) - 1ull)), na = (uint32_t)__popcll(act);
			for(uint32_t i = rank; i < n; i += na) {
				const uint4* src = (const uint4*)&s_br[wv][i];
				const uint4 w0 = src[0], w1 = src[1], w2 = src[2];
				if(qb + i < brq_cap) {
					uint4* dst = (uint4*)&brq[qb + i];
					dst[0] = w0; dst[1] = w1; dst[2] = w2;
				} else if(atomicExch(&slot_flag[w1.x], 1u) == 0u) {
					// queue full: the entry's item is redone whole by the in-place state
					// machine (its queued branches are skipped by their slot flag)
					const uint32_t f = atomicAdd(fb_n, 1u);
					fb_items[f] = items[w2.y];
					fb_st4[f] = st4[w2.y];
					fb_sdep[f] = sdep[w2.y];
				}
			}
			overflow = qb + n > brq_cap;
		}
	}
	if(overflow && !handed && atomicAdd(&slot_flag[slot], 0u)) return;   // redone by the state machine
	if(handed) {
		// queue full: the whole item goes to the in-place state machine (unless the
		// flush of another lane's entries already sent it there)
		if(claimed) {
			const uint32_t f = wave_alloc1(fb_n);
			fb_items[f] = item;
			fb_st4[f] = q4;
			fb_sdep[f] = sd;
		}
		return;
	}
	slot_counts[slot] = nh;
	if(ops) atomicAdd(&ops_out[r], ops);
	if(ops && loads_out) atomicAdd(&loads_out[r], loads);
}

template <bool EBWTFW>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BT2G_MM_FAR_WAVES)))
k_one_mm_far(DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, const uint8_t* __restrict__ quals,
             uint32_t stride, const uint32_t* __restrict__ lens, const int32_t* __restrict__ minscs, MmParams P,
             double ncl_const, double ncl_lin, const uint32_t* __restrict__ items,
             const uint32_t* __restrict__ nitems_p, const uint4* __restrict__ st4, const uint32_t* __restrict__ sdep,
             uint32_t cap, bt2g_mm1* __restrict__ slots, int32_t* __restrict__ slot_counts,
             uint32_t* __restrict__ ops_out, uint32_t* __restrict__ loads_out, MmBranch* __restrict__ brq,
             uint32_t* __restrict__ brq_n, uint32_t brq_cap, uint32_t* __restrict__ fb_items,
             uint4* __restrict__ fb_st4, uint32_t* __restrict__ fb_sdep, uint32_t* __restrict__ fb_n,
             uint32_t* __restrict__ slot_flag) {
	__shared__ MmBranch s_br[4][MM_BRBUF];
	__shared__ uint32_t s_brn[4];
	one_mm_far_body<EBWTFW>(blockIdx.x, s_br, s_brn, F, B, reads, quals, stride, lens, minscs, P, ncl_const, ncl_lin, items, nitems_p, st4, sdep, cap, slots, slot_counts, ops_out, loads_out, brq, brq_n, brq_cap, fb_items, fb_st4, fb_sdep, fb_n, slot_flag);
}

// Walk every queued far-half branch to the read's end (or its death), one
// lane per branch: exact steps on the read's remaining bases with the same LF
// operations and op counting as the in-place walk (ST_BR above).  A completed
// valid branch appends its hit to its slot (after the far kernel's own hits,
// slot_counts[] is the slot's running count).
template <bool EBWTFW>
__device__ __forceinline__ void one_mm_branch_body(const uint32_t blk_, DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, uint32_t stride,
                const uint32_t* __restrict__ lens, const MmBranch* __restrict__ brq,
                const uint32_t* __restrict__ brq_n, uint32_t brq_cap, uint32_t cap, bt2g_mm1* __restrict__ slots,
                int32_t* __restrict__ slot_counts, uint32_t* __restrict__ ops_out, uint32_t* __restrict__ loads_out,
                const uint32_t* __restrict__ slot_flag) {
	walk_prio();
	const uint32_t i = blk_ * blockDim.x + threadIdx.x;
	const uint32_t nq = *brq_n < brq_cap ? *brq_n : brq_cap;
	if(i >= nq) return;
	const MmBranch b = brq[i];
	// one launch per index direction: the index a lane walks is then uniform (a
	// per-lane choice between the two DevEbwt arguments put both on the stack)
	const bool ebwtfw = (b.meta >> 25) & 1u;
	if(ebwtfw != EBWTFW) return;
	if(slot_flag[b.slot]) return;                 // its item was redone whole by the state machine
	const DevEbwt& E = EBWTFW ? F : B;
	const uint32_t r = b.slot >> 2;
	const bool fw = ((b.slot >> 1) & 1u) == 0;
	const uint32_t len = lens[r];
	const SeqView sv{reads + (size_t)r * stride, len, fw ? !ebwtfw : ebwtfw, !fw};
	SeqWin seq{sv, ReadWin{sv.p, sv.p + stride}};
	uint32_t topm = b.rng.x, botm = b.rng.y, topmp = b.rng.z, botmp = b.rng.w;
	uint32_t depm = b.meta & 0xffffu;
	uint32_t ops = 0, loads = 0;
	bool done = false;
	while(depm < len) {
		const int c = seq[len - depm - 1];
		ops++;
		bool dead;
		if(botm - topm > 1) {
			uint32_t ot[4] = {0, 0, 0, 0}, ob[4] = {0, 0, 0, 0}, otp[4], obp[4];
			otp[0] = topmp;
			loads += bi_step(E, topm, botm, topmp, ot, ob, otp, obp);
			topm = at4(ot, c); botm = at4(ob, c); topmp = at4(otp, c); botmp = at4(obp, c);
			dead = botm <= topm;
		} else {
			SideData s1;
			load_side(E, topm / 192u, s1);
			loads++;
			const int rowl = side_rowL(s1, topm % 192u);
			dead = rowl != c || topm == E.zoff;
			if(!dead) { topm = occ1(E, s1, topm, rowl); botm = topm + 1; }
		}
		if(dead) break;
		if(++depm == len) done = true;
	}
	if(done && ((b.meta >> 24) & 1u)) {
		const int32_t p = atomicAdd(&slot_counts[b.slot], 1);
		if((uint32_t)p < cap)
			slots[(size_t)b.slot * cap + p] = bt2g_mm1{ebwtfw ? topm : topmp, ebwtfw ? botm : botmp, fw ? 1 : 0,
			                                           b.score, b.off5p, (int32_t)((b.meta >> 16) & 0xfu),
			                                           (int32_t)((b.meta >> 20) & 0xfu), (int32_t)b.seq};
	}
	if(ops) atomicAdd(&ops_out[r], ops);
	if(ops && loads_out) atomicAdd(&loads_out[r], loads);
}

template <bool EBWTFW>
__global__ void __launch_bounds__(256)
k_one_mm_branch(DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, uint32_t stride,
                const uint32_t* __restrict__ lens, const MmBranch* __restrict__ brq,
                const uint32_t* __restrict__ brq_n, uint32_t brq_cap, uint32_t cap, bt2g_mm1* __restrict__ slots,
                int32_t* __restrict__ slot_counts, uint32_t* __restrict__ ops_out, uint32_t* __restrict__ loads_out,
                const uint32_t* __restrict__ slot_flag) {
	one_mm_branch_body<EBWTFW>(blockIdx.x, F, B, reads, stride, lens, brq, brq_n, brq_cap, cap, slots, slot_counts, ops_out, loads_out, slot_flag);
}



// The near half and the branch walks with a quad of lanes per item / branch
// (fm_device.h, the cooperative step; $BT2G_FM_QUAD=0: one lane each).
template <bool EBWTFW>
__device__ __forceinline__ void one_mm_near_quad_body(const uint32_t blk_, DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, uint32_t stride,
              const uint32_t* __restrict__ lens, const uint32_t* __restrict__ items,
              const uint32_t* __restrict__ nitems_p, uint4* __restrict__ st4, uint32_t* __restrict__ sdep,
              uint32_t* __restrict__ ops_out, uint32_t* __restrict__ loads_out) {
	walk_prio();
	const uint32_t lane_ = blk_ * blockDim.x + threadIdx.x;
	const uint32_t qi = lane_ >> 2, q = lane_ & 3u;   // a quad of lanes per item
	if(qi >= *nitems_p) return;
	const DevEbwt& E = EBWTFW ? F : B;
	const DevEbwt& Ep = EBWTFW ? B : F;
	const uint32_t item = items[qi];
	const uint32_t r = item >> 3;
	const bool fw = ((item >> 2) & 1u) == 0;
	const uint32_t len = lens[r];
	// seq = fw ? (ebwtfw ? patFw : patFwRev) : (ebwtfw ? patRc : patRcRev)
	const SeqView seq{reads + (size_t)r * stride, len, fw ? !EBWTFW : EBWTFW, !fw};
	const uint32_t nea = EBWTFW ? (len >> 1) : (len >> 1) + (len & 1);
	const uint32_t flen = E.ftab_chars;
	uint32_t top = 0, bot = 0, topp = 0, botp = 0, dep = 0, ops = 0, loads = 0;
	bool alive = len != 0;
	if(item & 1u)                               // the read has an N: none may be in the near half
		for(uint32_t d = 0; alive && d < nea; d++)
			if(seq[len - d - 1] > 3) alive = false;
	if(alive) {
		if(flen > 1 && flen <= nea) {
			// ftabSeqToInt(seq, len-flen, rev=!ebwtfw) (bt2_idx.h:1383-1390)
			uint32_t fi = 0, fip = 0;
			for(uint32_t i = 0; i < flen; i++) {
				fi = (fi << 2) | (uint32_t)seq[len - flen + i];
				fip = (fip << 2) | (uint32_t)seq[len - 1 - i];
			}
			top = ftab_hi(E, fi); bot = ftab_lo(E, fi + 1);
			topp = ftab_hi(Ep, fip); botp = ftab_lo(Ep, fip + 1);
			dep = flen;
		} else {
			const int c = seq[len - 1];
			top = topp = fchr_at(E, c);
			bot = botp = fchr_at(E, c + 1);
			dep = 1;
		}
		alive = bot != top;
	}
	SeqWin sw{seq, ReadWin{seq.p, seq.p + stride}};
	while(alive && dep < nea) {
		const int c = sw[len - dep - 1];
		ops++;
		if(bot - top > 1) {
			uint32_t t[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0}, tp[4], bp[4];
			tp[0] = topp;
			loads += quad_bi_step(E, q, top, bot, topp, t, b, tp, bp);
			const uint32_t nt = at4(t, c), nb = at4(b, c);
			if(nb <= nt) { alive = false; break; }
			top = nt; bot = nb; topp = at4(tp, c); botp = at4(bp, c);
		} else {
			QuadSide s1;
			load_quad(E, top / 192u, q, s1);
			loads++;
			if(quad_rowL(s1, q, top % 192u) != c || top == E.zoff) { alive = false; break; }
			top = quad_occ1(E, s1, q, top, c);
			bot = top + 1;
		}
		dep++;
	}
	if(q != 0) return;
	st4[qi] = alive ? make_uint4(top, bot, topp, botp) : make_uint4(0, 0, 0, 0);
	sdep[qi] = dep | (alive ? 0x80000000u : 0u);
	if(ops) atomicAdd(&ops_out[r], ops);
	if(ops && loads_out) atomicAdd(&loads_out[r], loads);
}

template <bool EBWTFW>
__device__ __forceinline__ void one_mm_branch_quad_body(const uint32_t blk_, DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, uint32_t stride,
                const uint32_t* __restrict__ lens, const MmBranch* __restrict__ brq,
                const uint32_t* __restrict__ brq_n, uint32_t brq_cap, uint32_t cap, bt2g_mm1* __restrict__ slots,
                int32_t* __restrict__ slot_counts, uint32_t* __restrict__ ops_out, uint32_t* __restrict__ loads_out,
                const uint32_t* __restrict__ slot_flag) {
	walk_prio();
	const uint32_t lane_ = blk_ * blockDim.x + threadIdx.x;
	const uint32_t i = lane_ >> 2, q = lane_ & 3u;   // a quad of lanes per branch
	const uint32_t nq = *brq_n < brq_cap ? *brq_n : brq_cap;
	if(i >= nq) return;
	const MmBranch b = brq[i];
	// one launch per index direction: the index a lane walks is then uniform (a
	// per-lane choice between the two DevEbwt arguments put both on the stack)
	const bool ebwtfw = (b.meta >> 25) & 1u;
	if(ebwtfw != EBWTFW) return;
	if(slot_flag[b.slot]) return;                 // its item was redone whole by the state machine
	const DevEbwt& E = EBWTFW ? F : B;
	const uint32_t r = b.slot >> 2;
	const bool fw = ((b.slot >> 1) & 1u) == 0;
	const uint32_t len = lens[r];
	const SeqView sv{reads + (size_t)r * stride, len, fw ? !ebwtfw : ebwtfw, !fw};
	SeqWin seq{sv, ReadWin{sv.p, sv.p + stride}};
	uint32_t topm = b.rng.x, botm = b.rng.y, topmp = b.rng.z, botmp = b.rng.w;
	uint32_t depm = b.meta & 0xffffu;
	uint32_t ops = 0, loads = 0;
	bool done = false;
	while(depm < len) {
		const int c = seq[len - depm - 1];
		ops++;
		bool dead;
		if(botm - topm > 1) {
			uint32_t ot[4] = {0, 0, 0, 0}, ob[4] = {0, 0, 0, 0}, otp[4], obp[4];
			otp[0] = topmp;
			loads += quad_bi_step(E, q, topm, botm, topmp, ot, ob, otp, obp);
			topm = at4(ot, c); botm = at4(ob, c); topmp = at4(otp, c); botmp = at4(obp, c);
			dead = botm <= topm;
		} else {
			QuadSide s1;
			load_quad(E, topm / 192u, q, s1);
			loads++;
			const int rowl = quad_rowL(s1, q, topm % 192u);
			dead = rowl != c || topm == E.zoff;
			if(!dead) { topm = quad_occ1(E, s1, q, topm, rowl); botm = topm + 1; }
		}
		if(dead) break;
		if(++depm == len) done = true;
	}
	if(q != 0) return;
	if(done && ((b.meta >> 24) & 1u)) {
		const int32_t p = atomicAdd(&slot_counts[b.slot], 1);
		if((uint32_t)p < cap)
			slots[(size_t)b.slot * cap + p] = bt2g_mm1{ebwtfw ? topm : topmp, ebwtfw ? botm : botmp, fw ? 1 : 0,
			                                           b.score, b.off5p, (int32_t)((b.meta >> 16) & 0xfu),
			                                           (int32_t)((b.meta >> 20) & 0xfu), (int32_t)b.seq};
	}
	if(ops) atomicAdd(&ops_out[r], ops);
	if(ops && loads_out) atomicAdd(&loads_out[r], loads);
}

// Both index directions in one launch (round 6): blocks [0, g_) walk the BWT's
// items, [g_, 2 g_) the mirror index's (their lists at +half_, their item
// count at +2, their fallback lists at +half_ and count +1).  Two launches on a
// second stream had joined through events: ~0.1-0.3 ms of cross-queue waits
// per call in the batch server's trace (r06a), a near-half launch's worth.
__global__ void __launch_bounds__(256)
k_one_mm_near2(const uint32_t g_, const size_t half_, DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, uint32_t stride,
              const uint32_t* __restrict__ lens, const uint32_t* __restrict__ items,
              const uint32_t* __restrict__ nitems_p, uint4* __restrict__ st4, uint32_t* __restrict__ sdep,
              uint32_t* __restrict__ ops_out, uint32_t* __restrict__ loads_out) {
	if(blockIdx.x < g_) one_mm_near_body<true>(blockIdx.x, F, B, reads, stride, lens, items, nitems_p, st4, sdep, ops_out, loads_out);
	else one_mm_near_body<false>(blockIdx.x - g_, F, B, reads, stride, lens, items + half_, nitems_p + 2, st4 + half_, sdep + half_, ops_out, loads_out);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BT2G_MM_FAR_WAVES)))
k_one_mm_far2(const uint32_t g_, const size_t half_, DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, const uint8_t* __restrict__ quals,
             uint32_t stride, const uint32_t* __restrict__ lens, const int32_t* __restrict__ minscs, MmParams P,
             double ncl_const, double ncl_lin, const uint32_t* __restrict__ items,
             const uint32_t* __restrict__ nitems_p, const uint4* __restrict__ st4, const uint32_t* __restrict__ sdep,
             uint32_t cap, bt2g_mm1* __restrict__ slots, int32_t* __restrict__ slot_counts,
             uint32_t* __restrict__ ops_out, uint32_t* __restrict__ loads_out, MmBranch* __restrict__ brq,
             uint32_t* __restrict__ brq_n, uint32_t brq_cap, uint32_t* __restrict__ fb_items,
             uint4* __restrict__ fb_st4, uint32_t* __restrict__ fb_sdep, uint32_t* __restrict__ fb_n,
             uint32_t* __restrict__ slot_flag) {
	__shared__ MmBranch s_br[4][MM_BRBUF];
	__shared__ uint32_t s_brn[4];
	if(blockIdx.x < g_) one_mm_far_body<true>(blockIdx.x, s_br, s_brn, F, B, reads, quals, stride, lens, minscs, P, ncl_const, ncl_lin, items, nitems_p, st4, sdep, cap, slots, slot_counts, ops_out, loads_out, brq, brq_n, brq_cap, fb_items, fb_st4, fb_sdep, fb_n, slot_flag);
	else one_mm_far_body<false>(blockIdx.x - g_, s_br, s_brn, F, B, reads, quals, stride, lens, minscs, P, ncl_const, ncl_lin, items + half_, nitems_p + 2, st4 + half_, sdep + half_, cap, slots, slot_counts, ops_out, loads_out, brq, brq_n, brq_cap, fb_items + half_, fb_st4 + half_, fb_sdep + half_, fb_n + 1, slot_flag);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BT2G_MM_WAVES)))
k_one_mm_q2(const uint32_t g_, const size_t half_, DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, const uint8_t* __restrict__ quals,
           uint32_t stride, const uint32_t* __restrict__ lens, const int32_t* __restrict__ minscs, MmParams P,
           double ncl_const, double ncl_lin, const uint32_t* __restrict__ items,
           const uint32_t* __restrict__ nitems_p, const uint4* __restrict__ st4,
           const uint32_t* __restrict__ sdep, uint32_t cap, bt2g_mm1* __restrict__ slots, int32_t* __restrict__ slot_counts, uint32_t* __restrict__ ops_out,
           uint32_t* __restrict__ loads_out, MmBranch* __restrict__ brq, uint32_t* __restrict__ brq_n,
           uint32_t brq_cap) {
	__shared__ uint32_t alt_s[16][256];
	if(blockIdx.x < g_) one_mm_q_body<true>(blockIdx.x, alt_s, F, B, reads, quals, stride, lens, minscs, P, ncl_const, ncl_lin, items, nitems_p, st4, sdep, cap, slots, slot_counts, ops_out, loads_out, brq, brq_n, brq_cap);
	else one_mm_q_body<false>(blockIdx.x - g_, alt_s, F, B, reads, quals, stride, lens, minscs, P, ncl_const, ncl_lin, items + half_, nitems_p + 1, st4 + half_, sdep + half_, cap, slots, slot_counts, ops_out, loads_out, brq, brq_n, brq_cap);
}
__global__ void __launch_bounds__(256)
k_one_mm_branch2(const uint32_t g_, const size_t half_, DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, uint32_t stride,
                const uint32_t* __restrict__ lens, const MmBranch* __restrict__ brq,
                const uint32_t* __restrict__ brq_n, uint32_t brq_cap, uint32_t cap, bt2g_mm1* __restrict__ slots,
                int32_t* __restrict__ slot_counts, uint32_t* __restrict__ ops_out, uint32_t* __restrict__ loads_out,
                const uint32_t* __restrict__ slot_flag) {
	if(blockIdx.x < g_) one_mm_branch_body<true>(blockIdx.x, F, B, reads, stride, lens, brq, brq_n, brq_cap, cap, slots, slot_counts, ops_out, loads_out, slot_flag);
	else one_mm_branch_body<false>(blockIdx.x - g_, F, B, reads, stride, lens, brq, brq_n, brq_cap, cap, slots, slot_counts, ops_out, loads_out, slot_flag);
}

__global__ void __launch_bounds__(256)
k_one_mm_near2q(const uint32_t g_, const size_t half_, DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads,
                uint32_t stride, const uint32_t* __restrict__ lens, const uint32_t* __restrict__ items,
                const uint32_t* __restrict__ nitems_p, uint4* __restrict__ st4, uint32_t* __restrict__ sdep,
                uint32_t* __restrict__ ops_out, uint32_t* __restrict__ loads_out) {
	if(blockIdx.x < g_)
		one_mm_near_quad_body<true>(blockIdx.x, F, B, reads, stride, lens, items, nitems_p, st4, sdep, ops_out, loads_out);
	else
		one_mm_near_quad_body<false>(blockIdx.x - g_, F, B, reads, stride, lens, items + half_, nitems_p + 2, st4 + half_,
		                             sdep + half_, ops_out, loads_out);
}
__global__ void __launch_bounds__(256)
k_one_mm_branch2q(const uint32_t g_, const size_t half_, DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads,
                  uint32_t stride, const uint32_t* __restrict__ lens, const MmBranch* __restrict__ brq,
                  const uint32_t* __restrict__ brq_n, uint32_t brq_cap, uint32_t cap, bt2g_mm1* __restrict__ slots,
                  int32_t* __restrict__ slot_counts, uint32_t* __restrict__ ops_out, uint32_t* __restrict__ loads_out,
                  const uint32_t* __restrict__ slot_flag) {
	(void)half_;
	if(blockIdx.x < g_)
		one_mm_branch_quad_body<true>(blockIdx.x, F, B, reads, stride, lens, brq, brq_n, brq_cap, cap, slots, slot_counts,
		                              ops_out, loads_out, slot_flag);
	else
		one_mm_branch_quad_body<false>(blockIdx.x - g_, F, B, reads, stride, lens, brq, brq_n, brq_cap, cap, slots,
		                               slot_counts, ops_out, loads_out, slot_flag);
}

void launch_one_mm_q(const DevEbwt& F, const DevEbwt& B, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                     const uint32_t* lens, uint32_t n, const int32_t* minsc, const bt2g_scoring& sc, int nofw,
                     int norc, const uint32_t* gate, uint32_t cap, uint32_t* items, uint32_t* counters,
                     uint4* near_state, uint32_t* near_dep, bt2g_mm1* slots, int32_t* slot_counts, uint32_t* ops,
                     uint32_t* loads, MmBranch* brq, uint32_t brq_cap, uint32_t* fb_items, uint4* fb_st4,
                     uint32_t* fb_sdep, uint32_t* slot_flag, hipStream_t st, hipStream_t st2, hipEvent_t* ev) {
	MmParams P{sc.match, sc.mmp_max, sc.mmp_min, sc.npen, sc.local, 0, 0};
	// $BT2G_MM_MERGED=0: the two index directions as separate launches on two
	// streams (forked and joined by events), as before round 6; default: one
	// launch per stage for both (k_one_mm_*2)
	const char* me = getenv("BT2G_MM_MERGED");            // (read per call: A/B in one process)
	const bool merged = !(me && *me == '0');
	if(merged) {
		hipLaunchKernelGGL(k_one_mm_items, dim3((n + 255) / 256), dim3(256), 0, st, reads, stride, lens, n, gate, nofw,
		                   norc, items, counters, slot_counts, ops, loads, slot_flag);
		const uint32_t g = (2 * n + 255) / 256, gb = (brq_cap + 255) / 256;
		const size_t half = 2 * (size_t)n;
		// ($BT2G_FM_QUAD=0: one lane per item and branch, else a quad: fm_device.h)
		const char* qe = getenv("BT2G_FM_QUAD");
		const bool quad = !(qe && *qe == '0');
		if(quad)
			hipLaunchKernelGGL(k_one_mm_near2q, dim3(8 * g), dim3(256), 0, st, 4 * g, half, F, B, reads, stride, lens,
			                   items, counters, near_state, near_dep, ops, loads);
		else
			hipLaunchKernelGGL(k_one_mm_near2, dim3(2 * g), dim3(256), 0, st, g, half, F, B, reads, stride, lens, items,
			                   counters, near_state, near_dep, ops, loads);
		hipLaunchKernelGGL(k_one_mm_far2, dim3(2 * g), dim3(256), 0, st, g, half, F, B, reads, quals, stride, lens, minsc,
		                   P, sc.ncl_const, sc.ncl_lin, items, counters, near_state, near_dep, cap, slots, slot_counts,
		                   ops, loads, brq, counters + 4, brq_cap, fb_items, fb_st4, fb_sdep, counters + 5, slot_flag);
		hipLaunchKernelGGL(k_one_mm_q2, dim3(2 * g), dim3(256), 0, st, g, half, F, B, reads, quals, stride, lens, minsc,
		                   P, sc.ncl_const, sc.ncl_lin, fb_items, counters + 5, fb_st4, fb_sdep, cap, slots, slot_counts,
		                   ops, loads, brq, counters + 7, 0u);
		if(quad)
			hipLaunchKernelGGL(k_one_mm_branch2q, dim3(8 * gb), dim3(256), 0, st, 4 * gb, half, F, B, reads, stride, lens,
			                   brq, counters + 4, brq_cap, cap, slots, slot_counts, ops, loads, slot_flag);
		else
			hipLaunchKernelGGL(k_one_mm_branch2, dim3(2 * gb), dim3(256), 0, st, gb, half, F, B, reads, stride, lens, brq,
			                   counters + 4, brq_cap, cap, slots, slot_counts, ops, loads, slot_flag);
		return;
	}
	// the BWT' direction's kernels on s2 (st2, forked from st and joined back), or after the BWT ones on st
	const bool two = st2 != nullptr && ev != nullptr;
	hipStream_t s2 = two ? st2 : st;
	// counters[0]/[2] = item counts of the BWT / BWT' lists (zeroed by the caller)
	hipLaunchKernelGGL(k_one_mm_items, dim3((n + 255) / 256), dim3(256), 0, st, reads, stride, lens, n, gate, nofw,
	                   norc, items, counters, slot_counts, ops, loads, slot_flag);
	const uint32_t grid = (2 * n + 255) / 256;   // list capacity; lanes past the count exit
	const size_t half = 2 * (size_t)n;
	if(two) {
		(void)hipEventRecord(ev[0], st);
		(void)hipStreamWaitEvent(s2, ev[0], 0);
	}
	// near half, far half (lean; branches to the queue, shared by both directions),
	// then the state machine for the items that met a full queue (counters[5] / [6];
	// it walks in place: no queue, its own dummy head counters[7])
	hipLaunchKernelGGL(k_one_mm_near<true>, dim3(grid), dim3(256), 0, st, F, B, reads, stride, lens, items, counters,
	                   near_state, near_dep, ops, loads);
	hipLaunchKernelGGL(k_one_mm_near<false>, dim3(grid), dim3(256), 0, s2, F, B, reads, stride, lens, items + half,
	                   counters + 2, near_state + half, near_dep + half, ops, loads);
	hipLaunchKernelGGL(k_one_mm_far<true>, dim3(grid), dim3(256), 0, st, F, B, reads, quals, stride, lens, minsc, P,
	                   sc.ncl_const, sc.ncl_lin, items, counters, near_state, near_dep, cap, slots, slot_counts, ops,
	                   loads, brq, counters + 4, brq_cap, fb_items, fb_st4, fb_sdep, counters + 5, slot_flag);
	hipLaunchKernelGGL(k_one_mm_far<false>, dim3(grid), dim3(256), 0, s2, F, B, reads, quals, stride, lens, minsc, P,
	                   sc.ncl_const, sc.ncl_lin, items + half, counters + 2, near_state + half, near_dep + half, cap,
	                   slots, slot_counts, ops, loads, brq, counters + 4, brq_cap, fb_items + half, fb_st4 + half,
	                   fb_sdep + half, counters + 6, slot_flag);
	hipLaunchKernelGGL(k_one_mm_q<true>, dim3(grid), dim3(256), 0, st, F, B, reads, quals, stride, lens, minsc, P,
	                   sc.ncl_const, sc.ncl_lin, fb_items, counters + 5, fb_st4, fb_sdep, cap, slots, slot_counts, ops,
	                   loads, brq, counters + 7, 0u);
	hipLaunchKernelGGL(k_one_mm_q<false>, dim3(grid), dim3(256), 0, s2, F, B, reads, quals, stride, lens, minsc, P,
	                   sc.ncl_const, sc.ncl_lin, fb_items + half, counters + 6, fb_st4 + half, fb_sdep + half, cap,
	                   slots, slot_counts, ops, loads, brq, counters + 7, 0u);
	if(two) {
		// every branch is queued (both far kernels) before either branch kernel runs
		(void)hipEventRecord(ev[1], s2);
		(void)hipStreamWaitEvent(st, ev[1], 0);
		(void)hipEventRecord(ev[2], st);
		(void)hipStreamWaitEvent(s2, ev[2], 0);
	}
	hipLaunchKernelGGL(k_one_mm_branch<true>, dim3((brq_cap + 255) / 256), dim3(256), 0, st, F, B, reads, stride,
	                   lens, brq, counters + 4, brq_cap, cap, slots, slot_counts, ops, loads, slot_flag);
	hipLaunchKernelGGL(k_one_mm_branch<false>, dim3((brq_cap + 255) / 256), dim3(256), 0, s2, F, B, reads, stride,
	                   lens, brq, counters + 4, brq_cap, cap, slots, slot_counts, ops, loads, slot_flag);
	if(two) {
		(void)hipEventRecord(ev[3], s2);
		(void)hipStreamWaitEvent(st, ev[3], 0);
	}
}
