// fm_kernels.hip -- FM-index engines of the seed phase, gfx950.
//
// One lane owns one independent query (a read strand, one seed, one SA row);
// the work is a chain of dependent 64-B side gathers, so throughput comes from
// keeping many independent chains in flight (wave64, high occupancy, no LDS),
// not from intra-query parallelism.  Every kernel is a restatement of the
// reference control flow (file:line per kernel) so the per-query results are
// identical; oracle/oracle.c is the CPU twin used by the tests.
#include "fm_device.h"
#include "bt2g_kernels.h"

// --------------------------------------------------------------------------
// exactSweep (aligner_seed.cpp:750-968): one lane = one (read, strand).
// --------------------------------------------------------------------------
#ifndef BT2G_SWEEP_WAVES
#define BT2G_SWEEP_WAVES 7      // 8 (63 VGPRs, no spills) measured 4.47 vs 4.33 ms
#endif
#ifndef BT2G_SEED_WAVES
#define BT2G_SEED_WAVES 4
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BT2G_SWEEP_WAVES)))
k_exact_sweep(DevEbwt e, const uint8_t* __restrict__ reads, uint32_t stride, const uint32_t* __restrict__ lens,
              uint32_t n, uint32_t mine_max, int nofw, int norc, uint32_t* __restrict__ out) {
	walk_prio();
	// lanes 2r, 2r+1: the two strands of read r (strand-homogeneous waves
	// measured slower: half the reads of any wave come from either strand)
	const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t r = gid >> 1, strand = gid & 1;
	const bool valid = r < n;
	const bool active = valid && !((strand == 0 && nofw) || (strand == 1 && norc));
	const uint32_t len = active ? lens[r] : 0;
	SeqView seq{reads + (size_t)(active ? r : 0) * stride, len, strand == 1, strand == 1};
	// the LF loop's base at depth dep: fw row[len-dep-1], rc comp(row[dep]), via a register window
	ReadWin rw{reads, reads + (size_t)n * stride};
	const uint8_t* row = seq.p;
	// seq[k] through the window: fw row[k], rc comp(row[len-1-k])
	auto seq_at = [&](uint32_t k) -> int {
		const int c = rw.at(row + (strand == 1 ? len - 1 - k : k));
		return strand == 1 ? (c > 3 ? 4 : 3 - c) : c;
	};
	auto base_at = [&](uint32_t d) -> int { return seq_at(len - d - 1); };
	const uint32_t flen = e.ftab_chars;
	uint32_t dep = 0, nedit = 0, top = 0, bot = 0, mine = 0;
	uint32_t bwops = 0, loads = 0;
	bool doinit = true, done = !active;
	// (r05v: on an idle GPU a launch of 256-540 reads took 0.385 ms, 2.6 us per
	// step against 0.61 us for one dependent 64-B gather: the ftab characters were
	// byte loads one after another, the two ftab words and their eftab entries
	// were waited for in turn, and the single-row and range steps had a side-load
	// site each -- a wave whose lanes took both paid two latencies a step.  Now
	// every load of a step is issued before any of them is waited for.)
	while(dep < len && !done) {
		if(doinit) {
			top = bot = 0;
			uint32_t left = len - dep;
			bool doftab = flen > 1 && left >= flen;
			uint32_t fi = 0;
			if(doftab) {
				// ftabSeqToInt(seq, left-flen, rev=false) on the forward index
				for(uint32_t i = 0; i < flen; i++) {
					int c = seq_at(left - flen + i);
					if(c > 3) { doftab = false; break; }
					fi = (fi << 2) | (uint32_t)c;
				}
			}
			if(doftab) {
				// ftab_hi(fi), ftab_lo(fi + 1): both words, then both eftab entries
				const uint32_t v0 = e.ftab[fi], v1 = e.ftab[fi + 1];
				const bool x0 = v0 > e.len, x1 = v1 > e.len;
				const uint32_t et = x0 ? e.eftab[(v0 ^ BT2G_OFF_MASK) * 2 + 1] : v0;
				const uint32_t eb = x1 ? e.eftab[(v1 ^ BT2G_OFF_MASK) * 2] : v1;
				top = et;
				bot = eb;
				dep += flen;
			} else {
				int c = seq_at(len - dep - 1);
				if(c < 4) { top = fchr_at(e, c); bot = fchr_at(e, c + 1); }
				dep++;
			}
			if(bot <= top) {
				nedit++;
				if(nedit >= mine_max) { mine = nedit; done = true; }
				continue;
			}
			doinit = false;
		}
		if(dep < len) {
			const int c = base_at(dep);
			const bool rng = bot - top > 1;
			const uint32_t st = top / 192u, sb = rng ? bot / 192u : st;
			// the step's sides, issued together (the second is the first again
			// for a single row or a range inside one side: a hit on the same
			// line); both paths read both, so neither load sinks into one path
			SideData s1, s2;
			load_side(e, st, s1);
			load_side(e, sb, s2);
			if(c > 3) {
				top = bot = 0;
			} else if(rng) {
				bwops += 2;
				loads += sb == st ? 1u : 2u;
				const uint32_t nt = occ1(e, s1, top, c), nb = occ1(e, s2, bot, c);
				top = nt; bot = nb;
			} else {
				bwops += 1;
				loads++;
				uint32_t co = top % 192u;
				if(side_rowL(s1, co) != c || top == e.zoff) {
					top = bot = 0;
				} else {
					top = occ1(e, s2, top, c);     // (s2 holds side st here)
					bot = top + 1;
				}
			}
			if(bot <= top) {
				nedit++;
				if(nedit >= mine_max) { mine = nedit; done = true; }
				doinit = true;
			}
			dep++;
		}
	}
	uint32_t otop = 0, obot = 0;
	if(active && !done && dep >= len) {
		mine = nedit;
		if(nedit == 0 && bot > top) { otop = top; obot = bot; }
	}
	// bwops / side loads of the read = sum of both strands: the pair's lanes are
	// neighbours in one wave (2r, 2r+1), so the sum is a lane swap and the read's
	// words are plain stores (no memset of the output before the launch)
	const uint32_t bw2 = bwops + (uint32_t)__shfl_xor((int)bwops, 1);
	const uint32_t ld2 = loads + (uint32_t)__shfl_xor((int)loads, 1);
	if(!valid) return;
	out[(size_t)r * 8 + strand] = mine;
	out[(size_t)r * 8 + 2 + 2 * strand] = otop;
	out[(size_t)r * 8 + 3 + 2 * strand] = obot;
	out[(size_t)r * 8 + 6 + strand] = strand == 0 ? bw2 : ld2;
}

// The exact sweep with a quad of lanes per (read, strand) (fm_device.h, the
// cooperative step): lanes 8r..8r+3 strand 0 of read r, 8r+4..8r+7 strand 1.
// Same control flow and outputs as k_exact_sweep, lane for quad.
__global__ void __launch_bounds__(256)
k_exact_sweep_quad(DevEbwt e, const uint8_t* __restrict__ reads, uint32_t stride, const uint32_t* __restrict__ lens,
                   uint32_t n, uint32_t mine_max, int nofw, int norc, uint32_t* __restrict__ out) {
	walk_prio();
	const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t q = gid & 3u, chain = gid >> 2;
	const uint32_t r = chain >> 1, strand = chain & 1u;
	const bool valid = r < n;
	const bool active = valid && !((strand == 0 && nofw) || (strand == 1 && norc));
	const uint32_t len = active ? lens[r] : 0;
	ReadWin rw{reads, reads + (size_t)n * stride};
	const uint8_t* row = reads + (size_t)(active ? r : 0) * stride;
	auto seq_at = [&](uint32_t k) -> int {
		const int c = rw.at(row + (strand == 1 ? len - 1 - k : k));
		return strand == 1 ? (c > 3 ? 4 : 3 - c) : c;
	};
	auto base_at = [&](uint32_t d) -> int { return seq_at(len - d - 1); };
	const uint32_t flen = e.ftab_chars;
	uint32_t dep = 0, nedit = 0, top = 0, bot = 0, mine = 0;
	uint32_t bwops = 0, loads = 0;
	bool doinit = true, done = !active;
	while(dep < len && !done) {
		if(doinit) {
			top = bot = 0;
			uint32_t left = len - dep;
			bool doftab = flen > 1 && left >= flen;
			uint32_t fi = 0;
			if(doftab) {
				for(uint32_t i = 0; i < flen; i++) {
					int c = seq_at(left - flen + i);
					if(c > 3) { doftab = false; break; }
					fi = (fi << 2) | (uint32_t)c;
				}
			}
			if(doftab) {
				const uint32_t v0 = e.ftab[fi], v1 = e.ftab[fi + 1];
				const bool x0 = v0 > e.len, x1 = v1 > e.len;
				const uint32_t et = x0 ? e.eftab[(v0 ^ BT2G_OFF_MASK) * 2 + 1] : v0;
				const uint32_t eb = x1 ? e.eftab[(v1 ^ BT2G_OFF_MASK) * 2] : v1;
				top = et;
				bot = eb;
				dep += flen;
			} else {
				int c = seq_at(len - dep - 1);
				if(c < 4) { top = fchr_at(e, c); bot = fchr_at(e, c + 1); }
				dep++;
			}
			if(bot <= top) {
				nedit++;
				if(nedit >= mine_max) { mine = nedit; done = true; }
				continue;
			}
			doinit = false;
		}
		if(dep < len) {
			const int c = base_at(dep);
			const bool rng = bot - top > 1;
			const uint32_t st = top / 192u, sb = rng ? bot / 192u : st;
			QuadSide s1, s2;
			load_quad(e, st, q, s1);
			load_quad(e, sb, q, s2);
			if(c > 3) {
				top = bot = 0;
			} else if(rng) {
				bwops += 2;
				loads += sb == st ? 1u : 2u;
				uint32_t nt, nb;
				quad_occ2(e, s1, s2, q, top, bot, c, nt, nb);
				top = nt; bot = nb;
			} else {
				bwops += 1;
				loads++;
				if(quad_rowL(s1, q, top % 192u) != c || top == e.zoff) {
					top = bot = 0;
				} else {
					top = quad_occ1(e, s1, q, top, c);
					bot = top + 1;
				}
			}
			if(bot <= top) {
				nedit++;
				if(nedit >= mine_max) { mine = nedit; done = true; }
				doinit = true;
			}
			dep++;
		}
	}
	uint32_t otop = 0, obot = 0;
	if(active && !done && dep >= len) {
		mine = nedit;
		if(nedit == 0 && bot > top) { otop = top; obot = bot; }
	}
	// both strands' bwops / side loads: the other strand's quad is 4 lanes away
	const uint32_t bw2 = bwops + (uint32_t)__shfl_xor((int)bwops, 4);
	const uint32_t ld2 = loads + (uint32_t)__shfl_xor((int)loads, 4);
	if(!valid || q != 0) return;
	out[(size_t)r * 8 + strand] = mine;
	out[(size_t)r * 8 + 2 + 2 * strand] = otop;
	out[(size_t)r * 8 + 3 + 2 * strand] = obot;
	out[(size_t)r * 8 + 6 + strand] = strand == 0 ? bw2 : ld2;
}

// --------------------------------------------------------------------------
// Exact seeds: instantiateSeeds (aligner_seed.cpp:498-587, Seed::instantiate
// 214-358) + searchSeedBi for SEED_TYPE_EXACT (80-122, 1633-1714, 1854-2033).
// One lane = one (read, strand, seed offset).
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BT2G_SEED_WAVES)))
k_seed_search(DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, uint32_t stride,
              const uint32_t* __restrict__ lens, uint32_t n, uint32_t seedlen, uint32_t interval,
              uint32_t offset, uint32_t maxseeds, uint32_t* __restrict__ out, int32_t* __restrict__ nseeds,
              uint32_t* __restrict__ bwops, uint32_t* __restrict__ loads_out) {
	walk_prio();
	uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
	uint32_t per = 2 * maxseeds;
	uint32_t r = gid / per, rem = gid % per, strand = rem / maxseeds, s = rem % maxseeds;
	if(r >= n) return;
	const uint32_t len = lens[r];
	uint32_t* o = out + (((size_t)r * 2 + strand) * maxseeds + s) * 4;
	o[0] = o[1] = o[2] = o[3] = 0;
	bool skip = offset > 0 && seedlen + offset > len;
	int ns = 0;
	if(!skip) {
		ns = 1;
		if((int)len - (int)offset > (int)seedlen) ns += ((int)len - (int)offset - (int)seedlen) / (int)interval;
	}
	if(gid % per == 0) nseeds[r] = ns;
	uint32_t ops = 0, loads = 0;
	if(!skip && (int)s < ns) {
		const uint32_t L = seedlen < len ? seedlen : len;
		const uint32_t depth = s * interval + offset;
		const uint8_t* rd = reads + (size_t)r * stride;
		// seed string as aligned to Watson: fw -> rd[depth+i]; rc -> comp(rd[depth+L-1-i])
		SeqView seq{rd + depth, L, strand == 1, strand == 1};
		bool hasn = false;
		for(uint32_t i = 0; i < L; i++) hasn |= seq[i] > 3;
		if(!hasn) {
			uint32_t topf, botf, topb, botb, step;
			const uint32_t flen = F.ftab_chars;
			bool dead = false;
			if(flen > 1 && flen <= L) {
				uint32_t off = L - flen, fi = 0, bi = 0;
				for(uint32_t i = 0; i < flen; i++) {
					fi = (fi << 2) | (uint32_t)seq[off + i];
					bi = (bi << 2) | (uint32_t)seq[off + flen - 1 - i];
				}
				topf = ftab_hi(F, fi);
				botf = ftab_lo(F, fi + 1);
				dead = botf == topf;
				topb = ftab_hi(B, bi);
				botb = topb + (botf - topf);
				step = flen;
			} else {
				int c = seq[L - 1];
				topf = topb = fchr_at(F, c);
				botf = botb = fchr_at(F, c + 1);
				dead = botf == topf;
				step = 1;
			}
			for(; !dead && step < L; step++) {
				int c = seq[L - step - 1];
				ops++;
				if(botf - topf > 1) {
					uint32_t t[4], b[4], tp[4], bp[4];
					tp[0] = topb;
					loads += bi_step(F, topf, botf, topb, t, b, tp, bp);
					if(b[c] == t[c]) { dead = true; break; }
					topf = t[c]; botf = b[c]; topb = tp[c]; botb = bp[c];
				} else {
					SideData s1;
					load_side(F, topf / 192u, s1);
					loads++;
					uint32_t co = topf % 192u;
					if(side_rowL(s1, co) != c || topf == F.zoff) { dead = true; break; }
					topf = occ1(F, s1, topf, c);
					botf = topf + 1;
				}
			}
			if(!dead) { o[0] = topf; o[1] = botf; o[2] = topb; o[3] = botb; }
		}
	}
	// per-read FM-op total (SeedSearchMetrics::bwops): wave-level sum over the
	// read's lanes would need a segmented reduction; a device atomic is cheap here.
	if(ops) atomicAdd(&bwops[r], ops);
	if(loads && loads_out) atomicAdd(&loads_out[r], loads);
}

// --------------------------------------------------------------------------
// oneMmSearch: the search itself is fm_one_mm.hip (work-queue kernel); its
// per-(read, strand, index) slots are concatenated here in the reference's
// loop order (fw/BWT, fw/BWT', rc/BWT, rc/BWT').
// --------------------------------------------------------------------------
// Concatenate the 4 per-direction slots of each read in discovery order.  A
// slot's hits arrive out of order (branches finish in the branch kernel), each
// tagged with its discovery number in `pad`: they are put back in order here.
__global__ void k_one_mm_compact(bt2g_mm1* __restrict__ slots, const int32_t* __restrict__ slot_counts,
                                 uint32_t n, uint32_t cap, bt2g_mm1* __restrict__ hits, int32_t* __restrict__ counts,
                                 int32_t* __restrict__ overflow) {
	uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
	if(r >= n) return;
	int32_t k = 0;
	bool ovf = false;
	for(int s = 0; s < 4; s++) {
		const int32_t c = slot_counts[(size_t)r * 4 + s];
		if((uint32_t)c > cap) ovf = true;
		bt2g_mm1* sl = slots + ((size_t)r * 4 + s) * cap;
		const int32_t m = c < (int32_t)cap ? c : (int32_t)cap;
		for(int32_t i = 1; i < m; i++) {                 // insertion sort by discovery number (m <= cap)
			const bt2g_mm1 h = sl[i];
			int32_t j = i - 1;
			while(j >= 0 && (uint32_t)sl[j].pad > (uint32_t)h.pad) { sl[j + 1] = sl[j]; j--; }
			sl[j + 1] = h;
		}
		for(int32_t i = 0; i < m; i++) {
			if((uint32_t)k < cap) {
				bt2g_mm1 h = sl[i];
				h.pad = 0;
				hits[(size_t)r * cap + k] = h;
			}
			k++;
		}
		if((uint32_t)c > cap) k += c - (int32_t)cap;
	}
	counts[r] = k;
	if(ovf || (uint32_t)k > cap) atomicOr(overflow, 1);
}

// --------------------------------------------------------------------------
// Ebwt::getOffset (bt2_idx.cpp:150-171): one lane = one SA row.
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_get_offset(DevEbwt e, const uint32_t* __restrict__ rows, uint32_t n, uint32_t* __restrict__ offs,
             uint32_t* __restrict__ loads_out) {
	walk_prio();
	uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if(i >= n) return;
	uint32_t row = rows[i];
	const uint32_t mask = BT2G_OFF_MASK << e.off_rate;
	uint32_t res, jumps = 0, loads = 0;
	if(row == e.zoff) res = 0;
	else if((row & mask) == row) res = e.offs[row >> e.off_rate];
	else {
		for(;;) {
			SideData s;
			load_side(e, row / 192u, s);
			loads++;
			int c = side_rowL(s, row % 192u);
			row = occ1(e, s, row, c);
			jumps++;
			if(row == e.zoff) { res = jumps; break; }
			if((row & mask) == row) { res = jumps + e.offs[row >> e.off_rate]; break; }
		}
	}
	offs[i] = res;
	if(loads_out) loads_out[i] = loads;
}

// --------------------------------------------------------------------------
// launchers
// --------------------------------------------------------------------------
void launch_exact_sweep(const DevEbwt& e, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t n,
                        uint32_t mine_max, int nofw, int norc, uint32_t* out, hipStream_t st) {
	// $BT2G_FM_QUAD=0: one lane per (read, strand); default (round 6): a quad of
	// lanes per walk (k_exact_sweep_quad) -- read at every launch (A/B in one process)
	const char* qe = getenv("BT2G_FM_QUAD");
	if(!(qe && *qe == '0')) {
		const uint64_t threads = (uint64_t)n * 8;
		hipLaunchKernelGGL(k_exact_sweep_quad, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, st, e, reads,
		                   stride, lens, n, mine_max, nofw, norc, out);
		return;
	}
	const uint32_t threads = n * 2;
	hipLaunchKernelGGL(k_exact_sweep, dim3((threads + 255) / 256), dim3(256), 0, st, e, reads, stride, lens, n,
	                   mine_max, nofw, norc, out);
}

void launch_seed_search(const DevEbwt& F, const DevEbwt& B, const uint8_t* reads, uint32_t stride,
                        const uint32_t* lens, uint32_t n, uint32_t seedlen, uint32_t interval, uint32_t offset,
                        uint32_t maxseeds, uint32_t* out, int32_t* nseeds, uint32_t* bwops, uint32_t* loads,
                        hipStream_t st) {
	uint64_t threads = (uint64_t)n * 2 * maxseeds;
	hipLaunchKernelGGL(k_seed_search, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, st, F, B, reads,
	                   stride, lens, n, seedlen, interval, offset, maxseeds, out, nseeds, bwops, loads);
}

void launch_one_mm(const DevEbwt& F, const DevEbwt& B, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                   const uint32_t* lens, uint32_t n, const int32_t* minsc, const bt2g_scoring& sc, int nofw,
                   int norc, const uint32_t* gate, uint32_t cap, uint32_t* items, uint32_t* counters,
                   uint4* near_state, uint32_t* near_dep, bt2g_mm1* slots, int32_t* slot_counts, bt2g_mm1* hits,
                   int32_t* counts, uint32_t* ops, uint32_t* loads, int32_t* overflow, MmBranch* brq,
                   uint32_t brq_cap, uint32_t* fb_items, uint4* fb_st4, uint32_t* fb_sdep, uint32_t* slot_flag,
                   hipStream_t st, hipStream_t st2, hipEvent_t* ev) {
	launch_one_mm_q(F, B, reads, quals, stride, lens, n, minsc, sc, nofw, norc, gate, cap, items, counters,
	                near_state, near_dep, slots, slot_counts, ops, loads, brq, brq_cap, fb_items, fb_st4, fb_sdep,
	                slot_flag, st, st2, ev);
	hipLaunchKernelGGL(k_one_mm_compact, dim3((n + 255) / 256), dim3(256), 0, st, slots, slot_counts, n, cap, hits,
	                   counts, overflow);
}

void launch_get_offset(const DevEbwt& e, const uint32_t* rows, uint32_t n, uint32_t* offs, uint32_t* loads,
                       hipStream_t st) {
	hipLaunchKernelGGL(k_get_offset, dim3((n + 255) / 256), dim3(256), 0, st, e, rows, n, offs, loads);
}

// The offsets of the rows of every small SA range an up-front search reported
// (bt2g_exact_sweep_1mm): the exact end-to-end ranges of each strand (sweep
// n x 8: mine, range) and the 1-mm hits (hits n x cap, counts); one lane per
// (read, range, row), ranges of more than off_cap rows skipped.  offs: n x
// (2 + cap) x off_cap, BT2G_OFF_MASK where no row.  The same walk as
// k_get_offset (Ebwt::getOffset, bt2_idx.cpp:150-171).
__device__ __forceinline__ uint32_t row_offset(const DevEbwt& e, uint32_t row) {
	const uint32_t mask = BT2G_OFF_MASK << e.off_rate;
	if(row == e.zoff) return 0;
	if((row & mask) == row) return e.offs[row >> e.off_rate];
	for(uint32_t jumps = 1;; jumps++) {
		SideData sd;
		load_side(e, row / 192u, sd);
		const int c = side_rowL(sd, row % 192u);
		row = occ1(e, sd, row, c);
		if(row == e.zoff) return jumps;
		if((row & mask) == row) return jumps + e.offs[row >> e.off_rate];
	}
}

__global__ void __launch_bounds__(256)
k_range_offsets(DevEbwt e, const uint32_t* __restrict__ sweep, const bt2g_mm1* __restrict__ hits,
                const int32_t* __restrict__ counts, uint32_t n, uint32_t cap, uint32_t off_cap,
                uint32_t* __restrict__ offs) {
	walk_prio();
	const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	const uint64_t per = (uint64_t)(2u + cap) * off_cap;
	if(gid >= (uint64_t)n * per) return;
	const uint32_t i = (uint32_t)(gid / per), slot = (uint32_t)((gid % per) / off_cap), j = (uint32_t)(gid % off_cap);
	uint32_t top = 0, bot = 0;
	if(slot < 2) {
		const uint32_t* w = sweep + (size_t)i * 8;
		if(w[slot] == 0) { top = w[2 + 2 * slot]; bot = w[3 + 2 * slot]; }
	} else if(hits && (int32_t)(slot - 2) < (counts[i] < (int32_t)cap ? counts[i] : (int32_t)cap)) {
		const bt2g_mm1 h = hits[(size_t)i * cap + (slot - 2)];
		top = h.top;
		bot = h.bot;
	}
	offs[gid] = (bot > top && bot - top <= off_cap && j < bot - top) ? row_offset(e, top + j) : BT2G_OFF_MASK;
}

// The same for the seed ranges of one seed round (bt2g_seed_search_ext): out
// n x 2 x maxseeds x 4 as k_seed_search wrote it, offs n x 2 x maxseeds x off_cap.
__global__ void __launch_bounds__(256)
k_seed_offsets(DevEbwt e, const uint32_t* __restrict__ out, uint64_t nrange, uint32_t off_cap,
               uint32_t* __restrict__ offs) {
	walk_prio();
	const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if(gid >= nrange * off_cap) return;
	const uint64_t k = gid / off_cap;
	const uint32_t j = (uint32_t)(gid % off_cap), top = out[k * 4], bot = out[k * 4 + 1];
	offs[gid] = (bot > top && bot - top <= off_cap && j < bot - top) ? row_offset(e, top + j) : BT2G_OFF_MASK;
}

void launch_seed_offsets(const DevEbwt& e, const uint32_t* out, uint64_t nrange, uint32_t off_cap, uint32_t* offs,
                         hipStream_t st) {
	const uint64_t tot = nrange * off_cap;
	if(!tot) return;
	hipLaunchKernelGGL(k_seed_offsets, dim3((uint32_t)((tot + 255) / 256)), dim3(256), 0, st, e, out, nrange, off_cap,
	                   offs);
}

void launch_range_offsets(const DevEbwt& e, const uint32_t* sweep, const bt2g_mm1* hits, const int32_t* counts,
                          uint32_t n, uint32_t cap, uint32_t off_cap, uint32_t* offs, hipStream_t st) {
	const uint64_t tot = (uint64_t)n * (2u + cap) * off_cap;
	if(!tot) return;
	hipLaunchKernelGGL(k_range_offsets, dim3((uint32_t)((tot + 255) / 256)), dim3(256), 0, st, e, sweep, hits, counts,
	                   n, cap, off_cap, offs);
}

// --------------------------------------------------------------------------
// SwDriver::extend (aligner_sw_driver.cpp:299-483): one lane = one seed-hit
// range.  Left: the range walks leftward in the forward index while it keeps
// its size and its one extending character agrees with the read (an N in the
// read takes any single character); right: the same in the mirror index.
// A one-row range steps by mapLF1 (bt2_idx.h:2451-2470, no step from the '$'
// row); the loop stops at 255 positions per side, as the reference does.
// --------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ext_walk(const DevEbwt& e, uint32_t top, uint32_t bot, const uint8_t* row,
                                             uint32_t rdlen, bool fw, uint32_t lim, uint32_t i0, int dir,
                                             uint32_t& fmops, uint32_t& loads) {
	uint32_t n = 0;
	for(uint32_t ii = 0; ii < lim; ii++) {
		const uint32_t i = (uint32_t)((int64_t)i0 + (int64_t)dir * ii);
		int rdc = fw ? row[i] : row[rdlen - 1 - i];
		if(!fw) rdc = rdc > 3 ? 4 : 3 - rdc;
		fmops++;
		if(bot - top > 1) {
			uint32_t t[4], b[4];
			loads += (uint32_t)bi_step_tb(e, top, bot, t, b);
			int nonz = -1;
			bool abort = false;
			const uint32_t orig = bot - top;
			for(int j = 0; j < 4; j++) {
				if(b[j] > t[j]) {
					if(nonz >= 0) { abort = true; break; }
					nonz = j;
					top = t[j];
					bot = b[j];
				}
			}
			if(abort || (nonz != rdc && rdc <= 3) || bot - top < orig) break;
		} else {
			int c = -1;
			if(top != e.zoff) {
				SideData s;
				loads++;
				load_side(e, top / 192u, s);
				c = side_rowL(s, top % 192u);
				top = occ1(e, s, top, c);
			}
			if(c != rdc && rdc <= 3) break;
			bot = top + 1;
		}
		if(++n == 255u) break;
	}
	return n;
}

__device__ __forceinline__ bt2g_ext_out ext_one(const DevEbwt& F, const DevEbwt& B, int has_bw, const uint8_t* row,
                                                uint32_t rdlen, const bt2g_ext_in& q) {
	const bool fw = q.fw != 0;
	uint32_t fmops = 0, nlex = 0, nrex = 0, loads = 0;
	// left, forward index (aligner_sw_driver.cpp:335-408)
	uint32_t lim = fw ? q.off : rdlen - q.len - q.off;
	if(lim > 0)
		nlex = ext_walk(F, q.topf, q.botf, row, rdlen, fw, lim, fw ? q.off - 1 : rdlen - q.off - q.len - 1, -1, fmops, loads);
	// right, mirror index (aligner_sw_driver.cpp:411-475)
	lim = fw ? rdlen - q.len - q.off : q.off;
	if(lim > 0 && has_bw)
		nrex = ext_walk(B, q.topb, q.botb, row, rdlen, fw, lim, fw ? q.len + q.off : rdlen - q.off, 1, fmops, loads);
	return bt2g_ext_out{nlex, nrex, fmops, loads};
}

__global__ void __launch_bounds__(256)
k_extend(DevEbwt F, DevEbwt B, int has_bw, const uint8_t* __restrict__ reads, uint32_t stride,
         const uint32_t* __restrict__ lens, const bt2g_ext_in* __restrict__ in, uint32_t n, bt2g_ext_out* __restrict__ out) {
	walk_prio();
	const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
	if(k >= n) return;
	const bt2g_ext_in q = in[k];
	out[k] = ext_one(F, B, has_bw, reads + (size_t)q.read * stride, lens[q.read], q);
}

void launch_extend(const DevEbwt& F, const DevEbwt& B, int has_bw, const uint8_t* reads, uint32_t stride,
                   const uint32_t* lens, const bt2g_ext_in* in, uint32_t n, bt2g_ext_out* out, hipStream_t st) {
	if(n == 0) return;
	hipLaunchKernelGGL(k_extend, dim3((n + 255) / 256), dim3(256), 0, st, F, B, has_bw, reads, stride, lens, in, n, out);
}

// SwDriver::extend for every range of one seed round, as prioritizeSATups would
// ask it (bt2g_seed_search_ext): one lane = one (read, strand, seed); the seed
// at depth s * interval + offset, min(seedlen, len) long (k_seed_search).
// ext[k] = {0, 0, 0, 0} where the seed has no range.
__global__ void __launch_bounds__(256)
k_seed_extend(DevEbwt F, DevEbwt B, int has_bw, const uint8_t* __restrict__ reads, uint32_t stride,
              const uint32_t* __restrict__ lens, uint32_t n, uint32_t seedlen, uint32_t interval, uint32_t offset,
              uint32_t maxseeds, const uint32_t* __restrict__ out, bt2g_ext_out* __restrict__ ext) {
	walk_prio();
	const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if(gid >= (uint64_t)n * 2 * maxseeds) return;
	const uint32_t r = (uint32_t)(gid / (2u * maxseeds)), rem = (uint32_t)(gid % (2u * maxseeds));
	const uint32_t strand = rem / maxseeds, s = rem % maxseeds;
	const uint32_t* o = out + gid * 4;
	const uint32_t len = lens[r], L = seedlen < len ? seedlen : len, depth = s * interval + offset;
	bt2g_ext_out res{0u, 0u, 0u, 0u};
	if(o[1] > o[0] && depth + L <= len) {
		bt2g_ext_in q;
		q.read = r;
		q.fw = strand == 0 ? 1 : 0;
		q.off = depth;
		q.len = L;
		q.topf = o[0];
		q.botf = o[1];
		q.topb = o[2];
		q.botb = o[3];
		res = ext_one(F, B, has_bw, reads + (size_t)r * stride, len, q);
	}
	ext[gid] = res;
}

// ext_walk / ext_one with a quad of lanes per range (fm_device.h)
__device__ __forceinline__ uint32_t ext_walk_quad(const DevEbwt& e, uint32_t q, uint32_t top, uint32_t bot,
                                                  const uint8_t* row, uint32_t rdlen, bool fw, uint32_t lim, uint32_t i0,
                                                  int dir, uint32_t& fmops, uint32_t& loads) {
	uint32_t n = 0;
	for(uint32_t ii = 0; ii < lim; ii++) {
		const uint32_t i = (uint32_t)((int64_t)i0 + (int64_t)dir * ii);
		int rdc = fw ? row[i] : row[rdlen - 1 - i];
		if(!fw) rdc = rdc > 3 ? 4 : 3 - rdc;
		fmops++;
		if(bot - top > 1) {
			uint32_t t[4], b[4];
			loads += (uint32_t)quad_bi_step_tb(e, q, top, bot, t, b);
			int nonz = -1;
			bool abort = false;
			const uint32_t orig = bot - top;
			for(int j = 0; j < 4; j++) {
				if(b[j] > t[j]) {
					if(nonz >= 0) { abort = true; break; }
					nonz = j;
					top = t[j];
					bot = b[j];
				}
			}
			if(abort || (nonz != rdc && rdc <= 3) || bot - top < orig) break;
		} else {
			int c = -1;
			if(top != e.zoff) {
				QuadSide s;
				loads++;
				load_quad(e, top / 192u, q, s);
				c = quad_rowL(s, q, top % 192u);
				top = quad_occ1(e, s, q, top, c);
			}
			if(c != rdc && rdc <= 3) break;
			bot = top + 1;
		}
		if(++n == 255u) break;
	}
	return n;
}

__device__ __forceinline__ bt2g_ext_out ext_one_quad(const DevEbwt& F, const DevEbwt& B, int has_bw, uint32_t q,
                                                     const uint8_t* row, uint32_t rdlen, const bt2g_ext_in& x) {
	const bool fw = x.fw != 0;
	uint32_t fmops = 0, nlex = 0, nrex = 0, loads = 0;
	uint32_t lim = fw ? x.off : rdlen - x.len - x.off;
	if(lim > 0)
		nlex = ext_walk_quad(F, q, x.topf, x.botf, row, rdlen, fw, lim, fw ? x.off - 1 : rdlen - x.off - x.len - 1, -1,
		                     fmops, loads);
	lim = fw ? rdlen - x.len - x.off : x.off;
	if(lim > 0 && has_bw)
		nrex = ext_walk_quad(B, q, x.topb, x.botb, row, rdlen, fw, lim, fw ? x.len + x.off : rdlen - x.off, 1, fmops,
		                     loads);
	return bt2g_ext_out{nlex, nrex, fmops, loads};
}

// k_seed_extend with a quad per (read, strand, seed): lanes 4k..4k+3 for range k
__global__ void __launch_bounds__(256)
k_seed_extend_quad(DevEbwt F, DevEbwt B, int has_bw, const uint8_t* __restrict__ reads, uint32_t stride,
                   const uint32_t* __restrict__ lens, uint32_t n, uint32_t seedlen, uint32_t interval, uint32_t offset,
                   uint32_t maxseeds, const uint32_t* __restrict__ out, bt2g_ext_out* __restrict__ ext) {
	walk_prio();
	const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	const uint64_t gid = lane >> 2;
	const uint32_t q = (uint32_t)(lane & 3u);
	if(gid >= (uint64_t)n * 2 * maxseeds) return;
	const uint32_t r = (uint32_t)(gid / (2u * maxseeds)), rem = (uint32_t)(gid % (2u * maxseeds));
	const uint32_t strand = rem / maxseeds, s = rem % maxseeds;
	const uint32_t* o = out + gid * 4;
	const uint32_t len = lens[r], L = seedlen < len ? seedlen : len, depth = s * interval + offset;
	bt2g_ext_out res{0u, 0u, 0u, 0u};
	if(o[1] > o[0] && depth + L <= len) {
		bt2g_ext_in x;
		x.read = r;
		x.fw = strand == 0 ? 1 : 0;
		x.off = depth;
		x.len = L;
		x.topf = o[0];
		x.botf = o[1];
		x.topb = o[2];
		x.botb = o[3];
		res = ext_one_quad(F, B, has_bw, q, reads + (size_t)r * stride, len, x);
	}
	if(q == 0) ext[gid] = res;
}

// $BT2G_FM_QUAD=0: the one-lane FM kernels (read at every launch)
static bool fm_quad() {
	const char* e = getenv("BT2G_FM_QUAD");
	return !(e && *e == '0');
}

void launch_seed_extend(const DevEbwt& F, const DevEbwt& B, int has_bw, const uint8_t* reads, uint32_t stride,
                        const uint32_t* lens, uint32_t n, uint32_t seedlen, uint32_t interval, uint32_t offset,
                        uint32_t maxseeds, const uint32_t* out, bt2g_ext_out* ext, hipStream_t st) {
	const uint64_t tot = (uint64_t)n * 2 * maxseeds;
	if(!tot) return;
	if(fm_quad()) {
		hipLaunchKernelGGL(k_seed_extend_quad, dim3((uint32_t)((4 * tot + 255) / 256)), dim3(256), 0, st, F, B, has_bw,
		                   reads, stride, lens, n, seedlen, interval, offset, maxseeds, out, ext);
		return;
	}
	hipLaunchKernelGGL(k_seed_extend, dim3((uint32_t)((tot + 255) / 256)), dim3(256), 0, st, F, B, has_bw, reads, stride,
	                   lens, n, seedlen, interval, offset, maxseeds, out, ext);
}
