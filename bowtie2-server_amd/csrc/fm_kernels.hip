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
__global__ void __launch_bounds__(256)
k_exact_sweep(DevEbwt e, const uint8_t* __restrict__ reads, uint32_t stride, const uint32_t* __restrict__ lens,
              uint32_t n, uint32_t mine_max, int nofw, int norc, uint32_t* __restrict__ out) {
	uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
	uint32_t r = gid >> 1, strand = gid & 1;
	// lanes 2r and 2r+1 always share a wave; no early return before the shuffle
	const bool valid = r < n;
	const bool active = valid && !((strand == 0 && nofw) || (strand == 1 && norc));
	const uint32_t len = active ? lens[r] : 0;
	SeqView seq{reads + (size_t)(active ? r : 0) * stride, len, strand == 1, strand == 1};
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
				// ftabSeqToInt(seq, left-flen, rev=false) on the forward index
				for(uint32_t i = 0; i < flen; i++) {
					int c = seq[left - flen + i];
					if(c > 3) { doftab = false; break; }
					fi = (fi << 2) | (uint32_t)c;
				}
			}
			if(doftab) {
				top = ftab_hi(e, fi);
				bot = ftab_lo(e, fi + 1);
				dep += flen;
			} else {
				int c = seq[len - dep - 1];
				if(c < 4) { top = e.fchr[c]; bot = e.fchr[c + 1]; }
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
			int c = seq[len - dep - 1];
			if(c > 3) {
				top = bot = 0;
			} else if(bot - top > 1) {
				bwops += 2;
				uint32_t st = top / 192u, sb = bot / 192u;
				SideData s1;
				load_side(e, st, s1);
				loads++;
				uint32_t nt = occ1(e, s1, top, c), nb;
				if(sb == st) {
					nb = occ1(e, s1, bot, c);
				} else {
					SideData s2;
					load_side(e, sb, s2);
					loads++;
					nb = occ1(e, s2, bot, c);
				}
				top = nt; bot = nb;
			} else {
				bwops += 1;
				SideData s1;
				load_side(e, top / 192u, s1);
				loads++;
				uint32_t co = top % 192u;
				if(side_rowL(s1, co) != c || top == e.zoff) {
					top = bot = 0;
				} else {
					top = occ1(e, s1, top, c);
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
	// bwops / loads of the read = sum of both strands (the pair shares a wave)
	uint32_t ob = __shfl_xor(bwops, 1), ol = __shfl_xor(loads, 1);
	if(!valid) return;
	out[(size_t)r * 8 + strand] = mine;
	out[(size_t)r * 8 + 2 + 2 * strand] = otop;
	out[(size_t)r * 8 + 3 + 2 * strand] = obot;
	if(strand == 0) {
		out[(size_t)r * 8 + 6] = bwops + ob;
		out[(size_t)r * 8 + 7] = loads + ol;
	}
}

// --------------------------------------------------------------------------
// Exact seeds: instantiateSeeds (aligner_seed.cpp:498-587, Seed::instantiate
// 214-358) + searchSeedBi for SEED_TYPE_EXACT (80-122, 1633-1714, 1854-2033).
// One lane = one (read, strand, seed offset).
// --------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_seed_search(DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, uint32_t stride,
              const uint32_t* __restrict__ lens, uint32_t n, uint32_t seedlen, uint32_t interval,
              uint32_t offset, uint32_t maxseeds, uint32_t* __restrict__ out, int32_t* __restrict__ nseeds,
              uint32_t* __restrict__ bwops, uint32_t* __restrict__ loads_out) {
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
				topf = topb = F.fchr[c];
				botf = botb = F.fchr[c + 1];
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
// oneMmSearch (aligner_seed.cpp:973-1323) with rep1mm=true, repex=false.
// One lane = one (read, strand, index direction); the 4 lanes of a read write
// their hits into 4 slots that are concatenated in the reference's loop order
// (fw/BWT, fw/BWT', rc/BWT, rc/BWT') by k_one_mm_compact.
// --------------------------------------------------------------------------
struct MmParams {
	int32_t match, mmp_max, mmp_min, npen, local;
	int32_t nceil_const_x1000, nceil_lin_x1000;
};

__device__ __forceinline__ int mmpen_q(const MmParams& p, int q) {
	int ii = q < 40 ? q : 40;
	float frac = (float)ii / 40.0f;
	return p.mmp_min + (int)(frac * (float)(p.mmp_max - p.mmp_min));
}

__global__ void __launch_bounds__(256)
k_one_mm(DevEbwt F, DevEbwt B, const uint8_t* __restrict__ reads, const uint8_t* __restrict__ quals,
         uint32_t stride, const uint32_t* __restrict__ lens, uint32_t n, const int32_t* __restrict__ minscs,
         MmParams P, double ncl_const, double ncl_lin, int nofw, int norc, const uint32_t* __restrict__ gate,
         uint32_t cap, bt2g_mm1* __restrict__ slots, int32_t* __restrict__ slot_counts, uint32_t* __restrict__ ops_out,
         uint32_t* __restrict__ loads_out) {
	uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
	uint32_t r = gid >> 2, fwi = (gid >> 1) & 1, ebwtfwi = gid & 1;
	if(r >= n) return;
	int32_t nh = 0;
	uint32_t ops = 0, loads = 0;
	bt2g_mm1* myslot = slots + ((size_t)r * 4 + fwi * 2 + ebwtfwi) * cap;
	const bool fw = fwi == 0, ebwtfw = ebwtfwi == 0;
	const uint32_t len = lens[r];
	const uint8_t* rd = reads + (size_t)r * stride;
	const uint8_t* qd = quals + (size_t)r * stride;
	uint32_t ns = 0;
	for(uint32_t i = 0; i < len; i++) ns += rd[i] > 3;
	int nceil = (int)(ncl_const + ncl_lin * (double)len);
	if(nceil < 0) nceil = 0;
	const int64_t minsc = minscs[r];
	bool nofw_r = nofw, norc_r = norc, gated_off = false;
	if(gate) {
		// bt2_search.cpp:3476-3506, 3640-3667: skipped when an exact end-to-end hit
		// exists (bestmin == 0); otherwise nofw = !(mineFw <= 1), norc = !(mineRc <= 1).
		uint32_t mfw = gate[(size_t)r * 8 + 0], mrc = gate[(size_t)r * 8 + 1];
		uint32_t bestmin = mfw < mrc ? mfw : mrc;
		bool yfw = mfw <= 1 && !nofw, yrc = mrc <= 1 && !norc;
		gated_off = bestmin == 0 || !(yfw || yrc);
		nofw_r = !yfw; norc_r = !yrc;
	}
	bool run = !gated_off && ns <= 1 && !((fw && nofw_r) || (!fw && norc_r));
	if(run) {
		const DevEbwt& E = ebwtfw ? F : B;
		const DevEbwt& Ep = ebwtfw ? B : F;
		// seq = fw ? (ebwtfw ? patFw : patFwRev) : (ebwtfw ? patRc : patRcRev)
		SeqView seq{rd, len, fw ? !ebwtfw : ebwtfw, !fw};
		// qual = fw ? (ebwtfw ? qual : qualRev) : (ebwtfw ? qualRev : qual)
		const bool qrev = fw ? !ebwtfw : ebwtfw;
		const uint32_t halfFw = len >> 1, halfBw = (len >> 1) + (len & 1);
		const uint32_t nea = ebwtfw ? halfFw : halfBw;
		const uint32_t flen = E.ftab_chars;
		const int64_t matchsc = (int64_t)((float)P.match + 0.5f);
		bool skip = false;
		for(uint32_t dep = 0; dep < nea; dep++) if(seq[len - dep - 1] > 3) { skip = true; break; }
		uint32_t t[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0}, tp[4] = {0, 0, 0, 0}, bp[4] = {0, 0, 0, 0};
		uint32_t top = 0, bot = 0, topp = 0, botp = 0, dep = 0;
		if(!skip) {
			if(flen > 1 && flen <= nea) {
				// ftabSeqToInt(seq, len-flen, rev=!ebwtfw): for E it reads left-to-right,
				// for Ep right-to-left (bt2_idx.h:1383-1390)
				uint32_t fi = 0, fip = 0;
				for(uint32_t i = 0; i < flen; i++) {
					fi = (fi << 2) | (uint32_t)seq[len - flen + i];
					fip = (fip << 2) | (uint32_t)seq[len - 1 - i];
				}
				top = ftab_hi(E, fi); bot = ftab_lo(E, fi + 1);
				topp = ftab_hi(Ep, fip); botp = ftab_lo(Ep, fip + 1);
				if(bot - top == 0) skip = true;
				else {
					int c = seq[len - flen];
					t[c] = top; b[c] = bot; tp[c] = topp; bp[c] = botp;
					dep = flen;
				}
			} else {
				int c = seq[len - 1];
				top = topp = tp[c] = E.fchr[c];
				bot = botp = bp[c] = E.fchr[c + 1];
				if(bot - top == 0) skip = true;
				else dep = 1;
			}
		}
		if(!skip) {
			// near half: exact
			for(; dep < nea; dep++) {
				int rdc = seq[len - dep - 1];
				for(int i = 0; i < 4; i++) { tp[i] = topp; bp[i] = botp; }
				ops++;
				if(bot - top > 1) {
					for(int i = 0; i < 4; i++) t[i] = b[i] = 0;
					loads += bi_step(E, top, bot, topp, t, b, tp, bp);
					top = t[rdc]; bot = b[rdc];
					if(bot <= top) { skip = true; break; }
					topp = tp[rdc]; botp = bp[rdc];
				} else {
					SideData s1;
					load_side(E, top / 192u, s1);
					loads++;
					uint32_t co = top % 192u;
					if(side_rowL(s1, co) != rdc || top == E.zoff) { skip = true; break; }
					top = occ1(E, s1, top, rdc);
					bot = top + 1;
					t[rdc] = top; b[rdc] = bot; tp[rdc] = topp; bp[rdc] = botp;
				}
			}
		}
		if(!skip) {
			// far half: 1 mismatch allowed
			for(; dep < len; dep++) {
				int rdc = seq[len - dep - 1];
				int quc = qd[qrev ? dep : len - dep - 1];
				if(rdc > 3 && nceil == 0) break;
				for(int i = 0; i < 4; i++) { tp[i] = topp; bp[i] = botp; }
				int clo = 0, chi = 3;
				bool match = true;
				ops++;
				if(bot - top > 1) {
					for(int i = 0; i < 4; i++) t[i] = b[i] = 0;
					loads += bi_step(E, top, bot, topp, t, b, tp, bp);
					match = rdc < 4;
					if(rdc < 4) { top = t[rdc]; bot = b[rdc]; topp = tp[rdc]; botp = bp[rdc]; }
				} else {
					if(top == E.zoff) break;       // mapLF1(row&) hit the '$'
					SideData s1;
					load_side(E, top / 192u, s1);
					loads++;
					uint32_t co = top % 192u;
					clo = side_rowL(s1, co);
					top = occ1(E, s1, top, clo);
					match = clo == rdc;
					t[clo] = top;
					b[clo] = bot = top + 1;
					bp[clo] = botp; tp[clo] = topp;
					chi = clo;
				}
				if(ns == 0 || rdc > 3) {
					for(int j = clo; j <= chi; j++) {
						if(j == rdc || b[j] == t[j]) continue;
						uint32_t depm = dep + 1;
						uint32_t topm = t[j], botm = b[j], topmp = tp[j], botmp = bp[j];
						for(; depm < len; depm++) {
							int rdcm = seq[len - depm - 1];
							ops++;
							if(botm - topm > 1) {
								uint32_t tm[4] = {0, 0, 0, 0}, bm[4] = {0, 0, 0, 0}, tmp[4], bmp[4];
								tmp[0] = topmp;
								loads += bi_step(E, topm, botm, topmp, tm, bm, tmp, bmp);
								topm = tm[rdcm]; botm = bm[rdcm]; topmp = tmp[rdcm]; botmp = bmp[rdcm];
								if(botm <= topm) break;
							} else {
								SideData s1;
								load_side(E, topm / 192u, s1);
								loads++;
								uint32_t co = topm % 192u;
								if(side_rowL(s1, co) != rdcm || topm == E.zoff) break;
								topm = occ1(E, s1, topm, rdcm);
								botm = topm + 1;
							}
						}
						if(depm == len) {
							uint32_t off5p = dep;
							if(fw == ebwtfw) off5p = len - off5p - 1;
							int64_t score = (int64_t)(len - 1) * matchsc;
							int pen = rdc > 3 ? -P.npen : -mmpen_q(P, quc - 33);
							score += pen;
							bool valid = true;
							if(P.local) {
								int64_t lf = 0, lb = 0;
								for(uint32_t i = 0; i < len; i++) {
									if(i == dep) {
										if(lf + pen <= 0) { valid = false; break; }
										lf += pen;
									} else lf += matchsc;
									if(len - i - 1 == dep) {
										if(lb + pen <= 0) { valid = false; break; }
										lb += pen;
									} else lb += matchsc;
								}
							}
							if(valid) valid = score >= minsc;
							if(valid) {
								if((uint32_t)nh < cap) {
									bt2g_mm1 h;
									h.top = ebwtfw ? topm : topmp;
									h.bot = ebwtfw ? botm : botmp;
									h.fw = fw ? 1 : 0; h.score = (int32_t)score; h.pos = (int32_t)off5p;
									h.chr = j; h.qchr = rdc; h.pad = 0;
									myslot[nh] = h;
								}
								nh++;
							}
						}
					}
				}
				if(bot > top && match) {
					if(dep == len - 1) break;
				} else {
					break;
				}
			}
		}
	}
	slot_counts[(size_t)r * 4 + fwi * 2 + ebwtfwi] = nh;
	if(ops) atomicAdd(&ops_out[r], ops);
	if(loads && loads_out) atomicAdd(&loads_out[r], loads);
}

// Concatenate the 4 per-direction slots of each read in discovery order.
__global__ void k_one_mm_compact(const bt2g_mm1* __restrict__ slots, const int32_t* __restrict__ slot_counts,
                                 uint32_t n, uint32_t cap, bt2g_mm1* __restrict__ hits, int32_t* __restrict__ counts,
                                 int32_t* __restrict__ overflow) {
	uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
	if(r >= n) return;
	int32_t k = 0;
	bool ovf = false;
	for(int s = 0; s < 4; s++) {
		int32_t c = slot_counts[(size_t)r * 4 + s];
		if((uint32_t)c > cap) ovf = true;
		for(int32_t i = 0; i < c && i < (int32_t)cap; i++) {
			if((uint32_t)k < cap) hits[(size_t)r * cap + k] = slots[((size_t)r * 4 + s) * cap + i];
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
	uint32_t threads = n * 2;
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
                   int norc, const uint32_t* gate, uint32_t cap, bt2g_mm1* slots, int32_t* slot_counts,
                   bt2g_mm1* hits, int32_t* counts, uint32_t* ops, uint32_t* loads, int32_t* overflow,
                   hipStream_t st) {
	MmParams P{sc.match, sc.mmp_max, sc.mmp_min, sc.npen, sc.local, 0, 0};
	uint64_t threads = (uint64_t)n * 4;
	hipLaunchKernelGGL(k_one_mm, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, st, F, B, reads, quals,
	                   stride, lens, n, minsc, P, sc.ncl_const, sc.ncl_lin, nofw, norc, gate, cap, slots,
	                   slot_counts, ops, loads);
	hipLaunchKernelGGL(k_one_mm_compact, dim3((n + 255) / 256), dim3(256), 0, st, slots, slot_counts, n, cap, hits,
	                   counts, overflow);
}

void launch_get_offset(const DevEbwt& e, const uint32_t* rows, uint32_t n, uint32_t* offs, uint32_t* loads,
                       hipStream_t st) {
	hipLaunchKernelGGL(k_get_offset, dim3((n + 255) / 256), dim3(256), 0, st, e, rows, n, offs, loads);
}
