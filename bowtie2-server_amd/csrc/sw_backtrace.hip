// sw_backtrace.hip -- SwAligner::nextAlignment for a batch of filled DP
// problems: the driver's loop of nextAlignment calls
// (aligner_sw_driver.cpp:1157-1180) over each problem's sorted candidate list,
// with the reference's backtrace walk (backtraceNucleotides{End2End,Local}
// Sse{U8,I16}: aligner_swsse_ee_u8.cpp:1283-1780, aligner_swsse_loc_u8.cpp:
// 1588-2175, the i16 files walk identically) and candidate filters
// (aligner_sw.cpp:737-1146).
//
// One lane per problem; the walk is a chain of dependent loads, so the kernel
// is latency-bound and wants many waves in flight (few VGPRs, no LDS).
//
// What the fill leaves behind is only the H score of every cell (the "score
// plane", one byte per cell for u8 fills, written by the systolic fill in
// sw_ee_packed.hip, or the generic fill's H,E,F int16 triples).  The E and F
// values a walk consults are recomputed from H on demand:
//   E(r,c) = max_{k>=1, c-k>=0}   H(r,c-k) - rdgo - (k-1)*rdge
//   F(r,c) = max_{k>=1, rows r..r-k+1 outside the gap barrier} H(r-k,c) - rfgo - (k-1)*rfge
// which is exactly the fill's recurrence wherever the value is above the
// floor, and the walk only asks whether such a value equals a target above
// the floor (path cells score >= minsc; local: > 0).  Two facts keep that
// cheap: an H cell above the floor that is not a diagonal move equals its F
// or its E, so once the H-up and F-up tests fail the E side is decided by
// the H-left test alone (no E scan); and the F scan reads one column, i.e.
// contiguous bytes of the plane (three 16-B loads for 32 rows).  The E/F-state
// moves need no scan at all: the F (E) value of the cell is known from the
// move that entered it, and one of its two sources must match (both: the H one).
//
// reportedThrough: the first walk of a problem records, per row, the column
// interval it crossed (a walk visits one contiguous run of columns per row);
// later walks are checked against those intervals and against a bitmap whose
// rows are cleared lazily over the range they reach (the bottom rows, for
// end-to-end candidates).  All loads a step needs are issued together, so a
// diagonal step costs one memory round trip.
//
// The reference's branch stack (btnstack_) never changes an outcome: every
// popped frame restarts at a cell already marked reportedThrough, so a walk
// that meets a marked cell fails (proved against the reference by
// tests/test_oracle_golden.py::test_sw_backtrace, whose oracle keeps the
// stack, and tests/test_gpu_bt.py).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "bt2g_kernels.h"

namespace {


__device__ __forceinline__ char mask2dna(int m) {
	// alphabet.cpp:71-89
	switch(m) {
	case 1: return 'A'; case 2: return 'C'; case 3: return 'M'; case 4: return 'G'; case 5: return 'R';
	case 6: return 'S'; case 7: return 'V'; case 8: return 'T'; case 9: return 'W'; case 10: return 'Y';
	case 11: return 'H'; case 12: return 'K'; case 13: return 'D'; case 14: return 'B';
	case 15: case 16: return 'N';
	default: return '?';
	}
}

enum { ST_H = 0, ST_E = 1, ST_F = 2 };

// Score plane accessor: KIND 0 = u8 plane, 1 = u16 plane (systolic layout:
// problem slot, column-major with cstride rows, bottom-aligned), 2 = int16
// H,E,F triples at mat_off[p] (generic fill, row-major).
template <int KIND>
struct Plane {
	const uint8_t* base;
	uint32_t cstride, ncol;
	int32_t off;      // score = raw - off
	__device__ __forceinline__ int32_t h(uint32_t r, uint32_t c) const {
		if(KIND == 0) return (int32_t)base[(size_t)c * cstride + r] - off;
		if(KIND == 1) return (int32_t)((const uint16_t*)base)[(size_t)c * cstride + r] - off;
		return (int32_t)((const int16_t*)base)[((size_t)r * ncol + c) * 3] - off;
	}
};

}  // namespace

template <int KIND>
__global__ void __launch_bounds__(64)
k_sw_bt(BtArgs A) {
	const uint32_t p = blockIdx.x * 64u + threadIdx.x;
	if(p >= A.nprob) return;
	const bt2g_sw_result R = A.res[p];
	if(!R.aligned || R.ncand <= 0) { A.naln[p] = 0; return; }
	const bt2g_sw_problem P = A.probs[p];
	const uint32_t nrow = A.lens[P.read], ncol = P.ncol;
	const bool local = A.local != 0;
	const int variant = local ? (R.u8succ ? 2 : 3) : (R.u8succ ? 0 : 1);
	Plane<KIND> pl;
	pl.ncol = ncol;
	pl.cstride = A.cstride;
	uint32_t pad = 0;
	const uint8_t* slot = nullptr;
	if(KIND == 2) {
		pl.base = (const uint8_t*)(A.mat + A.mat_off[p]);
		pl.off = variant == 0 ? 0xff : variant == 1 ? 0x7fff : variant == 2 ? 0 : -0x8000;
	} else {
		if(KIND == 0 && variant != 0) { A.naln[p] = -4; return; }   // i16 fill, u8-only plane
		const size_t es = KIND == 0 ? 1 : 2;
		pad = A.cstride - nrow;
		slot = A.plane + (size_t)p * A.slot;
		pl.base = slot + (size_t)pad * es;
		pl.off = variant == 0 ? 0xff : 0xffff;
	}
	// SwAligner::initRead / initRef inputs of this problem
	const uint8_t* rd = A.reads + (size_t)P.read * A.stride;
	const uint8_t* qu = A.quals + (size_t)P.read * A.stride;
	const bool fw = P.fw != 0;
	const SwConst& C = A.C;
	auto readc = [&](uint32_t r) -> int {
		if(fw) return rd[r];
		const int c = rd[nrow - 1 - r];
		return c > 3 ? 4 : 3 - c;
	};
	auto qual = [&](uint32_t r) -> int {
		int q = (int)(fw ? qu[r] : qu[nrow - 1 - r]) - 33;
		return q < 0 ? 0 : (q > 40 ? 40 : q);
	};
	uint64_t rs = 0, rlen = 0;
	if(P.win_off < 0) { rs = A.ref_starts[P.refidx]; rlen = A.ref_starts[P.refidx + 1] - rs; }
	auto refm = [&](uint32_t c) -> int {   // reference mask of column c (aligner_sw.cpp:171-253)
		if(P.win_off >= 0) return A.windows[P.win_off + c];
		const int64_t o = P.refl + (int64_t)c;
		if(o < 0 || (uint64_t)o >= rlen) return 16;
		const int code = A.ref_codes[rs + (uint64_t)o];
		return code > 3 ? 16 : 1 << code;
	};
	// Scoring::score / Scoring::mm (scoring.h:232-254); match(30) is the bonus
	auto sdiag = [&](int rc, int m, int q) -> int {
		if(rc > 3 || m > 15) return -C.npen;
		return ((m >> rc) & 1) ? C.match : -C.mmpen[q];
	};
	const int32_t rdgo = C.rdgo, rdge = C.rdge, rfgo = C.rfgo, rfge = C.rfge;
	const int32_t gb = C.gapbar;
	auto gaps_ok = [&](uint32_t r) { return !(r < (uint32_t)gb || nrow - r - 1 < (uint32_t)gb); };
	auto okv = [&](int32_t v) { return !local || v > 0; };   // floorsc (0 in local mode)
	// highest score any H cell of row r can hold: 0 end-to-end; (r+1)*match local
	auto hmax = [&](int32_t r) -> int32_t { return local ? (r + 1) * C.match : 0; };
	// does H(r, c) == base + (x - r) * step hold for some r in [rlo, rhi]?  (column scan)
	auto col_hit = [&](uint32_t c, int32_t rlo, int32_t rhi, int32_t x, int32_t base, int32_t step) -> bool {
		if(rlo > rhi) return false;
		if(KIND == 0) {
			// bytes [pad+rlo, pad+rhi] of column block c: aligned 16-B loads
			const uint8_t* cb = slot + (size_t)c * A.cstride;
			bool hit = false;
#pragma unroll 1
			for(int32_t o0 = ((int32_t)pad + rlo) & ~15; o0 <= (int32_t)pad + rhi; o0 += 16) {
				const uint4 v = *(const uint4*)(cb + o0);
				const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
				for(int b = 0; b < 16; b++) {
					const int32_t r = o0 + b - (int32_t)pad;
					const int32_t val = (int32_t)((wv[b >> 2] >> (8 * (b & 3))) & 0xffu) - pl.off;
					hit = hit || (r >= rlo && r <= rhi && val == base + (x - r) * step);
				}
			}
			return hit;
		} else {
			for(int32_t r = rhi; r >= rlo; r--)
				if(pl.h((uint32_t)r, c) == base + (x - r) * step) return true;
			return false;
		}
	};
	// N ceiling, Scoring::nCeil.f<int>(len) (simple_func.h:90-115)
	int32_t nceil;
	{
		double v = A.ncl_const + A.ncl_lin * (double)nrow;
		v = v < 0.0 ? 0.0 : v;
		nceil = v >= 2147483647.0 ? 2147483647 : (int32_t)v;
	}
	int32_t triml = 0, corel = 0, corer = 0x7fffffff;
	if(A.rects) { const bt2g_sw_rect rc = A.rects[p]; triml = rc.triml; corel = rc.corel; corer = rc.corer; }
	// reportedThrough: the first walk's per-row column intervals + a lazily
	// cleared bitmap for the cells of later walks
	uint32_t* marks = A.marks + (size_t)p * A.mslot;
	uint32_t* path1 = marks + (size_t)A.mwords * A.mrows;      // mrows words after the bitmap
	const uint32_t mw = A.mwords;
	int32_t mlo = 0x7fffffff, mhi = -1;      // bitmap rows cleared so far
	int32_t p1lo = 0x7fffffff, p1hi = -1;    // rows holding first-walk intervals
	auto clear_row = [&](int32_t r) {
		uint4* q = (uint4*)(marks + (size_t)r * mw);
		for(uint32_t w = 0; w < mw / 4; w++) q[w] = make_uint4(0, 0, 0, 0);
	};
	auto touch_rows = [&](int32_t r) {
		if(mhi < 0) { mlo = mhi = r; clear_row(r); return; }
		while(r > mhi) clear_row(++mhi);
		while(r < mlo) clear_row(--mlo);
	};
	auto marked = [&](uint32_t r, uint32_t c) -> bool {
		bool m = false;
		if((int32_t)r >= p1lo && (int32_t)r <= p1hi) {
			const uint32_t iv = path1[r];
			m = c >= (iv & 0xffffu) && c <= (iv >> 16);
		}
		if((int32_t)r >= mlo && (int32_t)r <= mhi) m = m || ((marks[(size_t)r * mw + (c >> 5)] >> (c & 31)) & 1u);
		return m;
	};
	const uint32_t ncand = (uint32_t)R.ncand < A.cap ? (uint32_t)R.ncand : A.cap;
	const bt2g_sw_cand* cl = A.cands + (size_t)p * A.cap;
	int2* done = local ? A.done + (size_t)p * A.cap : nullptr;
	uint32_t ndone = 0;
	uint32_t SQ = nrow >> 4;
	if(SQ == 0) SQ = 1;
	int32_t nal = 0;
	bool first = true;
	for(uint32_t ci = 0; ci < ncand; ci++) {
		if(nal >= (int32_t)A.maxaln) break;
		const bt2g_sw_cand cd = cl[ci];
		int8_t fate;
		if(cd.score < P.minsc) {
			fate = 5;                                   // BT_CAND_FATE_FILT_SCORE
		} else if(marked((uint32_t)cd.row, (uint32_t)cd.col)) {
			fate = 3;                                   // BT_CAND_FATE_FILT_START
		} else {
			bool dom = false;
			if(local) {
				for(uint32_t i = 0; i < ndone && !dom; i++) {
					const int2 d = done[i];
					const uint32_t dr = d.x > cd.row ? d.x - cd.row : cd.row - d.x;
					const uint32_t dc = d.y > cd.col ? d.y - cd.col : cd.col - d.y;
					dom = dc <= SQ && dr <= SQ;
				}
			}
			if(dom) {
				fate = 4;                               // BT_CAND_FATE_FILT_DOMINATED
			} else {
				// ---- one backtrace from (row, col) ----
				const bool rec = first;                 // first walk: record intervals
				first = false;
				bt2g_edit* ed = A.edits + ((size_t)p * A.maxaln + (size_t)nal) * A.maxedit;
				uint32_t ned = 0;
				auto push = [&](uint32_t pos, int type, int chr, int qchr) {
					if(ned < A.maxedit) ed[ned] = bt2g_edit{pos, (uint8_t)type, (uint8_t)chr, (uint8_t)qchr, 0};
					ned++;
				};
				uint32_t row = (uint32_t)cd.row, col = (uint32_t)cd.col;
				const uint32_t origCol = col, trimEnd = nrow - row - 1;
				int32_t score = 0, ns = 0, gaps = 0;
				int st = ST_H;
				int32_t cur = pl.h(row, col);
				bool ok = true, core = false;
				uint32_t irow = row, ilo = col, ihi = col;   // first walk: the open row interval
				if(rec) p1hi = (int32_t)row;
				while(true) {
					// the loads of this step, issued together
					const bool inP1 = !rec && (int32_t)row >= p1lo && (int32_t)row <= p1hi;
					const bool inBM = !rec && (int32_t)row >= mlo && (int32_t)row <= mhi;
					uint32_t* mwp = marks + (size_t)row * mw + (col >> 5);
					const uint32_t iv = inP1 ? path1[row] : 0xffffu;
					const uint32_t w = inBM ? *mwp : 0u;
					const bool wantd = st == ST_H && row > 0 && col > 0;
					const int32_t hul = wantd ? pl.h(row - 1, col - 1) : 0;
					const int rc = readc(row), m = refm(col), q = qual(row);
					const uint32_t bit = 1u << (col & 31);
					// reportedThrough (aligner_swsse_ee_u8.cpp:1331-1336, 1556)
					if((w & bit) || (col >= (iv & 0xffffu) && col <= (iv >> 16))) { ok = false; break; }
					if(rec) {
						if(row != irow) {
							path1[irow] = ilo | (ihi << 16);
							irow = row; ihi = col;
						}
						ilo = col;
					} else {
						if(!inBM) touch_rows((int32_t)row);
						*mwp = w | bit;
					}
					{
						const int32_t dg = (int32_t)col - (int32_t)row + triml;
						core = core || (dg >= 0 && dg >= corel && dg <= corer);
					}
					if(row == 0) break;
					int mv = -1;   // 0 diag, 1 ref open, 2 ref extend, 3 read open, 4 read extend
					int32_t nxt = 0;
					if(st == ST_H) {
						// diag equality; local mode also wants H(up-left) > 0 (floorsc)
						const bool deq = wantd && cur == hul + sdiag(rc, m, q);
						if(deq && okv(hul)) { mv = 0; nxt = hul; }
						if(mv < 0 && gaps_ok(row)) {
							const int32_t hu = pl.h(row - 1, col);
							const int32_t hl = col > 0 ? pl.h(row, col - 1) : 0;
							// F(row-1, col) == cur + rfge: H(x-k, col) == cur + rfgo + k*rfge, x = row-1,
							// rows x..x-k+1 outside the barrier, x-k >= 0
							bool fup = false;
							const int32_t x = (int32_t)row - 1;
							if(okv(cur + rfge) && x >= gb && x <= (int32_t)nrow - gb - 1) {
								int32_t kmax = x - gb + 1;
								kmax = kmax < x ? kmax : x;
								if(rfge > 0) {
									const int32_t kh = (hmax(x - 1) - cur - rfgo) / rfge;   // need <= hmax
									kmax = kh < kmax ? kh : kmax;
								}
								fup = col_hit(col, x - kmax, x - 1, x, cur + rfgo, rfge);
							}
							if(okv(hu) && cur == hu - rfgo) { mv = 1; nxt = hu; }
							else if(fup) { mv = 2; nxt = cur + rfge; }
							else if(col > 0) {
								if(okv(hl) && cur == hl - rdgo) { mv = 3; nxt = hl; }
								else if(!deq && (!local || cur > 0)) {
									// above the floor, not diagonal, not from F: from E, and not
									// by an open -- an extension
									if(col > 1) { mv = 4; nxt = cur + rdge; }
								} else if(col > 1 && okv(cur + rdge)) {
									// H may come from a diagonal the walk may not take (local,
									// H(up-left) == 0) or from the local floor: E(row, col-1) ==
									// cur + rdge needs the row scan
									const int32_t cc = (int32_t)col - 1;
									const int32_t hm = hmax((int32_t)row);
									for(int32_t k = 1; cc - k >= 0; k++) {
										const int32_t need = cur + rdge + rdgo + (k - 1) * rdge;
										if(need > hm) break;
										if(pl.h(row, (uint32_t)(cc - k)) == need) { mv = 4; nxt = cur + rdge; break; }
									}
								}
							}
						}
						if(mv < 0) break;   // empty cell: the alignment starts here
					} else if(st == ST_E) {
						if(col == 0) break;   // unreachable: E(row, 0) is the floor
						const int32_t hl = pl.h(row, col - 1);
						if(okv(hl) && hl - rdgo == cur) { mv = 3; nxt = hl; }
						else { mv = 4; nxt = cur + rdge; }
					} else {
						const int32_t hu = pl.h(row - 1, col);
						if(okv(hu) && hu - rfgo == cur) { mv = 1; nxt = hu; }
						else { mv = 2; nxt = cur + rfge; }
					}
					if(mv == 0) {
						const int mt = (m >= 16 || rc > 3) ? -1 : ((m >> rc) & 1);
						if(mt != 1) {
							push(row, 3, mask2dna(m), "ACGTN"[rc]);
							score -= (rc > 3 || m > 15) ? C.npen : C.mmpen[q];
						} else {
							score += C.match;
						}
						if(mt == -1) ns++;
						row--; col--;
						st = ST_H;
					} else if(mv <= 2) {
						push(row, 2, '-', "ACGTN"[rc]);
						score -= mv == 1 ? rfgo : rfge;
						st = mv == 1 ? ST_H : ST_F;
						row--; gaps++;
					} else {
						push(row + 1, 1, mask2dna(m), '-');
						score -= mv == 3 ? rdgo : rdge;
						st = mv == 3 ? ST_H : ST_E;
						col--; gaps++;
					}
					cur = nxt;
				}
				if(rec) {
					// close the first walk's record: rows [row, start] hold intervals
					path1[irow] = ilo | (ihi << 16);
					p1lo = (int32_t)row;
				}
				if(ok && !core) ok = false;              // must touch a core diagonal
				if(ok) {
					const int rc = readc(row), m = refm(col);
					const int mt = (m >= 16 || rc > 3) ? -1 : ((m >> rc) & 1);
					if(mt != 1) {
						push(row, 3, mask2dna(m), "ACGTN"[rc]);
						score -= (rc > 3 || m > 15) ? C.npen : C.mmpen[qual(row)];
					} else {
						score += C.match;
					}
					if(mt == -1) ns++;
					if(ns > nceil) ok = false;
				}
				if(local) done[ndone++] = make_int2(cd.row, cd.col);
				if(ok) {
					const uint32_t trimBeg = row;
					// res.reverse(), AlnRes::setShape trim shift, invertEdits for !fw
					// (aligner_result.cpp:101-117, 822-828; edit.cpp:50-78)
					const uint32_t nst = ned < A.maxedit ? ned : A.maxedit;
					if(fw) {
						for(uint32_t i = 0; i < nst / 2; i++) {
							const bt2g_edit t = ed[i];
							ed[i] = ed[nst - 1 - i];
							ed[nst - 1 - i] = t;
						}
						for(uint32_t i = 0; i < nst; i++) ed[i].pos -= trimBeg;
					} else {
						const uint32_t sz = nrow - trimBeg - trimEnd;
						for(uint32_t i = 0; i < nst; i++)
							ed[i].pos = sz - (ed[i].pos - trimBeg) - (ed[i].type == 1 ? 0u : 1u);
					}
					int32_t refns = 0;
					for(uint32_t c = col; c <= origCol; c++) refns += refm(c) > 15;
					bt2g_sw_aln a;
					a.cand = (int32_t)ci; a.score = score; a.off = (int32_t)col; a.ns = ns; a.gaps = gaps;
					a.refns = refns; a.nedit = (int32_t)ned;
					a.trim5p = (int32_t)(fw ? trimBeg : trimEnd); a.trim3p = (int32_t)(fw ? trimEnd : trimBeg);
					a.pad = 0;
					A.alns[(size_t)p * A.maxaln + (size_t)nal] = a;
					nal++;
					fate = 1;                               // BT_CAND_FATE_SUCCEEDED
				} else {
					fate = 2;                               // BT_CAND_FATE_FAILED
				}
			}
		}
		if(A.fates) A.fates[(size_t)p * A.cap + ci] = fate;
	}
	A.naln[p] = nal;
}

void launch_sw_bt(int kind, const BtArgs& a, hipStream_t st) {
	if(a.nprob == 0) return;
	const dim3 grid((a.nprob + 63u) / 64u), block(64);
	switch(kind) {
	case 0: hipLaunchKernelGGL(k_sw_bt<0>, grid, block, 0, st, a); break;
	case 1: hipLaunchKernelGGL(k_sw_bt<1>, grid, block, 0, st, a); break;
	default: hipLaunchKernelGGL(k_sw_bt<2>, grid, block, 0, st, a); break;
	}
}
