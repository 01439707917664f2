// sw_backtrace_wg.hip -- the nextAlignment loop of one end-to-end DP per
// workgroup, its candidates walked in parallel (the batch driver's path:
// rounds of a few thousand DPs, where a DP's latency, not the batch's
// throughput, bounds the round).
//
// The reference walks the sorted candidates one after another
// (aligner_sw_driver.cpp:1157-1180 -> SwAligner::nextAlignment,
// aligner_sw.cpp:737-1146): a walk marks every cell it enters in
// reportedThrough and fails at the first cell an earlier walk marked
// (backtraceNucleotidesEnd2EndSseU8, aligner_swsse_ee_u8.cpp:1283-1780).  A
// walk's path does not depend on the marks -- only where it stops does -- so:
//
//   A. every lane walks one candidate (64 at a time) without marks, over the
//      fill's decision nibbles (sw_ee_packed.hip, kind 2), and records its
//      moves (2 bits each) and its outcome if nothing stops it: touched a core
//      diagonal, Ns within the ceiling;
//   B. the wave resolves the candidates in the reference's order: a candidate's
//      cells (cut into 64 chunks, each lane one chunk, positions from a prefix
//      scan of the moves) are tested against the marks; the first marked cell
//      is where the sequential walk would have failed; the cells before it are
//      marked.  Score filter, start filter, maxaln stop: as the reference;
//   C. the candidates that succeeded are walked again, one per lane, writing
//      their edits and alignment records as the lane-per-problem kernel does.
//
// Plane, marks, read, qualities and reference masks of the DP live in LDS.
// The end-to-end rules the kernel relies on: every cell of the bottom
// gap-barrier rows is left unmarked (sw_backtrace.hip: such walks stay on
// their diagonals); a cell in a gap-barrier row moves diagonally only.
#include <atomic>
#include <mutex>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include "bt2g_kernels.h"

namespace {

__device__ __forceinline__ char mask2dna_wg(int m) {
	// alphabet.cpp:71-89
	switch(m) {
	case 1: return 'A'; case 2: return 'C'; case 3: return 'M'; case 4: return 'G'; case 5: return 'R';
	case 6: return 'S'; case 7: return 'V'; case 8: return 'T'; case 9: return 'W'; case 10: return 'Y';
	case 11: return 'H'; case 12: return 'K'; case 13: return 'D'; case 14: return 'B';
	case 15: case 16: return 'N';
	default: return '?';
	}
}

__device__ __forceinline__ char acgtn(int c) { return c == 0 ? 'A' : c == 1 ? 'C' : c == 2 ? 'G' : c == 3 ? 'T' : 'N'; }

enum { WST_H = 0, WST_E = 1, WST_F = 2 };

// LDS layout of one workgroup (bytes; every part a multiple of 16):
struct WgLayout {
	uint32_t plane, marks, moves, info, rd, qu, rf, total;
	uint32_t mw;      // move words per lane
	uint32_t mkw;     // mark words
};

__host__ __device__ inline uint32_t r16(uint32_t x) { return (x + 15u) & ~15u; }

__host__ __device__ inline WgLayout wg_layout(uint32_t cstride, uint32_t pcols) {
	WgLayout L;
	L.mw = (cstride + pcols + 15u) / 16u;
	L.mkw = (cstride * pcols + 31u) / 32u;
	L.plane = 0;
	L.marks = L.plane + (cstride >> 4) * pcols * 8u;
	L.moves = L.marks + r16(L.mkw * 4u);
	L.info = L.moves + r16(64u * L.mw * 4u);
	L.rd = L.info + 64u * 32u;
	L.qu = L.rd + r16(cstride);
	L.rf = L.qu + r16(cstride);
	L.total = L.rf + r16(pcols + 4u);
	return L;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
	for(int o = 32; o > 0; o >>= 1) {
		const uint32_t w = (uint32_t)__shfl_xor((int)v, o, 64);
		v = w < v ? w : v;
	}
	return v;
}

__device__ __forceinline__ uint32_t wave_sum_excl(uint32_t v, uint32_t lane) {
	uint32_t x = v;
#pragma unroll
	for(int o = 1; o < 64; o <<= 1) {
		const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
		if(lane >= (uint32_t)o) x += y;
	}
	return x - v;
}

}  // namespace

__global__ void __launch_bounds__(64) k_sw_bt_wg(BtArgs A) {
	walk_prio();
	HIP_DYNAMIC_SHARED(uint4, s_wg)
	const uint32_t p = blockIdx.x, lane = threadIdx.x;
	if(p >= A.nprob) return;
	const bt2g_sw_result R = A.res[p];
	if(!R.aligned || R.ncand <= 0) { if(!lane) A.naln[p] = 0; return; }
	if((uint32_t)R.ncand > A.cap) { if(!lane) A.naln[p] = -5; return; }   // truncated list: not the reference's
	const bt2g_sw_problem P = A.probs[p];
	const uint32_t nrow = A.lens[P.read], ncol = P.ncol;
	const uint32_t pcols = A.pcols;
	const WgLayout L = wg_layout(A.cstride, pcols);
	uint8_t* const lds = (uint8_t*)s_wg;
	const uint32_t* const dec = (const uint32_t*)(lds + L.plane);
	uint32_t* const marks = (uint32_t*)(lds + L.marks);
	uint32_t* const moves = (uint32_t*)(lds + L.moves);
	uint32_t* const info = (uint32_t*)(lds + L.info);      // per lane: moves, ok, row0, col0, score
	uint8_t* const srd = lds + L.rd;
	uint8_t* const squ = lds + L.qu;
	uint8_t* const srf = lds + L.rf;
	const bool fw = P.fw != 0;
	// systolic end-to-end fill: the last row at the bottom of the strip stack
	const uint32_t pad = A.plane_top == 1 ? 0u : A.cstride - (A.plane_top == 2 ? ((nrow + 15u) & ~15u) : nrow);
	{
		// the decision plane (16-row blocks, 8 B per block column)
		const uint32_t n16 = (A.cstride >> 4) * pcols * 8u / 16u;
		const uint4* src = (const uint4*)(A.plane + (size_t)p * A.slot);
		uint4* dst = (uint4*)(lds + L.plane);
		for(uint32_t i = lane; i < n16; i += 64u) dst[i] = src[i];
		for(uint32_t i = lane; i < L.mkw; i += 64u) marks[i] = 0u;
		// the read in DP-row order (reverse complement for !fw), its qualities, the
		// reference masks of columns 0..ncol (aligner_sw.cpp:171-253)
		const uint8_t* rd = A.reads + (size_t)P.read * A.stride;
		const uint8_t* qu = A.quals + (size_t)P.read * A.stride;
		for(uint32_t r = lane; r < nrow; r += 64u) {
			const uint32_t s = fw ? r : nrow - 1 - r;
			const int raw = rd[s];
			srd[r] = (uint8_t)(fw ? raw : (raw > 3 ? 4 : 3 - raw));
			int q = (int)qu[s] - 33;
			squ[r] = (uint8_t)(q < 0 ? 0 : (q > 40 ? 40 : q));
		}
		uint64_t rs = 0, rlen = 0;
		if(P.win_off < 0) { rs = A.ref_starts[P.refidx]; rlen = A.ref_starts[P.refidx + 1] - rs; }
		for(uint32_t c = lane; c <= ncol; c += 64u) {
			int m;
			if(P.win_off >= 0) m = A.windows[P.win_off + c];
			else {
				const int64_t o = P.refl + (int64_t)c;
				if(o < 0 || (uint64_t)o >= rlen) m = 16;
				else { const int code = A.ref_codes[rs + (uint64_t)o]; m = code > 3 ? 16 : 1 << code; }
			}
			srf[c] = (uint8_t)m;
		}
	}
	__syncthreads();
	const SwConst& C = A.C;
	const int32_t gb = C.gapbar;
	auto gaps_ok = [&](uint32_t r) { return !(r < (uint32_t)gb || nrow - r - 1 < (uint32_t)gb); };
	auto bottom = [&](uint32_t r) { return r + (uint32_t)gb >= nrow; };
	// the fill's decision of cell (r, c) (sw_ee_packed.hip DEC): bit 0 not diag,
	// bit 1 not from F, bit 2 F not opened from H(up), bit 3 E not opened from H(left)
	auto nibble = [&](uint32_t r, uint32_t c) -> uint32_t {
		const uint32_t rsx = pad + r, b = rsx >> 4, rr = rsx & 15u, i7 = 7u - (rr & 7u);
		const uint32_t wd = dec[((size_t)b * pcols + c) * 2u + (rr >> 3)];
		const uint32_t t = wd >> (3u * i7);
		return ((t >> 2) & 1u) | (t & 2u) | ((t & 1u) << 2) | (((wd >> (24u + i7)) & 1u) << 3);
	};
	// one move from (row, col, st): -1 the walk ends here; 0 diag, 1 ref-gap open,
	// 2 ref-gap extend, 3 read-gap open, 4 read-gap extend
	auto move_of = [&](uint32_t row, uint32_t col, int st) -> int {
		const bool bar = !gaps_ok(row);
		const bool needd = (st != WST_H || !bar) && row > 0;
		const uint32_t nb = needd ? nibble(row, col) : 0u;
		int mv = -1;
		if(st == WST_H) {
			if(bar) { if(col > 0) mv = 0; }
			else if(!(nb & 1u) && col > 0) mv = 0;
			else if(!(nb & 2u)) mv = (nb & 4u) ? 2 : 1;
			else if(col > 0) mv = (nb & 8u) ? 4 : 3;
		} else if(st == WST_E) {
			if(col > 0) mv = (nb & 8u) ? 4 : 3;
		} else {
			mv = (nb & 4u) ? 2 : 1;
		}
		return mv;
	};
	auto mark_bit = [&](uint32_t r, uint32_t c) -> uint32_t { return r * pcols + c; };
	int32_t nceil;
	{
		double v = A.ncl_const + A.ncl_lin * (double)nrow;
		v = v < 0.0 ? 0.0 : v;
		nceil = v >= 2147483647.0 ? 2147483647 : (int32_t)v;
	}
	int32_t triml = 0, corel = 0, corer = 0x7fffffff;
	if(A.rects) { const bt2g_sw_rect rc = A.rects[p]; triml = rc.triml; corel = rc.corel; corer = rc.corer; }
	const uint32_t ncand = (uint32_t)R.ncand < A.cap ? (uint32_t)R.ncand : A.cap;
	const bt2g_sw_cand* cl = A.cands + (size_t)p * A.cap;
	uint32_t* const mymoves = moves + (size_t)lane * L.mw;
	int32_t nal = 0;
	bool stop = false;
	for(uint32_t c0 = 0; c0 < ncand && !stop; c0 += 64u) {
		// ---- A: this lane's candidate walked without marks --------------------------
		{
			const uint32_t ci = c0 + lane;
			uint32_t T = 0, ok = 0, r0 = 0, q0 = 0;
			int32_t sc0 = 0;
			if(ci < ncand) {
				const bt2g_sw_cand cd = cl[ci];
				r0 = (uint32_t)cd.row;
				q0 = (uint32_t)cd.col;
				sc0 = cd.score;
				if(cd.score >= P.minsc) {
					uint32_t row = r0, col = q0;
					int st = WST_H;
					bool core = false;
					int32_t ns = 0;
					uint32_t word = 0;
					for(;;) {
						const int32_t dg = (int32_t)col - (int32_t)row + triml;
						core = core || (dg >= 0 && dg >= corel && dg <= corer);
						if(row == 0) break;
						const int mv = move_of(row, col, st);
						if(mv < 0) break;
						uint32_t code;
						if(mv == 0) {
							ns += (srd[row] > 3 || srf[col] > 15) ? 1 : 0;
							row--; col--; st = WST_H; code = 0u;
						} else if(mv <= 2) {
							row--; st = mv == 1 ? WST_H : WST_F; code = 1u;
						} else {
							col--; st = mv == 3 ? WST_H : WST_E; code = 2u;
						}
						word |= code << (2u * (T & 15u));
						if((T & 15u) == 15u) { mymoves[T >> 4] = word; word = 0; }
						T++;
					}
					if(T & 15u) mymoves[T >> 4] = word;
					ns += (srd[row] > 3 || srf[col] > 15) ? 1 : 0;   // the cell the walk ends on
					ok = core && ns <= nceil ? 1u : 0u;
				}
			}
			// (phase B reads the candidates from here, not from global memory: a
			// dependent global load per candidate would be most of the loop)
			info[lane * 8u] = T;
			info[lane * 8u + 1u] = ok;
			info[lane * 8u + 2u] = r0;
			info[lane * 8u + 3u] = q0;
			info[lane * 8u + 4u] = (uint32_t)sc0;
		}
		__syncthreads();
		// ---- B: the candidates in the reference's order -----------------------------
		uint32_t succ = 0;                          // lane k: candidate index of this batch's k-th success
		uint32_t nsucc = 0;
		const uint32_t cend = c0 + 64u < ncand ? c0 + 64u : ncand;
		for(uint32_t ci = c0; ci < cend; ci++) {
			if(nal >= (int32_t)A.maxaln) { stop = true; break; }
			const uint32_t j = ci - c0;
			int8_t fate;
			const uint32_t r0 = info[j * 8u + 2u], q0 = info[j * 8u + 3u];
			if((int32_t)info[j * 8u + 4u] < P.minsc) {
				fate = 5;                               // BT_CAND_FATE_FILT_SCORE
			} else if(!bottom(r0) && ((marks[mark_bit(r0, q0) >> 5] >> (mark_bit(r0, q0) & 31u)) & 1u)) {
				fate = 3;                               // BT_CAND_FATE_FILT_START
			} else {
				const uint32_t T = info[j * 8u], ncell = T + 1u;
				const uint32_t* mv = moves + (size_t)j * L.mw;
				const uint32_t ch = (ncell + 63u) / 64u;
				const uint32_t lo = lane * ch < ncell ? lane * ch : ncell, hi = lo + ch < ncell ? lo + ch : ncell;
				// this lane's chunk start: the moves before it, by a scan of the chunks' moves
				uint32_t dr = 0, dc = 0;
				for(uint32_t t = lo; t < hi && t < T; t++) {
					const uint32_t code = (mv[t >> 4] >> (2u * (t & 15u))) & 3u;
					dr += code != 2u;
					dc += code != 1u;
				}
				uint32_t row = r0 - wave_sum_excl(dr, lane), col = q0 - wave_sum_excl(dc, lane);
				const uint32_t srow = row, scol = col;
				uint32_t hit = 0xffffffffu;
				for(uint32_t t = lo; t < hi; t++) {
					if(!bottom(row)) {
						const uint32_t b = mark_bit(row, col);
						if((marks[b >> 5] >> (b & 31u)) & 1u) { hit = t; break; }
					}
					if(t < T) {
						const uint32_t code = (mv[t >> 4] >> (2u * (t & 15u))) & 3u;
						row -= code != 2u;
						col -= code != 1u;
					}
				}
				const uint32_t tstar = wave_min_u32(hit);
				__syncthreads();
				// the cells the sequential walk marks: those before tstar
				row = srow;
				col = scol;
				for(uint32_t t = lo; t < hi && t < tstar; t++) {
					if(!bottom(row)) {
						const uint32_t b = mark_bit(row, col);
						atomicOr(&marks[b >> 5], 1u << (b & 31u));
					}
					if(t < T) {
						const uint32_t code = (mv[t >> 4] >> (2u * (t & 15u))) & 3u;
						row -= code != 2u;
						col -= code != 1u;
					}
				}
				__syncthreads();
				if(tstar == 0xffffffffu && info[j * 8u + 1u]) {
					fate = 1;                           // BT_CAND_FATE_SUCCEEDED
					if(lane == nsucc) succ = ci;
					nsucc++;
					nal++;
				} else {
					fate = 2;                           // BT_CAND_FATE_FAILED
				}
			}
			if(A.fates && lane == 0) A.fates[(size_t)p * A.cap + ci] = fate;
		}
		// ---- C: the successes walked again, writing edits and records -----------------
		if(lane < nsucc) {
			const uint32_t ci = succ;
			const uint32_t a = (uint32_t)nal - nsucc + lane;
			const bt2g_sw_cand cd = cl[ci];
			bt2g_edit* ed = A.edits + ((size_t)p * A.maxaln + a) * A.maxedit;
			uint32_t ned = 0;
			auto push = [&](uint32_t pos, int type, int chr, int qchr) {
				if(ned < A.maxedit) ed[ned] = bt2g_edit{pos, (uint8_t)type, (uint8_t)chr, (uint8_t)qchr, 0};
				ned++;
			};
			const uint32_t row0 = (uint32_t)cd.row, col0 = (uint32_t)cd.col;
			uint32_t row = row0, col = col0;
			int st = WST_H;
			int32_t score = 0, ns = 0, gaps = 0;
			for(;;) {
				if(row == 0) break;
				const int mv = move_of(row, col, st);
				if(mv < 0) break;
				const int rc = srd[row], m = srf[col];
				if(mv == 0) {
					const int mt = (m >= 16 || rc > 3) ? -1 : ((m >> rc) & 1);
					if(mt != 1) {
						push(row, 3, mask2dna_wg(m), acgtn(rc));
						score -= (rc > 3 || m > 15) ? C.npen : C.mmpen[squ[row]];
					} else {
						score += C.match;
					}
					if(mt == -1) ns++;
					row--; col--; st = WST_H;
				} else if(mv <= 2) {
					push(row, 2, '-', acgtn(rc));
					score -= mv == 1 ? C.rfgo : C.rfge;
					st = mv == 1 ? WST_H : WST_F;
					row--; gaps++;
				} else {
					push(row + 1, 1, mask2dna_wg(m), '-');
					score -= mv == 3 ? C.rdgo : C.rdge;
					st = mv == 3 ? WST_H : WST_E;
					col--; gaps++;
				}
			}
			{
				const int rc = srd[row], m = srf[col];
				const int mt = (m >= 16 || rc > 3) ? -1 : ((m >> rc) & 1);
				if(mt != 1) {
					push(row, 3, mask2dna_wg(m), acgtn(rc));
					score -= (rc > 3 || m > 15) ? C.npen : C.mmpen[squ[row]];
				} else {
					score += C.match;
				}
				if(mt == -1) ns++;
			}
			// res.reverse(), AlnRes::setShape trim shift, invertEdits for !fw
			// (aligner_result.cpp:101-117, 822-828; edit.cpp:50-78)
			const uint32_t trimBeg = row, trimEnd = nrow - row0 - 1;
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
				for(uint32_t i = 0; i < nst; i++) ed[i].pos = sz - (ed[i].pos - trimBeg) - (ed[i].type == 1 ? 0u : 1u);
			}
			int32_t refns = 0;
			for(uint32_t c = col; c <= col0; c++) refns += srf[c] > 15;
			bt2g_sw_aln al;
			al.cand = (int32_t)ci; al.score = score; al.off = (int32_t)col; al.ns = ns; al.gaps = gaps;
			al.refns = refns; al.nedit = (int32_t)ned;
			al.trim5p = (int32_t)(fw ? trimBeg : trimEnd); al.trim3p = (int32_t)(fw ? trimEnd : trimBeg);
			al.pad = 0;
			A.alns[(size_t)p * A.maxaln + a] = al;
		}
		__syncthreads();
	}
	if(lane == 0) A.naln[p] = nal;
}

// LDS bytes of k_sw_bt_wg for this launch (0: it does not apply)
uint32_t sw_bt_wg_lds(const BtArgs& a) {
	const WgLayout L = wg_layout(a.cstride, a.pcols);
	return L.total;
}

// The dynamic LDS a workgroup of k_sw_bt_wg may take on a device: what the
// device lets a block opt in to (up to the CU's 160 KiB; the kernel declares no
// static LDS, so dynamic is all of it) -- wide planes (mate searches, ~90 KB)
// then fit; 64 KiB with $BT2G_BT_WG_LDS=0 or before sw_bt_wg_lds_init.
// HIP keeps function attributes per device, so the opt-in is made for every
// device a context is opened on, from bt2g_open, before that context has a
// stream or any worker thread launches on it (it had been made lazily, once per
// process, on whichever device was current at the first walk).
static std::atomic<uint32_t> g_wg_lds_lim[64];
static std::mutex g_wg_lds_mu;

void sw_bt_wg_lds_init(int dev) {
	if(dev < 0 || dev >= 64) return;
	std::lock_guard<std::mutex> lk(g_wg_lds_mu);
	if(g_wg_lds_lim[dev].load()) return;
	uint32_t lim = 65536u;
	const char* e = getenv("BT2G_BT_WG_LDS");
	int v = 0;
	if(!(e && *e == '0') &&
	   hipDeviceGetAttribute(&v, hipDeviceAttributeSharedMemPerBlockOptin, dev) == hipSuccess && v > 65536) {
		// (the caller made `dev` current: bt2g_open_mem)
		if(hipFuncSetAttribute((const void*)k_sw_bt_wg, hipFuncAttributeMaxDynamicSharedMemorySize, v) == hipSuccess)
			lim = (uint32_t)v;
		else
			(void)hipGetLastError();
	}
	g_wg_lds_lim[dev].store(lim);
}

// (on the calling thread's current device: the caller's context device)
uint32_t sw_bt_wg_lds_limit() {
	// ($BT2G_BT_WG_LDS=0 read at every launch too: the parity tests run one batch
	// both ways)
	const char* e = getenv("BT2G_BT_WG_LDS");
	if(e && *e == '0') return 65536u;
	int dev = 0;
	if(hipGetDevice(&dev) != hipSuccess) return 65536u;
	const uint32_t v = dev >= 0 && dev < 64 ? g_wg_lds_lim[dev].load() : 0u;
	return v ? v : 65536u;
}

void launch_sw_bt_wg(const BtArgs& a, uint32_t lds, hipStream_t st) {
	hipLaunchKernelGGL(k_sw_bt_wg, dim3(a.nprob), dim3(64), lds, st, a);
}
