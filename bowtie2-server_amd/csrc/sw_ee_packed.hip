// sw_ee_packed.hip -- SW fills + candidate gather as a systolic array of
// lanes, two problems per lane in packed 16-bit arithmetic (gfx950 VOP3P:
// v_pk_sub_u16 clamp, v_pk_max_u16, v_perm_b32).
//
// Restates the fills selected by SwAligner::align (aligner_sw.cpp:500-620),
// bit for bit: end-to-end aligner_swsse_ee_u8.cpp:775-1146 and
// aligner_swsse_ee_i16.cpp:780-1200 with the last-row candidate gather
// (aligner_swsse_ee_u8.cpp:1176-1208); local (LOCAL) aligner_swsse_loc_u8.cpp:
// 927-1336 and aligner_swsse_loc_i16.cpp:938-1367 with their gathers
// (aligner_swsse_loc_u8.cpp:1389-1500, aligner_swsse_loc_i16.cpp:1420-1535) and
// the u8 -> i16 fallback on saturation (aligner_sw.cpp:570-605).
//
// Value domain.  Both reference domains run as unsigned 16-bit lanes with
// unsigned saturation:
//   u8  fill: value = 0xff + score, floor 0          -> ROW0 = 0x00ff, LO = 0
//   i16 fill: value = 0x7fff + score, floor -0x8000;  stored + 0x8000
//             (signed saturation at -0x8000 == unsigned saturation at 0)
//                                                    -> ROW0 = 0xffff, LO = 0
// so a lane may pair a u8 problem with an i16 one; the reference's veto of
// gap opens/extensions in the gap-barrier rows becomes an AND with 0 (LO).
//
// Local value domain: the score itself (floor 0 = the unsigned saturation of
// the subtract).  The u8 local fill's bias cancels unless a cell would reach
// 255 - bias, which is exactly its saturation test (column max + bias >= 255,
// then the i16 fill runs), and the i16 fill's 0x8000 offset drops out: one
// pass yields the H of both fills.  They differ only in the striped padding
// rows below the last row (score 0, no gap barrier; up to a multiple of 16
// rows for u8, of 8 for i16) that feed the per-column maxima driving
// lastsolcol_ / colstop_; a problem's padded rows end at the bottom of the
// strip stack and the bottom lane keeps both column maxima.  The diagonal term
// is H(up-left) + match - pen', the query profile holding pen' = match - score
// (0 for a match), so dead rows above the problem (profile = match) stay 0.
// Candidate cells (>= minsc, a match whose down-right neighbour is not) are
// found with per-character row bit masks, only in 16-row blocks whose maximum
// reaches minsc, and appended through an LDS counter per problem (the
// candidate sort that follows fixes the order).
//
// Layout.  A problem pair (low/high half of every register) is swept by a
// group of S lanes (S = ceil(stride/16)); lane k of the group owns register
// rows 16k..16k+15 of a 16*S-row strip stack in which each problem is
// bottom-aligned (its last row is row 16S-1, rows above its first row are
// dead rows that reproduce the virtual top row: H = ROW0 everywhere, so
// H(row 0) sees the reference's free top row).  At step t lane k computes
// column t-k of its 16 rows and hands its bottom row's H/F and the column's
// reference selector to lane k+1 by one cross-lane shift -- nothing goes
// through memory between rows, and the reference windows are staged once in
// LDS as per-column selectors.  The bottom lane holds both problems' last rows and gathers the
// candidates.  Per cell pair: 10 packed ops + 2 ANDs (query-profile byte
// select by v_perm_b32, diagonal, E, F, maxima, vetoes); an 'N' reference
// column adds the N penalty in real rows only.  On gfx950 v_pk_*, v_perm_b32
// and v_max_u32 issue at half the rate of v_add/v_and/v_max_u16
// (scripts/micro/valu_rate.hip), so a packed pair costs about what one
// 32-bit cell would: the packing pays through fewer lanes per problem, not
// through fewer issue slots.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "bt2g_kernels.h"

namespace {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
constexpr int R = 16;   // rows per lane

__device__ __forceinline__ uint32_t psub(uint32_t a, uint32_t b) {
	return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, a),
	                                                                  __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t pmin(uint32_t a, uint32_t b) {
	return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
	                                                              __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t pmax(uint32_t a, uint32_t b) {
	return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a),
	                                                              __builtin_bit_cast(u16x2, b)));
}

// score-plane stores (BT2G_SW_NT_STORE: non-temporal, measured 4x slower fill: 57.8 vs 13.9 ms)
__device__ __forceinline__ void st_plane(uint8_t* p, uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
#ifdef BT2G_SW_NT_STORE
	typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
	u32x4 v = {x, y, z, w};
	__builtin_nontemporal_store(v, (u32x4*)p);
#else
	*(uint4*)p = make_uint4(x, y, z, w);
#endif
}

// DEC: acc * 2 + (a != b) for the low / high 16-bit halves -- a compare into
// VCC and an add-with-carry that shifts the bit in: two full-rate ops per bit
// (v_pk_* ops issue at half rate; the compiler's form of a per-half test took
// about twice the instructions)
__device__ __forceinline__ uint32_t shl_ne_lo(uint32_t acc, uint32_t a, uint32_t b) {
	uint32_t r;
	asm("v_cmp_ne_u16_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, %3, %3, vcc" : "=v"(r) : "v"(a), "v"(b), "v"(acc) : "vcc");
	return r;
}
__device__ __forceinline__ uint32_t shl_ne_hi(uint32_t acc, uint32_t a, uint32_t b) {
	uint32_t r;
	asm("v_cmp_ne_u16_sdwa vcc, %1, %2 src0_sel:WORD_1 src1_sel:WORD_1\n\tv_addc_co_u32_e32 %0, vcc, %3, %3, vcc"
	    : "=v"(r) : "v"(a), "v"(b), "v"(acc) : "vcc");
	return r;
}

__device__ __forceinline__ int first5(int m) {
	return (m & 1) ? 0 : (m & 2) ? 1 : (m & 4) ? 2 : (m & 8) ? 3 : 4;
}

struct Half {
	const uint8_t* rd;
	const uint8_t* qu;
	int64_t refl, win_off;
	uint32_t nrow, ncol, pi, refidx;
	int32_t minsc;
	uint32_t row0;      // end-to-end: 0xff (u8 fill) or 0xffff (i16 fill); local: 0
	bool fw, live;
};

}  // namespace

#ifndef BT2G_SW_COLS
#define BT2G_SW_COLS 1          // columns per systolic step (1, or 2: measured slower, occupancy 2)
#endif
#ifndef BT2G_SW_WAVES
#define BT2G_SW_WAVES 3
#endif
#ifndef BT2G_SW_WAVES_STORE
#define BT2G_SW_WAVES_STORE 2      // the score-plane stores need registers: no spills at 2
#endif
// STORE: also write every cell's H to the score plane for the backtrace
// (sw_backtrace.hip), block-major: problem pi's stack rows 16k..16k+15 of
// column j at plane + pi*hslot + ((k*max_cols + j)*16)*hbytes, so that a
// backtrace step (up-left) usually stays inside one 128-B line; hbytes 1 keeps
// u8 fills only.
// DEC (end-to-end, u8 fills): instead of H, the backtrace's decision at every
// cell as 4 bits (the "decision plane", 8 B per 16-row block column: word
// w = row >> 3 holds, for row 8w+i, bits 0 / 1 / 2 below at bits 3(7-i)+2 /
// 3(7-i)+1 / 3(7-i) and bit 3 at bit 24+7-i): the reference's walk
// (aligner_swsse_ee_u8.cpp:1357-1540) picks, in H state, diag > H-up > F-up >
// H-left > E-left, in F state H-up > F-up, in E state H-left > E-left; with
// H = max(diag, E, F) and every walked cell above the floor that is
//   bit 0  H != diag              bit 1  H != F
//   bit 2  F != H(up) - rfgo      bit 3  E != H(left) - rdgo
// (F-up / E-left being then the other source of F / E).  A walk step reads
// one nibble and no neighbour, no column or row scan (sw_backtrace.hip KIND 2).
// WIDE (reads of 1025..2048 bases, S = 65..128): one problem pair per
// workgroup of two waves; lane 63 hands its bottom row to lane 64 through LDS
// (double-buffered, one barrier per step) where the DPP shift stops at the wave
// edge.  (Before: one problem per lane in k_sw_fill, ~200 ms per 2 kb DP.)
template <bool LOCAL, bool SAMEGO, bool STORE, bool DEC = false, bool WIDE = false>
__global__ void __launch_bounds__(WIDE ? 128 : 64) __attribute__((amdgpu_waves_per_eu((STORE || LOCAL) ? BT2G_SW_WAVES_STORE : BT2G_SW_WAVES)))
k_sw_sys(const bt2g_sw_problem* __restrict__ probs, uint32_t nprob, const uint8_t* __restrict__ reads,
            const uint8_t* __restrict__ quals, uint32_t stride, const uint32_t* __restrict__ lens,
            const uint8_t* __restrict__ windows, const uint8_t* __restrict__ ref_codes,
            const uint64_t* __restrict__ ref_starts, SwConst C, int enable8, uint32_t cap, uint32_t max_cols,
            uint32_t S, uint32_t ldsw, bt2g_sw_result* __restrict__ res, bt2g_sw_cand* __restrict__ cands,
            uint8_t* __restrict__ plane, uint64_t hslot, int hbytes) {
	const uint32_t lane = threadIdx.x;
	const uint32_t G = WIDE ? 1u : 64u / S;      // problem pairs per wave (WIDE: per workgroup)
	const uint32_t g = WIDE ? 0u : lane / S, k = WIDE ? lane : lane % S;
	const bool in_group = WIDE ? lane < S : g < G;
	const uint32_t base = blockIdx.x * 2u * G;
	Half h[2];
#pragma unroll
	for(int x = 0; x < 2; x++) {
		Half& H = h[x];
		const uint32_t pi = base + (x ? G : 0u) + g;
		H.live = in_group && pi < nprob;
		H.nrow = H.ncol = 0;
		H.row0 = LOCAL ? 0u : 0xffu;
		if(!H.live) continue;
		H.pi = pi;
		const bt2g_sw_problem p = probs[pi];
		H.nrow = lens[p.read];
		H.ncol = p.ncol;
		H.rd = reads + (size_t)p.read * stride;
		H.qu = quals + (size_t)p.read * stride;
		H.fw = p.fw != 0;
		H.refl = p.refl;
		H.win_off = p.win_off;
		H.refidx = p.refidx;
		H.minsc = p.minsc;
		// end-to-end: u8 fill iff enable8 && minsc >= -254 (aligner_sw.cpp:516-519);
		// local: both fills in one pass (score domain)
		if(!LOCAL) H.row0 = (enable8 && p.minsc >= -254) ? 0xffu : 0xffffu;
		if(H.ncol > max_cols || H.ncol == 0 || H.nrow == 0 || H.nrow > 16u * S) {
			if(k == 0) {
				bt2g_sw_result bad{};
				bad.flag = -3;
				bad.best = INT32_MIN;
				res[pi] = bad;
			}
			H.live = false;
			H.nrow = H.ncol = 0;
		}
	}
	// strip-stack row of a problem's row 0: end-to-end, the last row at the stack
	// bottom; local, the padding rows up to a multiple of 16 below it
	auto top_of = [&](const Half& H) -> uint32_t { return 16u * S - (LOCAL ? ((H.nrow + 15u) & ~15u) : H.nrow); };
	// wave-uniform sweep length
	uint32_t ncolmax = h[0].ncol > h[1].ncol ? h[0].ncol : h[1].ncol;
#pragma unroll
	for(int o = 32; o > 0; o >>= 1) {
		uint32_t v = (uint32_t)__shfl_xor((int)ncolmax, o);
		ncolmax = v > ncolmax ? v : ncolmax;
	}
	if(ncolmax == 0) return;

	// Scoring::mmpens (scoring.h:103-131) staged in LDS for per-lane lookups
	__shared__ uint8_t mmq[48];
	__shared__ uint32_t lcnt[128], lmaxc[128];     // LOCAL: candidates per problem, their largest column
	if(lane <= 40) mmq[lane] = (uint8_t)C.mmpen[lane];
	if(LOCAL && lane < 64u) {
		lcnt[lane] = lcnt[lane + 64u] = 0u;
		lmaxc[lane] = lmaxc[lane + 64u] = 0u;
	}
	// this lane's rows: global row 16k+i of the stack; problem row = that - (16S - nrow).
	// All read bytes and qualities are fetched first (independent loads, one
	// wait), then turned into query-profile words.
	uint32_t bq[2][R];
	uint32_t below[2] = {5u, 5u};    // LOCAL: read character of the row under this lane's block (5: none)
#pragma unroll
	for(int x = 0; x < 2; x++) {
		const Half& H = h[x];
		const int64_t rx0 = (int64_t)(16u * k) - (int64_t)top_of(H);
		if(LOCAL && H.live && rx0 + R >= 0 && rx0 + R < (int64_t)H.nrow) {
			const uint32_t rb = (uint32_t)(rx0 + R);
			const uint32_t c = H.rd[H.fw ? rb : H.nrow - 1u - rb];
			below[x] = H.fw ? c : (c > 3u ? 4u : 3u - c);
		}
#pragma unroll
		for(int i = 0; i < R; i++) {
			const int64_t rx = rx0 + i;
			const bool real = H.live && rx >= 0 && rx < (int64_t)H.nrow;
			const uint32_t o = real ? (H.fw ? (uint32_t)rx : H.nrow - 1 - (uint32_t)rx) : 0u;
			const uint8_t* rdp = real ? H.rd : reads;
			const uint8_t* qup = real ? H.qu : quals;
			bq[x][i] = (uint32_t)rdp[o] | ((uint32_t)qup[o] << 8);
		}
	}
	__syncthreads();
	const uint32_t row0p = h[0].row0 | (h[1].row0 << 16);
	uint32_t PA[R], PB[R], M[R], E[R], Hc[R];   // M: 0 in gap-barrier rows (veto)
	const int gb = C.gapbar;
	const uint32_t match4 = (uint32_t)C.match * 0x01010101u;
	// LOCAL: rows (bit i; +16 for the high problem) whose read character is c,
	// real rows >= minrow (gather-eligible), the u8 fill's bias per problem
	uint32_t rm0 = 0, rm1 = 0, rm2 = 0, rm3 = 0, rm4 = 0, rowok = 0;
	uint32_t biasl[2] = {0u, 0u};
	uint64_t minrow[2] = {~0ull, ~0ull};
	if(LOCAL) {
#pragma unroll
		for(int x = 0; x < 2; x++)
			minrow[x] = ((uint64_t)(int64_t)h[x].minsc + (uint64_t)C.match - 1u) / (uint64_t)(C.match > 0 ? C.match : 1) - 1u;
	}
#pragma unroll
	for(int i = 0; i < R; i++) {
		uint32_t pa = 0, pb = 0, v = 0, hi = 0;
#pragma unroll
		for(int x = 0; x < 2; x++) {
			const Half& H = h[x];
			const int64_t rx = (int64_t)(16u * k + i) - (int64_t)top_of(H);
			uint32_t prof = LOCAL ? match4 : 0u, veto = 0, hinit = 0;   // local dead/padding rows: score 0
			if(H.live) {
				if(rx < 0 || rx >= (int64_t)H.nrow) {
					if(!LOCAL && rx < 0) hinit = H.row0;  // dead row: H(col -1) = ROW0
				} else {
					// {pen(A), pen(C), pen(G), pen(T)} (Scoring::score, scoring.h:237-262, no match bonus)
					int c = (int)(bq[x][i] & 0xffu);
					if(!H.fw) c = c > 3 ? 4 : 3 - c;
					int q = (int)(bq[x][i] >> 8) - 33;
					q = q < 0 ? 0 : (q > 40 ? 40 : q);
					if(LOCAL) {
						// pen' = match - score: 0 for a match, match + mmpen / match + npen otherwise
						prof = c > 3 ? (uint32_t)(C.match + C.npen) * 0x01010101u
						             : (((uint32_t)(C.match + mmq[q]) * 0x01010101u) & ~(0xffu << (8 * c)));
						const uint32_t bit = 1u << (i + 16 * x);
						rm0 |= c == 0 ? bit : 0u;
						rm1 |= c == 1 ? bit : 0u;
						rm2 |= c == 2 ? bit : 0u;
						rm3 |= c == 3 ? bit : 0u;
						rm4 |= c > 3 ? bit : 0u;
						if((uint64_t)rx >= minrow[x]) rowok |= bit;
						// the u8 fill's bias: the largest penalty of the row's profile
						const uint32_t bl = c > 3 ? (uint32_t)C.npen
						                          : ((uint32_t)mmq[q] > (uint32_t)C.npen ? (uint32_t)mmq[q] : (uint32_t)C.npen);
						biasl[x] = bl > biasl[x] ? bl : biasl[x];
					} else {
						prof = c > 3 ? (uint32_t)C.npen * 0x01010101u
						             : ((uint32_t)mmq[q] * 0x01010101u) & ~(0xffu << (8 * c));
					}
					if(rx < gb || rx >= (int64_t)H.nrow - gb) veto = 0xffffu;
				}
			}
			if(x == 0) { pa = prof; v |= veto; hi |= hinit; }
			else { pb = prof; v |= veto << 16; hi |= hinit << 16; }
		}
		PA[i] = pa; PB[i] = pb; M[i] = ~v; E[i] = 0; Hc[i] = hi;
	}
	// LOCAL: rows whose down-right neighbour's read character is c (next row real)
	const uint32_t nm0 = ((rm0 >> 1) & 0x7fff7fffu) | (below[0] == 0u ? 0x8000u : 0u) | (below[1] == 0u ? 0x80000000u : 0u);
	const uint32_t nm1 = ((rm1 >> 1) & 0x7fff7fffu) | (below[0] == 1u ? 0x8000u : 0u) | (below[1] == 1u ? 0x80000000u : 0u);
	const uint32_t nm2 = ((rm2 >> 1) & 0x7fff7fffu) | (below[0] == 2u ? 0x8000u : 0u) | (below[1] == 2u ? 0x80000000u : 0u);
	const uint32_t nm3 = ((rm3 >> 1) & 0x7fff7fffu) | (below[0] == 3u ? 0x8000u : 0u) | (below[1] == 3u ? 0x80000000u : 0u);
	const uint32_t nm4 = ((rm4 >> 1) & 0x7fff7fffu) | (below[0] == 4u ? 0x8000u : 0u) | (below[1] == 4u ? 0x80000000u : 0u);
	// LOCAL: the bias of each problem over its group's lanes; the bottom lane's
	// u8-only padding rows (round16(nrow) - round8(nrow) = 8: its rows 8..15)
	uint32_t bias[2] = {0u, 0u}, u8o = 0u;
	if(LOCAL) {
		__shared__ uint32_t wbias[2];         // WIDE: the group spans both waves
		if(WIDE) {
			if(lane < 2u) wbias[lane] = 0u;
			__syncthreads();
			if(in_group) {
				atomicMax(&wbias[0], biasl[0]);
				atomicMax(&wbias[1], biasl[1]);
			}
			__syncthreads();
		}
#pragma unroll
		for(int x = 0; x < 2; x++) {
			uint32_t b = 0u;
			if(WIDE) {
				b = wbias[x];
			} else {
				for(uint32_t t = 0; t < S; t++) {
					const uint32_t o = (uint32_t)__shfl((int)biasl[x], (int)(g * S + t));
					b = o > b ? o : b;
				}
			}
			bias[x] = b;
			const uint32_t r = h[x].nrow & 15u;
			if(k == S - 1u && h[x].live && r != 0u && r <= 8u) u8o |= 0xffffu << (16 * x);
		}
	}
	// H(row above this lane's first row, column -1): ROW0 if that row is dead
	uint32_t hbprev = 0;
	if(k > 0) {
#pragma unroll
		for(int x = 0; x < 2; x++) {
			const int64_t rx = (int64_t)(16u * k) - 1 - (int64_t)top_of(h[x]);
			if(h[x].live && rx < 0) hbprev |= h[x].row0 << (16 * x);
		}
	}
	const uint32_t rdge2 = (uint32_t)C.rdge * 0x10001u, rdgo2 = (uint32_t)C.rdgo * 0x10001u;
	const uint32_t rfge2 = (uint32_t)C.rfge * 0x10001u, rfgo2 = (uint32_t)C.rfgo * 0x10001u;
	const uint32_t npen = (uint32_t)C.npen;
	const bool top = k == 0, bottom = k == S - 1 || !in_group;
	int lrmax[2] = {0, 0};
	uint32_t ncand[2] = {0, 0};
	// The pair's reference windows, once, as per-column v_perm_b32 selectors in
	// LDS ([group][column], aligner_sw.cpp:171-253 for the characters): byte 0
	// picks problem A's profile byte for its reference character, byte 2
	// problem B's (4 + c); 0x0c (zero) marks an 'N' column.  Columns past a
	// problem's width (and absent problems) get filler 'A' so that only real
	// 'N' columns send the wave down the N row loop.
	extern __shared__ uint32_t selw[];
	uint32_t* mysel = selw + (size_t)g * ldsw;
	uint32_t* mycm = selw + (size_t)(G + g) * ldsw;                                    // LOCAL: i16 column maxima
	uint16_t* mymsk = (uint16_t*)(selw + (size_t)2u * G * ldsw) + (size_t)g * ldsw;      // LOCAL: reference masks
	// local: also column ncol (the extra right column a gather's down-right test reads)
	const uint32_t ncl = ncolmax + (LOCAL ? 1u : 0u);
	if(in_group) {
		const uint8_t* src[2];
		int64_t lo[2], hi[2];
		bool masks[2];
#pragma unroll
		for(int x = 0; x < 2; x++) {
			const Half& H = h[x];
			masks[x] = H.win_off >= 0;
			lo[x] = 0;
			hi[x] = (int64_t)H.ncol + (LOCAL ? 1 : 0);
			src[x] = reads;
			if(!H.live) continue;
			if(masks[x]) {
				src[x] = windows + H.win_off;
			} else {
				const uint64_t rs = ref_starts[H.refidx], re = ref_starts[H.refidx + 1];
				src[x] = ref_codes + rs + H.refl;        // only dereferenced inside [lo, hi)
				lo[x] = H.refl < 0 ? -H.refl : 0;
				const int64_t end = (int64_t)(re - rs) - H.refl;
				hi[x] = end < hi[x] ? end : hi[x];
			}
		}
		// eight columns (two characters each) in flight per lane, then the selectors
		for(uint32_t c0 = k; c0 < ncl; c0 += 8u * S) {
			uint32_t v[2][8];
#pragma unroll
			for(int u = 0; u < 8; u++) {
				const int64_t c = (int64_t)c0 + (int64_t)u * S;
#pragma unroll
				for(int x = 0; x < 2; x++)
					v[x][u] = (c >= lo[x] && c < hi[x]) ? ((const __attribute__((address_space(1))) uint8_t*)src[x])[c]
					        : (c < (int64_t)h[x].ncol + (LOCAL ? 1 : 0) ? 0x100u : 0x200u);
			}
#pragma unroll
			for(int u = 0; u < 8; u++) {
				const uint32_t c = c0 + (uint32_t)u * S;
				if(c >= ncl) break;
				uint32_t sel = 0x0c000c00u, msk = 0u;
#pragma unroll
				for(int x = 0; x < 2; x++) {
					// 0x100: off the reference (N); 0x200: filler
					int code = v[x][u] == 0x100u ? 4 : v[x][u] == 0x200u ? 0
					         : (masks[x] ? first5((int)v[x][u]) : (int)v[x][u]);
					sel |= (code < 4 ? (uint32_t)(4 * x + code) : 0x0cu) << (16 * x);
					// DEC: an ambiguous reference mask (IUPAC, caller windows only) in the
					// otherwise unused selector byte: the fill scores its first base
					// (firsts5) but the walk's diagonal test matches any of its bases
					if(DEC && masks[x] && v[x][u] < 16u && __popc(v[x][u]) > 1)
						sel = (sel & ~(0xff00u << (16 * x))) | ((0x80u | v[x][u]) << (8 + 16 * x));
					// the gather's reference mask (aligner_sw.cpp:247-253: 1 << c, N -> 16)
					const uint32_t m = v[x][u] == 0x100u ? 16u : v[x][u] == 0x200u ? 0u
					                 : (masks[x] ? v[x][u] : (v[x][u] > 3u ? 16u : 1u << v[x][u]));
					msk |= m << (8 * x);
				}
				mysel[c] = sel;
				if(LOCAL) mymsk[c] = (uint16_t)msk;
			}
		}
	}
	__syncthreads();
#if BT2G_SW_COLS == 2
	static_assert(!LOCAL, "the two-column step is end-to-end only");
	// Two columns per step: cell (i, j+1) only waits for (i, j)'s E and
	// (i-1, j)'s H, so the two F chains of a step interleave (twice the ILP of
	// the dependent row recurrence) and the lane-to-lane hand-off is halved.
	uint32_t hout0 = 0, fout0 = 0, hout1 = 0, fout1 = 0;
	uint32_t nsel0 = in_group ? mysel[0] : 0u, nsel1 = in_group ? mysel[1] : 0u;
	const uint32_t ncp = (ncolmax + 1) / 2;     // column pairs
	const uint32_t T = ncp + S - 1;
	for(uint32_t t = 0; t < T; t++) {
		const uint32_t hin0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hout0, 0x138, 0xf, 0xf, false);
		const uint32_t fin0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fout0, 0x138, 0xf, 0xf, false);
		const uint32_t hin1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hout1, 0x138, 0xf, 0xf, false);
		const uint32_t fin1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fout1, 0x138, 0xf, 0xf, false);
		const int jp = (int)t - (int)k;
		if(jp < 0 || jp >= (int)ncp) continue;
		const uint32_t j = 2u * (uint32_t)jp;
		const uint32_t sel0 = nsel0, sel1 = nsel1;
		if(in_group && jp + 1 < (int)ncp) { nsel0 = mysel[j + 2]; nsel1 = mysel[j + 3]; }
		uint32_t hup0, fup0, hup1, fup1, diag0;
		if(top) {
			hup0 = fup0 = hup1 = fup1 = 0;
			diag0 = row0p;
		} else {
			hup0 = hin0; fup0 = fin0; hup1 = hin1; fup1 = fin1;
			diag0 = hbprev;
			hbprev = hup1;
		}
		uint32_t diag1 = top ? row0p : hup0;
		const uint32_t nf0 = ((sel0 & 0xffu) == 0x0cu ? npen : 0u) | (((sel0 >> 16) & 0xffu) == 0x0cu ? npen << 16 : 0u);
		const uint32_t nf1 = ((sel1 & 0xffu) == 0x0cu ? npen : 0u) | (((sel1 >> 16) & 0xffu) == 0x0cu ? npen << 16 : 0u);
		uint32_t fprev0 = fup0, hprev0 = hup0, fprev1 = fup1, hprev1 = hup1;
		auto rows = [&](auto n_tag) {
			constexpr bool NCOL = decltype(n_tag)::value;
#pragma unroll
			for(int i = 0; i < R; i++) {
				uint32_t pen0 = __builtin_amdgcn_perm(PB[i], PA[i], sel0);
				uint32_t pen1 = __builtin_amdgcn_perm(PB[i], PA[i], sel1);
				if(NCOL) {
					uint32_t pa = PA[i], pb = PB[i];
					asm volatile("" : "+v"(pa), "+v"(pb));
					const uint32_t real = (pa ? 0xffffu : 0u) | (pb ? 0xffff0000u : 0u);
					pen0 = pmax(pen0, nf0 & real);
					pen1 = pmax(pen1, nf1 & real);
				}
				// column j
				const uint32_t d0 = psub(diag0, pen0);
				const uint32_t f0 = pmax(psub(fprev0, rfge2), psub(hprev0, rfgo2)) & M[i];
				const uint32_t h0 = pmax(pmax(d0, E[i]), f0);
				const uint32_t e0 = pmax(psub(E[i], rdge2), psub(h0, rdgo2) & M[i]);
				// column j+1
				const uint32_t d1 = psub(diag1, pen1);
				const uint32_t f1 = pmax(psub(fprev1, rfge2), psub(hprev1, rfgo2)) & M[i];
				const uint32_t h1 = pmax(pmax(d1, e0), f1);
				E[i] = pmax(psub(e0, rdge2), psub(h1, rdgo2) & M[i]);
				diag0 = Hc[i];      // H(i, j-1): diagonal of (i+1, j)
				diag1 = h0;         // H(i, j):   diagonal of (i+1, j+1)
				Hc[i] = h1;
				fprev0 = f0; hprev0 = h0;
				fprev1 = f1; hprev1 = h1;
			}
		};
		if(__ballot((nf0 | nf1) != 0)) rows(std::true_type{});
		else rows(std::false_type{});
		hout0 = hprev0; fout0 = fprev0;
		hout1 = hprev1; fout1 = fprev1;
		// the bottom lane is the last reader of columns j, j+1: their slots now
		// keep both problems' last-row H for the gather below
		if(bottom && in_group) {
			mysel[j] = hprev0;
			if(j + 1 < ncolmax) mysel[j + 1] = hprev1;
		}
	}
#else
	uint32_t hout = 0, fout = 0, mout = 0, cmout = 0;
	uint32_t nsel = in_group ? mysel[0] : 0u;
	const uint32_t T = ncolmax + S - 1;
	// score plane: a 16-row block is written only when one of its cells can be
	// on a backtrace (end-to-end: H >= minsc, every value a walk compares for
	// equality is at least its own score; local: H > 0, unwritten blocks read
	// as 0, sw_backtrace.hip); per column, a 16-bit mask of the written blocks
	// (S <= 16; beyond that every block is written)
#ifdef BT2G_SW_NOMASK
	const bool use_mask = false;           // timing experiments only
#else
	const bool use_mask = S <= 16u;
#endif
	const uint32_t thr0 = LOCAL ? 1u : h[0].row0 + (uint32_t)h[0].minsc;
	const uint32_t thr1 = LOCAL ? 1u : h[1].row0 + (uint32_t)h[1].minsc;
	const uint32_t pitch = sw_plane_pitch(max_cols);       // plane columns per 16-row block
	uint8_t* const mplane = plane + (size_t)16u * S * pitch * (size_t)hbytes;
	// (staging 4 columns per lane in LDS and writing 64-B bursts measured
	// slower: 17.2 vs 15.4 ms; stores into an L2-resident 64 KB instead of the
	// plane: 12.4 ms, no stores 10.0 ms)
	// LOCAL: a block is searched for candidates when its maximum reaches minsc
	// (never for a problem without gather-eligible rows); cthr = minsc - 1 per half
	uint32_t ctest[2];
#pragma unroll
	for(int x = 0; x < 2; x++)
		ctest[x] = (LOCAL && ((rowok >> (16 * x)) & 0xffffu) != 0u && h[x].minsc > 0 && h[x].minsc <= 0xffff)
		               ? (uint32_t)h[x].minsc : 0x10000u;
	const uint32_t cthr = ((ctest[0] - 1u) & 0xffffu) | (((ctest[1] - 1u) & 0xffffu) << 16);
	const uint32_t match2 = (uint32_t)C.match * 0x10001u, npm2 = (uint32_t)(C.match + C.npen) * 0x10001u;
	// DEC: this column's decision bits per problem (rows 0-7 / 8-15 shifted into
	// DA/DB[0] / [1], 3 bits a row) and the E bits of the next column, known one
	// column early (NA / NB, one bit a row; older bits shift out and are masked)
	uint32_t DA[2] = {0u, 0u}, DB[2] = {0u, 0u}, NA = 0u, NB = 0u;
	auto dec_cell = [&](int i, uint32_t hh, uint32_t dw, uint32_t f, uint32_t hu) {
		const int w = i >> 3;
		DA[w] = shl_ne_lo(shl_ne_lo(shl_ne_lo(DA[w], hh, dw), hh, f), f, hu);
		DB[w] = shl_ne_hi(shl_ne_hi(shl_ne_hi(DB[w], hh, dw), hh, f), f, hu);
	};
	auto dec_next = [&](uint32_t en, uint32_t hgm) {
		NA = shl_ne_lo(NA, en, hgm);
		NB = shl_ne_hi(NB, en, hgm);
	};
	for(uint32_t t = 0; t < T; t++) {
		// the lane above computed this lane's column in the previous step (DPP wave_shr:1)
		uint32_t hin = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hout, 0x138, 0xf, 0xf, false);
		uint32_t fin = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fout, 0x138, 0xf, 0xf, false);
		uint32_t mskin = STORE ? (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mout, 0x138, 0xf, 0xf, false) : 0u;
		uint32_t cmin = LOCAL ? (uint32_t)__builtin_amdgcn_update_dpp(0, (int)cmout, 0x138, 0xf, 0xf, false) : 0u;
		if constexpr(WIDE) {
			// across the wave edge: lane 63's previous step to lane 64 (a slot is
			// rewritten two steps later, after lane 64 has passed the next barrier)
			__shared__ uint32_t xch[2][4];
			if(lane == 63u) {
				uint32_t* b = xch[t & 1u];
				b[0] = hout; b[1] = fout; b[2] = mout; b[3] = cmout;
			}
			__syncthreads();
			if(lane == 64u) {
				const uint32_t* b = xch[t & 1u];
				hin = b[0]; fin = b[1]; mskin = b[2]; cmin = b[3];
			}
		}
		const int j = (int)t - (int)k;
		if(j < 0 || j >= (int)ncolmax) continue;
		const uint32_t selx = nsel;
		// DEC: ambiguous columns of this step (bytes 1 / 3 of the selector); their
		// diagonal term for the decision nibble is H(up-left) - the smallest
		// profile penalty over the mask's bases (Scoring::score with the mask)
		const bool amb = DEC && __ballot((selx & 0x80008000u) != 0u);
		const uint32_t sel = DEC ? ((selx & 0x00ff00ffu) | 0x0c000c00u) : selx;
		if(in_group) nsel = mysel[(uint32_t)j + 1 < ncolmax ? j + 1 : j];   // next step's column
		const uint32_t XA = NA, XB = NB;   // DEC: bit 3 of this column's cells (previous column)
		uint32_t hup, fup, diag;
		if(top) {
			hup = 0;
			fup = 0;
			diag = row0p;
		} else {
			hup = hin;
			fup = fin;
			diag = hbprev;
			hbprev = hup;
		}
		// An 'N' reference column costs npen in every real row (the selector
		// picked 0 there) but nothing in dead rows, which must stay at ROW0
		// (local: pen' = match in dead and padding rows, match + npen in real ones).
		// N columns are rare: the wave takes the slower row loop only when one of
		// its lanes sees one.
		const uint32_t ncm = ((sel & 0xffu) == 0x0cu ? 0xffffu : 0u) | (((sel >> 16) & 0xffu) == 0x0cu ? 0xffff0000u : 0u);
		const uint32_t nfloor = ncm & ((uint32_t)npen * 0x10001u);
		uint32_t fprev = fup, hprev = SAMEGO ? psub(hup, rfgo2) : hup;
		auto rows = [&](auto n_tag, auto a_tag) {
			constexpr bool NCOL = decltype(n_tag)::value;
			constexpr bool AMB = DEC && decltype(a_tag)::value;
#pragma unroll
			for(int i = 0; i < R; i++) {
				uint32_t pen = __builtin_amdgcn_perm(PB[i], PA[i], sel);
				if(NCOL) {
					// real rows: end-to-end a non-zero profile (sw_packed_ok: mmpen >= 1,
					// npen >= 1), local one other than match4; kept opaque so the masks are
					// not hoisted into 16 more registers
					uint32_t pa = PA[i], pb = PB[i];
					asm volatile("" : "+v"(pa), "+v"(pb));
					if(LOCAL) {
						const uint32_t real = (pa != match4 ? 0xffffu : 0u) | (pb != match4 ? 0xffff0000u : 0u);
						pen = pmax(pen, ncm & ((npm2 & real) | (match2 & ~real)));
					} else {
						const uint32_t real = (pa ? 0xffffu : 0u) | (pb ? 0xffff0000u : 0u);
						pen = pmax(pen, nfloor & real);
					}
				}
				// local: H(up-left) + match - pen' (no carry between the halves: H < 2^15)
				const uint32_t d = LOCAL ? psub(diag + match2, pen) : psub(diag, pen);
				uint32_t dwalk = d;   // DEC: the walk's diagonal term
				if(AMB) {
					// (rare: recomputed per row rather than held in registers)
					uint32_t pm = 0xffffffffu;
#pragma unroll
					for(int c = 0; c < 4; c++) {
						const uint32_t nm = (((selx >> (8 + c)) & 1u) ? 0u : 0xffffu) | (((selx >> (24 + c)) & 1u) ? 0u : 0xffff0000u);
						pm = pmin(pm, __builtin_amdgcn_perm(PB[i], PA[i], 0x0c000c00u | (uint32_t)c | ((4u + (uint32_t)c) << 16)) | nm);
					}
					const uint32_t ah = ((selx & 0x8000u) ? 0xffffu : 0u) | ((selx & 0x80000000u) ? 0xffff0000u : 0u);
					dwalk = (psub(diag, pm) & ah) | (d & ~ah);
				}
				if(SAMEGO) {
					// read and reference gap opens equal: H - open serves the F of the
					// next row and the E of the next column (one subtract less)
					const uint32_t f = pmax(psub(fprev, rfge2), hprev) & M[i];
					const uint32_t hh = pmax(pmax(d, E[i]), f);
					const uint32_t hg = psub(hh, rdgo2);
					if(DEC) {
						dec_cell(i, hh, dwalk, f, hprev);   // hprev: H(up) - rfgo
						const uint32_t hgm = hg & M[i];
						const uint32_t en = pmax(psub(E[i], rdge2), hgm);
						dec_next(en, hgm);
						E[i] = en;
					} else {
						E[i] = pmax(psub(E[i], rdge2), hg & M[i]);
					}
					diag = Hc[i];
					Hc[i] = hh;
					fprev = f;
					hprev = hg;          // carries H - open
				} else {
					const uint32_t huo = psub(hprev, rfgo2);
					const uint32_t f = pmax(psub(fprev, rfge2), huo) & M[i];
					const uint32_t hh = pmax(pmax(d, E[i]), f);
					if(DEC) {
						dec_cell(i, hh, dwalk, f, huo);
						const uint32_t hgm = psub(hh, rdgo2) & M[i];
						const uint32_t en = pmax(psub(E[i], rdge2), hgm);
						dec_next(en, hgm);
						E[i] = en;
					} else {
						E[i] = pmax(psub(E[i], rdge2), psub(hh, rdgo2) & M[i]);
					}
					diag = Hc[i];
					Hc[i] = hh;
					fprev = f;
					hprev = hh;
				}
			}
		};
		if(amb) {
			if(__ballot(ncm != 0)) rows(std::true_type{}, std::true_type{});
			else rows(std::false_type{}, std::true_type{});
		} else {
			if(__ballot(ncm != 0)) rows(std::true_type{}, std::false_type{});
			else rows(std::false_type{}, std::false_type{});
		}
		// this lane's block maxima (rows 0..7 and all): block masks, local column maxima
		uint32_t mlo = 0, mx = 0;
		if(LOCAL || (STORE && use_mask)) {
			mlo = Hc[0];
#pragma unroll
			for(int i = 1; i < R / 2; i++) mlo = pmax(mlo, Hc[i]);
			uint32_t mhi = Hc[R / 2];
#pragma unroll
			for(int i = R / 2 + 1; i < R; i++) mhi = pmax(mhi, Hc[i]);
			mx = pmax(mlo, mhi);
		}
		if(LOCAL) {
			// column maxima down the group (the reference's vcolmax, padding rows
			// included): u8 fill all rows, i16 fill without the u8-only padding rows
			const uint32_t cm = top ? mx : pmax(cmin, mx);
			cmout = cm;
			if(bottom && in_group) {
				const uint32_t m16 = (mlo & u8o) | (mx & ~u8o);
				mysel[j] = cm;                  // the last reader of selector j has read it
				mycm[j] = top ? m16 : pmax(cmin, m16);
			}
			// candidate cells of this block (aligner_swsse_loc_i16.cpp:1483-1520)
			const bool g0 = h[0].live && (uint32_t)j < h[0].ncol && (mx & 0xffffu) >= ctest[0];
			const bool g1 = h[1].live && (uint32_t)j < h[1].ncol && (mx >> 16) >= ctest[1];
			if(g0 || g1) {
				const uint32_t mj = mymsk[j], mj1 = mymsk[j + 1];
				// H >= minsc per half as one bit per half: min(H -sat (minsc-1), 1) is
				// 0 or 1 in each half, shifted to bit i / 16 + i (3 ops per row pair)
				uint32_t ge = 0;
#pragma unroll
				for(int i = 0; i < R; i++) ge |= pmin(psub(Hc[i], cthr), 0x00010001u) << i;
				auto s2 = [](uint32_t m, int c) -> uint32_t {
					return (((m >> c) & 1u) ? 0xffffu : 0u) | (((m >> (8 + c)) & 1u) ? 0xffff0000u : 0u);
				};
				// the cell is a match, its down-right neighbour (next row, next column) is not
				const uint32_t mb = (rm0 & s2(mj, 0)) | (rm1 & s2(mj, 1)) | (rm2 & s2(mj, 2)) | (rm3 & s2(mj, 3)) |
				                    (rm4 & s2(mj, 4));
				const uint32_t nb = (nm0 & s2(mj1, 0)) | (nm1 & s2(mj1, 1)) | (nm2 & s2(mj1, 2)) | (nm3 & s2(mj1, 3)) |
				                    (nm4 & s2(mj1, 4));
				const uint32_t cand = ge & mb & ~nb & rowok & ((g0 ? 0xffffu : 0u) | (g1 ? 0xffff0000u : 0u));
#pragma unroll
				for(int x = 0; x < 2; x++) {
					const uint32_t bits = (cand >> (16 * x)) & 0xffffu;
					if(!bits) continue;
					uint32_t slot = atomicAdd(&lcnt[2u * g + x], (uint32_t)__popc(bits));
					atomicMax(&lmaxc[2u * g + x], (uint32_t)j);
					bt2g_sw_cand* dst = cands + (size_t)h[x].pi * cap;
					const int32_t rx0 = (int32_t)(16u * k) - (int32_t)top_of(h[x]);
#pragma unroll
					for(int i = 0; i < R; i++) {
						if(!((bits >> i) & 1u)) continue;
						if(slot < cap) dst[slot] = bt2g_sw_cand{rx0 + i, j, (int32_t)((Hc[i] >> (16 * x)) & 0xffffu)};
						slot++;
					}
				}
			}
		}
#ifdef BT2G_SW_NOSTORE
		if(false) {                                   // timing experiments only
#else
		if(STORE && in_group) {
#endif
			bool s0 = h[0].live && (uint32_t)j < h[0].ncol, s1 = h[1].live && (uint32_t)j < h[1].ncol;
			const size_t cell = ((size_t)k * pitch + (uint32_t)j) * 16u;
			if(use_mask) {
				s0 = s0 && (mx & 0xffffu) >= thr0;
				s1 = s1 && (mx >> 16) >= thr1;
				// block masks of column j travel down the group with the H hand-off
				mout = (top ? 0u : mskin) | ((uint32_t)s0 << k) | ((uint32_t)s1 << (16u + k));
				if(bottom) {
					if(h[0].live && (uint32_t)j < h[0].ncol)
						*(uint16_t*)(mplane + (size_t)h[0].pi * hslot + 2u * (uint32_t)j) = (uint16_t)(mout & 0xffffu);
					if(h[1].live && (uint32_t)j < h[1].ncol)
						*(uint16_t*)(mplane + (size_t)h[1].pi * hslot + 2u * (uint32_t)j) = (uint16_t)(mout >> 16);
				}
			}
#ifdef BT2G_SW_STORE_TINY
			const uint64_t hslot = 0;                 // timing experiments only: all writes in 64 KB
#endif
			if(DEC) {
				// the decision bits of 16 rows: 8 B per problem (24 shifted-in bits a
				// word; the E bits of rows 0-7 / 8-15 are bits 15-8 / 7-0 of XA, XB)
				const uint32_t a0 = (DA[0] & 0xffffffu) | ((XA << 16) & 0xff000000u);
				const uint32_t a1 = (DA[1] & 0xffffffu) | (XA << 24);
				const uint32_t b0 = (DB[0] & 0xffffffu) | ((XB << 16) & 0xff000000u);
				const uint32_t b1 = (DB[1] & 0xffffffu) | (XB << 24);
				const size_t cell8 = ((size_t)k * pitch + (uint32_t)j) * 8u;
				// (u8 and i16 fills alike: the decisions do not depend on the width)
				if(s0) *(uint2*)(plane + (size_t)h[0].pi * hslot + cell8) = make_uint2(a0, a1);
				if(s1) *(uint2*)(plane + (size_t)h[1].pi * hslot + cell8) = make_uint2(b0, b1);
			} else if(!LOCAL && hbytes == 1) {
				// bytes of 16 rows per problem: low halves -> a, high halves -> b
				uint32_t a[4], b[4];
#pragma unroll
				for(int qd = 0; qd < 4; qd++) {
					const uint32_t y0 = __builtin_amdgcn_perm(Hc[4 * qd + 1], Hc[4 * qd], 0x06020400u);
					const uint32_t y1 = __builtin_amdgcn_perm(Hc[4 * qd + 3], Hc[4 * qd + 2], 0x06020400u);
					a[qd] = __builtin_amdgcn_perm(y1, y0, 0x05040100u);
					b[qd] = __builtin_amdgcn_perm(y1, y0, 0x07060302u);
				}
				if(s0 && h[0].row0 == 0xffu)
					st_plane(plane + (size_t)h[0].pi * hslot + cell, a[0], a[1], a[2], a[3]);
				if(s1 && h[1].row0 == 0xffu)
					st_plane(plane + (size_t)h[1].pi * hslot + cell, b[0], b[1], b[2], b[3]);
			} else {
				uint32_t a[8], b[8];
#pragma unroll
				for(int i = 0; i < 8; i++) {
					a[i] = __builtin_amdgcn_perm(Hc[2 * i + 1], Hc[2 * i], 0x05040100u);
					b[i] = __builtin_amdgcn_perm(Hc[2 * i + 1], Hc[2 * i], 0x07060302u);
				}
				if(s0) {
					uint8_t* d = plane + (size_t)h[0].pi * hslot + cell * 2u;
					st_plane(d, a[0], a[1], a[2], a[3]);
					st_plane(d + 16, a[4], a[5], a[6], a[7]);
				}
				if(s1) {
					uint8_t* d = plane + (size_t)h[1].pi * hslot + cell * 2u;
					st_plane(d, b[0], b[1], b[2], b[3]);
					st_plane(d + 16, b[4], b[5], b[6], b[7]);
				}
			}
		}
		hout = Hc[R - 1];        // the strip's bottom row at column j (== hprev when !SAMEGO)
		fout = fprev;
		// end-to-end: the bottom lane is the last reader of column j's selector:
		// the slot now keeps both problems' last-row H for the gather below
		if(!LOCAL && bottom && in_group) mysel[j] = hout;
	}
#endif
	if(LOCAL) {
		__syncthreads();                  // every lane's candidates are counted
		if(!bottom || !in_group) return;
		// SwAligner::align local outcome per problem: the u8 fill's column scan
		// (saturation, early bail colstop_, lastsolcol_), the i16 fill's when
		// the u8 one saturates (aligner_swsse_loc_u8.cpp:1278-1336,
		// aligner_swsse_loc_i16.cpp:1296-1367, aligner_sw.cpp:570-605), as k_sw_fill
#pragma unroll
		for(int x = 0; x < 2; x++) {
			if(!h[x].live) continue;
			const int64_t minsc = h[x].minsc, match = C.match, bs = bias[x];
			const uint32_t ncol = h[x].ncol;
			int flag = 0;
			int64_t best = 0, colstop = ncol, lastsol = 0;
			auto pass = [&](bool u8) {
				int64_t vmax = 0;
				bool sat = false;
				colstop = ncol;
				lastsol = 0;
				for(uint32_t j = 0; j < ncol; j++) {
					const int64_t c = (int64_t)(((u8 ? mysel[j] : mycm[j]) >> (16 * x)) & 0xffffu);
					vmax = c > vmax ? c : vmax;
					if(u8 && c + bs >= 255) { sat = true; break; }
					if(c < minsc) {
						if(c + (int64_t)(ncol - j - 1u) * match < minsc) { colstop = j + 1; break; }
					} else {
						lastsol = j;
					}
				}
				if(u8) {
					if(sat || vmax + bs >= 255) { flag = -2; best = INT64_MIN; }
					else if(vmax == 0 || vmax < minsc) { flag = -1; best = vmax; }
					else { flag = 0; best = vmax; }
				} else {
					if(vmax == 0) { flag = -1; best = INT64_MIN; }       // native -32768
					else if(vmax < minsc) { flag = -1; best = vmax; }
					else { flag = 0; best = vmax; }
				}
			};
			bt2g_sw_result out;
			out.u8succ = out.i16succ = 0;
			bool wide = !enable8;
			if(enable8) {
				pass(true);
				if(flag == -2) wide = true;
				else out.u8succ = flag == 0;
			}
			if(wide) {
				pass(false);
				out.i16succ = flag == 0;
			}
			out.flag = flag;
			out.colstop = (int32_t)colstop;
			out.lastsolcol = (int32_t)lastsol;
			// gather only columns <= lastsolcol_; on overflow the count stays and the
			// caller reports it (the stored subset is not the reference's)
			uint32_t nc = lcnt[2u * g + x];
			if(nc <= cap && lmaxc[2u * g + x] > (uint32_t)lastsol) {
				bt2g_sw_cand* cl = cands + (size_t)h[x].pi * cap;
				uint32_t kk = 0;
				for(uint32_t i = 0; i < nc; i++) {
					const bt2g_sw_cand c = cl[i];
					if(c.col <= (int32_t)lastsol) cl[kk++] = c;
				}
				nc = kk;
			}
			const bool fail = best == INT64_MIN || best < minsc;
			out.best = best == INT64_MIN ? INT32_MIN : (int32_t)best;
			if(fail) nc = 0;
			out.ncand = (int32_t)nc;
			out.aligned = (!fail && nc > 0) ? 1 : 0;
			res[h[x].pi] = out;
		}
		return;
	}
	if(!bottom || !in_group) return;
	// last-row maximum and end-to-end candidates in column order
	// (aligner_swsse_ee_u8.cpp:1096-1100, 1176-1208)
	for(uint32_t c = 0; c < ncolmax; c++) {
		const uint32_t hv = mysel[c];
#pragma unroll
		for(int x = 0; x < 2; x++) {
			if(h[x].live && c < h[x].ncol) {
				const int v = (int)((hv >> (16 * x)) & 0xffffu);
				lrmax[x] = v > lrmax[x] ? v : lrmax[x];
				const int64_t sc = (int64_t)v - (int64_t)h[x].row0;
				if(sc >= h[x].minsc) {
					if(ncand[x] < cap)
						cands[(size_t)h[x].pi * cap + ncand[x]] =
						    bt2g_sw_cand{(int32_t)h[x].nrow - 1, (int32_t)c, (int32_t)sc};
					ncand[x]++;
				}
			}
		}
	}
	// SwAligner::align end-to-end outcome (aligner_sw.cpp:500-620), as k_sw_fill
#pragma unroll
	for(int x = 0; x < 2; x++) {
		if(!h[x].live) continue;
		const bool u8 = h[x].row0 == 0xffu;
		bt2g_sw_result out;
		out.u8succ = out.i16succ = 0;
		int64_t best;
		const int64_t score = (int64_t)lrmax[x] - (int64_t)h[x].row0;
		if(score < h[x].minsc) { out.flag = -1; best = score; }
		else if(lrmax[x] == 0) { out.flag = -2; best = INT64_MIN; }
		else { out.flag = 0; best = score; }
		out.colstop = (int32_t)h[x].ncol - 1;
		out.lastsolcol = 0;
		if(u8) out.u8succ = out.flag == 0; else out.i16succ = out.flag == 0;
		const bool fail = best == INT64_MIN || best < h[x].minsc;
		out.best = best == INT64_MIN ? INT32_MIN : (int32_t)best;
		const uint32_t nc = fail ? 0u : ncand[x];
		out.ncand = (int32_t)nc;
		out.aligned = (!fail && nc > 0) ? 1 : 0;
		res[h[x].pi] = out;
	}
}

// All problems, u8 and i16 fills together (no partition needed); local: the
// u8 and i16 local fills in one pass.  Reads up to 1024 bases: a wave holds
// 64/S problem pairs; 1025..2048 bases: a two-wave workgroup per pair (WIDE).
template <bool WIDE>
static void launch_sys(bool local, const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* reads,
                       const uint8_t* quals, uint32_t stride, const uint32_t* lens, const uint8_t* windows,
                       const uint8_t* ref_codes, const uint64_t* ref_starts, const SwConst& C, int enable8,
                       uint32_t cap, uint32_t max_cols, bt2g_sw_result* res, bt2g_sw_cand* cands, uint8_t* plane,
                       uint64_t hslot, int hbytes, hipStream_t st) {
	const uint32_t S = (stride + 15u) / 16u;     // <= 128 (stride <= BT2G_MAX_READ_LEN)
	const uint32_t per_block = WIDE ? 2u : 2u * (64u / S);
	const uint32_t ldsw = (max_cols + 1u) | 1u;   // >= ncol+1 (column pairs); odd: groups hit different banks
	const dim3 grid((nprob + per_block - 1) / per_block), block(WIDE ? 128 : 64);
	const size_t lds = (per_block / 2) * sw_packed_group_words(max_cols, local) * sizeof(uint32_t);
#define BT2G_SYS(LO, SG, STO, DE)                                                                              \
	hipLaunchKernelGGL((k_sw_sys<LO, SG, STO, DE, WIDE>), grid, block, lds, st, probs, nprob, reads, quals, stride, \
	                   lens, windows, ref_codes, ref_starts, C, enable8, cap, max_cols, S, ldsw, res, cands, plane,  \
	                   hslot, hbytes)
	const bool samego = C.rdgo == C.rfgo;
	if(local) {
		if(plane) {
			if(samego) BT2G_SYS(true, true, true, false); else BT2G_SYS(true, false, true, false);
		} else {
			if(samego) BT2G_SYS(true, true, false, false); else BT2G_SYS(true, false, false, false);
		}
	} else if(plane && hbytes == 3) {
		// decision nibbles (the plane's u8 layout: masks after 16S x pitch bytes)
		hbytes = 1;
		if(samego) BT2G_SYS(false, true, true, true); else BT2G_SYS(false, false, true, true);
	} else if(plane) {
		if(samego) BT2G_SYS(false, true, true, false); else BT2G_SYS(false, false, true, false);
	} else {
		if(samego) BT2G_SYS(false, true, false, false); else BT2G_SYS(false, false, false, false);
	}
#undef BT2G_SYS
}

void launch_sw_packed(bool local, const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* reads,
                      const uint8_t* quals, uint32_t stride, const uint32_t* lens, const uint8_t* windows,
                      const uint8_t* ref_codes, const uint64_t* ref_starts, const SwConst& C, int enable8,
                      uint32_t cap, uint32_t max_cols, bt2g_sw_result* res, bt2g_sw_cand* cands, uint8_t* plane,
                      uint64_t hslot, int hbytes, hipStream_t st) {
	if(nprob == 0) return;
	if((stride + 15u) / 16u > 64u)
		launch_sys<true>(local, probs, nprob, reads, quals, stride, lens, windows, ref_codes, ref_starts, C, enable8,
		                 cap, max_cols, res, cands, plane, hslot, hbytes, st);
	else
		launch_sys<false>(local, probs, nprob, reads, quals, stride, lens, windows, ref_codes, ref_starts, C, enable8,
		                  cap, max_cols, res, cands, plane, hslot, hbytes, st);
}
