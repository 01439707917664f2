// fm_device.h -- device-side FM-index primitives for gfx950.
//
// HBM layout (one copy per GPU, written once by index_load.cpp):
//   sides  : the .bt2 "ebwt" array unchanged -- 64-B sides, 48 B of 2-bit BWT
//            (192 rows, row k at bits 2*(k%4) of byte k/4) followed by 4 u32
//            occurrence counts of A,C,G,T before the side (bt2_idx.h:1753-1757,
//            2929-3081).  A side is exactly one 64-B HBM request: an LF step is
//            one (or two, when top/bot rows sit in different sides) 64-B gathers.
//   ftab/eftab/fchr/offs : the .bt2 arrays unchanged.
//
// Counting follows bt2_idx.h:1758-2080 (countBt2Side[Ex], countUpTo[Ex],
// '$'-as-'A' correction at 1766-1774/1891-1899), but per side it is done with
// 32-bit bit-plane masks and popcounts instead of the byte LUT.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define BT2G_OFF_MASK 0xffffffffu

struct DevEbwt {
	const uint8_t*  sides;
	const uint32_t* ftab;
	const uint32_t* eftab;
	const uint32_t* offs;
	uint32_t len;
	uint32_t zoff;
	uint32_t zbyte;      // _zEbwtByteOff (bt2_idx.h:1631-1641)
	int32_t  zbp;        // _zEbwtBpOff
	uint32_t ftab_chars;
	uint32_t off_rate;
	int32_t  fw;         // Ebwt::fw()
	uint32_t fchr[5];
};

// Field-wise per-lane choice between two indexes (a per-lane reference to one
// of two kernel arguments would have to live in scratch).
__device__ __forceinline__ DevEbwt pick_ebwt(bool first, const DevEbwt& a, const DevEbwt& b) {
	DevEbwt e;
	e.sides = first ? a.sides : b.sides;
	e.ftab = first ? a.ftab : b.ftab;
	e.eftab = first ? a.eftab : b.eftab;
	e.offs = first ? a.offs : b.offs;
	e.len = first ? a.len : b.len;
	e.zoff = first ? a.zoff : b.zoff;
	e.zbyte = first ? a.zbyte : b.zbyte;
	e.zbp = first ? a.zbp : b.zbp;
	e.ftab_chars = first ? a.ftab_chars : b.ftab_chars;
	e.off_rate = first ? a.off_rate : b.off_rate;
	e.fw = first ? a.fw : b.fw;
#pragma unroll
	for(int i = 0; i < 5; i++) e.fchr[i] = first ? a.fchr[i] : b.fchr[i];
	return e;
}

// One loaded side: 12 BWT words (16 rows each) + 4 occ counts.
struct SideData {
	uint32_t w[12];
	uint32_t occ[4];
};

__device__ __forceinline__ void load_side(const DevEbwt& e, uint32_t side, SideData& s) {
	typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
	// global address space, stated: through a DevEbwt picked at run time the
	// pointer is generic, and flat loads make every later wait a full drain
	typedef const __attribute__((address_space(1))) u32x4 gu32x4;
	const gu32x4* p = (const gu32x4*)(e.sides + (size_t)side * 64u);
	u32x4 a = p[0], b = p[1], c = p[2], d = p[3];
	s.w[0] = a.x; s.w[1] = a.y; s.w[2] = a.z; s.w[3] = a.w;
	s.w[4] = b.x; s.w[5] = b.y; s.w[6] = b.z; s.w[7] = b.w;
	s.w[8] = c.x; s.w[9] = c.y; s.w[10] = c.z; s.w[11] = c.w;
	s.occ[0] = d.x; s.occ[1] = d.y; s.occ[2] = d.z; s.occ[3] = d.w;
}

// Raw counts of A, C, G, T among the first `charOff` rows of the side (the '$'
// is still counted as an 'A' here).
__device__ __forceinline__ void side_counts(const SideData& s, uint32_t charOff, uint32_t cnt[4]) {
	uint32_t a = 0, c = 0, g = 0;
#pragma unroll
	for(int k = 0; k < 12; k++) {
		int nk = (int)charOff - 16 * k;
		nk = nk < 0 ? 0 : (nk > 16 ? 16 : nk);
		uint32_t m = nk >= 16 ? 0x55555555u : ((1u << (2 * nk)) - 1u) & 0x55555555u;
		uint32_t lo = s.w[k] & 0x55555555u;
		uint32_t hi = (s.w[k] >> 1) & 0x55555555u;
		a += __builtin_popcount(~(lo | hi) & m);
		c += __builtin_popcount(lo & ~hi & m);
		g += __builtin_popcount(hi & ~lo & m);
	}
	cnt[0] = a; cnt[1] = c; cnt[2] = g; cnt[3] = charOff - a - c - g;
}

__device__ __forceinline__ uint32_t side_count1(const SideData& s, uint32_t charOff, int ch) {
	uint32_t n = 0;
	const uint32_t x = (uint32_t)(3 - ch) * 0x55555555u;   // c_table[ch] restricted to 32 bits
#pragma unroll
	for(int k = 0; k < 12; k++) {
		int nk = (int)charOff - 16 * k;
		nk = nk < 0 ? 0 : (nk > 16 ? 16 : nk);
		uint32_t m = nk >= 16 ? 0x55555555u : ((1u << (2 * nk)) - 1u) & 0x55555555u;
		uint32_t y = s.w[k] ^ x;
		n += __builtin_popcount(y & (y >> 1) & m);
	}
	return n;
}

// Character of row charOff of the side.  The word is picked by a select chain
// over values made opaque to the optimiser: folded back into an indexed load,
// a data-dependent index would put the whole side in scratch.
__device__ __forceinline__ int side_rowL(const SideData& s, uint32_t charOff) {
	const uint32_t k = charOff >> 4;
	uint32_t v[12];
#pragma unroll
	for(int i = 0; i < 12; i++) v[i] = s.w[i];
	asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
	                  "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]));
	uint32_t w = v[0];
#pragma unroll
	for(int i = 1; i < 12; i++) w = k == (uint32_t)i ? v[i] : w;
	return (int)((w >> (2 * (charOff & 15))) & 3u);
}


// Issue priority of the latency-bound walkers ($BT2G_WALK_PRIO at build time,
// 0 = none): a walker wave issues a few instructions between dependent HBM
// gathers, and on a SIMD shared with VALU-heavy waves of another service's
// kernel (the SW fill) it loses issue arbitration to older waves (priority,
// then age: MI355X_MICROARCH.md, "Two waves per SIMD", item 2) -- s_setprio at
// entry puts its few instructions first.
#ifndef BT2G_WALK_PRIO
#define BT2G_WALK_PRIO 0
#endif
__device__ __forceinline__ void walk_prio() {
#if BT2G_WALK_PRIO > 0
	__builtin_amdgcn_s_setprio(BT2G_WALK_PRIO);
#endif
}

// fchr[c] without a data-dependent index into the (kernel-argument) array
__device__ __forceinline__ uint32_t fchr_at(const DevEbwt& e, int c) {
	return c == 0 ? e.fchr[0] : c == 1 ? e.fchr[1] : c == 2 ? e.fchr[2] : c == 3 ? e.fchr[3] : e.fchr[4];
}

// '$' correction of countBt2Side/Ex: true iff the '$' (stored as 'A') lies in
// this side strictly before <by,bp>.
__device__ __forceinline__ bool dollar_before(const DevEbwt& e, uint32_t side, uint32_t charOff) {
	uint32_t sbo = side * 64u, by = charOff >> 2, bp = charOff & 3u;
	if(sbo <= e.zbyte && sbo + by >= e.zbyte) {
		if(sbo + by > e.zbyte || (sbo + by == e.zbyte && (int)bp > e.zbp)) return true;
	}
	return false;
}

// countBt2SideEx for a row whose side is loaded in s.
__device__ __forceinline__ void occ4(const DevEbwt& e, const SideData& s, uint32_t row, uint32_t out[4]) {
	uint32_t side = row / 192u, co = row % 192u;
	uint32_t c[4];
	side_counts(s, co, c);
	if(dollar_before(e, side, co)) c[0]--;
#pragma unroll
	for(int i = 0; i < 4; i++) out[i] = c[i] + s.occ[i] + e.fchr[i];
}

// countBt2Side for one character.
__device__ __forceinline__ uint32_t occ1(const DevEbwt& e, const SideData& s, uint32_t row, int ch) {
	uint32_t side = row / 192u, co = row % 192u;
	uint32_t n = side_count1(s, co, ch);
	if(ch == 0 && dollar_before(e, side, co)) n--;
	uint32_t o0 = s.occ[0], o1 = s.occ[1], o2 = s.occ[2], o3 = s.occ[3];
	asm volatile("" : "+v"(o0), "+v"(o1), "+v"(o2), "+v"(o3));   // keep the select in registers
	const uint32_t occ = ch == 0 ? o0 : ch == 1 ? o1 : ch == 2 ? o2 : o3;
	return n + occ + fchr_at(e, ch);
}

__device__ __forceinline__ uint32_t ftab_hi(const DevEbwt& e, uint32_t i) {
	uint32_t v = e.ftab[i];
	return v <= e.len ? v : e.eftab[(v ^ BT2G_OFF_MASK) * 2 + 1];
}
__device__ __forceinline__ uint32_t ftab_lo(const DevEbwt& e, uint32_t i) {
	uint32_t v = e.ftab[i];
	return v <= e.len ? v : e.eftab[(v ^ BT2G_OFF_MASK) * 2];
}

// Bidirectional range state after one step.
struct BiRange {
	uint32_t t[4], b[4], tp[4], bp[4];
};

// INIT_LOCS + mapBiLFEx / mapLF1 as one step from [top,bot) (mirror start topp).
// Loads one side when both rows share it (initFromTopBot, bt2_idx.h:325-352).
// Returns the number of 64-B sides loaded.
__device__ __forceinline__ int bi_step(const DevEbwt& e, uint32_t top, uint32_t bot, uint32_t topp,
                                       uint32_t t[4], uint32_t b[4], uint32_t tp[4], uint32_t bp[4]) {
	uint32_t st = top / 192u, sb = bot / 192u;
	int loads = sb == st ? 1 : 2;
#ifndef BT2G_LEAN_BISTEP
	// both sides issued before either is consumed: one memory latency per step
	// (the second is the first again when both rows share a side: a hit on the
	// line in flight).  r05w: the split form paid two latencies whenever a
	// wave's lanes had both cases.
	SideData s1, s2;
	load_side(e, st, s1);
	load_side(e, sb, s2);
	occ4(e, s1, top, t);
	occ4(e, s2, bot, b);
#else
	SideData s1;
	load_side(e, st, s1);
	occ4(e, s1, top, t);
	if(sb == st) {
		occ4(e, s1, bot, b);
	} else {
		// second side only after the first is consumed: one SideData live
		uint32_t z;
		asm volatile("v_mov_b32 %0, 0" : "=v"(z) : "v"(t[0]), "v"(t[3]));
		sb += z;
		SideData s2;
		load_side(e, sb, s2);
		occ4(e, s2, bot, b);
	}
#endif
	bp[0] = tp[0] + (b[0] - t[0]);
	tp[1] = bp[0];
	bp[1] = tp[1] + (b[1] - t[1]);
	tp[2] = bp[1];
	bp[2] = tp[2] + (b[2] - t[2]);
	tp[3] = bp[2];
	bp[3] = tp[3] + (b[3] - t[3]);
	return loads;
}

// bi_step without the mirror ranges (a caller that needs few of them derives
// them: mirror top of character j = topp + sum of the range sizes below j)
__device__ __forceinline__ int bi_step_tb(const DevEbwt& e, uint32_t top, uint32_t bot, uint32_t t[4], uint32_t b[4]) {
	const uint32_t st = top / 192u, sb = bot / 192u;
	SideData s1, s2;
	load_side(e, st, s1);
	load_side(e, sb, s2);     // (as bi_step: both issued, then both consumed)
	occ4(e, s1, top, t);
	occ4(e, s2, bot, b);
	return sb == st ? 1 : 2;
}

// ---- the cooperative step: a quad of lanes per walk ------------------------
// north_star: LF mapping "via coalesced occ-table gathers with LDS-staged rank
// blocks".  In the batch server the FM calls carry a round's few hundred reads:
// one lane per walk leaves ~15 waves on 1 024 SIMDs, each issuing ~200 VALU
// instructions of side counting per dependent step (round 5: ~2.2 us per step
// against ~0.6 us for the gather).  Here a side is counted by the four lanes of
// a quad (countBt2Side, bt2_idx.h:1758-1919): lane q loads 16 B of the 64-B
// side -- q = 0..2 the BWT words 4q..4q+3 (rows 64q..64q+63), q = 3 the four
// occurrence counts -- in ONE coalesced 64-B request per quad, counts its four
// words, and the quad sums by DPP (quad_perm) in registers; lane 3's counts
// reach the others the same way.  Every lane of a quad runs the walk's control
// flow on identical values, so the quad never diverges.
struct QuadSide {
	uint32_t w[4];
};

__device__ __forceinline__ void load_quad(const DevEbwt& e, uint32_t side, uint32_t q, QuadSide& s) {
	typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
	typedef const __attribute__((address_space(1))) u32x4 gu32x4;
	const gu32x4* p = (const gu32x4*)(e.sides + (size_t)side * 64u) + q;
	const u32x4 a = *p;
	s.w[0] = a.x; s.w[1] = a.y; s.w[2] = a.z; s.w[3] = a.w;
}

// sum over the lane's quad (quad_perm [1,0,3,2] then [2,3,0,1])
__device__ __forceinline__ uint32_t quad_sum(uint32_t x) {
	x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
	x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);
	return x;
}
// lane 3's value in every lane of the quad (quad_perm [3,3,3,3])
__device__ __forceinline__ uint32_t quad_lane3(uint32_t x) {
	return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xFF, 0xF, 0xF, false);
}

// w[i] of a quad side without a data-dependent register index
__device__ __forceinline__ uint32_t quad_word(const QuadSide& s, uint32_t i) {
	uint32_t x0 = s.w[0], x1 = s.w[1], x2 = s.w[2], x3 = s.w[3];
	asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
	return i == 0 ? x0 : i == 1 ? x1 : i == 2 ? x2 : x3;
}

// this lane's share of the count of `ch` among the side's first charOff rows
// (lane 3, the occurrence counts: 0)
__device__ __forceinline__ uint32_t quad_part1(const QuadSide& s, uint32_t q, uint32_t charOff, int ch) {
	const uint32_t x = (uint32_t)(3 - ch) * 0x55555555u;
	const int rem = q < 3u ? (int)charOff - 64 * (int)q : 0;
	uint32_t n = 0;
#pragma unroll
	for(int k = 0; k < 4; k++) {
		int nk = rem - 16 * k;
		nk = nk < 0 ? 0 : (nk > 16 ? 16 : nk);
		const uint32_t m = nk >= 16 ? 0x55555555u : ((1u << (2 * nk)) - 1u) & 0x55555555u;
		const uint32_t y = s.w[k] ^ x;
		n += __builtin_popcount(y & (y >> 1) & m);
	}
	return n;
}

// countBt2Side for one character, the side in the quad (occ1's quad form)
__device__ __forceinline__ uint32_t quad_occ1(const DevEbwt& e, const QuadSide& s, uint32_t q, uint32_t row, int ch) {
	const uint32_t side = row / 192u, co = row % 192u;
	uint32_t n = quad_sum(quad_part1(s, q, co, ch));
	if(ch == 0 && dollar_before(e, side, co)) n--;
	return n + quad_lane3(quad_word(s, (uint32_t)ch)) + fchr_at(e, ch);
}

// top's count in side s1 and bot's in side s2 for one character: one packed
// quad sum (each share is <= 64)
__device__ __forceinline__ void quad_occ2(const DevEbwt& e, const QuadSide& s1, const QuadSide& s2, uint32_t q,
                                          uint32_t top, uint32_t bot, int ch, uint32_t& nt, uint32_t& nb) {
	const uint32_t st = top / 192u, ct = top % 192u, sb = bot / 192u, cb = bot % 192u;
	const uint32_t p = quad_sum(quad_part1(s1, q, ct, ch) | (quad_part1(s2, q, cb, ch) << 16));
	uint32_t a = p & 0xffffu, b = p >> 16;
	if(ch == 0 && dollar_before(e, st, ct)) a--;
	if(ch == 0 && dollar_before(e, sb, cb)) b--;
	const uint32_t f = fchr_at(e, ch);
	nt = a + quad_lane3(quad_word(s1, (uint32_t)ch)) + f;
	nb = b + quad_lane3(quad_word(s2, (uint32_t)ch)) + f;
}

// character of row charOff of the quad's side (side_rowL's quad form)
__device__ __forceinline__ int quad_rowL(const QuadSide& s, uint32_t q, uint32_t charOff) {
	const uint32_t k = charOff >> 4;                 // the word: lane k >> 2, its word k & 3
	const uint32_t v = ((k >> 2) == q) ? ((quad_word(s, k & 3u) >> (2 * (charOff & 15))) & 3u) + 1u : 0u;
	return (int)quad_sum(v) - 1;
}

// this lane's share of the A, C, G counts among the side's first charOff rows
// (side_counts' quad form; T follows from charOff)
__device__ __forceinline__ void quad_part3(const QuadSide& s, uint32_t q, uint32_t charOff, uint32_t& a, uint32_t& c,
                                           uint32_t& g) {
	const int rem = q < 3u ? (int)charOff - 64 * (int)q : 0;
	a = c = g = 0;
#pragma unroll
	for(int k = 0; k < 4; k++) {
		int nk = rem - 16 * k;
		nk = nk < 0 ? 0 : (nk > 16 ? 16 : nk);
		const uint32_t m = nk >= 16 ? 0x55555555u : ((1u << (2 * nk)) - 1u) & 0x55555555u;
		const uint32_t lo = s.w[k] & 0x55555555u, hi = (s.w[k] >> 1) & 0x55555555u;
		a += __builtin_popcount(~(lo | hi) & m);
		c += __builtin_popcount(lo & ~hi & m);
		g += __builtin_popcount(hi & ~lo & m);
	}
}

// countBt2SideEx of top (its side in s1) and bot (in s2), all four characters
// (bi_step_tb's counting, quad form): the six shares (<= 64 each, sums <= 192)
// packed into two quad sums, the occurrence counts from lane 3
__device__ __forceinline__ void quad_occ4x2(const DevEbwt& e, const QuadSide& s1, const QuadSide& s2, uint32_t q,
                                            uint32_t top, uint32_t bot, uint32_t t[4], uint32_t b[4]) {
	const uint32_t st = top / 192u, ct = top % 192u, sb = bot / 192u, cb = bot % 192u;
	uint32_t a1, c1, g1, a2, c2, g2;
	quad_part3(s1, q, ct, a1, c1, g1);
	quad_part3(s2, q, cb, a2, c2, g2);
	const uint32_t p1 = quad_sum(a1 | (c1 << 8) | (g1 << 16) | (a2 << 24));
	const uint32_t p2 = quad_sum(c2 | (g2 << 8));
	uint32_t A1 = p1 & 0xffu, C1 = (p1 >> 8) & 0xffu, G1 = (p1 >> 16) & 0xffu, A2 = p1 >> 24;
	uint32_t C2 = p2 & 0xffu, G2 = (p2 >> 8) & 0xffu;
	const uint32_t T1 = ct - A1 - C1 - G1, T2 = cb - A2 - C2 - G2;
	if(dollar_before(e, st, ct)) A1--;
	if(dollar_before(e, sb, cb)) A2--;
	t[0] = A1 + quad_lane3(s1.w[0]) + e.fchr[0];
	t[1] = C1 + quad_lane3(s1.w[1]) + e.fchr[1];
	t[2] = G1 + quad_lane3(s1.w[2]) + e.fchr[2];
	t[3] = T1 + quad_lane3(s1.w[3]) + e.fchr[3];
	b[0] = A2 + quad_lane3(s2.w[0]) + e.fchr[0];
	b[1] = C2 + quad_lane3(s2.w[1]) + e.fchr[1];
	b[2] = G2 + quad_lane3(s2.w[2]) + e.fchr[2];
	b[3] = T2 + quad_lane3(s2.w[3]) + e.fchr[3];
}

// bi_step_tb / bi_step in quad form: both sides issued together (lane q's
// 16 B of each), then counted; the mirror ranges as bi_step derives them
__device__ __forceinline__ int quad_bi_step_tb(const DevEbwt& e, uint32_t q, uint32_t top, uint32_t bot, uint32_t t[4],
                                               uint32_t b[4]) {
	const uint32_t st = top / 192u, sb = bot / 192u;
	QuadSide s1, s2;
	load_quad(e, st, q, s1);
	load_quad(e, sb, q, s2);
	quad_occ4x2(e, s1, s2, q, top, bot, t, b);
	return sb == st ? 1 : 2;
}
__device__ __forceinline__ int quad_bi_step(const DevEbwt& e, uint32_t q, uint32_t top, uint32_t bot, uint32_t topp,
                                            uint32_t t[4], uint32_t b[4], uint32_t tp[4], uint32_t bp[4]) {
	const int loads = quad_bi_step_tb(e, q, top, bot, t, b);
	tp[0] = topp;
	bp[0] = tp[0] + (b[0] - t[0]);
	tp[1] = bp[0];
	bp[1] = tp[1] + (b[1] - t[1]);
	tp[2] = bp[1];
	bp[2] = tp[2] + (b[2] - t[2]);
	tp[3] = bp[2];
	bp[3] = tp[3] + (b[3] - t[3]);
	return loads;
}

// A read (or its reverse complement / reversal) as the reference's BTDnaString
// views: patFw (rev=0,cmp=0), patRc (1,1), patFwRev (1,0), patRcRev (0,1).
struct SeqView {
	const uint8_t* p;
	uint32_t len;
	bool rev, cmp;
	__device__ __forceinline__ int operator[](uint32_t i) const {
		int c = p[rev ? len - 1 - i : i];
		return cmp ? (c > 3 ? 4 : 3 - c) : c;
	}
};

// A walk's next read base through a 16-byte register window: the LF loops
// consume one base per step in a fixed direction, so the read row is loaded
// once per 16 steps instead of one byte load per step inside the dependent
// gather chain.  `lo`/`hi` bound the row (windows never cross them: a window
// that would is replaced by single-byte loads).
struct ReadWin {
	const uint8_t* lo;
	const uint8_t* hi;
	uint64_t a = ~0ull;
	uint4 w = make_uint4(0, 0, 0, 0);
	__device__ __forceinline__ int at(const uint8_t* ptr) {
		const uint64_t addr = (uint64_t)ptr, aa = addr & ~15ull;
		if(aa != a) {
			if(aa < (uint64_t)lo || aa + 16u > (uint64_t)hi) return *ptr;
			a = aa;
			w = *(const uint4*)(ptr - (addr & 15u));   // pointer provenance: global, not flat
		}
		const uint32_t di = (uint32_t)(addr >> 2) & 3u;
		uint32_t x0 = w.x, x1 = w.y, x2 = w.z, x3 = w.w;
		asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));   // a select, not a scratch array
		const uint32_t d = di == 0 ? x0 : di == 1 ? x1 : di == 2 ? x2 : x3;
		return (int)((d >> ((addr & 3u) * 8u)) & 0xffu);
	}
};

// SeqView read through a ReadWin (row bounds [lo, hi)).
struct SeqWin {
	SeqView v;
	ReadWin w;
	__device__ __forceinline__ int operator[](uint32_t i) {
		const int c = w.at(v.p + (v.rev ? v.len - 1 - i : i));
		return v.cmp ? (c > 3 ? 4 : 3 - c) : c;
	}
};
