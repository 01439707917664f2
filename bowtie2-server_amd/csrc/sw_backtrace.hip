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
// Memory: 1M lanes each walking their own problem cannot share caches, so a
// step must not touch memory: reportedThrough lives in 8x8 bit tiles of which
// one is held in registers, the read / qualities / reference are read through
// 16-byte windows and the u8 plane through a copy of 4 columns x 16 rows (the
// plane is stored in 16-row blocks, sw_ee_packed.hip), both in the lane's
// region of LDS,
// so a diagonal run reloads every 4 steps and the later, short walks of a
// problem (all near its last rows) mostly hit registers.  Edits are written
// by the first walk (which usually succeeds) and by a replay of any later
// walk that succeeds.
//
// The reference's branch stack (btnstack_) never changes an outcome: every
// popped frame restarts at a cell already marked reportedThrough, so a walk
// that meets a marked cell fails (proved against the reference by
// tests/test_oracle_golden.py::test_sw_backtrace, whose oracle keeps the
// stack, and tests/test_gpu_bt.py).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <atomic>
#include <mutex>
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

// Score plane accessor: KIND 0 = u8 plane, 1 = u16 plane (problem slot,
// 16-row blocks of pcols columns; the systolic fill bottom-aligns the rows in
// its strip stack (pad dead rows on top), the one-problem-per-lane fills
// top-align them).
template <int KIND>
struct Plane {
	const uint8_t* base;   // kinds 0/1: the problem's slot; 2: its matrix
	const uint16_t* mask;  // kinds 0/1: written 16-row blocks per column (null: all)
	uint32_t pcols, ncol, pad;
	int32_t off;      // score = raw - off
	__device__ __forceinline__ size_t idx(uint32_t r, uint32_t c) const {
		const uint32_t rs = pad + r;
		return ((size_t)(rs >> 4) * pcols + c) * 16u + (rs & 15u);
	}
	// unwritten blocks hold cells below minsc: they read as the floor (raw 0)
	__device__ __forceinline__ bool blk(uint32_t r, uint32_t c) const {
		return !mask || ((mask[c] >> ((pad + r) >> 4)) & 1u);
	}
	__device__ __forceinline__ int32_t h(uint32_t r, uint32_t c) const {
		if(KIND == 0) return (blk(r, c) ? (int32_t)base[idx(r, c)] : 0) - off;
		return (blk(r, c) ? (int32_t)((const uint16_t*)base)[idx(r, c)] : 0) - off;
	}
};

}  // namespace

// work counters for the CPU emulation (tests/cpu_emul) and, with
// BT2G_BT_PROF, for a profiling build of the kernel (bt2g_bt_prof_read):
// 0 walks, 1 steps, 2 col_hit u16 block loads, 3 E-scan rounds, 4 candidates,
// 5 dominance tests, 6 replays, 7 hget calls, 8 u8 chunk reloads, 9 tile loads,
// 10 tile write-backs, 11 col_hit u8 block loads, 12 DPs walked; 15: sum over
// waves of 64 x the wave's largest per-lane step count
#ifdef BT2G_BT_COUNT
extern unsigned long long bt_counts[16];
#define BTC(i) (bt_counts[i]++)
#elif defined(BT2G_BT_PROF)
__device__ unsigned long long g_bt_prof[16];
__device__ unsigned int g_bt_wave_max[1u << 16];
__device__ unsigned long long g_bt_wave_t0[1u << 16], g_bt_wave_t1[1u << 16];   // wall_clock64 ticks
#define BTC(i) (pc[i]++)
#else
#define BTC(i) ((void)0)
#endif

// u8 plane columns held in the lane's LDS chunk; LDS dwords per lane (the
// chunk, then the read / quality / reference windows; odd: banks differ by lane)
#ifndef BT_CHUNK
#define BT_CHUNK 4u      // 4: 36.7 ms, 6: 36.8, 8: 39.8 (LDS occupancy)
#endif
#define BT_LDSW ((4u * BT_CHUNK + 12u) | 1u)
#ifndef BT2G_BT_WAVES
#define BT2G_BT_WAVES 4      // with the LDS caches: 3 waves 41.3 ms, 4 (12 B/lane spilled) 36.9, 5 (124 B) 43.8
#endif
#ifndef BT2G_BT_EE_STEPS
#define BT2G_BT_EE_STEPS 0xffffffffu   // end-to-end: a whole walk per iteration (4, 8, 16: same 32 ms)
#endif
// LOCAL: the alignment mode, compile-time (each mode's kernel keeps only its
// own filters and moves); FLAT: the loop shape, flat for local (see below).
// LDSRES (kind-2 end-to-end decision planes, kind-1 local u16 planes): a
// workgroup per problem -- its 64 lanes copy the problem's plane (local: with
// its block masks) into LDS and its mark tiles (reportedThrough; local also the
// FILT_DOMINATED squares) live there too, then lane 0 walks with every plane and
// mark access in LDS.  A batch of a few thousand DPs (the batch driver's rounds)
// is bound by the longest walk chain, one dependent HBM load after another in
// the lane-per-problem kernel (~3 ms per 400-DP call, r04d; local: ~55 walks and
// ~1 200 candidates per DP one after another): LDS latency is an order of
// magnitude lower.  For big batches the lane-per-problem kernel keeps the
// throughput.
// WPF (LDS-resident local only): the wave-parallel candidate filter.  Between
// two walks nothing a filter reads changes (the marks and the dominated squares
// are written by walks alone), so the wave's 64 lanes test the next 64
// candidates at once -- score, FILT_DOMINATED, FILT_START, in the reference's
// order (aligner_sw.cpp nextAlignment; aligner_swsse_loc_i16.cpp:1420-1500) --
// and a ballot finds the first that survives; one lane testing ~1 200
// candidates per DP, one after another, is what it replaces.  The walks
// themselves are then run by all 64 lanes on identical values (the same
// loads, the same stores to the same addresses): no lane leaves the loop, so
// the wave stays converged for the next filter's ballot.
// WPF 2 (the default): the walks themselves in parallel too, as the end-to-end
// workgroup walk does (sw_backtrace_wg.hip).  A walk's path does not depend on
// the marks -- only where it stops does -- and the filters only ever grow (a
// candidate filtered now stays filtered), so:
//   scan: the lanes test the next candidates 64 at a time against the current
//     marks and squares and collect up to 64 survivors, in order;
//   A: lane s walks survivor s without marks, recording its moves (2 bits each)
//     and whether the path itself succeeds (a core diagonal touched, Ns within
//     the ceiling) -- the plane reads and move decisions, in parallel;
//   B: the wave resolves the batch in the reference's order: the candidates
//     between two survivors get their fates at that point (in parallel, as the
//     scan), a survivor is tested again (an earlier walk of the batch may have
//     filtered it) and, if it still stands, its recorded path is replayed
//     against the marks, marking each cell, failing at the first marked one,
//     then its dominance square is set -- what the serial walk does, minus the
//     plane reads;
//   C: the lanes whose walks succeeded walk again writing their edits and
//     alignment records (as a later success is replayed in the serial walk).
template <int KIND, bool LOCAL, bool FLAT = LOCAL, bool LDSRES = false, int WPF = 0>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BT2G_BT_WAVES)))
k_sw_bt(BtArgs A) {
	static_assert(!LDSRES || (KIND == 2 && !LOCAL) || (KIND == 1 && LOCAL),
	              "LDS-resident walks: kind-2 end-to-end or kind-1 local planes");
	static_assert(WPF == 0 || (LDSRES && LOCAL && !FLAT), "the wave-parallel filter: LDS-resident local walks");
	const uint32_t p = LDSRES ? blockIdx.x : blockIdx.x * 64u + threadIdx.x;
	if(p >= A.nprob) return;
#ifdef BT2G_BT_PROF
	uint32_t pc[13] = {0};
	if(threadIdx.x == 0) g_bt_wave_t0[blockIdx.x & 0xffffu] = wall_clock64();
	struct Flush {
		uint32_t* pc;
		__device__ ~Flush() {
			for(int i = 0; i < 13; i++)
				if(pc[i]) atomicAdd(&g_bt_prof[i], (unsigned long long)pc[i]);
			atomicMax(&g_bt_wave_max[blockIdx.x & 0xffffu], pc[1]);
			atomicMax(&g_bt_wave_t1[blockIdx.x & 0xffffu], (unsigned long long)wall_clock64());
		}
	} flush_{pc};
#endif
	const bt2g_sw_result R = A.res[p];
	const bool writer = !LDSRES || threadIdx.x == 0;
	if(!R.aligned || R.ncand <= 0) { if(writer) A.naln[p] = 0; return; }
	if((uint32_t)R.ncand > A.cap) { if(writer) A.naln[p] = -5; return; }   // truncated list: not the reference's
	const bt2g_sw_problem P = A.probs[p];
	const uint32_t nrow = A.lens[P.read], ncol = P.ncol;
	constexpr bool local = LOCAL;
	const int variant = local ? (R.u8succ ? 2 : 3) : (R.u8succ ? 0 : 1);
	Plane<KIND> pl;
	pl.ncol = ncol;
	pl.pcols = A.pcols;
	pl.pad = 0;
	pl.mask = nullptr;
	uint32_t pad = 0;
	const uint8_t* slot = nullptr;
	{
		if(KIND == 0 && variant != 0) { if(writer) A.naln[p] = -4; return; }   // i16 fill, u8-only plane
		const size_t es = KIND == 1 ? 2 : 1;   // kind 2: the u8 plane's layout, 8 B per block column
		// systolic end-to-end: last row at the stack bottom; one-problem-per-lane
		// fills: top-aligned; systolic local: padded rows (round16) at the bottom
		pad = A.plane_top == 1 ? 0u : A.cstride - (A.plane_top == 2 ? ((nrow + 15u) & ~15u) : nrow);
		slot = A.plane + (size_t)p * A.slot;
		pl.base = slot;
		pl.pad = pad;
		if(A.use_mask) pl.mask = (const uint16_t*)(slot + (size_t)A.cstride * A.pcols * es);
		// u8 fill: 0xff + score; i16 end-to-end fill: 0xffff + score (offset-u16
		// domain); local fills: the score itself
		pl.off = variant == 0 ? 0xff : variant == 1 ? 0xffff : 0;
	}
	// SwAligner::initRead / initRef inputs of this problem
	const uint8_t* rd = A.reads + (size_t)P.read * A.stride;
	const uint8_t* qu = A.quals + (size_t)P.read * A.stride;
	const bool fw = P.fw != 0;
	const SwConst& C = A.C;
	uint64_t rs = 0, rlen = 0;
	if(P.win_off < 0) { rs = A.ref_starts[P.refidx]; rlen = A.ref_starts[P.refidx + 1] - rs; }
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
			// stack rows [pad+rlo, pad+rhi] of column c: one 16-B load per row block
			bool hit = false;
#pragma unroll 1
			for(int32_t o0 = ((int32_t)pad + rlo) & ~15; o0 <= (int32_t)pad + rhi; o0 += 16) {
				if(pl.mask && !((pl.mask[c] >> (o0 >> 4)) & 1u)) continue;   // below minsc: no hit
				BTC(11);
				const uint4 v = *(const uint4*)(slot + ((size_t)(o0 >> 4) * A.pcols + c) * 16u);
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
			// u16 plane: the 16 rows of a column block are 32 contiguous bytes
			bool hit = false;
#pragma unroll 1
			for(int32_t o0 = ((int32_t)pad + rlo) & ~15; o0 <= (int32_t)pad + rhi && !hit; o0 += 16) {
				if(pl.mask && !((pl.mask[c] >> (o0 >> 4)) & 1u)) continue;   // all below minsc / zero: no hit
				BTC(2);
				const uint4* q = (const uint4*)(slot + ((size_t)(o0 >> 4) * A.pcols + c) * 32u);
				const uint4 v0 = q[0], v1 = q[1];
				const uint32_t wv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
				for(int b = 0; b < 16; b++) {
					const int32_t r = o0 + b - (int32_t)pad;
					const int32_t val = (int32_t)((wv[b >> 1] >> (16 * (b & 1))) & 0xffffu) - pl.off;
					hit = hit || (r >= rlo && r <= rhi && val == base + (x - r) * step);
				}
			}
			return hit;
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
	// reportedThrough: 8x8-cell bit tiles (one u64 each), one tile cached in
	// registers at a time (a walk stays in a tile for several steps); a tile is
	// valid once written back (one valid bit per tile, cleared here; the current
	// valid word is cached in a register too), so nothing else is ever cleared.
	// (Valid bits in LDS instead: measured slower.)
	uint32_t* marks = A.marks + (size_t)p * A.mslot;
	const uint32_t tcols = A.rwords, trows = A.rrows, vw = (tcols + 31u) / 32u;
	const bt2g_sw_cand* lcl = nullptr;      // (LDSRES local: the candidate list's copy in LDS)
	uint32_t* lpath = nullptr;              // (WPF 2: 64 recorded paths, then the survivors' indices and infos)
	if constexpr(LDSRES) {
		// the plane's 16-row blocks (kind 2: 8 B per block column; kind 1: 32 B, then
		// the columns' block masks) and the marks, in LDS (layout: sw_bt_lds_bytes)
		HIP_DYNAMIC_SHARED(uint4, s_res)
		const uint32_t n16 = sw_bt_lds_plane16(A, KIND);
		const uint4* src = (const uint4*)slot;
		for(uint32_t i = threadIdx.x; i < n16; i += 64u) s_res[i] = src[i];
		uint32_t* lm = (uint32_t*)(s_res + n16);
		for(uint32_t i = threadIdx.x; i < trows * vw; i += 64u) lm[(size_t)trows * tcols * 2u + i] = 0u;
		if(KIND == 1 && A.cands_lds) {
			// local: the sorted candidate list too (~1 200 per DP, most of them only
			// tested against the marks: streamed from HBM one at a time by the walker,
			// each a dependent round trip), after the whole mark slot
			const uint32_t nc = (uint32_t)R.ncand < A.cap ? (uint32_t)R.ncand : A.cap;
			uint32_t* lc = lm + A.mslot;
			const uint32_t* gc = (const uint32_t*)(A.cands + (size_t)p * A.cap);
			for(uint32_t i = threadIdx.x; i < 3u * nc; i += 64u) lc[i] = gc[i];
			lcl = (const bt2g_sw_cand*)lc;
		}
		if(WPF == 2) lpath = lm + A.mslot + (A.cands_lds ? 3u * A.cap : 0u);
		__syncthreads();
		if(WPF == 0 && threadIdx.x != 0) return;
		if(n16) {
			slot = (const uint8_t*)s_res;
			pl.base = slot;
			if(KIND == 1 && A.use_mask) pl.mask = (const uint16_t*)(slot + (size_t)A.cstride * A.pcols * 2u);
		}
		marks = lm;
	}
	uint32_t* valid = marks + (size_t)trows * tcols * 2u;
	for(uint32_t i = 0; i < trows * vw; i++) valid[i] = 0u;
	uint32_t ttr = 0xffffffffu, ttc = 0;
	uint64_t tbits = 0;
	bool tdirty = false;
	uint32_t vidx = 0xffffffffu, vval = 0u;
	bool vdirty = false;
	auto vword = [&](uint32_t i) -> uint32_t& {
		if(i != vidx) {
			// load before the write-back: a wave's loads wait for every older
			// vector-memory op, stores included (vmcnt is in order)
			const uint32_t nv = valid[i];
			if(vdirty) valid[vidx] = vval;
			vdirty = false;
			vidx = i;
			vval = nv;
		}
		return vval;
	};
	auto tile_get = [&](uint32_t r, uint32_t c) {
		const uint32_t tr = r >> 3, tc = c >> 3;
		if(tr == ttr && tc == ttc) return;
		BTC(9);
		// the new tile is loaded first, with (not after) its valid word, and the
		// old one written back after: one round trip, not a store acknowledgement
		// and then a load (vmcnt counts loads and stores in order); an invalid
		// tile's stale bits are dropped
		const uint64_t tl = *(const uint64_t*)(marks + ((size_t)tr * tcols + tc) * 2u);
		if(tdirty) {
			BTC(10);
			*(uint64_t*)(marks + ((size_t)ttr * tcols + ttc) * 2u) = tbits;
			vword(ttr * vw + (ttc >> 5)) |= 1u << (ttc & 31u);
			vdirty = true;
			tdirty = false;
		}
		ttr = tr;
		ttc = tc;
		const bool v = (vword(tr * vw + (tc >> 5)) >> (tc & 31u)) & 1u;
		tbits = v ? tl : 0ull;
	};
	auto tbit = [](uint32_t r, uint32_t c) -> uint64_t { return 1ull << (((r & 7u) << 3) | (c & 7u)); };
	auto rbit = tbit;
	auto marked = [&](uint32_t r, uint32_t c) -> bool {
		tile_get(r, c);
		return (tbits & rbit(r, c)) != 0;
	};
	// 16-byte windows over the read, the qualities and the reference (aligned
	// uint4: a walk moves one row / column at a time); a window that would
	// leave [lo, hi) is not loaded (single byte instead).  Reads and
	// qualities: [buffer start, end of this row's stride); the resident
	// reference is padded by bt2g_open; explicit windows: their own extent.
	// The window bytes and the u8 plane chunk below live in LDS, 29 dwords per
	// lane (odd stride: the 64 lanes' regions start in different banks): LDS
	// reads wait on their own counter, not behind the walk's global loads, and
	// the 40 VGPRs they took are what kept the kernel at 3 waves/SIMD with
	// spills (measured: 2 waves 61 ms, 3 waves 48.8 ms, 4 waves + spills 46.6).
	__shared__ uint32_t s_cache[64u * BT_LDSW];
	uint32_t* const myc = s_cache + threadIdx.x * BT_LDSW;
	uint64_t w_rd = ~0ull, w_q = ~0ull, w_rf = ~0ull;   // address of the window each slot holds
	auto win = [&](uint64_t& Wa, uint32_t k, const uint8_t* ptr, const uint8_t* lo, const uint8_t* hi) -> int {
		const uint64_t addr = (uint64_t)ptr, aa = addr & ~15ull;
		if(aa != Wa) {
			if(aa < (uint64_t)lo || aa + 16u > (uint64_t)hi) return *ptr;
			Wa = aa;
			// through the kernel-argument pointer (global address space), not an
			// integer cast: a flat load would make every later wait a full drain
			const uint4 v = *(const uint4*)(ptr - (addr & 15u));
			uint32_t* d = myc + 4u * BT_CHUNK + 4u * k;
			d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
		}
		return ((const uint8_t*)(myc + 4u * BT_CHUNK + 4u * k))[addr & 15u];
	};
	auto rd_at = [&](uint32_t r) -> int {   // read character of DP row r
		const int raw = win(w_rd, 0u, rd + (fw ? r : nrow - 1 - r), A.reads, rd + A.stride);
		return fw ? raw : (raw > 3 ? 4 : 3 - raw);
	};
	auto q_at = [&](uint32_t r) -> int {
		const int q = win(w_q, 1u, qu + (fw ? r : nrow - 1 - r), A.quals, qu + A.stride) - 33;
		return q < 0 ? 0 : (q > 40 ? 40 : q);
	};
	const uint8_t* wlo = P.win_off >= 0 ? A.windows + P.win_off : A.ref_codes;
	const uint8_t* whi = P.win_off >= 0 ? wlo + ncol + 1 : A.ref_codes + rs + rlen + 16u;
	auto rf_at = [&](uint32_t c) -> int {   // reference mask of column c (aligner_sw.cpp:171-253)
		if(P.win_off >= 0) return win(w_rf, 2u, wlo + c, wlo, whi);
		const int64_t o = P.refl + (int64_t)c;
		if(o < 0 || (uint64_t)o >= rlen) return 16;
		const int code = win(w_rf, 2u, A.ref_codes + rs + (uint64_t)o, wlo, whi);
		return code > 3 ? 16 : 1 << code;
	};
	// H of a cell; the u8 plane goes through a copy of BT_CHUNK columns x 16
	// rows in the lane's LDS region (column cc0 + u at dwords 4u..4u+3)
	uint32_t cb = 0xffffffffu, cc0 = 0;
	auto hget = [&](uint32_t r, uint32_t c) -> int32_t {
		BTC(7);
		if(KIND != 0) return pl.h(r, c);   // u16 planes: direct (a chunk cache costs occupancy)
		const uint32_t rsx = pad + r, b = rsx >> 4;
		if(b != cb || c < cc0 || c > cc0 + (BT_CHUNK - 1u)) {
			BTC(8);
			cb = b;
			// the walk moves left: the chunk ends at column c
			cc0 = c >= BT_CHUNK - 1u ? c - (BT_CHUNK - 1u) : 0u;
			if(cc0 + BT_CHUNK > A.pcols) cc0 = A.pcols >= BT_CHUNK ? A.pcols - BT_CHUNK : 0u;
			const uint4* qp = (const uint4*)(slot + ((size_t)b * A.pcols + cc0) * 16u);
			// chunks and their block masks in one round trip, dead blocks zeroed after
			const uint4 z = make_uint4(0, 0, 0, 0);
			uint4 ch[BT_CHUNK];
#pragma unroll
			for(uint32_t u = 0; u < BT_CHUNK; u++) ch[u] = cc0 + u < A.pcols ? qp[u] : z;
			if(pl.mask) {
				// the columns' block masks from one or two aligned 16-B loads (8 masks each)
				const uint32_t ma = cc0 & ~7u, sh = cc0 & 7u;
				const uint4 lo = *(const uint4*)(pl.mask + ma);
				const uint4 hi = sh + BT_CHUNK > 8u && ma + 8u < A.pcols ? *(const uint4*)(pl.mask + ma + 8u)
				                                                         : make_uint4(0u, 0u, 0u, 0u);
				uint32_t mw[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};   // two masks per word
				asm volatile("" : "+v"(mw[0]), "+v"(mw[1]), "+v"(mw[2]), "+v"(mw[3]), "+v"(mw[4]), "+v"(mw[5]),
				             "+v"(mw[6]), "+v"(mw[7]));
#pragma unroll
				for(uint32_t u = 0; u < BT_CHUNK; u++) {
					const uint32_t jw = sh + u;                       // column cc0 + u = ma + jw
					uint32_t w = mw[0];
#pragma unroll
					for(uint32_t q = 1; q < 8; q++) w = (jw >> 1) == q ? mw[q] : w;
					const uint32_t m = cc0 + u < A.pcols ? (w >> ((jw & 1u) * 16u)) & 0xffffu : 0u;
					if(!((m >> b) & 1u)) ch[u] = z;
				}
			}
#pragma unroll
			for(uint32_t u = 0; u < BT_CHUNK; u++) {
				myc[4u * u] = ch[u].x; myc[4u * u + 1u] = ch[u].y; myc[4u * u + 2u] = ch[u].z; myc[4u * u + 3u] = ch[u].w;
			}
		}
		return (int32_t)((const uint8_t*)myc)[(c - cc0) * 16u + (rsx & 15u)] - pl.off;
	};
	// KIND 2: the decision nibbles (sw_ee_packed.hip DEC) through a copy of
	// BT_DCH columns x 16 rows (8 B per column) in the lane's LDS region, loaded
	// in the walk step together with its reportedThrough tile (one round trip)
	constexpr uint32_t BT_DCH = 2u * BT_CHUNK;
	uint32_t db = 0xffffffffu, dc0 = 0;
	const uint32_t ncand = (uint32_t)R.ncand < A.cap ? (uint32_t)R.ncand : A.cap;
	const bt2g_sw_cand* cl = lcl ? lcl : A.cands + (size_t)p * A.cap;
	// local mode, FILT_DOMINATED (aligner_sw.cpp nextAlignment): a candidate
	// within SQ rows and SQ columns of one already walked is skipped.  Each
	// walked candidate sets its (2SQ+1)^2 square in a second set of 8x8 bit
	// tiles, so the test is one bit, not a scan of the walked list.
	uint32_t SQ = nrow >> 4;
	if(SQ == 0) SQ = 1;
	uint32_t* dmarks = marks + A.mdom;
	const uint32_t dtcols = A.mwords, dtrows = A.mrows, dvw = (dtcols + 31u) / 32u;
	uint32_t* dvalid = dmarks + (size_t)dtrows * dtcols * 2u;
	if(local)
		for(uint32_t i = 0; i < dtrows * dvw; i++) dvalid[i] = 0u;
	auto dom_test = [&](uint32_t r, uint32_t c) -> bool {
		const uint32_t tr = r >> 3, tc = c >> 3;
		if(!((dvalid[tr * dvw + (tc >> 5)] >> (tc & 31u)) & 1u)) return false;
		return (*(const uint64_t*)(dmarks + ((size_t)tr * dtcols + tc) * 2u) & tbit(r, c)) != 0;
	};
	auto dom_add = [&](uint32_t r, uint32_t c) {
		const uint32_t r0 = r > SQ ? r - SQ : 0u, c0 = c > SQ ? c - SQ : 0u;
		uint32_t r1 = r + SQ, c1 = c + SQ;
		r1 = r1 < dtrows * 8u - 1u ? r1 : dtrows * 8u - 1u;
		c1 = c1 < dtcols * 8u - 1u ? c1 : dtcols * 8u - 1u;
		for(uint32_t tr = r0 >> 3; tr <= r1 >> 3; tr++) {
			// bytes (tile rows) inside [r0, r1], one bit each
			const uint32_t lo = tr * 8u > r0 ? 0u : r0 & 7u, hi = tr * 8u + 7u < r1 ? 7u : r1 & 7u;
			const uint64_t rows = (~0ull >> (8u * (7u - hi))) & (~0ull << (8u * lo)) & 0x0101010101010101ull;
			for(uint32_t tc = c0 >> 3; tc <= c1 >> 3; tc++) {
				const uint32_t cl0 = tc * 8u > c0 ? 0u : c0 & 7u, ch = tc * 8u + 7u < c1 ? 7u : c1 & 7u;
				const uint64_t cols = (0xffull >> (7u - ch)) & (0xffull << cl0);
				uint64_t* t = (uint64_t*)(dmarks + ((size_t)tr * dtcols + tc) * 2u);
				uint32_t& vwd = dvalid[tr * dvw + (tc >> 5)];
				const uint32_t vb = 1u << (tc & 31u);
				*t = (vwd & vb ? *t : 0ull) | rows * cols;
				vwd |= vb;
			}
		}
	};
	int32_t nal = 0;
	bool first = true;
	BTC(12);
	// FLAT (local mode): the candidate loop and the walks run as ONE loop: an
	// iteration either filters a candidate or takes one walk step, so a lane
	// never waits for the longest walk of its wave at every candidate (nested
	// loops reconverge at each walk's end; flat, a wave runs for the longest
	// lane's total): 3.8x faster with local's ~1,200 candidates and 55 uneven
	// walks per DP.  End-to-end (48 similar candidates) keeps each walk in an
	// inner loop, whose iterations are cheaper (measured 31.5 vs 34.4 ms).
	// A walk: one backtrace from (row0, col0); wmark: set/check reportedThrough
	// (off when replaying a successful walk to emit its edits -- the path does
	// not depend on the marks); wemit: write the edits (walk order) to ed.
	struct Walk {
		bool ok, core;
		uint32_t row, col, ned;
		int32_t score, ns, gaps;
	};
	Walk w{true, false, 0u, 0u, 0u, 0, 0, 0};
	bool walking = false, wmark = false, wemit = false, replay = false;
	uint32_t row = 0, col = 0, row0 = 0, col0 = 0;
	int32_t cur = 0;
	int st = ST_H;
	bt2g_edit* ed = A.edits;
	auto push = [&](uint32_t pos, int type, int chr, int qchr) {
		if(wemit && w.ned < A.maxedit) ed[w.ned] = bt2g_edit{pos, (uint8_t)type, (uint8_t)chr, (uint8_t)qchr, 0};
		w.ned++;
	};
	auto start_walk = [&](bool mark, bool emit) {
		w = Walk{true, false, row0, col0, 0u, 0, 0, 0};
		row = row0; col = col0; st = ST_H;
		wmark = mark; wemit = emit;
		walking = true;
		BTC(0);
	};
	// the alignment record of a walk that succeeded (its edits at ed): candidate
	// `cand`, alignment k of the problem
	auto record_aln = [&](uint32_t cand, uint32_t k) {
		const uint32_t trimBeg = w.row, trimEnd = nrow - row0 - 1;
		// res.reverse(), AlnRes::setShape trim shift, invertEdits for !fw
		// (aligner_result.cpp:101-117, 822-828; edit.cpp:50-78)
		const uint32_t ned = w.ned, nst = ned < A.maxedit ? ned : A.maxedit;
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
		for(uint32_t c = w.col; c <= col0; c++) refns += rf_at(c) > 15;
		bt2g_sw_aln a;
		a.cand = (int32_t)cand; a.score = w.score; a.off = (int32_t)w.col; a.ns = w.ns; a.gaps = w.gaps;
		a.refns = refns; a.nedit = (int32_t)ned;
		a.trim5p = (int32_t)(fw ? trimBeg : trimEnd); a.trim3p = (int32_t)(fw ? trimEnd : trimBeg);
		a.pad = 0;
		A.alns[(size_t)p * A.maxaln + (size_t)k] = a;
	};
	uint32_t ndone = 0, wq0 = 0, wq1 = 0, wq2 = 0, wq3 = 0;   // walked candidates: row << 16 | col
#ifdef BT2G_BT_WQ8
	uint32_t wq4 = 0, wq5 = 0, wq6 = 0, wq7 = 0;
#endif
	uint32_t ci = 0;
	// the next candidate is loaded one ahead (its load overlaps the current walk)
	bt2g_sw_cand nxt_cd = ncand ? cl[0] : bt2g_sw_cand{0, 0, 0};
	int32_t cscore = 0;
	// WPF 2: the batch (survivor s's candidate index sidx[s], its path's moves and
	// success winfo[s]), this lane's path words, its survivor and alignment index
	const uint32_t PW = ((A.rrows * 8u + A.pcols) >> 4) + 1u;      // >= (rows + cols) / 16 + 1
	uint32_t* const sidx = lpath + 64u * PW;
	uint32_t* const winfo = sidx + 64u;
	uint32_t* const mypath = lpath + threadIdx.x * PW;
	int wphase = 0;                          // 0 between batches, 1 speculative walks (A), 2 emitting walks (C)
	bool wdone = false, wrec = false, my_succ = false;
	uint32_t nsurv = 0, bend = 0, my_cj = 0, my_kk = 0, nmv = 0, pacc = 0;
	// the walker's cached reportedThrough tile and valid word back to LDS, where
	// the other lanes read them
	auto flush_tile = [&]() {
		if(tdirty) {
			*(uint64_t*)(marks + ((size_t)ttr * tcols + ttc) * 2u) = tbits;
			vword(ttr * vw + (ttc >> 5)) |= 1u << (ttc & 31u);
			vdirty = true;
			tdirty = false;
		}
		if(vdirty) { valid[vidx] = vval; vdirty = false; }
		__syncthreads();
	};
	// a candidate's filter at this point, from LDS (after flush_tile): 5 score,
	// 4 dominated, 3 start marked, 0 none -- in the reference's order
	auto filt_lds = [&](const bt2g_sw_cand& c) -> int8_t {
		const uint32_t r = (uint32_t)c.row, cc = (uint32_t)c.col;
		const uint32_t tr = r >> 3, tc = cc >> 3;
		const bool mk = ((valid[tr * vw + (tc >> 5)] >> (tc & 31u)) & 1u) &&
		                (*(const uint64_t*)(marks + ((size_t)tr * tcols + tc) * 2u) & rbit(r, cc));
		if(c.score < P.minsc) return 5;                      // BT_CAND_FATE_FILT_SCORE
		if(!A.fates && dom_test(r, cc)) return 4;            // BT_CAND_FATE_FILT_DOMINATED
		if(mk) return 3;                                     // BT_CAND_FATE_FILT_START
		if(A.fates && dom_test(r, cc)) return 4;
		return 0;
	};
	while(true) {
		if constexpr(WPF == 2) {
			if(__ballot(walking) == 0ull) {
				if(wphase == 1) {
					// ---- B: the batch in the reference's order -------------------------
					__syncthreads();                     // (the lanes' paths and infos)
					uint32_t pos = ci;
					my_succ = false;
					for(uint32_t sv = 0; sv <= nsurv; sv++) {
						if(nal >= (int32_t)A.maxaln) { wdone = true; break; }
						const uint32_t cj = sv < nsurv ? sidx[sv] : bend;
						// the candidates up to the survivor: filtered at the scan, so filtered
						// now; their fates as of this point
						flush_tile();
						if(A.fates)
							for(uint32_t x = pos; x < cj; x += 64u) {
								const uint32_t j = x + threadIdx.x;
								if(j < cj) A.fates[(size_t)p * A.cap + j] = filt_lds(cl[j]);
							}
						pos = cj;
						if(sv == nsurv) break;
						const bt2g_sw_cand c = cl[cj];
						int8_t fate = filt_lds(c);
						if(!fate) {
							// its walk: the recorded path against the marks
							const uint32_t info = winfo[sv], nm = info >> 1;
							const uint32_t* pp = lpath + sv * PW;
							uint32_t r = (uint32_t)c.row, cc = (uint32_t)c.col;
							bool ok = true;
							for(uint32_t i = 0;; i++) {
								tile_get(r, cc);
								const uint64_t bt = rbit(r, cc);
								if(tbits & bt) { ok = false; break; }
								tbits |= bt;
								tdirty = true;
								if(i == nm) break;
								const uint32_t code = (pp[i >> 4] >> (2u * (i & 15u))) & 3u;
								// (a walk never moves past row or column 0: a guard, not a case)
								if((code != 2u && r == 0u) || (code != 1u && cc == 0u)) { ok = false; break; }
								if(code != 2u) r--;          // diagonal or up
								if(code != 1u) cc--;         // diagonal or left
							}
							dom_add((uint32_t)c.row, (uint32_t)c.col);
							if(ok && (info & 1u)) {
								if(threadIdx.x == sv) { my_succ = true; my_kk = (uint32_t)nal; }
								nal++;
								fate = 1;                        // BT_CAND_FATE_SUCCEEDED
							} else {
								fate = 2;                        // BT_CAND_FATE_FAILED
							}
						}
						if(A.fates && threadIdx.x == 0) A.fates[(size_t)p * A.cap + cj] = fate;
						pos = cj + 1u;
					}
					ci = pos;
					// ---- C: the successes walked again, writing their edits ------------
					if(my_succ) {
						const bt2g_sw_cand c = cl[my_cj];
						ed = A.edits + ((size_t)p * A.maxaln + (size_t)my_kk) * A.maxedit;
						row0 = (uint32_t)c.row; col0 = (uint32_t)c.col; cur = c.score;
						wrec = false;
						start_walk(false, true);
					}
					wphase = 2;
				} else {
					// ---- the next batch: up to 64 survivors of the filters as they stand --
					if(wdone || ci >= ncand || nal >= (int32_t)A.maxaln) break;
					flush_tile();
					nsurv = 0;
					bool full = false;
					uint32_t wpos = ci;
					while(nsurv < 64u && wpos < ncand) {
						const uint32_t j = wpos + threadIdx.x;
						const bool sv = j < ncand && filt_lds(cl[j]) == 0;
						const uint64_t m = __ballot(sv);
						const uint32_t nm = (uint32_t)__popcll(m), take = nm < 64u - nsurv ? nm : 64u - nsurv;
						const uint32_t rk = (uint32_t)__popcll(m & ((1ull << threadIdx.x) - 1ull));
						if(sv && rk < take) sidx[nsurv + rk] = j;
						nsurv += take;
						wpos += 64u;
						if(take < nm) { full = true; break; }
					}
					__syncthreads();
					// (a full batch ends at its last survivor; else at the scanned end)
					bend = full ? sidx[63] + 1u : (wpos < ncand ? wpos : ncand);
					if(threadIdx.x < nsurv) {
						my_cj = sidx[threadIdx.x];
						const bt2g_sw_cand c = cl[my_cj];
						row0 = (uint32_t)c.row; col0 = (uint32_t)c.col; cur = c.score;
						wrec = true;
						nmv = 0;
						pacc = 0;
						start_walk(false, false);
					}
					wphase = 1;
				}
			}
			if(!walking) continue;
		}
		if(WPF == 1 && !walking) {
			if(ci >= ncand || nal >= (int32_t)A.maxaln) break;
			// the cached reportedThrough tile and valid word back to LDS, where the
			// other lanes read them
			if(tdirty) {
				*(uint64_t*)(marks + ((size_t)ttr * tcols + ttc) * 2u) = tbits;
				vword(ttr * vw + (ttc >> 5)) |= 1u << (ttc & 31u);
				vdirty = true;
				tdirty = false;
			}
			if(vdirty) { valid[vidx] = vval; vdirty = false; }
			__syncthreads();
			for(;;) {
				const uint32_t j = ci + threadIdx.x;
				int8_t fj = 0;
				if(j < ncand) {
					const bt2g_sw_cand c = cl[j];
					const uint32_t r = (uint32_t)c.row, cc = (uint32_t)c.col;
					const uint32_t tr = r >> 3, tc = cc >> 3;
					const bool mk = ((valid[tr * vw + (tc >> 5)] >> (tc & 31u)) & 1u) &&
					                (*(const uint64_t*)(marks + ((size_t)tr * tcols + tc) * 2u) & rbit(r, cc));
					if(c.score < P.minsc) fj = 5;                      // BT_CAND_FATE_FILT_SCORE
					else if(!A.fates && dom_test(r, cc)) fj = 4;        // BT_CAND_FATE_FILT_DOMINATED
					else if(mk) fj = 3;                                 // BT_CAND_FATE_FILT_START
					else if(A.fates && dom_test(r, cc)) fj = 4;
				}
				const uint64_t stop = __ballot(j >= ncand || fj == 0);
				const uint32_t f = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;
				if(A.fates && threadIdx.x < f) A.fates[(size_t)p * A.cap + j] = fj;
				ci += f;
				if(stop) break;
			}
			if(ci >= ncand) break;
			const bt2g_sw_cand cd = cl[ci];
			ed = A.edits + ((size_t)p * A.maxaln + (size_t)nal) * A.maxedit;
			row0 = (uint32_t)cd.row; col0 = (uint32_t)cd.col; cur = cd.score; cscore = cd.score;
			replay = false;
			start_walk(true, first);
		} else if(!walking) {
			if(ci >= ncand || nal >= (int32_t)A.maxaln) break;
			const bt2g_sw_cand cd = nxt_cd;
			nxt_cd = cl[ci + 1u < ncand ? ci + 1u : ci];
			int8_t fate = 0;
			BTC(4);
			// Local mode: most candidates (~95 % at 150 bp) lie within SQ of a walked
			// one.  The squares of the first and the last three walked candidates
			// are tested in registers first (exact: a hit is a dominated candidate);
			// without a fates array the dominance test also runs before the start
			// mark (either filter only skips the candidate; fates alone tell them apart).
			const uint32_t cr = (uint32_t)cd.row, cc = (uint32_t)cd.col;
			auto near = [&](uint32_t wv) {
				const uint32_t wr = wv >> 16, wc = wv & 0xffffu;
				return (wr > cr ? wr - cr : cr - wr) <= SQ && (wc > cc ? wc - cc : cc - wc) <= SQ;
			};
#ifdef BT2G_BT_WQ8
			const bool dom_reg = local && ndone > 0 && (near(wq0) || near(wq1) || near(wq2) || near(wq3) ||
			                                            near(wq4) || near(wq5) || near(wq6) || near(wq7));
#else
			const bool dom_reg = local && ndone > 0 && (near(wq0) || near(wq1) || near(wq2) || near(wq3));
#endif
			const bool dom_first = local && !A.fates && (dom_reg || (BTC(5), dom_test(cr, cc)));
			if(cd.score < P.minsc) {
				fate = 5;                                   // BT_CAND_FATE_FILT_SCORE
			} else if(dom_first) {
				fate = 4;                                   // BT_CAND_FATE_FILT_DOMINATED
			} else if((local || cr + (uint32_t)gb < nrow) && marked(cr, cc)) {
				// (end-to-end starts in the bottom barrier rows are never marked: see walk)
				fate = 3;                                   // BT_CAND_FATE_FILT_START
			} else if(local && A.fates && (dom_reg || (BTC(5), dom_test(cr, cc)))) {
				fate = 4;                                   // BT_CAND_FATE_FILT_DOMINATED
			}
			if(fate) {
				if(A.fates) A.fates[(size_t)p * A.cap + ci] = fate;
				ci++;
				continue;
			}
			// the first walk writes its edits as it goes (it usually succeeds);
			// a later walk that succeeds is walked again to write them.  The
			// candidate's score is its cell's H.
			ed = A.edits + ((size_t)p * A.maxaln + (size_t)nal) * A.maxedit;
			row0 = cr; col0 = cc; cur = cd.score; cscore = cd.score;
			replay = false;
			start_walk(true, first);
		}
		// ---- one walk step (FLAT), or up to BT2G_BT_EE_STEPS steps ---------------
		bool ended = false;
		uint32_t ks = 0;
		do {
		uint32_t nb2 = 0;   // KIND 2: the cell's decision nibble
		if constexpr(KIND == 2) {
			// Gap-barrier rows allow diagonal moves only (E and F are vetoed there):
			// no nibble.  The bottom ones are never marked (see below).  Every load
			// of the step (tile, its valid word, the nibble chunk and its block
			// masks) is issued before any store or use: one round trip per step.
			const bool bbar = row + (uint32_t)gb >= nrow, bar = bbar || row < (uint32_t)gb;
			const bool mk = wmark && !bbar;
			const uint32_t tr = row >> 3, tc = col >> 3;
			const bool tnew = mk && (tr != ttr || tc != ttc);
			const uint32_t vi = tr * vw + (tc >> 5);
			const bool vnew = tnew && vi != vidx;
			uint64_t tl = 0;
			uint32_t nv = 0;
			if(tnew) tl = *(const uint64_t*)(marks + ((size_t)tr * tcols + tc) * 2u);
			if(vnew) nv = valid[vi];
			const bool needd = (st != ST_H || !bar) && row > 0;
			const uint32_t rsx = pad + row, b = rsx >> 4;
			const bool dnew = needd && (b != db || col < dc0 || col > dc0 + (BT_DCH - 1u));
			// (leaving the inner loop at the first step that needs a load, so that
			// a wave's loads go out together: measured slower, 28.2 vs 25.1 ms)
			BTC(1);
			uint4 ch[BT_DCH / 2u];
			uint32_t ndc0 = dc0;
			if(dnew) {
				// the walk moves left: the chunk ends near column col (even start: 16-B loads)
				ndc0 = (col >= BT_DCH - 2u ? col - (BT_DCH - 2u) : 0u) & ~1u;
				if(ndc0 + BT_DCH > A.pcols) ndc0 = A.pcols >= BT_DCH ? A.pcols - BT_DCH : 0u;
				const uint4* qp = (const uint4*)(slot + ((size_t)b * A.pcols + ndc0) * 8u);
#pragma unroll
				for(uint32_t u = 0; u < BT_DCH / 2u; u++) ch[u] = ndc0 + 2u * u < A.pcols ? qp[u] : make_uint4(0u, 0u, 0u, 0u);
			}
			if(tnew) {
				BTC(9);
				// the cached valid word is the old tile's (it was switched in with it)
				if(tdirty) {
					BTC(10);
					*(uint64_t*)(marks + ((size_t)ttr * tcols + ttc) * 2u) = tbits;
					vval |= 1u << (ttc & 31u);
					vdirty = true;
					tdirty = false;
				}
				if(vnew) {
					if(vdirty) valid[vidx] = vval;
					vidx = vi;
					vval = nv;
					vdirty = false;
				}
				ttr = tr;
				ttc = tc;
				tbits = ((vval >> (tc & 31u)) & 1u) ? tl : 0ull;
			}
			if(dnew) {
				BTC(8);
				db = b;
				dc0 = ndc0;
				// (no block masks: a walked cell is >= the candidate's score >= minsc,
				// so its block was written; unwritten columns of a chunk are never read)
#pragma unroll
				for(uint32_t u = 0; u < BT_DCH / 2u; u++) {
					myc[4u * u] = ch[u].x; myc[4u * u + 1u] = ch[u].y; myc[4u * u + 2u] = ch[u].z; myc[4u * u + 3u] = ch[u].w;
				}
			}
			if(mk) {
				// reportedThrough (aligner_swsse_ee_u8.cpp:1331-1336, 1556)
				const uint64_t bt = rbit(row, col);
				if(tbits & bt) { w.ok = false; ended = true; }
				else { tbits |= bt; tdirty = true; }
			}
			if(needd) {
				// row 8w+i of the block: word w of the column's 8 bytes, bits 0-2 of
				// the decision at 3(7-i)+2, +1, +0, bit 3 at 24+7-i (sw_ee_packed.hip)
				const uint32_t rr = rsx & 15u, i7 = 7u - (rr & 7u);
				const uint32_t wd = myc[(col - dc0) * 2u + (rr >> 3)];
				const uint32_t t = wd >> (3u * i7);
				nb2 = ((t >> 2) & 1u) | ((t & 2u)) | ((t & 1u) << 2) | (((wd >> (24u + i7)) & 1u) << 3);
			}
		} else {
			BTC(1);
			// end-to-end: every candidate starts in the last row and the bottom
			// gap-barrier rows allow only diagonal moves, so walks there stay on
			// their own diagonals and can neither meet nor be met: no marks
			const bool bottom_bar = !local && row + (uint32_t)gb >= nrow;
			if(wmark && !bottom_bar) {
				// reportedThrough (aligner_swsse_ee_u8.cpp:1331-1336, 1556)
				tile_get(row, col);
				const uint64_t bt = rbit(row, col);
				if(tbits & bt) { w.ok = false; ended = true; }
				else { tbits |= bt; tdirty = true; }
			}
		}
		if(!ended) {
			const int32_t dg = (int32_t)col - (int32_t)row + triml;
			w.core = w.core || (dg >= 0 && dg >= corel && dg <= corer);
			if(row == 0) ended = true;
		}
		if(!ended) {
			int rc = 0, m = 0, q = 0;
			int mv = -1;   // 0 diag, 1 ref open, 2 ref extend, 3 read open, 4 read extend
			int32_t nxt = 0;
			if constexpr(KIND == 2) {
			// the fill's decision (sw_ee_packed.hip DEC): bit 0 not diag, bit 1 not
			// from F, bit 2 F not opened from H(up), bit 3 E not opened from H(left)
			const uint32_t nb = nb2;
			if(st == ST_H) {
				if(!gaps_ok(row)) { if(col > 0) mv = 0; }   // barrier rows: diagonal only
				else if(!(nb & 1u) && col > 0) mv = 0;
				else if(gaps_ok(row)) {
					if(!(nb & 2u)) mv = (nb & 4u) ? 2 : 1;
					else if(col > 0) mv = (nb & 8u) ? 4 : 3;
				}
				if(mv < 0) ended = true;   // empty cell: the alignment starts here
			} else if(st == ST_E) {
				if(col == 0) ended = true;   // unreachable: E(row, 0) is the floor
				mv = (nb & 8u) ? 4 : 3;
			} else {
				mv = (nb & 4u) ? 2 : 1;
			}
			// characters only for a walk that writes its edits (a failing walk
			// needs none; a later walk that succeeds is replayed with them)
			if(!ended && wemit) { rc = rd_at(row); m = rf_at(col); if(mv == 0) q = q_at(row); }
			} else {
			rc = rd_at(row); m = rf_at(col); q = q_at(row);
			// in gap-barrier rows H is the diagonal term itself when above the
			// floor (E and F are the floor there): H(up-left) = cur - score, no load
			const bool derive = st == ST_H && !gaps_ok(row) && (!local || cur > 0);
			// one plane read site for the neighbour the state tests first:
			// H -> up-left, E -> left, F -> up
			const bool need1 = st == ST_H ? (col > 0 && !derive) : (st == ST_E ? col > 0 : true);
			const int32_t v1 = need1 ? hget(st == ST_E ? row : row - 1, st == ST_F ? col : col - 1) : 0;
			if(st == ST_H) {
				const bool wantd = col > 0;
				const int32_t hul = !wantd ? 0 : derive ? cur - sdiag(rc, m, q) : v1;
				// diag equality; local mode also wants H(up-left) > 0 (floorsc)
				const bool deq = wantd && cur == hul + sdiag(rc, m, q);
				if(deq && okv(hul)) { mv = 0; nxt = hul; }
				if(mv < 0 && gaps_ok(row)) {
					int32_t hu = 0, hl = 0;
#pragma unroll 1
					for(int t = 0; t < 2; t++) {          // one read site for up and left
						if(t == 1 && col == 0) break;
						const int32_t v = hget(t == 0 ? row - 1 : row, t == 0 ? col : col - 1);
						if(t == 0) hu = v; else hl = v;
					}
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
							// eight independent loads in flight per round (only existence matters)
							bool found = false;
#pragma unroll 1
							for(int32_t k0 = 1; !found && cc - k0 >= 0 && cur + rdge + rdgo + (k0 - 1) * rdge <= hm;
							    k0 += 8) {
								int32_t v[8];
								BTC(3);
#pragma unroll
								for(int u = 0; u < 8; u++)
									v[u] = cc - (k0 + u) >= 0 ? pl.h(row, (uint32_t)(cc - (k0 + u))) : -1;
#pragma unroll
								for(int u = 0; u < 8; u++) {
									const int32_t need = cur + rdge + rdgo + (k0 + u - 1) * rdge;
									found = found || (cc - (k0 + u) >= 0 && need <= hm && v[u] == need);
								}
							}
							if(found) { mv = 4; nxt = cur + rdge; }
						}
					}
				}
				if(mv < 0) ended = true;   // empty cell: the alignment starts here
			} else if(st == ST_E) {
				if(col == 0) ended = true;   // unreachable: E(row, 0) is the floor
				const int32_t hl = v1;
				if(okv(hl) && hl - rdgo == cur) { mv = 3; nxt = hl; }
				else { mv = 4; nxt = cur + rdge; }
			} else {
				const int32_t hu = v1;
				if(okv(hu) && hu - rfgo == cur) { mv = 1; nxt = hu; }
				else { mv = 2; nxt = cur + rfge; }
			}
			}   // KIND
			if(!ended) {
				if(mv == 0) {
					const int mt = (m >= 16 || rc > 3) ? -1 : ((m >> rc) & 1);
					if(mt != 1) {
						push(row, 3, mask2dna(m), "ACGTN"[rc]);
						w.score -= (rc > 3 || m > 15) ? C.npen : C.mmpen[q];
					} else {
						w.score += C.match;
					}
					if(mt == -1) w.ns++;
					row--; col--;
					st = ST_H;
				} else if(mv <= 2) {
					push(row, 2, '-', "ACGTN"[rc]);
					w.score -= mv == 1 ? rfgo : rfge;
					st = mv == 1 ? ST_H : ST_F;
					row--; w.gaps++;
				} else {
					push(row + 1, 1, mask2dna(m), '-');
					w.score -= mv == 3 ? rdgo : rdge;
					st = mv == 3 ? ST_H : ST_E;
					col--; w.gaps++;
				}
				cur = nxt;
				if(WPF == 2 && wrec) {
					// the move, for the replay against the marks: 0 diagonal, 1 up, 2 left
					pacc |= (uint32_t)(mv == 0 ? 0 : mv <= 2 ? 1 : 2) << (2u * (nmv & 15u));
					if((++nmv & 15u) == 0u) { mypath[(nmv >> 4) - 1u] = pacc; pacc = 0u; }
				}
			}
		}
		} while(!ended && ++ks < (FLAT ? 1u : (uint32_t)BT2G_BT_EE_STEPS));
		if(!ended) continue;
		// ---- the walk ended --------------------------------------------------
		w.row = row;
		w.col = col;
		if(w.ok && !w.core) w.ok = false;            // must touch a core diagonal
		if(w.ok && (KIND != 2 || wemit)) {
			const int rc = rd_at(row), m = rf_at(col);
			const int mt = (m >= 16 || rc > 3) ? -1 : ((m >> rc) & 1);
			if(mt != 1) {
				push(row, 3, mask2dna(m), "ACGTN"[rc]);
				w.score -= (rc > 3 || m > 15) ? C.npen : C.mmpen[q_at(row)];
			} else {
				w.score += C.match;
			}
			if(mt == -1) w.ns++;
			if(w.ns > nceil) w.ok = false;
		}
		if constexpr(WPF == 2) {
			walking = false;
			if(wphase == 1) {
				// A: the path and whether it succeeds where no mark stops it
				if(nmv & 15u) mypath[nmv >> 4] = pacc;
				winfo[threadIdx.x] = (nmv << 1) | (w.ok ? 1u : 0u);
			} else if(w.ok) {
				record_aln(my_cj, my_kk);           // C (the same path: it succeeds)
			}
			continue;
		}
		if(w.ok && !first && !replay) {
			// a later walk that succeeded: walk it again, unmarked, writing its edits
			BTC(6);
			replay = true;
			cur = cscore;
			start_walk(false, true);
			continue;
		}
		walking = false;
		first = false;
		int8_t fate;
		if(local) {
			dom_add(row0, col0);
			// register copies: the first walked candidate stays, the others rotate
			const uint32_t wv = (row0 << 16) | col0;
#ifdef BT2G_BT_WQ8
			if(ndone == 0) wq0 = wq1 = wq2 = wq3 = wq4 = wq5 = wq6 = wq7 = wv;
			else { wq7 = wq6; wq6 = wq5; wq5 = wq4; wq4 = wq3; wq3 = wq2; wq2 = wq1; wq1 = wv; }
#else
			if(ndone == 0) wq0 = wq1 = wq2 = wq3 = wv;
			else { wq3 = wq2; wq2 = wq1; wq1 = wv; }
#endif
			ndone++;
		}
		if(w.ok) {
			record_aln(ci, (uint32_t)nal);
			nal++;
			fate = 1;                                       // BT_CAND_FATE_SUCCEEDED
		} else {
			fate = 2;                                       // BT_CAND_FATE_FAILED
		}
		if(A.fates) A.fates[(size_t)p * A.cap + ci] = fate;
		ci++;
	}
	A.naln[p] = nal;
}

#ifdef BT2G_BT_PROF
// profiling build: counters since the last call (then cleared); out[15] is the
// wave-divergence sum described above
// per-wave start / end (wall_clock64 ticks, 100 MHz) of the last launch, for
// waves 0..n-1 (n <= 65536)
extern "C" int bt2g_bt_prof_waves(unsigned long long* t0, unsigned long long* t1, unsigned int* steps, uint32_t n) {
	if(n > (1u << 16)) return -1;
	if(hipMemcpyFromSymbol(t0, HIP_SYMBOL(g_bt_wave_t0), sizeof(unsigned long long) * n) != hipSuccess) return -1;
	if(hipMemcpyFromSymbol(t1, HIP_SYMBOL(g_bt_wave_t1), sizeof(unsigned long long) * n) != hipSuccess) return -1;
	if(hipMemcpyFromSymbol(steps, HIP_SYMBOL(g_bt_wave_max), sizeof(unsigned int) * n) != hipSuccess) return -1;
	return 0;
}

extern "C" int bt2g_bt_prof_read(unsigned long long* out) {
	unsigned long long h[16];
	static unsigned int w[1u << 16];
	if(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_bt_prof), sizeof(h)) != hipSuccess) return -1;
	if(hipMemcpyFromSymbol(w, HIP_SYMBOL(g_bt_wave_max), sizeof(w)) != hipSuccess) return -1;
	h[15] = 0;
	for(uint32_t i = 0; i < (1u << 16); i++) h[15] += 64ull * w[i];
	for(int i = 0; i < 16; i++) out[i] = h[i];
	const unsigned long long z[16] = {0};
	(void)hipMemcpyToSymbol(HIP_SYMBOL(g_bt_prof), z, sizeof(z));
	static const unsigned int zw[1u << 16] = {0};
	(void)hipMemcpyToSymbol(HIP_SYMBOL(g_bt_wave_max), zw, sizeof(zw));
	static const unsigned long long zt[1u << 16] = {0};
	(void)hipMemcpyToSymbol(HIP_SYMBOL(g_bt_wave_t1), zt, sizeof(zt));
	return 0;
}
#endif

// LDS bytes of an LDS-resident walk (k_sw_bt<., ., ., true>): the plane's
// blocks (sw_bt_lds_plane16: local with the block masks) and the problem's
// whole mark slot (reportedThrough tiles with their valid words; local also the
// FILT_DOMINATED tiles, A.mdom words in)
static uint32_t bt_lds_bytes(const BtArgs& a, int kind) {
	const uint64_t plane = (uint64_t)sw_bt_lds_plane16(a, kind) * 16u;
	const uint64_t marks = (kind == 1 ? a.mslot
	                                  : (uint64_t)a.rrows * a.rwords * 2u + (uint64_t)a.rrows * ((a.rwords + 31u) / 32u)) * 4u;
	// (local: the candidate list, but for the wave-parallel filter, which reads it
	// from HBM 64 candidates at a time: ~24 KB less per workgroup at cap 2 048)
	const uint64_t cands = kind == 1 && a.cands_lds ? (uint64_t)a.cap * sizeof(bt2g_sw_cand) : 0u;
	// (the parallel walks: 64 recorded paths of (rows + cols) / 16 + 1 words, the
	// survivors' indices and infos)
	const uint64_t paths = kind == 1 && a.wpf == 2 ? (64ull * (((a.rrows * 8u + a.pcols) >> 4) + 1u) + 128u) * 4u : 0u;
	const uint64_t n = plane + marks + cands + paths;
	return n > 0xffffffffull ? 0xffffffffu : (uint32_t)n;
}

// The dynamic LDS the LDS-resident local walk may take on a device: its opt-in
// (up to the CU's 160 KiB less the kernel's static LDS, the lanes' window cache),
// made per device at context open (bt2g_open_mem), as for the workgroup walk.
static std::atomic<uint32_t> g_loc_lds_lim[64];
static std::mutex g_loc_lds_mu;
static constexpr uint32_t BT_STATIC_LDS = 64u * BT_LDSW * 4u;

void sw_bt_lds_init(int dev) {
	if(dev < 0 || dev >= 64) return;
	std::lock_guard<std::mutex> lk(g_loc_lds_mu);
	if(g_loc_lds_lim[dev].load()) return;
	uint32_t lim = 65536u - BT_STATIC_LDS;
	int v = 0;
	if(hipDeviceGetAttribute(&v, hipDeviceAttributeSharedMemPerBlockOptin, dev) == hipSuccess && v > 65536 &&
	   hipFuncSetAttribute((const void*)k_sw_bt<1, true, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
	                       v - (int)BT_STATIC_LDS) == hipSuccess &&
	   hipFuncSetAttribute((const void*)k_sw_bt<1, true, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
	                       v - (int)BT_STATIC_LDS) == hipSuccess &&
	   hipFuncSetAttribute((const void*)k_sw_bt<1, true, false, true, 1>,
	                       hipFuncAttributeMaxDynamicSharedMemorySize, v - (int)BT_STATIC_LDS) == hipSuccess &&
	   hipFuncSetAttribute((const void*)k_sw_bt<1, true, false, true, 2>,
	                       hipFuncAttributeMaxDynamicSharedMemorySize, v - (int)BT_STATIC_LDS) == hipSuccess)
		lim = (uint32_t)v - BT_STATIC_LDS;
	else
		(void)hipGetLastError();
	g_loc_lds_lim[dev].store(lim);
}

static uint32_t bt_loc_lds_limit() {
	const char* e = getenv("BT2G_BT_WG_LDS");           // (0: no opt-in, as for the workgroup walk)
	if(e && *e == '0') return 65536u - BT_STATIC_LDS;
	int dev = 0;
	if(hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 65536u - BT_STATIC_LDS;
	const uint32_t v = g_loc_lds_lim[dev].load();
	return v ? v : 65536u - BT_STATIC_LDS;
}

// batches up to $BT2G_BT_LDS_MAX problems (default 65536; 0: never) walk
// LDS-resident (the workgroup walk, else the one-walker kernel when a problem's
// plane and marks fit in 64 KB)
// (read at every launch: the parity tests run one batch both ways)
static uint32_t bt_lds_max() {
	const char* e = getenv("BT2G_BT_LDS_MAX");
	// (the workgroup walk at any batch-server size: r04x, 76 DP calls over 8 192
	// problems took the lane-per-DP walk at ~11 ms each against ~0.3 ms)
	return e ? (uint32_t)atol(e) : 65536u;
}

void launch_sw_bt(int kind, const BtArgs& a, hipStream_t st) {
	if(a.nprob == 0) return;
	if(kind == 2 && !a.local && !a.queue && a.nprob <= bt_lds_max()) {
		// $BT2G_BT_WG=0: the LDS-resident one-walker kernel instead of the
		// parallel-candidate one (sw_backtrace_wg.hip)
		const char* e = getenv("BT2G_BT_WG");
		if(!(e && *e == '0')) {
			const uint32_t lw = sw_bt_wg_lds(a);
			if(lw <= sw_bt_wg_lds_limit()) {
				launch_sw_bt_wg(a, lw, st);
				return;
			}
		}
		const uint32_t lds = bt_lds_bytes(a, 2);
		if(lds <= 65536u - BT_STATIC_LDS) {
			hipLaunchKernelGGL((k_sw_bt<2, false, false, true>), dim3(a.nprob), dim3(64), lds, st, a);
			return;
		}
	}
	if(kind == 1 && a.local && !a.queue && a.nprob <= bt_lds_max()) {
		// $BT2G_BT_LOC_LDS: 0 local walks stay lane-per-problem; "plane" the u16 plane
		// in LDS too (one workgroup per CU at ~80 KB); default: the marks only, the
		// plane read in place (just written by the fill: mostly cache hits), so a CU
		// holds many walkers
		const char* e = getenv("BT2G_BT_LOC_LDS");
		if(!(e && *e == '0')) {
			BtArgs b = a;
			b.lds_marks_only = !(e && !strcmp(e, "plane"));
			// (one walker per workgroup: no lanes to diverge, so a walk runs to its
			// end in the inner loop -- the flat loop's one body per step is the
			// union of the filter and the walk; $BT2G_BT_LOC_FLAT=1 keeps it)
			// $BT2G_BT_LOC_WPF (read at every launch: A/B in one process): 0 the
			// candidates filtered and walked by the walker alone, one at a time (round
			// 5); 1 filtered by the wave, walked one at a time; default: filtered and
			// walked by the wave (the recorded paths take LDS: a batch whose paths do
			// not fit takes form 1)
			const char* fl = getenv("BT2G_BT_LOC_FLAT");
			const char* wp = getenv("BT2G_BT_LOC_WPF");
			// $BT2G_BT_LOC_CANDS=lds: the wave-parallel forms' candidates copied to LDS
			// as the serial filter's are (one dependent load per candidate there)
			const char* cl = getenv("BT2G_BT_LOC_CANDS");
			for(int form = (fl && *fl == '1') ? 0 : (wp && *wp == '0') ? 1 : (wp && *wp == '1') ? 2 : 3; form >= 0;) {
				b.wpf = form == 3 ? 2 : form == 2 ? 1 : 0;
				b.cands_lds = form < 2 || (cl && !strcmp(cl, "lds"));
				const uint32_t lds = bt_lds_bytes(b, 1);
				if(lds > bt_loc_lds_limit()) {
					if(form == 3) { form = 2; continue; }
					break;
				}
				if(form == 0) hipLaunchKernelGGL((k_sw_bt<1, true, true, true>), dim3(b.nprob), dim3(64), lds, st, b);
				else if(form == 1) hipLaunchKernelGGL((k_sw_bt<1, true, false, true>), dim3(b.nprob), dim3(64), lds, st, b);
				else if(form == 2) hipLaunchKernelGGL((k_sw_bt<1, true, false, true, 1>), dim3(b.nprob), dim3(64), lds, st, b);
				else hipLaunchKernelGGL((k_sw_bt<1, true, false, true, 2>), dim3(b.nprob), dim3(64), lds, st, b);
				return;
			}
		}
	}
	const dim3 grid((a.nprob + 63u) / 64u), block(64);
	if(a.local) {
		// local fills leave a u16 plane
		hipLaunchKernelGGL((k_sw_bt<1, true>), grid, block, 0, st, a);
	} else {
		if(kind == 0) hipLaunchKernelGGL((k_sw_bt<0, false>), grid, block, 0, st, a);
		else if(kind == 2) hipLaunchKernelGGL((k_sw_bt<2, false>), grid, block, 0, st, a);
		else hipLaunchKernelGGL((k_sw_bt<1, false>), grid, block, 0, st, a);
	}
}
