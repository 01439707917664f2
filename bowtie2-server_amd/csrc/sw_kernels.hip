// sw_kernels.hip -- Smith-Waterman fill + candidate gather, gfx950.
//
// Inter-task layout: one lane owns one DP problem (a wave64 = 64 problems in
// lock-step); the problem is swept in horizontal strips of R rows kept in
// VGPRs, column by column, so the vertical (F) dependency stays inside a lane
// and no cross-lane traffic is needed.  Between strips only the last row's H/F
// and the running column maxima cross, through a per-problem boundary buffer
// laid out [column][lane] so each column step is one coalesced 256-B access per
// wave.  This is integer VALU work (no MFMA): ~12 ops per cell.
//
// Values are computed in the native domain of the reference kernel selected
// by SwAligner::align (aligner_sw.cpp:500-620) and saturate exactly like the
// SSE2 ops they restate:
//   V=0 end-to-end u8  : 0xff = score 0, subs_epu8 floors at 0  (aligner_swsse_ee_u8.cpp:775-1146)
//   V=1 end-to-end i16 : 0x7fff = score 0, signed saturation    (aligner_swsse_ee_i16.cpp:780-1200)
//   V=2 local u8       : score + bias, adds/subs_epu8            (aligner_swsse_loc_u8.cpp:927-1336)
//   V=3 local i16      : 0x8000 = score 0, signed saturation     (aligner_swsse_loc_i16.cpp:938-1367)
// The striped kernels' lazy-F loop converges to the plain Gotoh recurrence, so
// the H/E/F of every real cell equal the reference's.  Local mode also
// reproduces the striped padding rows (rows nrow..ceil(nrow/W)*W-1, W = 16 for
// u8 and 8 for i16, score 0, no gap barrier) because their H feeds the column
// maximum (vcolmax) that drives lastsolcol_/colstop_.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "bt2g_kernels.h"

namespace {

constexpr int R = 16;           // rows per strip held in registers

template <int V> struct Dom;
template <> struct Dom<0> {   // EE u8
	static constexpr int LO = 0, ROW0 = 255;
	static __device__ __forceinline__ int sub(int a, int b) { int r = a - b; return r < 0 ? 0 : r; }
	static __device__ __forceinline__ int diag(int h, int s, int) { return sub(h, -s); }
	static constexpr int W = 16;
};
template <> struct Dom<1> {   // EE i16
	static constexpr int LO = -32768, ROW0 = 32767;
	static __device__ __forceinline__ int sat(int x) { return x < -32768 ? -32768 : (x > 32767 ? 32767 : x); }
	static __device__ __forceinline__ int sub(int a, int b) { return sat(a - b); }
	static __device__ __forceinline__ int diag(int h, int s, int) { return sat(h + s); }
	static constexpr int W = 8;
};
template <> struct Dom<2> {   // local u8
	static constexpr int LO = 0, ROW0 = 0;
	static __device__ __forceinline__ int sub(int a, int b) { int r = a - b; return r < 0 ? 0 : r; }
	static __device__ __forceinline__ int diag(int h, int s, int bias) {
		int t = h + s + bias; t = t > 255 ? 255 : t;
		return sub(t, bias);
	}
	static constexpr int W = 16;
};
template <> struct Dom<3> {   // local i16
	static constexpr int LO = -32768, ROW0 = -32768;
	static __device__ __forceinline__ int sat(int x) { return x < -32768 ? -32768 : (x > 32767 ? 32767 : x); }
	static __device__ __forceinline__ int sub(int a, int b) { return sat(a - b); }
	static __device__ __forceinline__ int diag(int h, int s, int) { return sat(h + s); }
	static constexpr int W = 8;
};

__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }

__device__ __forceinline__ int firsts5(int m) {
	return (m & 1) ? 0 : (m & 2) ? 1 : (m & 4) ? 2 : (m & 8) ? 3 : 4;
}

struct ProbView {
	const uint8_t* rd;
	const uint8_t* qu;
	uint32_t len;
	bool fw;
	// rd_ = fw ? rdfw_ : rdrc_, qu_ = fw ? qufw_ : qurc_ (aligner_sw.cpp:98-99)
	__device__ __forceinline__ int base(uint32_t r) const {
		if(fw) return rd[r];
		int c = rd[len - 1 - r];
		return c > 3 ? 4 : 3 - c;
	}
	__device__ __forceinline__ int qual(uint32_t r) const { return fw ? qu[r] : qu[len - 1 - r]; }
};

// Reference mask of column j (0..ncol): explicit window, or the resident
// reference with N outside [0, reflen) (aligner_sw.cpp:171-253).
__device__ __forceinline__ int refmask(const bt2g_sw_problem& p, const uint8_t* windows, const uint8_t* ref_codes,
                                       const uint64_t* ref_starts, uint32_t j) {
	if(p.win_off >= 0) return windows[p.win_off + j];
	int64_t o = p.refl + (int64_t)j;
	uint64_t s = ref_starts[p.refidx], e = ref_starts[p.refidx + 1];
	int c = (o < 0 || (uint64_t)o >= e - s) ? 4 : ref_codes[s + (uint64_t)o];
	return 1 << c;
}

__device__ __forceinline__ int score_of(const SwConst& C, int rdc, int refc, int q) {
	if(rdc > 3 || refc > 3) return -C.npen;
	if(rdc == refc) return C.match;
	return -C.mmpen[q < 0 ? 0 : (q > 40 ? 40 : q)];
}

}  // namespace

// One lane per problem.  `list` (optional) selects which problems to run and
// `list_n` (device) how many; otherwise problems 0..nprob-1.
template <int V>
__global__ void __launch_bounds__(64)
k_sw_fill(const bt2g_sw_problem* __restrict__ probs, uint32_t nprob, const uint32_t* __restrict__ list,
          const uint32_t* __restrict__ list_n, const uint8_t* __restrict__ reads, const uint8_t* __restrict__ quals,
          uint32_t stride, const uint32_t* __restrict__ lens, const uint8_t* __restrict__ windows,
          const uint8_t* __restrict__ ref_codes, const uint64_t* __restrict__ ref_starts, SwConst C,
          uint32_t cap, uint32_t* __restrict__ bnd, uint32_t bnd_cols, bt2g_sw_result* __restrict__ res,
          bt2g_sw_cand* __restrict__ cands, int16_t* __restrict__ mat, const uint64_t* __restrict__ mat_off,
          uint32_t* __restrict__ sat_list, uint32_t* __restrict__ sat_n, PlaneOut po) {
	using D = Dom<V>;
	const uint32_t lane = threadIdx.x;
	const uint32_t gi = blockIdx.x * 64u + lane;
	const uint32_t cnt = list ? *list_n : nprob;
	if(gi >= cnt) return;
	const uint32_t pi = list ? list[gi] : gi;
	const bt2g_sw_problem p = probs[pi];
	const uint32_t nrow = lens[p.read];
	const uint32_t ncol = p.ncol;
	if(ncol > bnd_cols || ncol == 0 || nrow == 0) {
		bt2g_sw_result bad{};
		bad.flag = -3;
		bad.best = INT32_MIN;
		res[pi] = bad;
		return;
	}
	ProbView pv{reads + (size_t)p.read * stride, quals + (size_t)p.read * stride, nrow, p.fw != 0};
	constexpr bool LOCAL = V >= 2;
	const uint32_t nrowp = LOCAL ? ((nrow + D::W - 1) / D::W) * D::W : nrow;
	// boundary buffer: [col][64 lanes] of {H:16 | F:16} and [col][64] column max
	uint32_t* bhf = bnd + (size_t)blockIdx.x * bnd_cols * 64u * 2u;
	uint32_t* bcm = bhf + (size_t)bnd_cols * 64u;
	int bias = 0;
	if(V == 2) {
		for(uint32_t r = 0; r < nrow; r++) {
			int rdc = pv.base(r), q = pv.qual(r) - 33;
			for(int c = 0; c < 5; c++) {
				int s = score_of(C, rdc, c, q);
				if(s < 0 && s < bias) bias = s;
			}
		}
		bias = -bias;
	}
	const int64_t minsc = p.minsc;
	const int64_t matchsc = C.match;
	uint64_t minrow = 0;
	if(LOCAL) minrow = (((uint64_t)minsc + (uint64_t)matchsc - 1) / (uint64_t)matchsc) - 1;
	bt2g_sw_cand* mycands = cands + (size_t)pi * cap;
	uint32_t ncand = 0;
	int16_t* mymat = mat ? mat + mat_off[pi] : nullptr;
	int lrmax = D::LO;   // EE: max of the last real row

	for(uint32_t s0 = 0; s0 < nrowp; s0 += R) {
		int rdc[R], mmq[R];
		uint32_t barmask = 0, realmask = 0;
#pragma unroll
		for(int k = 0; k < R; k++) {
			uint32_t r = s0 + k;
			bool real = r < nrow;
			rdc[k] = real ? pv.base(r) : 0;
			int q = real ? pv.qual(r) - 33 : 0;
			mmq[k] = C.mmpen[q < 0 ? 0 : (q > 40 ? 40 : q)];
			if(real) realmask |= 1u << k;
			if(real && ((int)r < C.gapbar || (int)(nrow - r - 1) < C.gapbar)) barmask |= 1u << k;
		}
		int E[R], Hl[R];
#pragma unroll
		for(int k = 0; k < R; k++) { E[k] = D::LO; Hl[k] = D::LO; }
		int hb_prev = D::LO;              // H of row s0-1 at column j-1
		int refm_next = refmask(p, windows, ref_codes, ref_starts, 0);
		for(uint32_t j = 0; j < ncol; j++) {
			const int refm = refm_next;
			refm_next = refmask(p, windows, ref_codes, ref_starts, j + 1);
			const int refc = firsts5(refm);
			int hup, fup, diag0;
			if(s0 == 0) {
				hup = D::LO; fup = D::LO; diag0 = D::ROW0;
			} else {
				uint32_t w = bhf[(size_t)j * 64u + lane];
				hup = (int)(int16_t)(w >> 16);
				fup = (int)(int16_t)(w & 0xffff);
				diag0 = hb_prev;
				hb_prev = hup;
			}
			int cm = D::LO;
			int fprev = fup, hprev = hup, diag = diag0;
			uint32_t hs[R / 2];                    // the strip's H as u16 pairs (score plane)
#pragma unroll
			for(int k = 0; k < R / 2; k++) hs[k] = 0;
#pragma unroll
			for(int k = 0; k < R; k++) {
				const uint32_t r = s0 + k;
				if(r < nrowp) {
					const bool real = (realmask >> k) & 1u;
					const bool bar = (barmask >> k) & 1u;
					int s;
					if(real) s = (rdc[k] > 3 || refc > 3) ? -C.npen : (rdc[k] == refc ? C.match : -mmq[k]);
					else s = 0;
					int f;
					if(r == 0) f = (V == 0 || V == 2) ? 0 : -32768;
					else if(bar) f = (V == 0 || V == 2) ? 0 : -32768;
					else f = imax(D::sub(fprev, C.rfge), D::sub(hprev, C.rfgo));
					int h = imax(imax(D::diag(diag, s, bias), E[k]), f);
					int eold = E[k];
					E[k] = imax(D::sub(E[k], C.rdge), bar ? D::LO : D::sub(h, C.rdgo));
					diag = Hl[k];
					Hl[k] = h;
					fprev = f; hprev = h;
					cm = imax(cm, h);
					hs[k / 2] |= (uint32_t)(uint16_t)(h + ((V & 1) ? 0x8000 : 0)) << (16 * (k & 1));
					if(mymat && real) {
						size_t o = ((size_t)r * ncol + j) * 3;
						mymat[o] = (int16_t)h; mymat[o + 1] = (int16_t)eold; mymat[o + 2] = (int16_t)f;
					}
					if(!LOCAL) {
						if(r == nrow - 1) {
							lrmax = imax(lrmax, h);
							int64_t sc = (int64_t)h - (V == 0 ? 0xff : 0x7fff);
							if(sc >= minsc) {
								if(ncand < cap) mycands[ncand] = bt2g_sw_cand{(int32_t)r, (int32_t)j, (int32_t)sc};
								ncand++;
							}
						}
					} else if(real && (uint64_t)r >= minrow) {
						int64_t sc = (int64_t)h + (V == 2 ? 0 : 0x8000);
						if(sc >= minsc) {
							bool m = (refm & (1 << rdc[k])) != 0;
							bool ms = false;
							if(r < nrow - 1) {
								int rn = (k + 1 < R) ? rdc[(k + 1) & (R - 1)] : pv.base(r + 1);
								ms = (refm_next & (1 << rn)) != 0;
							}
							if(m && !ms) {
								if(ncand < cap) mycands[ncand] = bt2g_sw_cand{(int32_t)r, (int32_t)j, (int32_t)sc};
								ncand++;
							}
						}
					}
				}
			}
			if(po.plane) {
				// score plane (sw_backtrace.hip), rows top-aligned: this strip is block s0/16
				uint4* d = (uint4*)(po.plane + (size_t)pi * po.hslot + (((size_t)(s0 / R) * po.pcols + j) * R) * 2u);
				d[0] = make_uint4(hs[0], hs[1], hs[2], hs[3]);
				d[1] = make_uint4(hs[4], hs[5], hs[6], hs[7]);
			}
			// hand the strip's last row and the column max to the next strip
			bhf[(size_t)j * 64u + lane] = ((uint32_t)(uint16_t)(int16_t)hprev << 16) | (uint16_t)(int16_t)fprev;
			if(LOCAL) {
				int prev = s0 == 0 ? D::LO : (int)(int16_t)bcm[(size_t)j * 64u + lane];
				bcm[(size_t)j * 64u + lane] = (uint32_t)(uint16_t)(int16_t)imax(prev, cm);
			}
		}
	}

	bt2g_sw_result out;
	out.u8succ = out.i16succ = 0;
	out.flag = 0;
	int64_t best;
	if(!LOCAL) {
		int64_t score = (int64_t)lrmax - (V == 0 ? 0xff : 0x7fff);
		if(score < minsc) { out.flag = -1; best = score; }
		else if(lrmax == D::LO) { out.flag = -2; best = INT64_MIN; }
		else { out.flag = 0; best = score; }
		out.colstop = (int32_t)ncol - 1;
		out.lastsolcol = 0;
		if(V == 0) out.u8succ = out.flag == 0; else out.i16succ = out.flag == 0;
	} else {
		// column bail / lastsolcol_ / saturation exactly as the per-column code
		int vmax = D::LO;
		int64_t colstop = ncol, lastsol = 0;
		bool sat = false;
		for(uint32_t j = 0; j < ncol; j++) {
			int c = (int)(int16_t)bcm[(size_t)j * 64u + lane];
			vmax = imax(vmax, c);
			int64_t sc = (int64_t)c + (V == 2 ? 0 : 0x8000);
			if(V == 2 && c + bias >= 255) { sat = true; break; }
			if(sc < minsc) {
				int64_t ncolleft = (int64_t)ncol - j - 1;
				if(sc + ncolleft * matchsc < minsc) { colstop = j + 1; break; }
			} else {
				lastsol = j;
			}
		}
		if(V == 2) {
			if(sat || vmax + bias >= 255) { out.flag = -2; best = INT64_MIN; }
			else if(vmax == 0 || vmax < minsc) { out.flag = -1; best = vmax; }
			else { out.flag = 0; best = vmax; }
			out.u8succ = out.flag == 0;
		} else {
			if(vmax == -32768) { out.flag = -1; best = INT64_MIN; }
			else {
				int64_t score = (int64_t)vmax + 0x8000;
				if(score < minsc) { out.flag = -1; best = score; }
				else if(vmax == 32767) { out.flag = -2; best = INT64_MIN; }
				else { out.flag = 0; best = score; }
			}
			out.i16succ = out.flag == 0;
		}
		out.colstop = (int32_t)colstop;
		out.lastsolcol = (int32_t)lastsol;
		// gather only columns <= lastsolcol_ (aligner_swsse_loc_*.cpp gather loop).
		// On overflow (ncand > cap) the count is left as is and the caller
		// reports BT2G_ERR_OVERFLOW: the stored subset is not the reference's.
		if(ncand <= cap) {
			uint32_t k = 0;
			for(uint32_t i = 0; i < ncand; i++) {
				bt2g_sw_cand c = mycands[i];
				if(c.col <= lastsol) mycands[k++] = c;
			}
			ncand = k;
		}
	}
	const bool fail = best == INT64_MIN || best < minsc;
	out.best = best == INT64_MIN ? INT32_MIN : (int32_t)best;
	if(fail) ncand = 0;
	out.ncand = (int32_t)ncand;
	out.aligned = (!fail && ncand > 0) ? 1 : 0;
	if(V == 2 && out.flag == -2) {
		// local u8 saturated: SwAligner::align falls back to the i16 fill
		uint32_t slot = atomicAdd(sat_n, 1u);
		sat_list[slot] = pi;
	}
	res[pi] = out;
}

// Split problems by the fill SwAligner::align picks first (aligner_sw.cpp:516-586):
// end-to-end u8 iff enable8 && minsc >= -254, else i16; local u8 iff enable8.
// One atomic per wave and list (ballot + prefix popcount), not per problem.
__global__ void __launch_bounds__(256)
k_sw_partition(const bt2g_sw_problem* __restrict__ probs, uint32_t nprob, int local, int enable8,
               uint32_t* __restrict__ list8, uint32_t* __restrict__ n8, uint32_t* __restrict__ list16,
               uint32_t* __restrict__ n16) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t lane = threadIdx.x & 63u;
	const bool valid = i < nprob;
	const bool u8 = valid && enable8 && (local || probs[i].minsc >= -254);
	const bool w16 = valid && !u8;
	const uint64_t m8 = __ballot(u8), m16 = __ballot(w16);
	uint32_t b8 = 0, b16 = 0;
	if(lane == 0) {
		if(m8) b8 = atomicAdd(n8, (uint32_t)__popcll(m8));
		if(m16) b16 = atomicAdd(n16, (uint32_t)__popcll(m16));
	}
	b8 = __shfl(b8, 0);
	b16 = __shfl(b16, 0);
	const uint64_t below = (1ull << lane) - 1ull;
	if(u8) list8[b8 + (uint32_t)__popcll(m8 & below)] = i;
	if(w16) list16[b16 + (uint32_t)__popcll(m16 & below)] = i;
}

void launch_sw_partition(const bt2g_sw_problem* probs, uint32_t nprob, int local, int enable8, uint32_t* list8,
                         uint32_t* n8, uint32_t* list16, uint32_t* n16, hipStream_t st) {
	if(nprob == 0) return;
	hipLaunchKernelGGL(k_sw_partition, dim3((nprob + 255) / 256), dim3(256), 0, st, probs, nprob, local, enable8,
	                   list8, n8, list16, n16);
}

// Sort each problem's candidates by the DpBtCandidate total order
// (score desc, row desc, col desc; aligner_sw_nuc.h:149-157) on packed 64-bit
// keys: key = ~((score ^ sign) << 32 | row << 16 | col), ascending.
__device__ __forceinline__ unsigned long long cand_key(const bt2g_sw_cand& c) {
	return ~(((unsigned long long)(uint32_t)(c.score ^ 0x80000000) << 32) |
	         ((unsigned long long)(uint32_t)c.row << 16) | (uint32_t)c.col);
}
__device__ __forceinline__ bt2g_sw_cand cand_of(unsigned long long key) {
	const unsigned long long k = ~key;
	bt2g_sw_cand o;
	o.score = (int32_t)((uint32_t)(k >> 32) ^ 0x80000000u);
	o.row = (int32_t)((k >> 16) & 0xffff);
	o.col = (int32_t)(k & 0xffff);
	return o;
}

// One wave per problem: up to 64 candidates sorted in registers by a bitonic
// network over lanes (shuffles); larger lists are queued for k_sort_big.
__global__ void __launch_bounds__(256)
k_sort_small(const bt2g_sw_result* __restrict__ res, bt2g_sw_cand* __restrict__ cands, uint32_t nprob,
             uint32_t cap, uint32_t* __restrict__ big, uint32_t* __restrict__ nbig) {
	const uint32_t pi = blockIdx.x * 4u + (threadIdx.x >> 6);
	const uint32_t lane = threadIdx.x & 63u;
	if(pi >= nprob) return;
	const int n0 = res[pi].ncand;
	const uint32_t n = (uint32_t)(n0 < 0 ? 0 : (n0 > (int)cap ? cap : n0));
	if(n <= 1) return;
	if(n > 64) {
		if(lane == 0) big[atomicAdd(nbig, 1u)] = pi;
		return;
	}
	bt2g_sw_cand* c = cands + (size_t)pi * cap;
	unsigned long long key = lane < n ? cand_key(c[lane]) : ~0ull;
	for(uint32_t size = 2; size <= 64; size <<= 1) {
		for(uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
			const unsigned long long other = __shfl_xor(key, (int)stride);
			const bool up = (lane & size) == 0 || size == 64;
			const bool lower = (lane & stride) == 0;
			const unsigned long long lo = key < other ? key : other, hi = key < other ? other : key;
			key = (lower == up) ? lo : hi;
		}
	}
	if(lane < n) c[lane] = cand_of(key);
}

// Lists longer than 64: one workgroup per queued problem (grid-stride over
// the queue, whose length is only known on the device).  Lists of >= 128 whose
// scores span <= SORT_BUCKETS values (local mode: ~1200 candidates over a few
// hundred scores) are counting-sorted by score (histogram, scan, scatter into
// buckets, then each bucket -- a few candidates -- insertion-sorted by the full
// key by one thread); others go through an LDS bitonic network.
constexpr uint32_t SORT_BUCKETS = 2048;
__global__ void __launch_bounds__(256)
k_sort_big(const bt2g_sw_result* __restrict__ res, bt2g_sw_cand* __restrict__ cands, uint32_t cap, uint32_t P2max,
           int counting, const uint32_t* __restrict__ big, const uint32_t* __restrict__ nbig) {
	extern __shared__ __attribute__((aligned(16))) unsigned long long keys[];
	unsigned long long* tmp = keys + P2max;
	uint32_t* start = (uint32_t*)(tmp + P2max);
	uint32_t* cur = start + SORT_BUCKETS;
	__shared__ uint32_t part[256];
	__shared__ int smin, smax;
	const uint32_t tid = threadIdx.x;
	const uint32_t nq = *nbig;
	for(uint32_t qi = blockIdx.x; qi < nq; qi += gridDim.x) {
		const uint32_t pi = big[qi];
		const int n0 = res[pi].ncand;
		const uint32_t n = (uint32_t)(n0 > (int)cap ? cap : n0);
		uint32_t P2 = 1;
		while(P2 < n) P2 <<= 1;
		bt2g_sw_cand* c = cands + (size_t)pi * cap;
		if(tid == 0) { smin = INT32_MAX; smax = INT32_MIN; }
		__syncthreads();
		int lmin = INT32_MAX, lmax = INT32_MIN;
		for(uint32_t i = tid; i < P2; i += blockDim.x) {
			if(i < n) {
				const bt2g_sw_cand x = c[i];
				keys[i] = cand_key(x);
				lmin = x.score < lmin ? x.score : lmin;
				lmax = x.score > lmax ? x.score : lmax;
			} else {
				keys[i] = ~0ull;
			}
		}
		if(lmin <= lmax) { atomicMin(&smin, lmin); atomicMax(&smax, lmax); }
		__syncthreads();
		const int hi = smax;
		const uint32_t range = (uint32_t)((int64_t)smax - (int64_t)smin + 1);
		if(counting && n >= 128u && range <= SORT_BUCKETS) {
			for(uint32_t b = tid; b < range; b += blockDim.x) cur[b] = 0u;
			__syncthreads();
			for(uint32_t i = tid; i < n; i += blockDim.x)
				atomicAdd(&cur[(uint32_t)(hi - cand_of(keys[i]).score)], 1u);
			__syncthreads();
			// exclusive scan of the bucket counts (chunk per thread + block scan)
			const uint32_t chunk = (range + 255u) / 256u, b0 = tid * chunk;
			const uint32_t b1 = b0 + chunk < range ? b0 + chunk : range;
			uint32_t sum = 0;
			for(uint32_t b = b0; b < b1; b++) sum += cur[b];
			part[tid] = sum;
			__syncthreads();
			for(uint32_t off = 1; off < 256u; off <<= 1) {
				const uint32_t v = tid >= off ? part[tid - off] : 0u;
				__syncthreads();
				part[tid] += v;
				__syncthreads();
			}
			uint32_t run = tid ? part[tid - 1] : 0u;
			for(uint32_t b = b0; b < b1; b++) {
				const uint32_t h = cur[b];
				start[b] = run;
				cur[b] = run;
				run += h;
			}
			__syncthreads();
			for(uint32_t i = tid; i < n; i += blockDim.x) {
				const unsigned long long k = keys[i];
				tmp[atomicAdd(&cur[(uint32_t)(hi - cand_of(k).score)], 1u)] = k;
			}
			__syncthreads();
			for(uint32_t b = tid; b < range; b += blockDim.x) {
				const uint32_t s0 = start[b], e0 = b + 1u < range ? start[b + 1u] : n;
				for(uint32_t i = s0 + 1u; i < e0; i++) {
					const unsigned long long x = tmp[i];
					uint32_t j = i;
					while(j > s0 && tmp[j - 1u] > x) { tmp[j] = tmp[j - 1u]; j--; }
					tmp[j] = x;
				}
			}
			__syncthreads();
			for(uint32_t i = tid; i < n; i += blockDim.x) c[i] = cand_of(tmp[i]);
		} else {
			for(uint32_t size = 2; size <= P2; size <<= 1) {
				for(uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
					for(uint32_t i = tid; i < P2; i += blockDim.x) {
						const uint32_t jx = i ^ stride;
						if(jx > i) {
							const bool up = (i & size) == 0;
							const unsigned long long a = keys[i], b = keys[jx];
							if((a > b) == up) { keys[i] = b; keys[jx] = a; }
						}
					}
					__syncthreads();
				}
			}
			for(uint32_t i = tid; i < n; i += blockDim.x) c[i] = cand_of(keys[i]);
		}
		__syncthreads();
	}
}

void sw_fill_consts(const bt2g_scoring& sc, SwConst& h) {
	h.match = sc.match; h.npen = sc.npen; h.gapbar = sc.gapbar;
	h.rdgo = sc.rdg_const + sc.rdg_lin; h.rdge = sc.rdg_lin;
	h.rfgo = sc.rfg_const + sc.rfg_lin; h.rfge = sc.rfg_lin;
	for(int q = 0; q <= 40; q++) {
		float frac = (float)q / 40.0f;
		h.mmpen[q] = sc.mmp_min + (int)(frac * (sc.mmp_max - sc.mmp_min));
	}
}

// Launch one variant over `nprob` problems (or the device list).
void launch_sw_fill(int variant, const bt2g_sw_problem* probs, uint32_t nprob, const uint32_t* list,
                    const uint32_t* list_n, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                    const uint32_t* lens, const uint8_t* windows, const uint8_t* ref_codes,
                    const uint64_t* ref_starts, const SwConst& C, uint32_t cap, uint32_t* bnd,
                    uint32_t bnd_cols, bt2g_sw_result* res, bt2g_sw_cand* cands, int16_t* mat,
                    const uint64_t* mat_off, uint32_t* sat_list, uint32_t* sat_n, PlaneOut po, hipStream_t st) {
	dim3 grid((nprob + 63) / 64), block(64);
	if(nprob == 0) return;
	switch(variant) {
	case 0: hipLaunchKernelGGL(k_sw_fill<0>, grid, block, 0, st, probs, nprob, list, list_n, reads, quals, stride,
	                           lens, windows, ref_codes, ref_starts, C, cap, bnd, bnd_cols, res, cands, mat, mat_off,
	                           sat_list, sat_n, po); break;
	case 1: hipLaunchKernelGGL(k_sw_fill<1>, grid, block, 0, st, probs, nprob, list, list_n, reads, quals, stride,
	                           lens, windows, ref_codes, ref_starts, C, cap, bnd, bnd_cols, res, cands, mat, mat_off,
	                           sat_list, sat_n, po); break;
	case 2: hipLaunchKernelGGL(k_sw_fill<2>, grid, block, 0, st, probs, nprob, list, list_n, reads, quals, stride,
	                           lens, windows, ref_codes, ref_starts, C, cap, bnd, bnd_cols, res, cands, mat, mat_off,
	                           sat_list, sat_n, po); break;
	default: hipLaunchKernelGGL(k_sw_fill<3>, grid, block, 0, st, probs, nprob, list, list_n, reads, quals, stride,
	                            lens, windows, ref_codes, ref_starts, C, cap, bnd, bnd_cols, res, cands, mat, mat_off,
	                            sat_list, sat_n, po); break;
	}
}

void launch_sort_cands(const bt2g_sw_result* res, bt2g_sw_cand* cands, uint32_t nprob, uint32_t cap,
                       uint32_t* big, uint32_t* nbig, hipStream_t st) {
	if(nprob == 0) return;
	hipLaunchKernelGGL(k_sort_small, dim3((nprob + 3) / 4), dim3(256), 0, st, res, cands, nprob, cap, big, nbig);
	if(cap <= 64) return;
	uint32_t P2 = 1;
	while(P2 < cap) P2 <<= 1;
	// enough workgroups to fill every CU's LDS (48 KB each at cap 2048); the
	// queue length is only known on the device, idle groups exit at once
	const uint32_t grid = nprob < 4096u ? nprob : 4096u;
	// counting sort needs the keys twice plus the buckets (48 KB at cap 2048);
	// larger caps keep the bitonic network only
	size_t lds = 2u * P2 * sizeof(unsigned long long) + 2u * SORT_BUCKETS * sizeof(uint32_t);
	const int counting = lds <= 65536u ? 1 : 0;
	if(!counting) lds = P2 * sizeof(unsigned long long);
	hipLaunchKernelGGL(k_sort_big, dim3(grid), dim3(256), lds, st, res, cands, cap, P2, counting, big, nbig);
}
