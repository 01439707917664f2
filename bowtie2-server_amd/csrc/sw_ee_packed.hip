// sw_ee_packed.hip -- end-to-end SW fill + last-row gather, two problems per
// lane in packed 16-bit arithmetic (gfx950 VOP3P: v_pk_sub_{u16,i16} clamp,
// v_pk_max_{u16,i16}, v_perm_b32).
//
// Same recurrence, value domains and saturation as k_sw_fill<0/1> (and so as
// aligner_swsse_ee_u8.cpp:775-1146 / aligner_swsse_ee_i16.cpp:780-1200), but:
//   * lane l of a wave owns problems 2 of a 128-problem block: the low half of
//     every 32-bit register is problem base+l, the high half problem
//     base+64+l.  The u8 domain (0xff = score 0, floor 0) runs in u16 lanes
//     with unsigned saturation, the i16 domain in i16 lanes with signed
//     saturation -- each packed op is exactly the SSE2 op of the reference.
//   * the substitution penalty of a cell is one v_perm_b32: each row keeps a
//     per-problem 4-byte profile {pen(A),pen(C),pen(G),pen(T)} (the reference's
//     query profile, aligner_swsse_ee_u8.cpp:56-190, row-major instead of
//     striped) and each column a byte selector built from the two reference
//     characters; an 'N' column selects 0 and is lifted to the N penalty.
//   * strips of R rows live in VGPRs; strip 0 gathers the reference once and
//     leaves the per-column selector in the boundary buffer, later strips read
//     it back coalesced together with the strip above's last H/F.
// Cost per cell pair: 13 VALU ops (7 more per row in the <= 2 strips that hold
// gap-barrier rows or a problem's last row).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "bt2g_kernels.h"

namespace {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

template <int V> struct Pk;
template <> struct Pk<0> {   // end-to-end u8 domain
	typedef u16x2 T;
	static constexpr uint32_t LO = 0x00000000u, ROW0 = 0x00ff00ffu;
	static constexpr int LOS = 0, ROW0S = 0xff;
	static __device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b) {
		return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(T, a), __builtin_bit_cast(T, b)));
	}
	static __device__ __forceinline__ uint32_t max(uint32_t a, uint32_t b) {
		return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(T, a), __builtin_bit_cast(T, b)));
	}
	static __device__ __forceinline__ int lo(uint32_t v) { return (int)(v & 0xffffu); }
	static __device__ __forceinline__ int hi(uint32_t v) { return (int)(v >> 16); }
};
template <> struct Pk<1> {   // end-to-end i16 domain
	typedef i16x2 T;
	static constexpr uint32_t LO = 0x80008000u, ROW0 = 0x7fff7fffu;
	static constexpr int LOS = -32768, ROW0S = 0x7fff;
	static __device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b) {
		return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(T, a), __builtin_bit_cast(T, b)));
	}
	static __device__ __forceinline__ uint32_t max(uint32_t a, uint32_t b) {
		return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(T, a), __builtin_bit_cast(T, b)));
	}
	static __device__ __forceinline__ int lo(uint32_t v) { return (int)(int16_t)(v & 0xffffu); }
	static __device__ __forceinline__ int hi(uint32_t v) { return (int)(int16_t)(v >> 16); }
};

// (m & a) | (~m & b): v_bfi_b32
__device__ __forceinline__ uint32_t msel(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }

__device__ __forceinline__ int first5(int m) {
	return (m & 1) ? 0 : (m & 2) ? 1 : (m & 4) ? 2 : (m & 8) ? 3 : 4;
}

struct Half {
	const uint8_t* rd;
	const uint8_t* qu;
	uint32_t nrow, ncol, pi;
	int32_t minsc;
	bool fw, live;
	int64_t refl, win_off;
	uint32_t refidx;
	__device__ __forceinline__ int base(uint32_t r) const {
		if(fw) return rd[r];
		int c = rd[nrow - 1 - r];
		return c > 3 ? 4 : 3 - c;
	}
	__device__ __forceinline__ int qual(uint32_t r) const { return fw ? qu[r] : qu[nrow - 1 - r]; }
	// reference character of column j (0..3, 4 = N / off the reference)
	__device__ __forceinline__ int refc(uint32_t j, const uint8_t* windows, const uint8_t* ref_codes,
	                                    const uint64_t* ref_starts) const {
		if(!live || j >= ncol) return 4;
		if(win_off >= 0) return first5(windows[win_off + j]);
		int64_t o = refl + (int64_t)j;
		uint64_t s = ref_starts[refidx], e = ref_starts[refidx + 1];
		return (o < 0 || (uint64_t)o >= e - s) ? 4 : ref_codes[s + (uint64_t)o];
	}
	// {pen(A), pen(C), pen(G), pen(T)} of row r (Scoring::score, scoring.h:237-262; match bonus 0)
	__device__ __forceinline__ uint32_t profile(uint32_t r, const SwConst& C) const {
		if(!live || r >= nrow) return 0;
		int rdc = base(r);
		if(rdc > 3) return (uint32_t)C.npen * 0x01010101u;
		int q = qual(r) - 33;
		q = q < 0 ? 0 : (q > 40 ? 40 : q);
		uint32_t w = (uint32_t)C.mmpen[q] * 0x01010101u;
		return w & ~(0xffu << (8 * rdc));
	}
	__device__ __forceinline__ bool bar(uint32_t r, int gapbar) const {
		return r < nrow && ((int)r < gapbar || (int)(nrow - r - 1) < gapbar);
	}
};

}  // namespace

template <int V, int R>
__global__ void __launch_bounds__(64)
k_sw_ee_pk(const bt2g_sw_problem* __restrict__ probs, uint32_t nprob, const uint32_t* __restrict__ list,
           const uint32_t* __restrict__ list_n, const uint8_t* __restrict__ reads, const uint8_t* __restrict__ quals,
           uint32_t stride, const uint32_t* __restrict__ lens, const uint8_t* __restrict__ windows,
           const uint8_t* __restrict__ ref_codes, const uint64_t* __restrict__ ref_starts, SwConst C, uint32_t cap,
           uint32_t* __restrict__ bnd, uint32_t bnd_cols, bt2g_sw_result* __restrict__ res,
           bt2g_sw_cand* __restrict__ cands) {
	using D = Pk<V>;
	const uint32_t lane = threadIdx.x;
	const uint32_t cnt = list ? *list_n : nprob;
	const uint32_t ga = blockIdx.x * 128u + lane, gb = ga + 64u;
	if(ga >= cnt) return;
	Half h[2];
#pragma unroll
	for(int x = 0; x < 2; x++) {
		const uint32_t g = x ? gb : ga;
		Half& H = h[x];
		H.live = g < cnt;
		H.nrow = H.ncol = 0;
		if(!H.live) continue;
		H.pi = list ? list[g] : g;
		const bt2g_sw_problem p = probs[H.pi];
		H.nrow = lens[p.read];
		H.ncol = p.ncol;
		H.rd = reads + (size_t)p.read * stride;
		H.qu = quals + (size_t)p.read * stride;
		H.fw = p.fw != 0;
		H.refl = p.refl;
		H.win_off = p.win_off;
		H.refidx = p.refidx;
		H.minsc = p.minsc;
		if(H.ncol > bnd_cols || H.ncol == 0 || H.nrow == 0) {
			bt2g_sw_result bad{};
			bad.flag = -3;
			bad.best = INT32_MIN;
			res[H.pi] = bad;
			H.live = false;
			H.nrow = H.ncol = 0;
		}
	}
	const uint32_t nrowmax = h[0].nrow > h[1].nrow ? h[0].nrow : h[1].nrow;
	const uint32_t ncolmax = h[0].ncol > h[1].ncol ? h[0].ncol : h[1].ncol;
	uint32_t* hf = bnd + (size_t)blockIdx.x * bnd_cols * 64u * 3u;   // [col][lane] {H pair, F pair}
	uint32_t* selb = hf + (size_t)bnd_cols * 64u * 2u;                // [col][lane] selector
	const uint32_t rdge2 = (uint32_t)C.rdge * 0x10001u, rdgo2 = (uint32_t)C.rdgo * 0x10001u;
	const uint32_t rfge2 = (uint32_t)C.rfge * 0x10001u, rfgo2 = (uint32_t)C.rfgo * 0x10001u;
	const uint32_t npen = (uint32_t)C.npen;
	int lrmax[2] = {D::LOS, D::LOS};
	uint32_t ncand[2] = {0, 0};

	for(uint32_t s0 = 0; s0 < nrowmax; s0 += R) {
		uint32_t PA[R], PB[R], E[R], Hc[R];
#pragma unroll
		for(int k = 0; k < R; k++) {
			PA[k] = h[0].profile(s0 + k, C);
			PB[k] = h[1].profile(s0 + k, C);
			E[k] = D::LO;
			Hc[k] = D::LO;
		}
		const bool first = s0 == 0;
		const bool store = s0 + R < nrowmax;
		bool full = false, has_last[2];
#pragma unroll
		for(int x = 0; x < 2; x++) {
			const uint32_t nr = h[x].nrow;
			has_last[x] = nr > 0 && nr - 1 >= s0 && nr - 1 < s0 + R;
			const bool top = (int)s0 < C.gapbar && s0 < nr;
			const bool bot = nr > 0 && (int64_t)s0 + R > (int64_t)nr - C.gapbar && s0 < nr;
			full |= has_last[x] || top || bot;
		}
		auto sweep = [&](auto full_tag) {
			constexpr bool FULL = decltype(full_tag)::value;
			uint32_t BM[R], LM[R];
			if(FULL) {
#pragma unroll
				for(int k = 0; k < R; k++) {
					const uint32_t r = s0 + k;
					BM[k] = (h[0].bar(r, C.gapbar) ? 0u : 0xffffu) | (h[1].bar(r, C.gapbar) ? 0u : 0xffff0000u);
					LM[k] = (h[0].nrow > 0 && r == h[0].nrow - 1 ? 0xffffu : 0u) |
					        (h[1].nrow > 0 && r == h[1].nrow - 1 ? 0xffff0000u : 0u);
				}
			}
			uint32_t hbprev = D::LO;
			// software pipeline: column j+1's inputs are fetched while j computes
			int ca = 4, cb = 4;
			uint32_t nsel = 0, nh = 0, nf = 0;
			if(first) {
				ca = h[0].refc(0, windows, ref_codes, ref_starts);
				cb = h[1].refc(0, windows, ref_codes, ref_starts);
			} else {
				nsel = selb[lane];
				nh = hf[2u * lane];
				nf = hf[2u * lane + 1];
			}
			for(uint32_t j = 0; j < ncolmax; j++) {
				uint32_t sel, hup, fup, diag;
				if(first) {
					sel = (ca < 4 ? (uint32_t)ca : 0x0cu) | 0x0c00u | ((cb < 4 ? 4u + (uint32_t)cb : 0x0cu) << 16) |
					      0x0c000000u;
					if(j + 1 < ncolmax) {
						ca = h[0].refc(j + 1, windows, ref_codes, ref_starts);
						cb = h[1].refc(j + 1, windows, ref_codes, ref_starts);
					}
					if(store) selb[(size_t)j * 64u + lane] = sel;
					hup = fup = D::LO;
					diag = D::ROW0;
				} else {
					sel = nsel; hup = nh; fup = nf;
					if(j + 1 < ncolmax) {
						const size_t o = (size_t)(j + 1) * 64u + lane;
						nsel = selb[o];
						nh = hf[2u * o];
						nf = hf[2u * o + 1];
					}
					diag = hbprev;
					hbprev = hup;
				}
				const uint32_t nfloor = ((sel & 0xffu) == 0x0cu ? npen : 0u) |
				                        (((sel >> 16) & 0xffu) == 0x0cu ? npen << 16 : 0u);
				uint32_t fprev = fup, hprev = hup, lastv = D::LO;
#pragma unroll
				for(int k = 0; k < R; k++) {
					uint32_t pen = D::max(__builtin_amdgcn_perm(PB[k], PA[k], sel), nfloor);
					const uint32_t d = D::sub(diag, pen);
					uint32_t f = D::max(D::sub(fprev, rfge2), D::sub(hprev, rfgo2));
					if(FULL) f = msel(BM[k], f, D::LO);
					const uint32_t hh = D::max(D::max(d, E[k]), f);
					uint32_t eo = D::sub(hh, rdgo2);
					if(FULL) eo = msel(BM[k], eo, D::LO);
					E[k] = D::max(D::sub(E[k], rdge2), eo);
					diag = Hc[k];
					Hc[k] = hh;
					fprev = f;
					hprev = hh;
					if(FULL) lastv = D::max(lastv, msel(LM[k], hh, D::LO));
				}
				if(store) {
					const size_t o = (size_t)j * 64u + lane;
					hf[2u * o] = hprev;
					hf[2u * o + 1] = fprev;
				}
				if(FULL) {
#pragma unroll
					for(int x = 0; x < 2; x++) {
						if(has_last[x] && j < h[x].ncol) {
							const int v = x ? D::hi(lastv) : D::lo(lastv);
							lrmax[x] = v > lrmax[x] ? v : lrmax[x];
							const int64_t sc = (int64_t)v - D::ROW0S;
							if(sc >= h[x].minsc) {
								if(ncand[x] < cap)
									cands[(size_t)h[x].pi * cap + ncand[x]] =
									    bt2g_sw_cand{(int32_t)h[x].nrow - 1, (int32_t)j, (int32_t)sc};
								ncand[x]++;
							}
						}
					}
				}
			}
		};
		if(full) sweep(std::true_type{});
		else sweep(std::false_type{});
	}

	// SwAligner::align end-to-end outcome (aligner_sw.cpp:500-620), as k_sw_fill
#pragma unroll
	for(int x = 0; x < 2; x++) {
		if(!h[x].live) continue;
		bt2g_sw_result out;
		out.u8succ = out.i16succ = 0;
		int64_t best;
		const int64_t score = (int64_t)lrmax[x] - D::ROW0S;
		if(score < h[x].minsc) { out.flag = -1; best = score; }
		else if(lrmax[x] == D::LOS) { out.flag = -2; best = INT64_MIN; }
		else { out.flag = 0; best = score; }
		out.colstop = (int32_t)h[x].ncol - 1;
		out.lastsolcol = 0;
		if(V == 0) out.u8succ = out.flag == 0; else out.i16succ = out.flag == 0;
		const bool fail = best == INT64_MIN || best < h[x].minsc;
		out.best = best == INT64_MIN ? INT32_MIN : (int32_t)best;
		uint32_t nc = fail ? 0u : ncand[x];
		out.ncand = (int32_t)nc;
		out.aligned = (!fail && nc > 0) ? 1 : 0;
		res[h[x].pi] = out;
	}
}

// Packed end-to-end fill over a device list (V=0 u8 domain, V=1 i16 domain).
void launch_sw_ee_packed(int variant, const bt2g_sw_problem* probs, uint32_t nprob, const uint32_t* list,
                         const uint32_t* list_n, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                         const uint32_t* lens, const uint8_t* windows, const uint8_t* ref_codes,
                         const uint64_t* ref_starts, const SwConst& C, uint32_t cap, uint32_t* bnd,
                         uint32_t bnd_cols, bt2g_sw_result* res, bt2g_sw_cand* cands, hipStream_t st) {
	if(nprob == 0) return;
	dim3 grid((nprob + 127) / 128), block(64);
	if(variant == 0)
		hipLaunchKernelGGL((k_sw_ee_pk<0, 16>), grid, block, 0, st, probs, nprob, list, list_n, reads, quals, stride,
		                   lens, windows, ref_codes, ref_starts, C, cap, bnd, bnd_cols, res, cands);
	else
		hipLaunchKernelGGL((k_sw_ee_pk<1, 16>), grid, block, 0, st, probs, nprob, list, list_n, reads, quals, stride,
		                   lens, windows, ref_codes, ref_starts, C, cap, bnd, bnd_cols, res, cands);
}
