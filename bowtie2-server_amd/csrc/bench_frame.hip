// bench_frame.hip -- batch glue between the seed-phase engines and the SW
// engine, on the device: gather every read's hit rows, and after getOffset
// turn them into seed-extension DP rectangles.
//
// These are NOT reference seams: the reference decides which hits to extend
// in SwDriver::extendSeeds with RNG-driven prioritisation and extension
// limits (aligner_sw_driver.cpp:756-1297).  The bench's policy is documented
// in DESIGN.md section 5: one rectangle per distinct (read, strand, reference,
// diagonal), at most two per read, the two smallest by (strand, reference,
// diagonal).  k_frame emits seed-extension frame inputs (kind 0); the
// rectangles themselves come from bt2g_frame_dev, the restatement of
// DynProgFramer::frameSeedExtensionRect (dp_framer.cpp:81-129) with its
// trimming at the reference ends and its core diagonals.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "bt2g_kernels.h"
#include "bt2g_bench.h"
#include "dev_util.h"

namespace {

// meta of a hit row: fw << 31 | depth << 16 | hit length
__device__ __forceinline__ uint32_t meta_of(bool fw, uint32_t dep, uint32_t hitlen) {
	return (fw ? 0x80000000u : 0u) | (dep << 16) | (hitlen & 0xffffu);
}

}  // namespace

// One thread per read: the top SA row of its exact end-to-end hit, of every
// one-mismatch hit and of every exact seed hit, contiguous per read.
__global__ void __launch_bounds__(256)
k_collect_rows(uint32_t n, const uint32_t* __restrict__ lens, const uint32_t* __restrict__ sweep,
               const bt2g_mm1* __restrict__ mm, const int32_t* __restrict__ mm_cnt, uint32_t mm_cap,
               const uint32_t* __restrict__ seeds, const int32_t* __restrict__ inv, uint32_t maxseeds,
               uint32_t seedlen, uint32_t interval, uint32_t* __restrict__ rows, uint32_t* __restrict__ meta,
               uint32_t* __restrict__ read_base, uint32_t* __restrict__ read_cnt, uint32_t* __restrict__ total,
               uint32_t cap) {
	const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
	const bool valid = r < n;
	uint32_t cnt = 0, len = 0;
	bool exact = false;
	int32_t si = -1, nm = 0;
	if(valid) {
		len = lens[r];
		const uint32_t* sw = sweep + (size_t)r * 8;
		exact = (sw[0] < sw[1] ? sw[0] : sw[1]) == 0;
		cnt += exact ? 1u : 0u;
		nm = mm_cnt[r];
		nm = nm < 0 ? 0 : (nm > (int32_t)mm_cap ? (int32_t)mm_cap : nm);
		cnt += (uint32_t)nm;
		si = inv ? inv[r] : -1;
		if(si >= 0) {
			const uint32_t* sd = seeds + (size_t)si * 2 * maxseeds * 4;
			for(uint32_t k = 0; k < 2 * maxseeds; k++) cnt += sd[k * 4 + 1] > sd[k * 4] ? 1u : 0u;
		}
	}
	uint32_t base = block_alloc<256>(cnt, total);
	if(!valid) return;
	if(base + cnt > cap) cnt = base < cap ? cap - base : 0;   // overflow: truncated (caller checks total)
	read_base[r] = base;
	read_cnt[r] = cnt;
	uint32_t k = 0;
	const uint32_t* sw = sweep + (size_t)r * 8;
	if(exact && k < cnt) {
		const bool fw = sw[3] > sw[2];
		rows[base + k] = fw ? sw[2] : sw[4];
		meta[base + k] = meta_of(fw, 0, len);
		k++;
	}
	for(int32_t i = 0; i < nm && k < cnt; i++, k++) {
		const bt2g_mm1 h = mm[(size_t)r * mm_cap + i];
		rows[base + k] = h.top;
		meta[base + k] = meta_of(h.fw != 0, 0, len);
	}
	if(si >= 0) {
		const uint32_t* sd = seeds + (size_t)si * 2 * maxseeds * 4;
		for(uint32_t q = 0; q < 2 * maxseeds && k < cnt; q++) {
			if(sd[q * 4 + 1] > sd[q * 4]) {
				const uint32_t strand = q / maxseeds, s = q % maxseeds;
				rows[base + k] = sd[q * 4];
				meta[base + k] = meta_of(strand == 0, s * interval, seedlen);
				k++;
			}
		}
	}
}

// One thread per read: joined offsets -> (reference, offset) (Ebwt::joinedToTextOff,
// bt2_idx.cpp:54, rejecting hits that straddle a fragment end), read start on
// the reference, two smallest distinct (strand, reference, start) -> frame
// inputs for bt2g_frame_dev.
__global__ void __launch_bounds__(256)
k_frame(uint32_t n, const uint32_t* __restrict__ lens, const uint32_t* __restrict__ offs,
        const uint32_t* __restrict__ meta, const uint32_t* __restrict__ read_base,
        const uint32_t* __restrict__ read_cnt, const uint32_t* __restrict__ fr_joff,
        const uint32_t* __restrict__ fr_tid, const uint32_t* __restrict__ fr_toff,
        const uint32_t* __restrict__ fr_end, uint32_t nfrag, int32_t minsc,
        bt2g_frame_in* __restrict__ fin, uint32_t* __restrict__ nprob, uint32_t cap) {
	const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
	const bool valid = r < n;
	const uint64_t NONE = ~0ull;
	uint64_t k1 = NONE, k2 = NONE;
	uint32_t len = 0;
	if(valid) {
		len = lens[r];
		const uint32_t b = read_base[r], c = read_cnt[r];
		for(uint32_t k = b; k < b + c; k++) {
			const uint32_t off = offs[k], m = meta[k];
			// last fragment with joff <= off
			uint32_t lo = 0, hi = nfrag;
			while(hi - lo > 1) {
				const uint32_t mid = (lo + hi) >> 1;
				if(fr_joff[mid] <= off) lo = mid; else hi = mid;
			}
			const bool fw = m >> 31;
			const uint32_t dep = (m >> 16) & 0x7fffu, hitlen = m & 0xffffu;
			if((uint64_t)off + hitlen > fr_end[lo]) continue;      // straddles a fragment boundary
			const int64_t toff = (int64_t)fr_toff[lo] + (int64_t)(off - fr_joff[lo]);
			const int64_t start = fw ? toff - dep : toff - ((int64_t)len - dep - hitlen);
			const uint64_t key = ((uint64_t)(fw ? 1 : 0) << 62) | ((uint64_t)fr_tid[lo] << 40) |
			                     (uint64_t)(start + (1ll << 39));
			if(key == k1 || key == k2) continue;
			if(key < k1) { k2 = k1; k1 = key; }
			else if(key < k2) k2 = key;
		}
	}
	const uint32_t np = (k1 != NONE ? 1u : 0u) + (k2 != NONE ? 1u : 0u);
	const uint32_t base = block_alloc<256>(np, nprob);
	if(!valid) return;
	for(uint32_t i = 0; i < np; i++) {
		if(base + i >= cap) break;
		const uint64_t key = i ? k2 : k1;
		bt2g_frame_in f;
		f.off = (int64_t)(key & ((1ull << 40) - 1)) - (1ll << 39);
		f.read = r;
		f.refidx = (uint32_t)((key >> 40) & 0x3fffffu);
		f.minsc = minsc;
		f.fw = (int32_t)(key >> 62);
		f.kind = 0;
		f.anchor1 = 0;
		f.alen = 0;
		f.pad = 0;
		fin[base + i] = f;
	}
}

extern "C" {

int bt2g_bench_collect_rows_dev(uint32_t n, const uint32_t* lens, const uint32_t* sweep, const bt2g_mm1* mm,
                                const int32_t* mm_cnt, uint32_t mm_cap, const uint32_t* seeds, const int32_t* inv,
                                uint32_t maxseeds, uint32_t seedlen, uint32_t interval, uint32_t* rows,
                                uint32_t* meta, uint32_t* read_base, uint32_t* read_cnt, uint32_t* total,
                                uint32_t cap, void* stream) {
	if(n == 0) return BT2G_OK;
	hipLaunchKernelGGL(k_collect_rows, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, lens, sweep, mm,
	                   mm_cnt, mm_cap, seeds, inv, maxseeds, seedlen, interval, rows, meta, read_base, read_cnt,
	                   total, cap);
	return hipGetLastError() == hipSuccess ? BT2G_OK : BT2G_ERR_HIP;
}

int bt2g_bench_frame_dev(uint32_t n, const uint32_t* lens, const uint32_t* offs, const uint32_t* meta,
                         const uint32_t* read_base, const uint32_t* read_cnt, const uint32_t* fr_joff,
                         const uint32_t* fr_tid, const uint32_t* fr_toff, const uint32_t* fr_end, uint32_t nfrag,
                         int32_t minsc, bt2g_frame_in* fin, uint32_t* nprob, uint32_t cap, void* stream) {
	if(n == 0) return BT2G_OK;
	if(nfrag == 0) return BT2G_ERR_ARG;
	hipLaunchKernelGGL(k_frame, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, lens, offs, meta,
	                   read_base, read_cnt, fr_joff, fr_tid, fr_toff, fr_end, nfrag, minsc, fin, nprob, cap);
	return hipGetLastError() == hipSuccess ? BT2G_OK : BT2G_ERR_HIP;
}

}  // extern "C"
