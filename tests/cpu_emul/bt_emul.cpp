// tests/cpu_emul/bt_emul.cpp -- TEST INFRASTRUCTURE ONLY.
// Runs the backtrace kernel of bowtie2-server_amd/csrc/sw_backtrace.hip (the
// same source file, compiled for the host against stub/hip/hip_runtime.h)
// over a batch on the CPU, so tests/test_bt_emul.py can check its indexing and
// its results against the oracle without a GPU.  The product never uses this.
#include "../../bowtie2-server_amd/csrc/sw_backtrace.hip"
#include <string.h>
#include <stdlib.h>

thread_local uint3v threadIdx, blockIdx;
// the workgroup kernel (sw_backtrace_wg.hip) runs in tests/cpu_emul/wg_emul.cpp
uint32_t sw_bt_wg_lds(const BtArgs&) { return 0xffffffffu; }
uint32_t sw_bt_wg_lds_limit() { return 65536u; }
void launch_sw_bt_wg(const BtArgs&, uint32_t, hipStream_t) { abort(); }
#ifdef BT2G_BT_COUNT
unsigned long long bt_counts[16];
extern "C" unsigned long long* bt_emul_counts() { return bt_counts; }
#endif

extern "C" int bt_emul_run(int kind, const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* reads,
                           const uint8_t* quals, uint32_t stride, const uint32_t* lens, const uint8_t* windows,
                           const bt2g_sw_rect* rects, const bt2g_sw_result* res, const bt2g_sw_cand* cands,
                           uint32_t cap, const uint8_t* plane, uint64_t slot, uint32_t cstride, int plane_top, uint32_t maxrow, uint32_t maxcol, const SwConst* C, int local,
                           double ncl_const, double ncl_lin, uint32_t maxaln, uint32_t maxedit, int32_t* naln,
                           bt2g_sw_aln* alns, bt2g_edit* edits, int8_t* fates) {
	BtArgs a{};
	a.probs = probs; a.nprob = nprob; a.reads = reads; a.quals = quals; a.stride = stride; a.lens = lens;
	a.windows = windows; a.ref_codes = nullptr; a.ref_starts = nullptr; a.rects = rects;
	a.res = res; a.cands = cands; a.cap = cap; a.plane = plane; a.slot = slot; a.cstride = cstride; a.pcols = maxcol; a.use_mask = plane_top != 1 && cstride <= 256u;
	a.plane_top = plane_top;
	a.rwords = sw_bt_rcols(maxrow, maxcol); a.rrows = sw_bt_rrows(maxrow);
	a.mwords = sw_bt_tcols(maxcol); a.mrows = sw_bt_trows(maxrow); a.mslot = sw_bt_mslot(maxrow, maxcol, local != 0);
	a.mdom = local ? sw_bt_mdom(maxrow, maxcol) : 0u;
	// garbage-filled scratch: the kernel must not rely on zeroed memory
	std::vector<uint32_t> marks(a.mslot * nprob + 4, 0xdeadbeefu);
	a.marks = marks.data();
	a.C = *C; a.local = local; a.ncl_const = ncl_const; a.ncl_lin = ncl_lin;
	a.maxaln = maxaln; a.maxedit = maxedit; a.naln = naln; a.alns = alns; a.edits = edits; a.fates = fates;
	// DP queue (the lanes of the emulation run one after another: lane 0 of each
	// block takes every DP left; BT_EMUL_STATIC=1: one DP per lane)
	uint32_t queue = 0;
	const char* st = getenv("BT_EMUL_STATIC");
	a.queue = st && *st == '1' ? nullptr : &queue;
	setenv("BT2G_BT_LDS_MAX", "0", 1);          // lane-per-problem kernels only (one lane at a time here)
	launch_sw_bt(kind, a, nullptr);
	return 0;
}
