// tests/cpu_emul/wg_emul.cpp -- TEST INFRASTRUCTURE ONLY.
// Runs the workgroup backtrace kernel of bowtie2-server_amd/csrc/sw_backtrace_wg.hip
// (the same source file, compiled for the host against stub_wg/hip/hip_runtime.h:
// 64 threads per workgroup) so tests/test_bt_emul.py can check it against the
// reference's alignments without a GPU.  The product never uses this.
#include "../../bowtie2-server_amd/csrc/sw_backtrace_wg.hip"

thread_local uint3v threadIdx, blockIdx;
thread_local EmulGroup* t_group;

extern "C" int wg_emul_run(const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* reads, const uint8_t* quals,
                           uint32_t stride, const uint32_t* lens, const uint8_t* windows, const bt2g_sw_rect* rects,
                           const bt2g_sw_result* res, const bt2g_sw_cand* cands, uint32_t cap, const uint8_t* plane,
                           uint64_t slot, uint32_t cstride, uint32_t maxcol, const SwConst* C, double ncl_const,
                           double ncl_lin, uint32_t maxaln, uint32_t maxedit, int32_t* naln, bt2g_sw_aln* alns,
                           bt2g_edit* edits, int8_t* fates) {
	BtArgs a{};
	a.probs = probs; a.nprob = nprob; a.reads = reads; a.quals = quals; a.stride = stride; a.lens = lens;
	a.windows = windows; a.rects = rects; a.res = res; a.cands = cands; a.cap = cap; a.plane = plane; a.slot = slot;
	a.cstride = cstride; a.pcols = maxcol; a.plane_top = 0;
	a.C = *C; a.local = 0; a.ncl_const = ncl_const; a.ncl_lin = ncl_lin;
	a.maxaln = maxaln; a.maxedit = maxedit; a.naln = naln; a.alns = alns; a.edits = edits; a.fates = fates;
	launch_sw_bt_wg(a, sw_bt_wg_lds(a), nullptr);
	return 0;
}
