// bt2g_kernels.h -- launchers shared by the kernel files and the host API.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/bt2g.h"
#include "fm_device.h"

// Scoring constants of the SW fills (Scoring, scoring.h:103-131, 417-440).
struct SwConst {
	int32_t match, npen, gapbar;
	int32_t rdgo, rdge, rfgo, rfge;
	int32_t mmpen[41];          // Scoring::mmpens for Phred 0..40 (capped at 40)
};

void sw_fill_consts(const bt2g_scoring& sc, SwConst& h);

void launch_exact_sweep(const DevEbwt& e, const uint8_t* reads, uint32_t stride, const uint32_t* lens, uint32_t n,
                        uint32_t mine_max, int nofw, int norc, uint32_t* out, hipStream_t st);
void launch_seed_search(const DevEbwt& F, const DevEbwt& B, const uint8_t* reads, uint32_t stride,
                        const uint32_t* lens, uint32_t n, uint32_t seedlen, uint32_t interval, uint32_t offset,
                        uint32_t maxseeds, uint32_t* out, int32_t* nseeds, uint32_t* bwops, uint32_t* loads,
                        hipStream_t st);
// oneMmSearch scoring inputs (aligner_seed.cpp:973-1323)
struct MmParams {
	int32_t match, mmp_max, mmp_min, npen, local;
	int32_t nceil_const_x1000, nceil_lin_x1000;
};
// One far-half branch (a one-mismatch alternative still to be walked to the
// read's end) handed from the far-half kernel to the branch kernel.
struct MmBranch {
	uint4 rng;          // topm, botm, topmp, botmp after the mismatch step
	uint32_t slot;      // read * 4 + fwi * 2 + ebwtfw index
	uint32_t seq;       // discovery order within the slot
	uint32_t meta;      // depm | j << 16 | rdc << 20 | valid << 24 | ebwtfw << 25
	int32_t score;      // the hit's score
	int32_t off5p;      // the mismatch's offset from the 5' end
	uint32_t pad[3];
};
// items: n*4 u32 scratch; counters: 8 u32 zeroed by the caller (item counts
// at [0] / [2], branch queue head at [4], fallback item counts at [5] / [6]);
// near_state / near_dep / fb_items / fb_st4 / fb_sdep / slot_flag: n*4 each;
// brq: brq_cap branch records (items meeting a full queue are redone whole by
// the in-place state machine k_one_mm_q)
// launch_one_mm's nofw with this bit and a gate: the reference's rule alone
// (bt2_search.cpp:3649-3650), no skip of reads with an exact end-to-end hit
const int MM_GATE_KEEP_EXACT = 2;
void launch_one_mm_q(const DevEbwt& F, const DevEbwt& B, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                     const uint32_t* lens, uint32_t n, const int32_t* minsc, const bt2g_scoring& sc, int nofw,
                     int norc, const uint32_t* gate, uint32_t cap, uint32_t* items, uint32_t* counters,
                     uint4* near_state, uint32_t* near_dep, bt2g_mm1* slots, int32_t* slot_counts, uint32_t* ops,
                     uint32_t* loads, MmBranch* brq, uint32_t brq_cap, uint32_t* fb_items, uint4* fb_st4,
                     uint32_t* fb_sdep, uint32_t* slot_flag, hipStream_t st, hipStream_t st2 = nullptr,
                     hipEvent_t* ev = nullptr);
// st2 / ev (4 events, optional): the second index direction's kernels on st2
// (fork from st, join back): each direction's kernels last as long as their
// longest walk, so the two directions overlap instead of running back to back
void launch_one_mm(const DevEbwt& F, const DevEbwt& B, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                   const uint32_t* lens, uint32_t n, const int32_t* minsc, const bt2g_scoring& sc, int nofw,
                   int norc, const uint32_t* gate, uint32_t cap, uint32_t* items, uint32_t* counters,
                   uint4* near_state, uint32_t* near_dep, bt2g_mm1* slots, int32_t* slot_counts, bt2g_mm1* hits,
                   int32_t* counts, uint32_t* ops, uint32_t* loads, int32_t* overflow, MmBranch* brq,
                   uint32_t brq_cap, uint32_t* fb_items, uint4* fb_st4, uint32_t* fb_sdep, uint32_t* slot_flag,
                   hipStream_t st, hipStream_t st2 = nullptr, hipEvent_t* ev = nullptr);
void launch_extend(const DevEbwt& F, const DevEbwt& B, int has_bw, const uint8_t* reads, uint32_t stride,
                   const uint32_t* lens, const bt2g_ext_in* in, uint32_t n, bt2g_ext_out* out, hipStream_t st);
void launch_get_offset(const DevEbwt& e, const uint32_t* rows, uint32_t n, uint32_t* offs, uint32_t* loads,
                       hipStream_t st);
// offsets of the rows of the small ranges of an exact sweep + 1-mm search (bt2g_exact_sweep_1mm)
void launch_seed_offsets(const DevEbwt& e, const uint32_t* out, uint64_t nrange, uint32_t off_cap, uint32_t* offs,
                         hipStream_t st);
void launch_seed_extend(const DevEbwt& F, const DevEbwt& B, int has_bw, const uint8_t* reads, uint32_t stride,
                        const uint32_t* lens, uint32_t n, uint32_t seedlen, uint32_t interval, uint32_t offset,
                        uint32_t maxseeds, const uint32_t* out, bt2g_ext_out* ext, hipStream_t st);
void launch_range_offsets(const DevEbwt& e, const uint32_t* sweep, const bt2g_mm1* hits, const int32_t* counts,
                          uint32_t n, uint32_t cap, uint32_t off_cap, uint32_t* offs, hipStream_t st);
void launch_sw_partition(const bt2g_sw_problem* probs, uint32_t nprob, int local, int enable8, uint32_t* list8,
                         uint32_t* n8, uint32_t* list16, uint32_t* n16, hipStream_t st);
// Score plane written by the one-problem-per-lane fills: u16 per cell (score
// + 0x8000 for the i16 fills' offset domain), rows top-aligned in 16-row
// blocks of pcols columns, hslot bytes per problem (null plane: none).
struct PlaneOut {
	uint8_t* plane;
	uint64_t hslot;
	uint32_t pcols;
};
void launch_sw_fill(int variant, const bt2g_sw_problem* probs, uint32_t nprob, const uint32_t* list,
                    const uint32_t* list_n, const uint8_t* reads, const uint8_t* quals, uint32_t stride,
                    const uint32_t* lens, const uint8_t* windows, const uint8_t* ref_codes,
                    const uint64_t* ref_starts, const SwConst& c, uint32_t cap, uint32_t* bnd,
                    uint32_t bnd_cols, bt2g_sw_result* res, bt2g_sw_cand* cands, int16_t* mat,
                    const uint64_t* mat_off, uint32_t* sat_list, uint32_t* sat_n, PlaneOut po, hipStream_t st);
void launch_sw_packed(bool local, const bt2g_sw_problem* probs, uint32_t nprob, const uint8_t* reads,
                      const uint8_t* quals, uint32_t stride, const uint32_t* lens, const uint8_t* windows,
                      const uint8_t* ref_codes, const uint64_t* ref_starts, const SwConst& C, int enable8,
                      uint32_t cap, uint32_t max_cols, bt2g_sw_result* res, bt2g_sw_cand* cands, uint8_t* plane,
                      uint64_t hslot, int hbytes, hipStream_t st);
// LDS words per problem pair of the systolic fill: per-column selectors, and in
// local mode the i16 column maxima and the reference masks (u16) too
inline uint32_t sw_packed_group_words(uint32_t max_cols, bool local) {
	const uint32_t w = (max_cols + 1u) | 1u;
	return local ? 2u * w + (w + 1u) / 2u : w;
}
// Rows per strip stack of the systolic fill (its score-plane column stride).
inline uint32_t sw_packed_rows(uint32_t stride) { return 16u * ((stride + 15u) / 16u); }
// Score-plane column pitch: a multiple of 4, so that the u8 fill's 4-column
// bursts (64 B) start on 64-B boundaries
__host__ __device__ inline uint32_t sw_plane_pitch(uint32_t cols) { return (cols + 3u) & ~3u; }
// Score-plane bytes per problem: 16-row blocks x pitch x hbytes, then one u16
// mask of written blocks per column (sw_ee_packed.hip); a multiple of 64 B
inline uint64_t sw_plane_slot(uint32_t stride, uint32_t cols, int hbytes) {
	const uint64_t pc = sw_plane_pitch(cols);
	return ((uint64_t)sw_packed_rows(stride) * pc * (uint64_t)hbytes + ((pc * 2u + 15u) & ~(uint64_t)15u) + 63u) &
	       ~(uint64_t)63u;
}

// Backtrace (sw_backtrace.hip): one lane per problem.
struct BtArgs {
	const bt2g_sw_problem* probs;
	uint32_t nprob;
	const uint8_t* reads;
	const uint8_t* quals;
	uint32_t stride;
	const uint32_t* lens;
	const uint8_t* windows;
	const uint8_t* ref_codes;
	const uint64_t* ref_starts;
	const bt2g_sw_rect* rects;        // may be null
	const bt2g_sw_result* res;
	const bt2g_sw_cand* cands;
	uint32_t cap;
	const uint8_t* plane;             // kinds 0/1: systolic score plane
	uint64_t slot;                    //   bytes per problem
	uint32_t cstride;                 //   rows per column (16-row blocks)
	uint32_t pcols;                   //   columns per row block
	int use_mask;                     //   per-column masks of written blocks (<= 16 blocks)
	int plane_top;                    //   0 systolic end-to-end, 1 top-aligned (per-lane fills), 2 systolic local
	uint32_t* marks;                  // per problem (mslot words): reportedThrough tiles
	uint64_t mslot;
	uint32_t rwords, rrows;           //   reportedThrough: diagonal tiles per tile row, tile rows
	uint32_t mwords, mrows;           //   FILT_DOMINATED squares: 8x8 tiles per tile row, tile rows
	uint64_t mdom;                    // local mode: word offset of the FILT_DOMINATED tiles
	SwConst C;
	int local;
	double ncl_const, ncl_lin;
	uint32_t maxaln, maxedit;
	int32_t* naln;
	bt2g_sw_aln* alns;
	bt2g_edit* edits;
	int8_t* fates;                    // may be null
	uint32_t* queue;                  // null: one DP per lane; else a zeroed counter: lanes take DPs from it
	int lds_marks_only;               // LDS-resident local walk: marks in LDS, the plane read in place
	int cands_lds;                    // LDS-resident local walk: the candidate list copied to LDS too
	int wpf;                          // LDS-resident local walk: 2 the walks in parallel (64 paths in LDS)
};
// kind: 0 u8 score plane, 1 u16 score plane, 2 decision nibbles (end-to-end u8 fills)
void launch_sw_bt(int kind, const BtArgs& a, hipStream_t st);
// sw_backtrace_wg.hip: one end-to-end kind-2 DP per workgroup, candidates walked
// in parallel; LDS bytes it needs for this launch's geometry
uint32_t sw_bt_wg_lds(const BtArgs& a);
void sw_bt_wg_lds_init(int dev);          // once per device, from bt2g_open
void sw_bt_lds_init(int dev);             // the LDS-resident local walk's opt-in, likewise
uint32_t sw_bt_wg_lds_limit();             // on the current device
void launch_sw_bt_wg(const BtArgs& a, uint32_t lds, hipStream_t st);

// uint4s of a problem's plane an LDS-resident walk copies (sw_backtrace.hip):
// kind 2 (decision planes) 8 B per 16-row block column; kind 1 (local u16
// planes) 32 B per block column, then the block masks (2 B per column) that the
// fill stores right after the plane
__host__ __device__ inline uint32_t sw_bt_lds_plane16(const BtArgs& a, int kind) {
	if(kind == 2) return (a.cstride >> 4) * a.pcols * 8u / 16u;
	if(a.lds_marks_only) return 0u;
	const uint64_t b = (uint64_t)(a.cstride >> 4) * a.pcols * 32u + (a.use_mask ? (uint64_t)a.pcols * 2u : 0u);
	return (uint32_t)((b + 15u) / 16u);
}

// backtrace mark scratch per problem of <= rows x cols (sw_backtrace.hip):
// reportedThrough in 8x8-cell bit tiles (2 words each) + one valid bit per
// tile; dom (local mode's dominated-candidate squares): a second set of the
// same shape.  (16-row x 4-diagonal reportedThrough tiles: 9 % more tile
// loads, the short failing walks are not diagonal runs.)
inline uint32_t sw_bt_rcols(uint32_t rows, uint32_t cols) { (void)rows; return (cols + 7u) / 8u; }
inline uint32_t sw_bt_rrows(uint32_t rows) { return (rows + 7u) / 8u; }
inline uint32_t sw_bt_tcols(uint32_t cols) { return (cols + 7u) / 8u; }
inline uint32_t sw_bt_trows(uint32_t rows) { return (rows + 7u) / 8u; }
inline uint64_t sw_bt_tiles_words(uint64_t tr, uint64_t tc) {
	return (tr * tc * 2u + tr * ((tc + 31u) / 32u) + 3u) & ~(uint64_t)3u;
}
// word offset of the dom tiles = the reportedThrough part
inline uint64_t sw_bt_mdom(uint32_t rows, uint32_t cols) {
	return sw_bt_tiles_words(sw_bt_rrows(rows), sw_bt_rcols(rows, cols));
}
inline uint64_t sw_bt_mslot(uint32_t rows, uint32_t cols, bool dom) {
	return sw_bt_mdom(rows, cols) + (dom ? sw_bt_tiles_words(sw_bt_trows(rows), sw_bt_tcols(cols)) : 0u);
}
// sw_pack.hip: outputs of launch_sw_bt packed per problem (cnt: 3n scratch,
// off: 3n + 3, totals last) into pc / pf (fates, may be null) / pe
void launch_sw_pack(const bt2g_sw_result* res, const int32_t* naln, const bt2g_sw_aln* alns,
                    const bt2g_sw_cand* cands, const int8_t* fates, const bt2g_edit* edits, uint32_t n, uint32_t cap,
                    uint32_t maxaln, uint32_t maxedit, uint32_t* cnt, uint32_t* off, bt2g_sw_cand* pc, int8_t* pf,
                    bt2g_edit* pe, hipStream_t st);
void launch_sort_cands(const bt2g_sw_result* res, bt2g_sw_cand* cands, uint32_t nprob, uint32_t cap,
                       uint32_t* big, uint32_t* nbig, hipStream_t st);

// DP framing (frame.hip): the scoring and framer parameters of one batch
struct FrameConst {
	int32_t match, rdgo, rdge, rfgo, rfge;   // bonus and gap open (incl. extension) / extension
	int32_t maxhalf, trim_to_ref;
	double ncl_const, ncl_lin;
};
void launch_frame(const bt2g_frame_in* in, uint32_t n, const uint32_t* lens, const uint64_t* ref_starts,
                  const FrameConst& F, const bt2g_pe_policy& P, bt2g_sw_problem* probs, bt2g_sw_rect* rects,
                  int32_t* ok, hipStream_t st);

void launch_ungapped(const bt2g_ug_problem* probs, uint32_t n, const uint8_t* reads, const uint8_t* quals,
                     uint32_t stride, const uint32_t* lens, const uint8_t* ref_codes, const uint64_t* ref_starts,
                     const SwConst& C, int local, double ncl_const, double ncl_lin, int ohang, uint32_t maxedit,
                     bt2g_ug_result* res, bt2g_edit* edits, hipStream_t st);
