/* bt2g_bench.h -- bench.py's device glue, NOT part of the product ABI.
 *
 * libbt2g_bench.so (built from bowtie2-server_amd/csrc/bench_frame.hip beside
 * libbt2g.so) exports these two functions for bench.py's kernel chain
 * (kernel_chain in the bench line): they stand in for the host logic between
 * the seed-phase calls and bt2g_sw_align_dev with a fixed policy, where the
 * reference chooses hits with RNG-driven prioritisation
 * (aligner_sw_driver.cpp:756-1297).  Nothing of the drop-in servers calls them.
 * Types: include/bt2g.h. */
#ifndef BT2G_BENCH_H
#define BT2G_BENCH_H
#include "bt2g.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Device-side glue used by bench.py between the seed-phase calls and
 * bt2g_sw_align_dev.  The reference's SwDriver::extendSeeds chooses hits with
 * RNG-driven prioritisation (aligner_sw_driver.cpp:756-1297); the bench's
 * fixed policy is documented in DESIGN.md section 5. */

/* Top SA rows of each read's exact end-to-end hit (sweep, as returned by
 * bt2g_exact_sweep_dev), 1-mm hits (mm, mm_cnt; cap mm_cap per read) and exact
 * seed hits (seeds of bt2g_seed_search_dev over the reads with inv[r] >= 0 at
 * compacted index inv[r]); contiguous per read at rows[read_base[r] ..
 * + read_cnt[r]), meta = fw << 31 | seed depth << 16 | hit length.  *total
 * (zeroed by the caller) receives the row count; beyond cap rows are dropped. */
int bt2g_bench_collect_rows_dev(uint32_t n, const uint32_t* lens, const uint32_t* sweep, const bt2g_mm1* mm,
                                const int32_t* mm_cnt, uint32_t mm_cap, const uint32_t* seeds, const int32_t* inv,
                                uint32_t maxseeds, uint32_t seedlen, uint32_t interval, uint32_t* rows,
                                uint32_t* meta, uint32_t* read_base, uint32_t* read_cnt, uint32_t* total,
                                uint32_t cap, void* stream);
/* Rows' joined offsets (bt2g_get_offset_dev) -> seed-extension frame inputs
 * (kind 0, off = the read's start on the reference) for bt2g_frame_dev: one
 * per distinct (strand, reference, diagonal), the two smallest per read;
 * fragments as in the .1.bt2 rstarts (joined offset, text id, text offset) plus
 * each fragment's joined end.  *nprob (zeroed by the caller) receives the
 * count. */
int bt2g_bench_frame_dev(uint32_t n, const uint32_t* lens, const uint32_t* offs, const uint32_t* meta,
                         const uint32_t* read_base, const uint32_t* read_cnt, const uint32_t* fr_joff,
                         const uint32_t* fr_tid, const uint32_t* fr_toff, const uint32_t* fr_end, uint32_t nfrag,
                         int32_t minsc, bt2g_frame_in* fin, uint32_t* nprob, uint32_t cap, void* stream);

#ifdef __cplusplus
}
#endif
#endif
