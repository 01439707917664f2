#!/usr/bin/env python3
"""bench.py -- reads aligned/sec of the bowtie2 seed-and-extend hot path on MI355X.

One "step" pushes a batch of synthetic 150 bp reads (resident in HBM) through
the GPU engines in the order bt2_search.cpp:3440-4020 chains the reference's
seams for an unpaired --end-to-end --sensitive read:

  1. exact end-to-end sweep, both strands     SeedAligner::exactSweep
  2. 1-mismatch end-to-end search, gated by 1  SeedAligner::oneMmSearch
  3. exact 22-mer seeds every 15 bp, round 0  instantiateSeeds + searchAllSeeds
     (reads without an exact end-to-end hit: those are EXTEND_PERFECT_SCORE)
  4. SA row -> text offset of the top row of every seed / exact / 1-mm hit
                                               Ebwt::getOffset (GroupWalk's job)
  5. one seed-extension DP rectangle per distinct hit diagonal (<= 2 per read),
     150 x 210, end-to-end u8 fill + candidate gather   SwAligner::align
  6. the driver's nextAlignment loop over every candidate of every aligned DP
     (backtrace, edits, core-diagonal / N-ceiling checks)  SwAligner::nextAlignment
  A read counts as aligned when it has an exact end-to-end hit or a DP that
  yields an alignment.  Glue between the stages is device code on the same stream.

The host decision logic of SwDriver (RNG-ranked seed prioritisation, streak
limits, MAPQ, SAM) is not on the GPU path; hg38
cannot be fetched, so the genome is a synthetic one of --genome-mb Mbp with
planted near-duplicate repeats and N runs, indexed byte-exactly as
bowtie2-build would (tools/bt2_index.py).

Multi-GPU: one process per GPU (torchrun), reads sharded by rank (weak
scaling), each GPU holds a full index replica; the only collective is the
all-reduce of the aligned-read counters and the max of the timings.
"""
import argparse
import concurrent.futures as cf
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "bowtie2-server_amd")
for _p in (ROOT, PKG, os.path.join(PKG, "tools"), os.path.join(ROOT, "tests", "golden")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# SW fill (VALU-bound): VALU lane-ops issued per DP cell by the systolic
# end-to-end fill incl. its decision plane (r02o, scripts/pmc_fill.sh:
# SQ_INSTS_VALU x 64 lanes / 3.15e10 cells per launch = 22.0; 11.9 with the H
# score plane, BT2G_BT_HPLANE=1), against two ceilings: the chip's VALU peak (256
# CUs x 128 lanes x 2.4 GHz = 78.6 T lane-ops/s) and the issue rate measured
# on the box for packed u16 / v_perm ops, which issue at half rate (37 T;
# profiles/r01_valu_rates.txt, full-rate ops 70 T)
VALU_OPS_PER_CELL = 11.9 if os.environ.get("BT2G_BT_HPLANE") == "1" else 22.0
VALU_PEAK_TOPS = 78.6
# algorithmic integer ops per DP cell: H = max(Hdiag - pen, E, F),
# E = max(E - ext, H - open), F likewise, with the gap-barrier vetoes
SW_OPS_PER_CELL = 10
# the kernel whose PMC counters make roofline.traffic (per bench kernel id)
PMC_KERNEL = {0: "k_exact_sweep", 1: "k_seed_search", 2: "k_one_mm", 3: "k_get_offset", 4: "k_sw_sys",
              12: "k_seed_extend"}
VALU_PACKED_TOPS = 37.0
SEEDLEN, INTERVAL = 22, 15     # --sensitive, 150 bp: -L 22, -i S,1,1.15 -> 1+1.15*sqrt(150) = 15


class Policy:
    """Per-mode seed and score policy (bt2_search.cpp presets).
    ee:     --end-to-end --sensitive: -L 22, -i S,1,1.15, --score-min L,-0.6,-0.6
    local:  --local --sensitive-local: -L 20, -i S,1,0.75, --score-min G,20,8, --ma 2
    paired: ee with the paired-end seed interval, --fr -I 0 -X 500 mate search
    preset "very-sensitive" (BASELINE configs[4]): -L 20, -i S,1,0.50 in every mode
    (bt2_search.cpp preset table; --very-sensitive-local has the same seed
    policy).  Its -D 20 -R 3 extension / re-seed limits belong to the host
    driver loop (row A11), which the bench does not model: round 0 only."""

    def __init__(self, mode, length, preset="sensitive"):
        import math
        self.mode, self.local, self.paired = mode, mode == "local", mode == "paired"
        self.preset = preset
        if preset == "very-sensitive":
            seedlen, interval = 20, int(1 + 0.50 * math.sqrt(length))
        elif self.local:
            seedlen, interval = 20, int(1 + 0.75 * math.sqrt(length))
        else:
            seedlen, interval = SEEDLEN, int(1 + 1.15 * math.sqrt(length))
        if self.paired:
            # paired-end: the seed interval is boosted (bt2_search.cpp:3392-3395)
            interval = int(interval * 1.2 + 0.5)
        self.seedlen, self.interval = seedlen, interval
        if self.local:
            self.minsc = int(20 + 8 * math.log(length))
        else:
            self.minsc = int(-0.6 - 0.6 * length)
MAXALN, MAXEDIT = 8, 64        # alignments kept per DP (the loop stops there); edits per alignment
                               # (150 bp, minsc -90, n-ceil 22: <= 22 N + 34 mismatches = 56)
MAXGAP = 15                    # min(max(read gaps, ref gaps), maxhalf=15), dp_framer.cpp:95-100
MAXHALF = 15                   # --dpad (bt2_search.cpp:486)
PE_MAXFRAG = 500               # -X (bt2_search.cpp:378); -I 0, --fr
MATE_CHUNK = 262_144           # mate-search DPs per fill + backtrace call (their score planes: 114 KB each)


def gap_budget(minsc, length):
    """max(Scoring::maxReadGaps, maxRefGaps) (scoring.cpp:42-98) for the
    default end-to-end scoring: gap open 8, extension 3, no match bonus."""
    return 1 + (0 - 8 - minsc) // 3 if -8 >= minsc else 0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_genome(mb, seed=2024, model="hg38like"):
    """Synthetic genome of mb Mbp in 8 references (2 below 8 Mbp).  model
    "hg38like" (default): tests/golden/synth.genome_hg38like -- Alu/L1-like
    interspersed repeat families with 3-20 % divergence, segmental duplications,
    microsatellites and N gaps at hg38's genome fractions; "simple": random
    sequence with planted 2 kb near-duplicates (round 1's bench genome)."""
    import synth
    n = int(mb * 1_000_000)
    if model == "hg38like":
        g = synth.genome_hg38like(seed, n)
    else:
        g = synth.genome(seed, n, n_repeats=max(1, n // 200_000), rep_len=2000, n_copies=3,
                         n_runs=max(1, n // 2_000_000))
    nref = 8 if n >= 8_000_000 else 2
    cuts = np.linspace(0, n, nref + 1).astype(np.int64)
    parts = [g[cuts[i]:cuts[i + 1]] for i in range(nref)]
    return parts, [b"chr%d" % (i + 1) for i in range(nref)]


def _reads_at(g, gpos, rc, length, rng):
    """Reads whose forward-strand windows start at genome positions gpos
    (BASELINE.md section 3 model: 1-bp indel in 5 %, 0.4 % substitutions,
    0.05 % N, Phred 2..40), reverse-complemented where rc."""
    n = len(gpos)
    win = g[gpos[:, None] + np.arange(length + 1)[None, :]]
    out = win[:, :length].copy()
    ind = np.nonzero(rng.random(n) < 0.05)[0]
    for i in ind:                                   # 1-bp indel in 5 % of reads
        k = rng.integers(1, length - 1)
        if rng.random() < 0.5:
            out[i, k:] = win[i, k + 1:length + 1]
        else:
            out[i, k + 1:] = win[i, k:length - 1]
            out[i, k] = rng.integers(0, 4)
    out[rc] = np.where(out[rc] > 3, 4, 3 - out[rc])[:, ::-1]
    m = rng.random((n, length)) < 0.004
    out[m] = (out[m] + rng.integers(1, 4, m.sum(), dtype=np.uint8)) % 4
    out[rng.random((n, length)) < 0.0005] = 4
    quals = (rng.integers(2, 41, (n, length), dtype=np.uint8) + 33).astype(np.uint8)
    return out.astype(np.uint8), quals


def _n_free_starts(rng, g, sizes, starts, n, span):
    """n fragment starts uniform over the genome's positions whose next `span`
    bases lie in one reference and hold no N (uniform over
    non-N positions)."""
    isn = np.concatenate([[0], np.cumsum(g == 4, dtype=np.int64)])
    out = np.empty(0, np.int64)
    while len(out) < n:
        m = int((n - len(out)) * 1.2) + 16
        ref = rng.choice(len(sizes), m, p=sizes / sizes.sum())
        pos = starts[ref] + (rng.random(m) * (sizes[ref] - span - 2)).astype(np.int64)
        ok = isn[pos + span] == isn[pos]
        out = np.concatenate([out, pos[ok]])
    return out[:n]


def make_reads(parts, n, length, seed):
    """Vectorised version of tests/golden/synth.reads (BASELINE.md section 3 model)."""
    rng = np.random.default_rng(seed)
    sizes = np.array([len(p) for p in parts], np.int64)
    starts = np.concatenate([[0], np.cumsum(sizes)])[:-1]
    g = np.concatenate(parts)
    gpos = _n_free_starts(rng, g, sizes, starts, n, length + 1)
    win = g[gpos[:, None] + np.arange(length + 1)[None, :]]
    out = win[:, :length].copy()
    ind = np.nonzero(rng.random(n) < 0.05)[0]
    for i in ind:                                   # 1-bp indel in 5 % of reads
        k = rng.integers(1, length - 1)
        if rng.random() < 0.5:
            out[i, k:] = win[i, k + 1:length + 1]
        else:
            out[i, k + 1:] = win[i, k:length - 1]
            out[i, k] = rng.integers(0, 4)
    fw = rng.random(n) >= 0.5
    rc = ~fw
    out[rc] = np.where(out[rc] > 3, 4, 3 - out[rc])[:, ::-1]
    m = rng.random((n, length)) < 0.004
    out[m] = (out[m] + rng.integers(1, 4, m.sum(), dtype=np.uint8)) % 4
    out[rng.random((n, length)) < 0.0005] = 4
    quals = (rng.integers(2, 41, (n, length), dtype=np.uint8) + 33).astype(np.uint8)
    return out.astype(np.uint8), quals


def make_pairs(parts, n, length, seed):
    """n read pairs (fragment ~N(300, 50) clipped to [200, 500],
    mates 2 x length in --fr orientation, the fragment from either strand).
    Returns 2n reads: mate 1 of pair i in row i, mate 2 in row n + i."""
    rng = np.random.default_rng(seed)
    sizes = np.array([len(p) for p in parts], np.int64)
    frag = np.clip(np.rint(rng.normal(300, 50, n)), 200, 500).astype(np.int64)
    frag = np.maximum(frag, length)
    starts = np.concatenate([[0], np.cumsum(sizes)])[:-1]
    g = np.concatenate(parts)
    left = _n_free_starts(rng, g, sizes, starts, n, 502)
    right = left + frag - length
    flip = rng.random(n) < 0.5                      # fragment from the reverse strand: mate 1 on the right
    r1, q1 = _reads_at(g, np.where(flip, right, left), flip, length, rng)
    r2, q2 = _reads_at(g, np.where(flip, left, right), ~flip, length, rng)
    return np.concatenate([r1, r2]), np.concatenate([q1, q2])


class Pipeline:
    """The per-step GPU work (see module docstring), torch glue on one stream."""

    def __init__(self, eng, idx, reads, quals, length, mode="ee", preset="sensitive"):
        import torch
        import bt2g
        self.pol = pol = Policy(mode, length, preset)
        self.torch, self.bt2g, self.L = torch, bt2g, bt2g.lib()
        self.eng = eng
        self.dev = reads.device
        self.n = reads.shape[0]
        self.len = length
        self.reads, self.quals = reads, quals
        self.lens = torch.full((self.n,), length, dtype=torch.int32, device=self.dev)
        self.minsc = torch.full((self.n,), pol.minsc, dtype=torch.int32, device=self.dev)
        self.sc = bt2g.scoring(pol.local)
        n = self.n
        self.maxseeds = 1 + (length - pol.seedlen) // pol.interval
        self.sweep = torch.empty((n, 8), dtype=torch.int32, device=self.dev)
        self.mm_cap = 16
        self.mm_hits = torch.empty((n, self.mm_cap, 8), dtype=torch.int32, device=self.dev)
        self.mm_cnt = torch.empty(n, dtype=torch.int32, device=self.dev)
        self.mm_ops = torch.empty(n, dtype=torch.int32, device=self.dev)
        self.mm_loads = torch.empty(n, dtype=torch.int32, device=self.dev)
        self.seeds = torch.empty((n, 2, self.maxseeds, 4), dtype=torch.int32, device=self.dev)
        self.nseeds = torch.empty(n, dtype=torch.int32, device=self.dev)
        self.sd_ops = torch.empty(n, dtype=torch.int32, device=self.dev)
        self.sd_loads = torch.empty(n, dtype=torch.int32, device=self.dev)
        rs = idx.fw.rstarts.astype(np.int64).reshape(-1, 3)
        self.fr_joff = torch.tensor(rs[:, 0], device=self.dev)
        self.fr_tid = torch.tensor(rs[:, 1], device=self.dev)
        self.fr_toff = torch.tensor(rs[:, 2], device=self.dev)
        fr_end = np.concatenate([rs[1:, 0], [idx.fw.length]])
        self.fr_end = torch.tensor(fr_end, device=self.dev)
        self.fr = [torch.tensor(a.astype(np.uint32), device=self.dev)
                   for a in (rs[:, 0], rs[:, 1], rs[:, 2], fr_end)]      # joff, tid, toff, end
        self.nfrag = int(rs.shape[0])
        self.inv = torch.empty(n, dtype=torch.int32, device=self.dev)
        self.row_cap = n * (1 + self.mm_cap + 2 * self.maxseeds)
        self.rows = torch.empty(self.row_cap, dtype=torch.int32, device=self.dev)
        self.meta = torch.empty(self.row_cap, dtype=torch.int32, device=self.dev)
        self.offs = torch.empty(self.row_cap, dtype=torch.int32, device=self.dev)
        self.loads_off = torch.empty(self.row_cap, dtype=torch.int32, device=self.dev)
        self.read_base = torch.empty(n, dtype=torch.int32, device=self.dev)
        self.read_cnt = torch.empty(n, dtype=torch.int32, device=self.dev)
        self.counters = torch.zeros(2, dtype=torch.int32, device=self.dev)   # rows, problems
        self.ncol = length + 4 * MAXGAP
        self.max_probs = 2 * n
        self.probs = torch.zeros((self.max_probs, 5), dtype=torch.int64, device=self.dev)
        _chk = bt2g._chk
        # fill + backtrace scratch: u8 score plane (end-to-end, minsc >= -254);
        # u16 for the local fills
        _chk(self.L.bt2g_reserve_sw_bt(eng.h, self.max_probs, length, self.ncol, 2 if pol.local else 1))
        # candidate cells per DP: end-to-end gathers the last row only; local
        # gathers every match-then-mismatch cell >= minsc (~1200 per 150 bp hit)
        self.sw_cap = 2048 if pol.local else 256
        self.res = torch.empty((self.max_probs, 8), dtype=torch.int32, device=self.dev)
        self.cands = torch.empty((self.max_probs, self.sw_cap, 3), dtype=torch.int32, device=self.dev)
        # seed-extension frame inputs (bt2g_frame_in) -> rectangles of DynProgFramer::
        # frameSeedExtensionRect (trimmed at the reference ends, core diagonals; dp_framer.cpp:81-129)
        self.fin0 = torch.zeros((self.max_probs, 10), dtype=torch.int32, device=self.dev)
        self.probs0 = torch.zeros((self.max_probs, 5), dtype=torch.int64, device=self.dev)
        self.rects0 = torch.zeros((self.max_probs, 4), dtype=torch.int32, device=self.dev)
        self.fok = torch.zeros(self.max_probs, dtype=torch.int32, device=self.dev)
        self.maxaln, self.maxedit = MAXALN, MAXEDIT
        self.naln = torch.empty(self.max_probs, dtype=torch.int32, device=self.dev)
        self.alns = torch.empty((self.max_probs, self.maxaln, 10), dtype=torch.int32, device=self.dev)
        self.edits = torch.empty((self.max_probs, self.maxaln, self.maxedit, 2), dtype=torch.int32, device=self.dev)
        self.stats = {}
        self._timing = None
        if pol.paired:
            # mate search (SwDriver::extendSeedsPaired, aligner_sw_driver.cpp:1975-2100):
            # its own context on the same index, reserved for the mate rectangles
            # (otherMate + frameFindMateRect: maxfrag + len - 1 + 2 max(gaps, maxhalf) columns)
            self.npairs = P = n // 2
            self.mate_cols = PE_MAXFRAG + length - 1 + 2 * max(gap_budget(pol.minsc, length), MAXHALF)
            self.mate_chunk = ch = min(P, MATE_CHUNK)
            self.eng2 = bt2g.Engine(index=idx, device=self.dev.index or 0)
            _chk(self.L.bt2g_reserve_sw_bt(self.eng2.h, ch, length, self.mate_cols, 1))
            self.pe = bt2g.pe_policy()
            self.fin = torch.zeros((P, 10), dtype=torch.int32, device=self.dev)     # bt2g_frame_in
            self.mprobs = torch.zeros((P, 5), dtype=torch.int64, device=self.dev)
            self.mrects = torch.zeros((P, 4), dtype=torch.int32, device=self.dev)
            self.mok = torch.zeros(P, dtype=torch.int32, device=self.dev)
            self.mres = torch.empty((ch, 8), dtype=torch.int32, device=self.dev)
            self.mcands = torch.empty((ch, self.sw_cap, 3), dtype=torch.int32, device=self.dev)
            self.mnaln = torch.empty(ch, dtype=torch.int32, device=self.dev)
            self.malns = torch.empty((ch, self.maxaln, 10), dtype=torch.int32, device=self.dev)
            self.medits = torch.empty((ch, self.maxaln, self.maxedit, 2), dtype=torch.int32, device=self.dev)

    def _p(self, t):
        return C.c_void_p(t.data_ptr())

    def _mark(self, name):
        """Phase boundary: the stream is drained here (measured faster than letting
        the host run ahead into the next phase's glue: 196 vs 268-303 ms per paired
        step); BT2G_BENCH_TIMING=1 also logs the phase times."""
        self.torch.cuda.current_stream().synchronize()
        if self._timing is not None:
            self._timing.append((name, time.perf_counter()))

    def _overflow(self, h, probs, rects, npb, res, naln, alns, edits, S):
        """DPs whose candidate list outgrew the call's cap (naln -5, the engine's
        'list truncated' mark) are run again with room for all of them, as the
        reference keeps every candidate (SwAligner::align; the drop-in binding
        does the same): the local fill finds > 2048 candidates in some repeat
        windows of the hg38-like genome."""
        torch, L, bt2g = self.torch, self.L, self.bt2g
        over = torch.nonzero(naln[:npb] == -5).squeeze(1)
        k = int(over.numel())
        if k == 0:
            return
        cap = min(8192, int(res[:npb, 6].index_select(0, over).max()))
        dev, P = self.dev, self._p
        r2 = torch.empty((k, 8), dtype=torch.int32, device=dev)
        c2 = torch.empty((k, cap, 3), dtype=torch.int32, device=dev)
        n2 = torch.empty(k, dtype=torch.int32, device=dev)
        a2 = torch.empty((k, self.maxaln, 10), dtype=torch.int32, device=dev)
        e2 = torch.empty((k, self.maxaln, self.maxedit, 2), dtype=torch.int32, device=dev)
        p2, q2 = probs.index_select(0, over).contiguous(), rects.index_select(0, over).contiguous()
        bt2g._chk(L.bt2g_sw_align_bt_dev(h, P(self.reads), P(self.quals), self.len, P(self.lens), P(p2), k, None,
                                         P(q2), C.byref(self.sc), 1, cap, P(r2), P(c2), self.maxaln, self.maxedit,
                                         P(n2), P(a2), P(e2), None, S))
        res[over] = r2
        naln[over] = n2
        alns[over] = a2
        edits[over] = e2
        self.stats["cand_overflow_reruns"] = self.stats.get("cand_overflow_reruns", 0) + k

    def step(self, keep=False):
        torch, L, bt2g = self.torch, self.L, self.bt2g
        self._timing = [("start", time.perf_counter())] if os.environ.get("BT2G_BENCH_TIMING") else None
        if self._timing is not None:
            torch.cuda.synchronize()
        S = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        h, n, stride = self.eng.h, self.n, self.len
        chk = bt2g._chk
        u32 = 0xFFFFFFFF
        # 1. exact end-to-end sweep
        chk(L.bt2g_exact_sweep_dev(h, self._p(self.reads), stride, self._p(self.lens), n, 2, 0, 0,
                                   self._p(self.sweep), S))
        # 2. 1-mismatch search gated by the sweep (bt2_search.cpp:3640-3667)
        chk(L.bt2g_one_mm_gated_dev(h, self._p(self.reads), self._p(self.quals), stride, self._p(self.lens), n,
                                    self._p(self.minsc), C.byref(self.sc), self._p(self.sweep), self.mm_cap,
                                    self._p(self.mm_hits), self._p(self.mm_cnt), self._p(self.mm_ops),
                                    self._p(self.mm_loads), S))
        self._mark("sweep+1mm")
        sw = self.sweep.to(torch.int64) & u32
        exact = torch.minimum(sw[:, 0], sw[:, 1]) == 0
        # 3. seed round 0 for reads without an exact end-to-end hit
        sel = torch.nonzero(~exact).squeeze(1)
        m = int(sel.numel())
        sreads = self.reads.index_select(0, sel)
        pol = self.pol
        chk(L.bt2g_seed_search_dev(h, self._p(sreads), stride, self._p(self.lens), m, pol.seedlen, pol.interval, 0,
                                   self.maxseeds, self._p(self.seeds), self._p(self.nseeds), self._p(self.sd_ops),
                                   self._p(self.sd_loads), S))
        self._mark("seeds")
        # 4. every read's hit rows (exact, 1-mm, seeds) -> one list, contiguous per read
        self.inv.fill_(-1)
        self.inv[sel] = torch.arange(m, dtype=torch.int32, device=self.dev)
        self.counters.zero_()
        P = self._p
        chk(self.bt2g.bench_lib().bt2g_bench_collect_rows_dev(n, P(self.lens), P(self.sweep), P(self.mm_hits), P(self.mm_cnt),
                                          self.mm_cap, P(self.seeds), P(self.inv), self.maxseeds, pol.seedlen,
                                          pol.interval,
                                          P(self.rows), P(self.meta), P(self.read_base), P(self.read_cnt),
                                          P(self.counters), self.row_cap, S))
        nrows = int(self.counters[0])
        self._mark("rows")
        # 5. SA rows -> joined-text offsets
        chk(L.bt2g_get_offset_dev(h, P(self.rows), nrows, P(self.offs), P(self.loads_off), S))
        self._mark("offsets")
        # 6. joinedToTextOff + straddle filter, <= 2 diagonals per read (device), framed by
        #    frameSeedExtensionRect (bt2g_frame_dev kind 0)
        chk(self.bt2g.bench_lib().bt2g_bench_frame_dev(n, P(self.lens), P(self.offs), P(self.meta), P(self.read_base),
                                   P(self.read_cnt), P(self.fr[0]), P(self.fr[1]), P(self.fr[2]), P(self.fr[3]),
                                   self.nfrag, pol.minsc, P(self.fin0),
                                   P(self.counters[1:]), self.max_probs, S))
        nfin = min(int(self.counters[1]), self.max_probs)
        chk(L.bt2g_frame_dev(h, P(self.fin0), nfin, P(self.lens), C.byref(self.sc), None, MAXHALF, 1,
                             P(self.probs0), P(self.rects0), P(self.fok), S))
        okp = torch.nonzero(self.fok[:nfin]).squeeze(1)
        npb = int(okp.numel())
        if npb == nfin:
            probs, self.rects = self.probs0[:npb], self.rects0[:npb]
        else:                                           # rectangles trimmed away entirely
            probs, self.rects = self.probs0.index_select(0, okp), self.rects0.index_select(0, okp)
        self._mark("frame")
        # 7. fill + candidates + the nextAlignment loop (backtraces)
        chk(L.bt2g_sw_align_bt_dev(h, P(self.reads), P(self.quals), stride, P(self.lens),
                                   P(probs), npb, None, P(self.rects), C.byref(self.sc), 1, self.sw_cap,
                                   P(self.res), P(self.cands), self.maxaln, self.maxedit, P(self.naln),
                                   P(self.alns), P(self.edits), None, S))
        self._overflow(h, probs, self.rects, npb, self.res, self.naln, self.alns, self.edits, S)
        self._mark("sw")
        # end-to-end: an exact end-to-end hit is the alignment (EXTEND_PERFECT_SCORE);
        # local: every read's hits, the exact ones included, go through the DP
        aligned = torch.zeros_like(exact) if pol.local else exact.clone()
        al = self.naln[:npb] > 0
        aligned[probs.view(torch.int32)[:, 0][al].to(torch.int64)] = True
        ns = 0
        if keep:
            self.last = dict(sel=sel, rows=self.rows[:nrows], offs=self.offs[:nrows], probs=probs, npb=npb,
                             rects=self.rects, nrows=nrows, m=m, ns=ns, loads_off=self.loads_off[:nrows],
                             meta=self.meta[:nrows], read_base=self.read_base, read_cnt=self.read_cnt)
        if pol.paired:
            aligned = self.mates(probs, npb, aligned, keep, S)
        self._mark("end")
        if self._timing is not None:
            t = self._timing
            log("[timing] " + ", ".join(f"{t[i][0]} {1e3 * (t[i][1] - t[i - 1][1]):.1f}" for i in range(1, len(t))))
        return aligned

    def mates(self, probs, npb, aligned, keep, S):
        """Mate search for every pair with an aligned mate: the first alignment of
        mate 1 (else mate 2) is the anchor; otherMate + frameFindMateRect frame the
        opposite mate's window (bt2g_frame_dev, on the device) and the mate DPs
        run fill + nextAlignment loop in chunks.  Returns the pairs with an
        aligned mate; counts the pairs whose mate search found the opposite mate."""
        torch, L, chk, P = self.torch, self.L, self.bt2g._chk, self._p
        npairs, dev = self.npairs, self.dev
        rid = probs.view(torch.int32)[:, 0].to(torch.int64)
        dpi = torch.arange(npb, device=dev)
        al = self.naln[:npb] > 0
        first = torch.full((self.n,), npb, dtype=torch.int64, device=dev)
        first.scatter_reduce_(0, rid[al], dpi[al], reduce="amin")
        f1, f2 = first[:npairs], first[npairs:]
        has1, has2 = f1 < npb, f2 < npb
        use = torch.nonzero(has1 | has2).squeeze(1)
        a1 = has1[use]
        dp = torch.where(a1, f1[use], f2[use])
        pw = probs.view(torch.int32)
        na = int(use.numel())
        fin = self.fin[:na]
        fin.zero_()
        fin.view(torch.int64)[:, 0] = probs[dp, 1] + self.alns[dp, 0, 2].to(torch.int64)   # anchor refoff
        fin[:, 2] = torch.where(a1, use + npairs, use).to(torch.int32)                       # opposite mate
        fin[:, 3] = pw[dp, 6]                                                                # refidx
        fin[:, 4] = self.pol.minsc
        fin[:, 5] = pw[dp, 1]                                                                # anchor strand
        fin[:, 6] = 1                                                                        # mate search
        fin[:, 7] = a1.to(torch.int32)
        fin[:, 8] = self.len
        self._mark("anchors")
        chk(L.bt2g_frame_dev(self.eng2.h, P(fin), na, P(self.lens), C.byref(self.sc), C.byref(self.pe), MAXHALF,
                             1, P(self.mprobs), P(self.mrects), P(self.mok), S))
        kept = torch.nonzero(self.mok[:na]).squeeze(1)
        nm = int(kept.numel())
        mp = self.mprobs[:na].index_select(0, kept)
        mr = self.mrects[:na].index_select(0, kept)
        if nm and int(mp.view(torch.int32)[:, 7].max()) > self.mate_cols:
            raise RuntimeError("mate rectangle wider than the reservation")
        found = torch.zeros(npairs, dtype=torch.bool, device=dev)
        pair_of = use.index_select(0, kept)
        self._mark("mate_frame")
        for c0 in range(0, nm, self.mate_chunk):
            c1 = min(nm, c0 + self.mate_chunk)
            chk(L.bt2g_sw_align_bt_dev(self.eng2.h, P(self.reads), P(self.quals), self.len, P(self.lens),
                                       P(mp[c0:c1]), c1 - c0, None, P(mr[c0:c1]), C.byref(self.sc), 1, self.sw_cap,
                                       P(self.mres), P(self.mcands), self.maxaln, self.maxedit, P(self.mnaln),
                                       P(self.malns), P(self.medits), None, S))
            self._overflow(self.eng2.h, mp[c0:c1], mr[c0:c1], c1 - c0, self.mres, self.mnaln, self.malns,
                           self.medits, S)
            found[pair_of[c0:c1][self.mnaln[:c1 - c0] > 0]] = True
        self._mark("mate_dps")
        if keep:
            self.last.update(m_anchors=na, m_dps=nm, m_found=int(found.sum()), m_probs=mp, m_rects=mr,
                             m_pairs=pair_of, m_fin=fin.index_select(0, kept))
        return aligned[:npairs] | aligned[npairs:]


def pmc_traffic(fetch_csv, write_csv, kernel):
    """HBM bytes per launch of `kernel` from separate rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes of the same command (counter values in KiB per dispatch;
    FETCH_SIZE is uncalibrated for 64-B gathers on gfx950)."""
    import csv
    if not fetch_csv or not write_csv:
        return None
    import collections
    total = 0.0
    for path in (fetch_csv, write_csv):
        per = collections.defaultdict(list)          # every kernel of the API call (k_one_mm_near<true>, ...)
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            if name == kernel or name.startswith(kernel + "_") or name.startswith(kernel + "<"):
                per[name].append(float(r["Counter_Value"]))
        if not per:
            return None
        total += sum(sum(v) / len(v) for v in per.values()) * 1024
    return total


# ($BT2G_BENCH_SERVER_BIN: another build of it, for A/B runs on one lease)
BATCH_SERVER = os.environ.get("BT2G_BENCH_SERVER_BIN") or os.path.join(ROOT, "integration", "bin",
                                                                     "bowtie2-align-server-batch")
# HBM traffic per launch of the batch server's kernels: the summary of separate
# rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this same bench command
# (scripts/gpu_r06.sh prof -> scripts/pmc_summary.py), committed under profiles/
SERVER_PMC = os.path.join(ROOT, "profiles", "r06", "server_pmc.json")


def server_traffic(path, kernel):
    """(bytes per launch, note) of `kernel` (name prefix) from a pmc_summary.py
    file: FETCH_SIZE doubled (gfx950 counts 64 B per 128-B request) + WRITE_SIZE,
    summed over the kernel's instantiations weighted by their dispatches."""
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    tot, n = 0.0, 0
    for name, v in d.get("kernels", {}).items():
        if not (name == kernel or name.startswith(kernel + "<") or name.startswith(kernel + "_")):
            continue
        if v.get("fetch_bytes_x2") is None or v.get("write_bytes") is None:
            continue
        tot += (v["fetch_bytes_x2"] + v["write_bytes"]) * v["dispatches"]
        n += v["dispatches"]
    if not n:
        return None, None
    note = (f"{os.path.relpath(path, ROOT)}: FETCH_SIZE x 2 + WRITE_SIZE per dispatch of {kernel}* "
            f"({n} dispatches of separate --pmc passes of bench.py with rocprofv3 in front of the server)")
    lib = os.path.join(PKG, "libbt2g.so")
    want = (d.get("build_sha256") or {}).get("bowtie2-server_amd/libbt2g.so")
    if want is None:
        note += "; STALE? the summary records no build"
    elif os.path.exists(lib) and binary_id(lib)["sha256"] != want:
        note += "; STALE: taken on another build of libbt2g.so than the one benchmarked"
    return tot / n, note
# the engine services' kernel ids (bt2g_api.cpp ProfScope) by call kind, the
# kernels' names in the line, and their bound (None: no roofline, e.g. the DP
# call's whole stream span); the algorithmic work of each comes from the server
# per kernel id (FM kernels: bytes; the fill: DP cells)
SERVER_KERNELS = [("exact_sweep", 0, "k_exact_sweep", "hbm"),
                  ("exact_sweep", 2, "k_one_mm (items/q/near/far/branch/compact) in the sweep's call "
                                     "(bt2g_exact_sweep_1mm)", "hbm"),
                  ("exact_sweep", 3, "k_range_offsets (the sweep's small ranges' rows)", None),
                  ("seed_search", 1, "k_seed_search", "hbm"),
                  ("seed_search", 12, "k_seed_extend (SwDriver::extend of every seed range, bt2g_seed_search_ext)",
                   "hbm"),
                  ("seed_search", 3, "k_seed_offsets (the seed ranges' small rows)", None),
                  ("one_mm", 2, "k_one_mm (items/q/near/far/branch/compact)", "hbm"),
                  ("get_offset", 3, "k_get_offset", "hbm"), ("extend", 12, "k_extend", "hbm"),
                  ("ungapped", 6, "k_ungapped", None), ("sw_dp", 4, "k_sw_sys (fill, with the candidate gather)", "valu"),
                  ("sw_dp", 11, "k_sort_small / k_sort_big (candidate sort)", None),
                  ("sw_dp", 5, "k_sw_bt_wg / k_sw_bt (nextAlignment loop)", None),
                  ("sw_dp", 8, "host: the DP call's staging (packing into pinned memory)", "span"),
                  ("sw_dp", 9, "host: the DP call's enqueueing (copies and launches)", "span"),
                  ("sw_dp", 10, "host: the DP call's wait and copy out", "span"),
                  ("sw_dp", 7, "the DP call's whole stream span (copies, fill, walk, pack)", "span")]


def policy_args(mode, preset):
    """Server options of a bench mode (BASELINE.json configs)."""
    a = ["--local"] if mode == "local" else []
    if preset == "very-sensitive":
        a.append("--very-sensitive-local" if mode == "local" else "--very-sensitive")
    return a


def count_aligned(sam_texts, paired):
    """Reads (pairs) with an alignment in SAM text: primary records (no 0x100 /
    0x800) without 0x4; a pair counts when either mate aligned (its first
    mate's record: 0x4 or 0x8 clear)."""
    n = 0
    for t in sam_texts:
        for ln in t.split(b"\n"):
            if not ln or ln[:1] == b"@":
                continue
            a = ln.index(b"\t")
            flag = int(ln[a + 1:ln.index(b"\t", a + 1)])
            if flag & 0x900:
                continue
            if paired:
                if flag & 0x40 and (flag & 0xC) != 0xC:
                    n += 1
            elif not flag & 0x4:
                n += 1
    return n


def server_kernels(st):
    """Kernel times and algorithmic work of a batch-server run (its BT2G_KPROF
    stats: per engine service and kernel id, the HIP-event time of every launch
    and the algorithmic work of the requests it carried).  FM kernels: bytes =
    64 B per occurrence-table side gathered + the read bytes walked (SURVEY.md
    8(d), the figures of the chain below); the SW fill: SW_OPS_PER_CELL integer
    ops per DP cell."""
    out = {}
    ks = (st or {}).get("kernels") or {}
    for kind, kid, name, bound in SERVER_KERNELS:
        k = ks.get(kind)
        if not k:
            continue
        row = k["ids"][kid]
        launches, ms = row[0], row[1]
        work, items = (row[2], row[3]) if len(row) > 3 else (0, 0)
        if not launches:
            continue
        e = {"kernel": name, "launches": launches, "ms_total": ms, "ms_per_launch": ms / launches,
             "items": items}
        if bound == "span":
            e["span"] = True
        if (kind, kid) in FAMILY_IDS:
            e["family"] = True
        if bound == "hbm" and work:
            e.update(bound="hbm", bytes_total=work, bytes_per_launch=work / launches,
                     achieved=work / (ms / 1e3) / 1e9, unit="GB/s", peak=HBM_PEAK_GBS)
        elif bound == "valu" and work:
            e.update(bound="valu", cells_total=work, cells_per_launch=work / launches,
                     achieved=work * SW_OPS_PER_CELL / (ms / 1e3) / 1e12, unit="T int-ops/s", peak=VALU_PEAK_TOPS,
                     ops_per_cell=SW_OPS_PER_CELL)
        if "achieved" in e:
            e["frac"] = e["achieved"] / e["peak"]
        out[f"{kind}:{kid}"] = e
    return out


# ids whose time spans several kernels (the 1-mm search's items / near / far /
# branch / compact launches): a family, not one kernel
FAMILY_IDS = {("exact_sweep", 2), ("one_mm", 2)}

# kernel-name prefixes of each id in a rocprofv3 --pmc summary (the 1-mm family's
# kernels serve both the sweep's fused call and the rare standalone 1-mm call)
PMC_NAMES = {"exact_sweep:0": ("k_exact_sweep",), "exact_sweep:2": ("k_one_mm_",), "one_mm:2": ("k_one_mm_",),
             "exact_sweep:3": ("k_range_offsets",), "seed_search:1": ("k_seed_search",),
             "seed_search:12": ("k_seed_extend",), "seed_search:3": ("k_seed_offsets",),
             "get_offset:3": ("k_get_offset",), "extend:12": ("k_extend",), "ungapped:6": ("k_ungapped",),
             "sw_dp:4": ("k_sw_sys",), "sw_dp:5": ("k_sw_bt",), "sw_dp:11": ("k_sort_",)}


def dominant_kernel(kern):
    """The kernel -- or multi-kernel family, such as the 1-mm search's five
    launches per call -- with the largest total time over the run (the DP call's
    whole stream span is not one kernel).  round 6: families are candidates
    (the 1-mm family was the largest GPU consumer, ~28 % of kernel
    time, and the line named k_sw_sys)."""
    ks = [k for k in kern if not kern[k].get("span")]
    return max(ks, key=lambda k: kern[k]["ms_total"], default=None)


def line_rooflines(kern, server_pmc):
    """(roofline, rooflines) of a line: the largest consumer's roofline object and
    every kernel (family) with a bound, largest total time first.  When the
    largest consumer has no bound (--local: the backtrace, dependent plane reads
    and LDS mark tests whose per-step work the host does not see), the
    roofline is the largest kernel WITH one and names that consumer in
    `largest_consumer`."""
    dom_k = dominant_kernel(kern)
    rl, rls, largest = None, [], None
    if dom_k and "achieved" not in kern[dom_k]:
        largest = {"id": dom_k, "kernel": kern[dom_k]["kernel"], "ms_per_launch": kern[dom_k]["ms_per_launch"],
                   "share_of_kernel_time": kern[dom_k]["ms_total"] / max(1e-9, sum(
                       v["ms_total"] for v in kern.values() if not v.get("span"))),
                   "why_no_roofline": "dependent plane reads and LDS mark tests per DP (one workgroup per DP; "
                                      "local: ~55 walks over ~1 200 candidates, up to 64 walked at once, then "
                                      "resolved in the reference's order): latency-bound, and the host sees no "
                                      "per-step byte or op count"}
        bounded = [k for k in kern if "achieved" in kern[k] and not kern[k].get("span")]
        dom_k = max(bounded, key=lambda k: kern[k]["ms_total"], default=None)
    if dom_k:
        rl = roofline_entry(kern, dom_k, server_pmc)
        if largest:
            rl["largest_consumer"] = largest
        rl["note"] = ("kernel times: HIP events around every launch of the batch server's engine services "
                      "over warmup + timed passes (BT2G_KPROF); a family's time is its call's launches from "
                      "the first kernel's start to the last one's end; per-launch work: the algorithmic figure "
                      "of SURVEY.md 8(d) for the requests of each call.  Latency-bound here: the batch "
                      "server's calls carry a round's requests (hundreds to a few thousand items); the "
                      "throughput regime of the same kernels is kernel_chain.roofline")
    for k in sorted(kern, key=lambda k: -kern[k]["ms_total"]):
        if "achieved" in kern[k]:
            e = roofline_entry(kern, k, server_pmc)
            rls.append({"id": k, **{x: e[x] for x in ("kernel", "bound", "frac", "achieved", "unit",
                                                      "ms_per_launch", "share_of_kernel_time", "traffic",
                                                      "traffic_ratio", "per_launch_work")}})
    return rl, rls


def work_by_kernel(st):
    """{kind:id: [algorithmic work total, items]} of a run's server statistics
    (bytes for the FM kernels, DP cells for the fill): with a --pmc pass of the
    same command, the PMC-to-algorithmic traffic ratio of every kernel."""
    out = {}
    for kind, kid, _name, _bound in SERVER_KERNELS:
        row = (((st or {}).get("kernels") or {}).get(kind) or {}).get("ids")
        if row and len(row[kid]) > 3 and row[kid][2]:
            out[f"{kind}:{kid}"] = [row[kid][2], row[kid][3]]
    return out


def pmc_ratio(path, key):
    """(HBM bytes per algorithmic byte, note) of kernel id `key` from a
    pmc_summary.py file that carries the algorithmic work of its own passes:
    FETCH_SIZE x 2 over every dispatch of the id's kernels in the FETCH pass,
    over the algorithmic bytes the server counted in that pass, plus the same
    for WRITE_SIZE in the WRITE pass (each --pmc pass is its own run of the
    same bench command)."""
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    works = d.get("work_by_kernel") or {}
    names = PMC_NAMES.get(key)
    if not names or not all(key in (works.get(c) or {}) for c in ("fetch", "write")):
        return None, None

    def alg(c):                     # the id's work, with the ids sharing its kernels
        w = works[c]
        return sum(w[k][0] for k in w if k == key or PMC_NAMES.get(k) == names)

    fx2, wr, nd = 0.0, 0.0, 0
    for name, v in d.get("kernels", {}).items():
        if not any(name.startswith(p) for p in names):
            continue
        if v.get("fetch_bytes_x2") is None or v.get("write_bytes") is None:
            continue
        fx2 += v["fetch_bytes_x2"] * v["dispatches"]
        wr += v["write_bytes"] * v["dispatches"]
        nd += v["dispatches"]
    if not nd or not alg("fetch") or not alg("write"):
        return None, None
    ratio = fx2 / alg("fetch") + wr / alg("write")
    note = (f"{os.path.relpath(path, ROOT)}: FETCH_SIZE x 2 + WRITE_SIZE over {nd} dispatches of "
            f"{'/'.join(names)}* in separate rocprofv3 --pmc passes of bench.py, each over the algorithmic bytes the "
            f"server counted in the same pass (ratio {ratio:.2f}; traffic = ratio x this run's bytes per launch)")
    lib = os.path.join(PKG, "libbt2g.so")
    want = (d.get("build_sha256") or {}).get("bowtie2-server_amd/libbt2g.so")
    if want is None:
        note += "; STALE? the summary records no build"
    elif os.path.exists(lib) and binary_id(lib)["sha256"] != want:
        note += "; STALE: taken on another build of libbt2g.so than the one benchmarked"
    return ratio, note


def roofline_entry(kern, key, server_pmc):
    """The line's roofline object for kernel id `key` of server_kernels."""
    d = kern[key]
    ratio, tnote = pmc_ratio(server_pmc, key)
    per = (d.get("bytes_total") or d.get("cells_total")) / d["launches"]
    if ratio is not None and d["bound"] == "hbm":
        traffic = ratio * per
    elif d.get("family"):
        ratio, traffic, tnote = None, None, "no PMC summary with this run's algorithmic work (work_by_kernel)"
    else:
        ratio = None
        traffic, tnote = server_traffic(server_pmc, PMC_KERNEL.get(int(key.split(":")[1]), "?"))
    return {"bound": d["bound"], "kernel": d["kernel"], "family": bool(d.get("family")), "achieved": d["achieved"],
            "peak": d["peak"], "unit": d["unit"], "frac": d["frac"], "traffic": traffic, "traffic_ratio": ratio,
            "traffic_source": tnote, "ms_per_launch": d["ms_per_launch"], "launches": d["launches"],
            "ms_total": d["ms_total"],
            "share_of_kernel_time": d["ms_total"] / sum(v["ms_total"] for v in kern.values() if not v.get("span")),
            "per_launch_work": per, "work_unit": "bytes" if d["bound"] == "hbm" else "DP cells"}


# host memory of one batch server (r05d, 16 drivers, hg38-like genome): ~12 GB
# without slots (the reference's index on the host, the engines' pinned staging,
# the HIP runtime) + ~2.8 MB per read slot (the reference's per-read objects and
# the slot's cache pools after pool_trim), plus ~10 GB for the bench process
SERVER_BASE_GB, SLOT_MB, BENCH_PROC_GB = 12.0, 2.8, 10.0


def slots_per_driver(world, drivers, rank_mem_gb=0.0, mode="ee"):
    """Reads in flight per driver thread ($BT2G_BATCH_SLOTS) within a per-rank
    host-memory budget: one GPU keeps the server's default (1 024; --local 2 048:
    its rounds wait on ~12 ms DP calls -- the local walks, one per workgroup -- with
    the drivers' CPU mostly idle, so reads in flight are its throughput: r05n 45 k
    -> 65 k aligned reads/s at 64 -> 108 GB of host memory); with several ranks
    per node every rank's server and bench process must fit rank_mem_gb (default
    56 GB: 8 ranks in ~450 GB of the node's host memory)."""
    if world <= 1 and not rank_mem_gb:
        return 2048 if mode == "local" else 1024
    budget = rank_mem_gb or 56.0
    per = int((budget - BENCH_PROC_GB - SERVER_BASE_GB) * 1024 / (drivers * SLOT_MB))
    return max(128, min(1024, per // 64 * 64))


def schedule_run(args, rank, world, local, base, reads_np, quals_np, workdir, binary=None):
    """The north-star number: the reference's real schedule -- its server,
    client, per-read logic and SAM -- with the batch-first driver
    (integration/bt2g_batch.cpp) on this rank's GPU.  The reads go out in
    <= 10 000-read client connections, args.clients at a time (BASELINE.md
    section 3; the same k as the stock server below).  Warmup: the first
    args.warmup_chunks chunks, args.warmup times (the server's slots and
    caches reach their working size); then args.steps timed passes over every
    chunk, bracketed by barriers across ranks.  Returns the timing, the
    aligned count (from the SAM), the last pass's SAM texts and the server's
    engine statistics."""
    import torch
    import torch.distributed as dist
    import serve as rs
    binary = binary or BATCH_SERVER
    client = client_binary(args)
    if not os.path.exists(binary):
        raise RuntimeError(f"{binary} is not built (python -c 'import __graft_entry__ as g; g.build()')")
    gpu = torch.cuda.is_available()
    paired = args.mode == "paired"
    n = args.reads
    if paired:
        chunks = rs.write_fastq_chunks(workdir, reads_np[:n], quals_np[:n], codes2=reads_np[n:], quals2=quals_np[n:])
    else:
        chunks = rs.write_fastq_chunks(workdir, reads_np, quals_np)
    stats = os.path.join(workdir, "stats.json")
    env = rs.dropin_env(base, stats, device=local)
    env["BT2G_KPROF"] = "1"
    slots = int(os.environ.get("BT2G_BATCH_SLOTS") or
                slots_per_driver(world, args.drivers, getattr(args, "rank_mem_gb", 0.0), args.mode))
    env["BT2G_BATCH_SLOTS"] = str(slots)
    # $BT2G_BENCH_SERVER_PREFIX: a profiler in front of the batch server's command line
    # (e.g. "rocprofv3 --kernel-trace --stats -d DIR -o run --"); the server then exits
    # through exit() at SIGTERM so that the profile is written
    import shlex
    prefix = tuple(shlex.split(os.environ.get("BT2G_BENCH_SERVER_PREFIX", "")))
    if prefix:
        env["BT2G_EXIT_CLEAN"] = "1"
        # the profiler times the kernels itself; the engines' own HIP-event timing
        # under rocprofv3 faulted inside librocprofiler-sdk (r04ag, r05h: SIGSEGV under
        # hipEventRecord of ProfScope::~ProfScope, DP service threads) -- off unless
        # $BT2G_BENCH_KPROF=1
        env["BT2G_KPROF"] = os.environ.get("BT2G_BENCH_KPROF", "0")
        # (the algorithmic work by kernel id is still counted: a --pmc pass sets its
        # counters against the work of the same dispatches, bench.pmc_ratio)
        env["BT2G_KWORK"] = "1"
    multi = world > 1 and dist.is_initialized()
    with rs.Server(base, threads=args.drivers, args=policy_args(args.mode, args.preset), binary=binary,
                   env=env, log_path=os.path.join(workdir, "server.log"), prefix=prefix) as srv:
        log(f"[rank {rank}] batch server ready in {srv.load_s:.1f}s (-p {args.drivers})")
        for _ in range(args.warmup):
            srv.run(chunks[:args.warmup_chunks] if args.warmup_chunks > 0 else chunks, k=args.clients, client=client)
        if multi:
            dist.barrier()
        if gpu:
            torch.cuda.synchronize()
        rss = [srv.last_rss_gb]                 # after the warmup, then after every timed pass
        native = os.path.basename(client) == os.path.basename(rs.NATIVE_CLIENT)
        t0 = time.perf_counter()
        aligned, outs, cpu_s, client_s, host_s, thr_s, run_s = 0, None, 0.0, 0.0, 0.0, 0.0, 0.0
        pass_s, client_aligned = [], []
        for i in range(args.steps):
            last = i + 1 == args.steps
            # (the aligned reads of a pass are counted by the native client as the SAM
            # arrives; only the last pass's SAM is kept, for sam_parity, and counted
            # again here after the timed region -- counting 1 M records in Python took
            # ~1 s per pass, inside the timed region, with the server idle)
            dt_i, outs = srv.run(chunks, k=args.clients, client=client, keep=last or not native)
            cpu_s += srv.last_cpu_s
            client_s += srv.last_client_cpu_s
            host_s += srv.last_host_cpu_s
            thr_s += srv.last_throttled_s
            run_s += dt_i
            pass_s.append(dt_i)
            rss.append(srv.last_rss_gb)
            if native:
                client_aligned.append(srv.last_aligned)
                aligned += srv.last_aligned
            else:
                aligned += count_aligned(outs, paired)
            log(f"[rank {rank}] pass {i + 1}/{args.steps}: {dt_i:.3f} s, server RSS {rss[-1]:.1f} GB")
        if gpu:
            torch.cuda.synchronize()
        if multi:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if native and outs is not None:
            # the client's count of the last pass against the SAM it returned
            py = count_aligned(outs, paired)
            if py != client_aligned[-1]:
                raise RuntimeError(f"aligned count: client {client_aligned[-1]} vs SAM {py}")
        threads_cpu = srv.last_threads
        smaps = srv.smaps_top()
    st = None
    for _ in range(50):                         # written by the server at SIGTERM
        if os.path.exists(stats):
            try:
                st = json.load(open(stats))
                break
            except ValueError:
                pass
        time.sleep(0.1)
    return {"elapsed": elapsed, "aligned": aligned, "outs": outs, "chunks": chunks, "stats": st, "slots_per_driver": slots,
            "server_cpu_s": cpu_s, "client_cpu_s": client_s, "host_cpu_s": host_s, "throttled_s": thr_s,
            "passes_s": run_s, "pass_s": pass_s, "server_threads_cpu": threads_cpu, "server_rss_gb": rss[-1],
            "server_rss_gb_per_pass": rss, "binary": binary_id(binary), "client": binary_id(client),
            "smaps_top": smaps}


def client_binary(args):
    """The client that sends the reads: this repository's multi-connection client
    (integration/bin/bt2g-client, row (f)-4: one process, args.clients
    connections, SAM identical to the reference client's, tests/test_client.py)
    or, with --client reference, one reference client process per chunk
    (oracle/_ref/bowtie2-align-l, A/B runs)."""
    if getattr(args, "client", "native") == "reference":
        return os.path.join(ROOT, "oracle", "_ref", "bowtie2-align-l")
    import serve
    if not os.path.exists(serve.NATIVE_CLIENT):
        raise RuntimeError(f"{serve.NATIVE_CLIENT} is not built (make -C integration client)")
    return serve.NATIVE_CLIENT


def binary_id(path):
    """Which server binary ran: its path, size and sha256 (the box runs the
    prebuilt file the snapshot carried)."""
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return {"path": os.path.relpath(path, ROOT), "bytes": os.path.getsize(path), "sha256": h.hexdigest()}


def stock_baseline(args, base, chunks, batch_outs, workdir):
    """cpu_baseline: the stock reference server (oracle/_ref/bowtie2-align-server-s,
    built from /root/reference by oracle/ref/Makefile, -p <usable cores>) on
    the first args.stock_sample reads of the same chunks, same k and warmup,
    through the reference's own client (bowtie2-align-l, one process per
    connection); args.stock_runs timed runs, the median reported (BASELINE.md
    section 3).  Its sorted SAM against the batch server's for those chunks
    (which bt2g-client received): the engines and the client are checked
    against the reference server and client together."""
    from oracle import ref_server as rs
    host = rs.host_cpus()
    threads = args.cpu_threads or host["usable"]
    m = max(1, min(len(chunks), (args.stock_sample + rs.CHUNK - 1) // rs.CHUNK))
    sample = chunks[:m]
    paired = args.mode == "paired"
    runs = []
    cpus = rs.serve.pinned_cpus()     # (the CPUs the batch server pinned itself to, if it did)
    with rs.Server(base, threads=threads, args=policy_args(args.mode, args.preset), binary=rs.SERVER,
                   log_path=os.path.join(workdir, "server_stock.log"), cpus=cpus) as srv:
        for _ in range(args.warmup):
            srv.run(sample[:min(args.warmup_chunks, m)] if args.warmup_chunks > 0 else sample, k=args.clients)
        for _ in range(max(1, getattr(args, "stock_runs", 3))):
            dt, outs = srv.run(sample, k=args.clients)
            runs.append({"seconds": dt, "aligned": count_aligned(outs, paired), "server_cpu_s": srv.last_cpu_s,
                         "client_cpu_s": srv.last_client_cpu_s})
    a, b = rs.sorted_records(outs), rs.sorted_records(batch_outs[:m])
    differ = sum(1 for x, y in zip(a, b) if x != y) + abs(len(a) - len(b))
    nreads = min(args.reads, m * rs.CHUNK)
    unit = "read pairs/s" if paired else "reads/s"
    med = sorted(runs, key=lambda r: r["seconds"])[len(runs) // 2]
    dt = med["seconds"]
    return {"value": med["aligned"] / dt, "unit": "aligned " + unit, "cores": threads,
            "kind": "reference", "host": host, "reads_per_s": nreads / dt, "seconds": dt,
            "server_cpu_s": med["server_cpu_s"], "client_cpu_s": med["client_cpu_s"],
            "runs": [{"value": r["aligned"] / r["seconds"], "seconds": r["seconds"]} for r in runs],
            "sample": f"the stock reference server (bowtie2-align-server-s built from the reference's sources, "
                      f"-p {threads} = the usable cores of this host, {host['model']}) on the first {nreads} "
                      f"{'pairs' if paired else 'reads'} of the batch through the reference client "
                      f"(bowtie2-align-l), <= 10 000 per client connection, {args.clients} connections at a time, "
                      f"after {args.warmup} warmup pass(es) over "
                      f"{min(args.warmup_chunks, m) if args.warmup_chunks > 0 else m} chunk(s); median of "
                      f"{len(runs)} timed runs" + (f"; server pinned to the {len(cpus)} CPUs the batch server uses"
                                                   if cpus else ""),
            "cpus": cpus}, \
        {"sample_reads": nreads, "records": len(a), "records_differing": differ, "identical": differ == 0,
         "batch_client": "integration/bin/bt2g-client", "stock_client": "oracle/_ref/bowtie2-align-l"}


def combine_ranks(elapsed, n_aligned, dev, eng=None):
    """Max of the per-rank times, sum of the aligned-read counters: the path's
    only collective.  On the GPUs the counters go through the
    engines' own RCCL all-reduce (bt2g_allreduce_counts, communicator from
    comm_setup); the max of the times, a harness figure, through torch.distributed
    (RCCL); in the CPU tests both through gloo."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return elapsed, n_aligned
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if eng is not None:
        return float(el[0]), int(eng.allreduce_counts([n_aligned])[0])
    na = torch.tensor([float(n_aligned)], dtype=torch.float64, device=dev)
    dist.all_reduce(na, op=dist.ReduceOp.SUM)
    return float(el[0]), int(na[0])


def comm_setup(eng, rank, world):
    """The engines' communicator over the ranks: rank 0 makes the RCCL id, the
    others receive it over torch.distributed, every rank joins (bt2g_comm_init)."""
    import torch.distributed as dist
    obj = [eng.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    eng.comm_init(world, rank, obj[0])


def shard_seed(rank):
    """Weak scaling: every rank aligns its own batch of reads (seed 42 + rank)."""
    return 42 + rank


def cpu_baseline(idx, reads, quals, pipe, sample, threads, base=None):
    """Reference code (oracle/_ref/libbt2ref.so = /root/reference built by
    oracle/ref/Makefile) on the same per-read work for `sample` reads (paired:
    `sample` pairs, both mates, plus their mate searches), split over `threads`
    host threads.  The seed-extension chain runs on the reference's OWN
    intermediates (oracle/ref_chain.py: its exact sweep, 1-mm hits, seeds, hit
    rows, getOffset, joinedToTextOff, frameSeedExtensionRect, SwAligner), never
    on the GPU's; the mate searches start from the GPU's anchors (reference
    framing + DPs).  Returns (seconds, chain outputs, mate outputs or None,
    per-stage seconds)."""
    import bt2_index as bi
    import tempfile
    import synth
    from oracle.ref_chain import RefChain
    from oracle.ref_harness import score_params
    if not base or not os.path.exists(base + ".rev.2.bt2"):
        base = os.path.join(tempfile.mkdtemp(prefix="bt2bench_"), "g")
        bi.write_index(base, idx)
    chain = RefChain(base)
    L, R = chain.L, chain.R
    pol = pipe.pol
    ids = np.arange(sample)
    if pol.paired:
        ids = np.concatenate([ids, pipe.npairs + ids])
    n = len(ids)
    asc = synth.to_ascii(reads[ids])
    seqs = [bytes(asc[i]) for i in range(n)]
    qs = [bytes(quals[i]) for i in ids]
    lens = np.full(n, pipe.len, np.int64)
    ref = chain.run(seqs, qs, lens, pol, pipe.maxseeds, pipe.mm_cap, MAXHALF, idx.ref_codes, threads)
    ref["ids"] = ids
    dt = sum(chain.secs.values())
    secs = dict(chain.secs)
    mate = None
    if pol.paired:
        # mate searches of the sampled pairs from the GPU's anchors: the reference frames
        # them again (otherMate + frameFindMateRect) and runs the mate DPs
        sp = score_params(pol.local)
        last = pipe.last
        gen_codes = idx.ref_codes
        L.bt2ref_sw_bt_batch_rects.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                               C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        mpairs = last["m_pairs"].cpu().numpy()
        sel_m = np.nonzero(mpairs < sample)[0]
        mfin = last["m_fin"].cpu().numpy()[sel_m]
        mp = last["m_probs"].cpu().numpy()[sel_m]
        mr = np.ascontiguousarray(last["m_rects"].cpu().numpy()[sel_m])
        fin64 = mfin.view(np.int64)
        opp = mfin[:, 2].astype(np.int64)
        fx = np.zeros((len(sel_m), 8), np.int64)
        fx[:, 0] = 1
        fx[:, 1] = fin64[:, 0]
        fx[:, 2] = pipe.len
        fx[:, 3] = [len(gen_codes[r]) for r in mfin[:, 3]]
        fx[:, 4] = pol.minsc
        fx[:, 5] = mfin[:, 5]
        fx[:, 6] = mfin[:, 7]
        fx[:, 7] = pipe.len
        mncol = mp.view(np.int32)[:, 7].astype(np.int64)
        rf_all, rf_off = [], [0]
        for p_, nc in zip(mp, mncol):
            refidx, refl = int(p_.view(np.int32)[6]), int(p_[1])
            g = gen_codes[refidx]
            o = np.arange(refl, refl + nc + 1)
            cc = np.where((o >= 0) & (o < len(g)), g[np.clip(o, 0, len(g) - 1)], 4)
            rf_all.append((1 << cc).astype(np.uint8))
            rf_off.append(rf_off[-1] + nc + 1)
        mrf = np.concatenate(rf_all) if rf_all else np.zeros(1, np.uint8)
        mrf_off = np.array(rf_off, np.int64)
        pos_of = {int(r): i for i, r in enumerate(ids)}
        mseq = [seqs[pos_of[int(r)]] for r in opp]
        mq = [qs[pos_of[int(r)]] for r in opp]
        mfw = np.ascontiguousarray(mp.view(np.int32)[:, 1].astype(np.uint8))
        mnc32 = np.ascontiguousarray(mncol.astype(np.int32))

        def work_mate(lo, hi):
            k = hi - lo
            fxk = np.ascontiguousarray(fx[lo:hi])
            fo = np.zeros((k, 7), np.int64)
            pev = np.array([3, 0, PE_MAXFRAG, 0, 0, 1, 1], np.int32)
            L.bt2ref_frame(k, fxk.ctypes.data, C.byref(sp), pev.ctypes.data, MAXHALF, 1, fo.ctypes.data)
            out = np.zeros((k, 8), np.int64)
            ms = np.full(k, pol.minsc, np.int64)
            L.bt2ref_sw_bt_batch_rects(k, (C.c_char_p * k)(*mseq[lo:hi]), (C.c_char_p * k)(*mq[lo:hi]),
                                       mfw[lo:].ctypes.data, mrf.ctypes.data,
                                       np.ascontiguousarray(mrf_off[lo:hi + 1]).ctypes.data,
                                       mnc32[lo:].ctypes.data, ms.ctypes.data, C.byref(sp),
                                       np.ascontiguousarray(mr[lo:hi]).ctypes.data, out.ctypes.data)
            return fo, out

        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(threads) as ex_:
            b_ = np.linspace(0, len(fx), threads + 1).astype(int)
            mts = list(ex_.map(lambda a: work_mate(*a),
                               [(int(b_[i]), int(b_[i + 1])) for i in range(threads) if b_[i + 1] > b_[i]]))
        secs["mate_search"] = time.perf_counter() - t0
        dt += secs["mate_search"]
        mate = dict(mp=mp, mr=mr, sel=sel_m)
        mate["frame_ref"] = np.concatenate([m[0] for m in mts]) if mts else np.zeros((0, 7), np.int64)
        mate["out_ref"] = np.concatenate([m[1] for m in mts]) if mts else np.zeros((0, 8), np.int64)
    chain.close()
    ref["index_base"] = base
    return dt, ref, mate, secs


def gpu_chain(pipe, ids):
    """The GPU's buffers of the sampled reads, in the shapes oracle/ref_chain.compare expects."""
    import torch
    dev = pipe.dev
    last = pipe.last
    tid = torch.from_numpy(ids).to(dev)
    n_all = pipe.n
    pos = np.full(n_all, -1, np.int64)
    pos[ids] = np.arange(len(ids))
    g = {"sweep": pipe.sweep.index_select(0, tid).cpu().numpy(),
         "mm_cnt": pipe.mm_cnt.index_select(0, tid).cpu().numpy(),
         "mm_hits": pipe.mm_hits.index_select(0, tid).cpu().numpy()}
    sd = np.zeros((len(ids), 2, pipe.maxseeds, 4), np.uint32)
    inv = pipe.inv.cpu().numpy()[ids]
    has = inv >= 0
    if has.any():
        sd[has] = pipe.seeds[:last["m"]].cpu().numpy()[inv[has]].view(np.uint32)
    g["seeds"] = sd
    # hit rows of the sampled reads: contiguous per read at read_base
    rb = last["read_base"].cpu().numpy().astype(np.int64)[ids]
    rc = last["read_cnt"].cpu().numpy().astype(np.int64)[ids]
    tot = int(rc.sum())
    within = np.arange(tot) - np.repeat(np.cumsum(rc) - rc, rc)
    at = np.repeat(rb, rc) + within
    g["rows"] = last["rows"].cpu().numpy()[at]
    g["offs"] = last["offs"].cpu().numpy()[at]
    g["row_read"] = np.repeat(np.arange(len(ids)), rc)
    pr = last["probs"].cpu().numpy()
    rt = last["rects"].cpu().numpy()
    pw = pr.view(np.int32)
    r_all = pw[:, 0].astype(np.int64)
    keep = pos[r_all] >= 0
    g["probs"] = dict(read=pos[r_all[keep]], fw=pw[keep, 1].astype(np.int64), refidx=pw[keep, 6].astype(np.int64),
                      refl=pr[keep, 1], ncol=pw[keep, 7].astype(np.int64), triml=rt[keep, 0].astype(np.int64),
                      corel=rt[keep, 1].astype(np.int64), corer=rt[keep, 2].astype(np.int64))
    g["probs_index"] = np.nonzero(keep)[0]
    return g


def bt_mismatches(naln, alns, ed, ref, maxaln, maxedit):
    """DPs whose GPU nextAlignment results differ from the reference's
    (bt2ref_sw_bt_batch rows): alignment count, first alignment (candidate,
    score, offset, edit count) and a checksum over every alignment's edits.  DPs
    that hit maxaln compare their first maxaln only."""
    import torch
    dev = naln.device
    naln = naln.to(torch.int64)
    alns = alns.to(torch.int64)
    k = torch.arange(maxaln, device=dev)[None, :, None]
    e = torch.arange(maxedit, device=dev)[None, None, :]
    cks = []
    for s0 in range(0, len(naln), 65536):          # int64 temporaries: 4 KB per DP per tensor
        s1 = min(s0 + 65536, len(naln))
        pos = ed[s0:s1, ..., 0].to(torch.int64)
        w = ed[s0:s1, ..., 1].to(torch.int64) & 0xFFFFFFFF
        typ, chr_, qchr = w & 0xFF, (w >> 8) & 0xFF, (w >> 16) & 0xFF
        live = (k < naln[s0:s1, None, None]) & (e < alns[s0:s1, :, 6][:, :, None])
        term = (k + 1) * (pos * 131 + typ * 31 + chr_ * 7 + qchr)
        cks.append((torch.where(live, term, torch.zeros_like(term)).sum((1, 2)) & 0x7FFFFFFFFFFFFFFF).cpu().numpy())
    ck = np.concatenate(cks) if cks else np.zeros(0, np.int64)
    naln = naln.cpu().numpy()
    first = alns[:, 0][:, [0, 1, 2, 6]].cpu().numpy()
    bad = np.minimum(ref[:, 2], maxaln) != naln
    bad |= (naln > 0) & (first != ref[:, 3:7]).any(1)
    bad |= (naln < maxaln) & (ck != ref[:, 7])
    if os.environ.get("BT2G_BENCH_DEBUG"):
        for i in np.nonzero(bad)[0][:8]:
            print(f"[bt mismatch] dp {i}: gpu naln {naln[i]} first {first[i].tolist()} ck {ck[i]} | "
                  f"ref {ref[i].tolist()}", flush=True)
    return int(bad.sum())


def chain_parity(pipe, ref, mate):
    """Stage-by-stage comparison of the GPU's buffers of the last kept step with
    the reference's own chain on the same reads (cpu_baseline): every count
    ending in "_mismatch" is 0 when the two agree."""
    from oracle.ref_chain import compare
    g = gpu_chain(pipe, ref["ids"])
    parity = compare(ref, g)
    parity["reads"] = int(len(ref["ids"]))
    if parity["frame_mismatch"] == 0:
        # the same rectangles on both sides: pair them up and compare fill + backtraces
        rp, gp = ref["probs"], g["probs"]
        kr = np.lexsort([rp[k] for k in ("refl", "refidx", "fw", "read")])
        kg = np.lexsort([gp[k] for k in ("refl", "refidx", "fw", "read")])
        gidx = g["probs_index"][kg]
        sw_ref = ref["sw"][kr]
        res = pipe.res[:pipe.last["npb"]].cpu().numpy()[gidx]
        parity["sw_mismatch"] = int((res[:, 0] != sw_ref[:, 0]).sum() + (res[:, 6] != sw_ref[:, 1]).sum())
        parity["backtrace_mismatch"] = backtrace_parity(pipe, gidx, sw_ref)
        parity["ref_alignments"] = int(sw_ref[:, 2].sum())
    if pipe.pol.paired:
        parity.update(mate_parity(pipe, mate))
    return parity


def backtrace_parity(pipe, kp_all, sw_ref):
    """The seed-extension DPs kp_all (GPU problem indices) nextAlignment results
    vs the reference's rows sw_ref (same order)."""
    import torch
    npb = pipe.last["npb"]
    bad = 0
    for s0 in range(0, len(kp_all), 262144):       # bounded copies of the edit rows
        kp = torch.from_numpy(kp_all[s0:s0 + 262144]).to(pipe.dev)
        bad += bt_mismatches(pipe.naln[:npb].index_select(0, kp), pipe.alns[:npb].index_select(0, kp),
                             pipe.edits[:npb].index_select(0, kp), sw_ref[s0:s0 + 262144], pipe.maxaln,
                             pipe.maxedit)
    return bad


def mate_parity(pipe, mate):
    """The sampled pairs' mate searches: rectangles (bt2g_frame vs the
    reference's otherMate + frameFindMateRect) and the mate DPs' fill +
    nextAlignment results, re-run on the GPU for the sample (outside the
    timed steps) vs the reference's."""
    import torch
    bt2g, L = pipe.bt2g, pipe.L
    mp, mr = mate["mp"], mate["mr"]
    fr = mate["frame_ref"]
    got = np.stack([np.ones(len(mp), np.int64), mp.view(np.int32)[:, 1], mp[:, 1], mp.view(np.int32)[:, 7],
                    mr[:, 0], mr[:, 1], mr[:, 2]], 1)
    frame_bad = int((got != fr).any(1).sum())
    k = len(mp)
    if k == 0:
        return {"mate_dps": 0, "mate_frame_mismatch": frame_bad, "mate_backtrace_mismatch": 0}
    k = min(k, pipe.mate_chunk)
    dev = pipe.dev
    tp = torch.from_numpy(np.ascontiguousarray(mp[:k])).to(dev)
    tr = torch.from_numpy(np.ascontiguousarray(mr[:k])).to(dev)
    S = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    bt2g._chk(L.bt2g_sw_align_bt_dev(pipe.eng2.h, pipe._p(pipe.reads), pipe._p(pipe.quals), pipe.len,
                                     pipe._p(pipe.lens), pipe._p(tp), k, None, pipe._p(tr), C.byref(pipe.sc), 1,
                                     pipe.sw_cap, pipe._p(pipe.mres), pipe._p(pipe.mcands), pipe.maxaln,
                                     pipe.maxedit, pipe._p(pipe.mnaln), pipe._p(pipe.malns), pipe._p(pipe.medits),
                                     None, S))
    torch.cuda.synchronize()
    ref = mate["out_ref"][:k]
    res = pipe.mres[:k].cpu().numpy()
    sw_bad = int((res[:, 0] != ref[:, 0]).sum() + (res[:, 6] != ref[:, 1]).sum())
    bt_bad = bt_mismatches(pipe.mnaln[:k], pipe.malns[:k], pipe.medits[:k], ref, pipe.maxaln, pipe.maxedit)
    return {"mate_dps": k, "mate_frame_mismatch": frame_bad, "mate_sw_mismatch": sw_bad,
            "mate_backtrace_mismatch": bt_bad, "mate_ref_alignments": int(ref[:, 2].sum())}


def workload(args):
    size = "hg38-size; " if args.genome_mb >= 3000 else ""
    model = ("hg38-like repeat landscape: Alu/L1-like families at 10 %/17 % with 3-20 % divergence, segmental "
             "duplications, microsatellites, N gaps" if args.genome_model == "hg38like" else
             "random sequence with planted 2 kb near-repeats")
    genome = (f"vs a {args.genome_mb:.0f} Mbp synthetic genome ({size}{model}; hg38 itself is unavailable offline), "
              f"index built like bowtie2-build (offRate 4, ftabChars 10)")
    vs = args.preset == "very-sensitive"
    seed = ("exact sweep + gated 1-mm + seed round 0 + SA offsets + <=2 seed-extension DPs/read "
            "(fill + nextAlignment loop)")
    if args.mode == "paired":
        cfg = "BASELINE configs[4] policy, --end-to-end --very-sensitive" if vs else \
            "BASELINE configs[2], --end-to-end --sensitive"
        return (f"{args.reads} synthetic 2 x {args.read_len} bp read pairs per GPU per step ({cfg}), "
                f"{genome}; both mates: {seed}; then per pair with an aligned mate one "
                f"mate search: otherMate + frameFindMateRect (--fr -I 0 -X 500) + the mate DP "
                f"({args.read_len} x <=705, fill + nextAlignment loop)")
    mode = "--local --sensitive-local (configs[3])" if args.mode == "local" else "--end-to-end --sensitive (configs[1])"
    if vs:
        mode = "--local --very-sensitive-local" if args.mode == "local" else "--end-to-end --very-sensitive"
    return f"{args.reads} synthetic {args.read_len} bp unpaired reads per GPU per step, {mode} policy, {genome}; {seed}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1, help="timed passes of the batch server over every read")
    ap.add_argument("--warmup", type=int, default=1, help="untimed passes over the first --warmup-chunks chunks")
    ap.add_argument("--reads", type=int, default=1_000_000, help="reads (paired: read pairs) per GPU per step")
    ap.add_argument("--drivers", type=int, default=int(os.environ.get("BT2G_BENCH_DRIVERS") or 16),
                    help="batch server driver threads (-p; $BT2G_BENCH_DRIVERS for A/B runs)")
    ap.add_argument("--clients", type=int, default=32, help="concurrent client connections (both servers)")
    ap.add_argument("--client", choices=("native", "reference"), default="native",
                    help="client of the timed passes: native = integration/bin/bt2g-client (row (f)-4, SAM "
                         "identical to the reference client's); reference = one bowtie2-align-l per chunk")
    ap.add_argument("--rank-mem-gb", type=float, default=0.0,
                    help="host-memory budget per rank (batch server + this process) that sizes the server's "
                         "read slots (0: 1 024 slots per driver on one GPU, 56 GB per rank with several)")
    ap.add_argument("--warmup-chunks", type=int, default=0,
                    help="chunks of a warmup pass (0: all of them -- a warmup step is a whole pass)")
    ap.add_argument("--stock-sample", type=int, default=200_000,
                    help="reads (pairs) timed through the stock server for cpu_baseline and SAM parity (0: skip)")
    ap.add_argument("--chain-steps", type=int, default=2, help="timed steps of the kernel chain (0: skip it)")
    ap.add_argument("--chain-warmup", type=int, default=1)
    ap.add_argument("--chain-cpu-baseline", action="store_true",
                    help="also time the reference's own chain on the host (oracle/ref_chain.py) for the kernel chain")
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--mode", choices=("ee", "local", "paired"), default="ee",
                    help="ee: BASELINE configs[1] (--end-to-end --sensitive); local: configs[3] (--local); "
                         "paired: configs[2] (2 x 150 bp pairs, --end-to-end, mate search)")
    ap.add_argument("--preset", choices=("sensitive", "very-sensitive"), default="sensitive",
                    help="seed policy; very-sensitive: -L 20 -i S,1,0.50 (with --mode paired: BASELINE "
                         "configs[4]'s policy, sharded by torchrun across GPUs)")
    ap.add_argument("--genome-mb", type=float, default=3100.0,
                    help="synthetic genome size (default: hg38's 3.1 Gbp; the index is built on the GPU, ~160 s)")
    ap.add_argument("--genome-model", choices=("hg38like", "simple"), default="hg38like")
    ap.add_argument("--cpu-sample", type=int, default=200_000, help="reads of the chain's CPU baseline")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: the usable cores of the host (cgroup quota / "
                                                                   "affinity)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--index-cache", default="auto",
                    help="reuse/write the built index at this base path ('auto': under $TMPDIR keyed by the "
                         "genome model and size; '': always build)")
    ap.add_argument("--pmc-fetch", default="", help="rocprofv3 --pmc FETCH_SIZE counter_collection.csv of this "
                                                    "command: fills roofline.traffic")
    ap.add_argument("--server-pmc", default=SERVER_PMC, help="pmc_summary.py file for the batch server's kernels "
                    "(roofline.traffic)")
    ap.add_argument("--pmc-write", default="", help="same for WRITE_SIZE")
    ap.add_argument("--allow-fallbacks", action="store_true",
                    help="do not fail the run when the server's reference-CPU fallbacks served requests")
    ap.add_argument("--stock-runs", type=int, default=3, help="timed runs of the stock server's sample (median)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import bt2g
    import bt2_index as bi

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    t0 = time.time()
    parts, names = make_genome(args.genome_mb, model=args.genome_model)
    log(f"[rank {rank}] genome {sum(len(p) for p in parts)/1e6:.0f} Mbp in {time.time()-t0:.1f}s")
    t1 = time.time()
    cache = args.index_cache
    if cache == "auto":
        import tempfile
        cache = os.path.join(tempfile.gettempdir(), "bt2g_bench_index",
                             f"{args.genome_model}_{args.genome_mb:g}mb", "g")
    if not cache:
        import tempfile
        cache = os.path.join(tempfile.mkdtemp(prefix="bt2g_bench_index_"), "g")   # (the servers read it from disk)
    if world > 1 and not os.path.exists(cache + ".rev.2.bt2"):
        # rank 0 builds and writes the index; the others read it
        if rank != 0:
            dist.barrier()
    if os.path.exists(cache + ".rev.2.bt2"):
        idx = bi.read_index(cache)                  # same seed -> same genome -> same index
        log(f"[rank {rank}] index read from {cache}")
    else:
        idx = bi.build_index_device(parts, names=names, device=str(dev))
        if rank == 0:
            # written beside, then renamed into place: a reader never sees half an index
            import shutil
            d = os.path.dirname(cache)
            tmpd = f"{d}.tmp{os.getpid()}"
            os.makedirs(tmpd, exist_ok=True)
            bi.write_index(os.path.join(tmpd, os.path.basename(cache)), idx)
            if os.path.isdir(d):
                shutil.rmtree(d, ignore_errors=True)
            os.makedirs(os.path.dirname(d), exist_ok=True)
            os.rename(tmpd, d)
        if world > 1:
            dist.barrier()
    torch.cuda.synchronize()
    log(f"[rank {rank}] index built on GPU in {time.time()-t1:.1f}s")
    torch.cuda.empty_cache()
    t2 = time.time()
    if args.mode == "paired":
        reads_np, quals_np = make_pairs(parts, args.reads, args.read_len, seed=shard_seed(rank))
    else:
        reads_np, quals_np = make_reads(parts, args.reads, args.read_len, seed=shard_seed(rank))
    del parts                                   # (3.1 GB: the reads are made, the index holds the rest)
    log(f"[rank {rank}] {args.reads} reads in {time.time()-t2:.1f}s")

    # ---- the north-star number: the reference's real schedule on the batch server ----
    import tempfile
    wd = tempfile.mkdtemp(prefix=f"bt2g_sched_r{rank}_")
    sched = schedule_run(args, rank, world, local, cache, reads_np, quals_np, wd)
    elapsed, n_aligned = combine_ranks(sched["elapsed"], sched["aligned"], dev)
    value = n_aligned / elapsed
    total_reads = args.reads * args.steps * world
    log(f"[rank {rank}] real schedule: {sched['aligned']} aligned of {args.reads * args.steps} in "
        f"{sched['elapsed']:.2f}s; whole job {value:.0f} aligned/s")
    kern = server_kernels(sched["stats"])
    cpu, sam = None, None
    if rank == 0 and world == 1 and args.stock_sample and not args.no_cpu_baseline:
        try:
            cpu, sam = stock_baseline(args, cache, sched["chunks"], sched["outs"], wd)
            log(f"[rank 0] stock server {cpu['value']:.0f} {cpu['unit']} on {cpu['cores']} cores; SAM {sam}")
        except Exception as e:        # a checker: its failure must not hide the measurement
            import traceback
            traceback.print_exc()
            cpu = {"error": repr(e)[:500]}
    sched["outs"] = None
    chain = None
    if args.chain_steps > 0:
        chain = run_chain(args, rank, world, local, dev, idx, cache, reads_np, quals_np)
    if rank == 0:
        unit = "read pairs/s" if args.mode == "paired" else "reads/s"
        st = sched["stats"] or {}
        rl, rls = line_rooflines(kern, args.server_pmc)
        calls = {k: st.get(k) for k in ("exact_sweep", "one_mm", "seed_search", "extend", "get_offset", "ungapped",
                                        "sw_dp")}
        # the reference's CPU code inside the product server (bt2g_batch.cpp's live
        # fallbacks: exactSweep, oneMmSearch, ungappedAlign, SwAligner::align,
        # Ebwt::getOffset) must not have served any request of the run
        fallbacks = {k: v[1] for k, v in calls.items() if v and v[1]}
        dp = st.get("dp") or [0, 0, 0, 0]
        out = {
            "metric": "reads aligned/sec (whole node), 150 bp vs hg38, at 1/2/4/8 MI355X",
            "value": value, "unit": "aligned " + unit, "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8/i16 DP, u32 FM", "data": "synthetic",
            "config": {"workload": schedule_workload(args), "global_batch": args.reads * world,
                       "seq_len": args.read_len, "parallelism": f"dp{world} (a batch server per GPU)",
                       "aligned_frac": n_aligned / total_reads, "drivers": args.drivers,
                       "slots_per_driver": sched["slots_per_driver"],
                       "client_connections": args.clients, "reads_per_connection": 10_000,
                       "warmup_chunks": args.warmup_chunks},
            "roofline": rl,
            "rooflines": rls,
            "reads_per_s": total_reads / elapsed,
            "server_kernels": kern,
            "server": {k: st.get(k) for k in ("reads", "rounds", "slots", "slots_live", "slots_rebuilt",
                                              "slot_kib_hist", "pool_trims", "steps", "idle_ms", "phases_ms",
                                              "ext_speculative", "ext_prefetched")
                       if k in st} |
                      {"binary": sched["binary"], "server_cpu_s": sched["server_cpu_s"],
                       "server_rss_gb": sched["server_rss_gb"], "server_rss_gb_per_pass": sched["server_rss_gb_per_pass"],
                       "smaps_top": sched["smaps_top"],
                       "cpu_us_per_read": sched["server_cpu_s"] / max(1, args.reads * args.steps) * 1e6,
                       # the client side (read parsing, the wire, SAM receipt) on the same CPU
                       # quota: bt2g-client, or the reference's client processes (--client reference)
                       "client": sched["client"],
                       # the whole CPU share's use over the timed passes (cgroup cpu.stat: every
                       # process of the job) and the time its quota throttled it
                       "host_cores_busy": sched["host_cpu_s"] / max(1e-9, sched["passes_s"]),
                       "throttled_s": sched["throttled_s"],
                       "client_cpu_s": sched["client_cpu_s"],
                       "client_cpu_us_per_read": sched["client_cpu_s"] / max(1, args.reads * args.steps) * 1e6,
                       "calls": calls,
                       "cpu_fallbacks": fallbacks,
                       # speculative DPs (bt2g_batch.cpp: the first DP an extension loop needs
                       # goes out with up to 7 of its others): filled, taken by the loops, taken
                       # at a tightened minimum score, and DPs asked for that were not ready
                       "dp_speculation": {"speculated": dp[0], "used": dp[1], "reused": dp[2], "missed": dp[3],
                                          "consumed_frac": dp[1] / dp[0] if dp[0] else None},
                       "pass_s": sched["pass_s"], "passes_s": sched["passes_s"],
                       "work_by_kernel": work_by_kernel(st),
                       "threads_cpu": sched["server_threads_cpu"]},
            "cpu_baseline": cpu,
            "sam_parity": sam,
            "vs_cpu_baseline": value / cpu["value"] if cpu and cpu.get("value") else None,
            "kernel_chain": chain,
        }
        print(json.dumps(out), flush=True)
        if fallbacks and not args.allow_fallbacks:
            # (after the line, so that what ran is on record; the exit status fails the run)
            log(f"[rank 0] FAIL: the reference's CPU code served requests in the product server: {fallbacks}")
            sys.exit(3)
    if world > 1:
        dist.destroy_process_group()


def schedule_workload(args):
    vs = args.preset == "very-sensitive"
    if args.mode == "paired":
        cfg = "configs[4] policy, --end-to-end --very-sensitive" if vs else "configs[2], --end-to-end --sensitive"
        what = f"{args.reads} synthetic 2 x {args.read_len} bp read pairs per GPU per step ({cfg})"
    else:
        mode = "--local (configs[3])" if args.mode == "local" else "--end-to-end --sensitive (configs[1])"
        if vs:
            mode = "--local --very-sensitive-local" if args.mode == "local" else "--end-to-end --very-sensitive"
        what = f"{args.reads} synthetic {args.read_len} bp unpaired reads per GPU per step, {mode}"
    size = "hg38-size " if args.genome_mb >= 3000 else ""
    clt = ("the reference's own client, one process per connection" if getattr(args, "client", "native") == "reference"
           else "read by this repository's multi-connection client (integration/bin/bt2g-client, one process)")
    return (f"{what}, vs a {args.genome_mb:.0f} Mbp {size}synthetic genome ({args.genome_model}; hg38 is "
            f"unavailable offline), through the reference's own server and per-read logic with the "
            f"batch-first driver on the engines (integration/bin/bowtie2-align-server-batch), SAM output, "
            f"{clt}; <= 10 000 reads per client connection, {args.clients} connections at a time")


def run_chain(args, rank, world, local, dev, idx, cache, reads_np, quals_np):
    """The kernel chain (the module docstring's fixed policy, reads resident in
    HBM): the engines in their throughput regime, with the roofline of its
    dominant kernel.  Returns the kernel_chain block of the bench line."""
    import torch
    import torch.distributed as dist
    import bt2g
    eng = bt2g.Engine(index=idx, device=local)
    if world > 1:
        comm_setup(eng, rank, world)
    info = eng.info()
    log(f"[rank {rank}] chain engine: index resident {info[12]/1e9:.2f} GB")
    reads = torch.from_numpy(reads_np).to(dev)
    quals = torch.from_numpy(quals_np).to(dev)
    pipe = Pipeline(eng, idx, reads, quals, args.read_len, args.mode, args.preset)

    engs = [eng] + ([pipe.eng2] if args.mode == "paired" else [])
    for _ in range(args.chain_warmup):
        pipe.step()
    torch.cuda.synchronize()
    for e in engs:
        e.reset_stats()
        e.set_profiling(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ts = time.perf_counter()
    n_aligned = 0
    for k in range(args.chain_steps):
        aligned = pipe.step(keep=(k == args.chain_steps - 1))
        n_aligned += int(aligned.sum())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - ts
    for e in engs:
        e.set_profiling(False)
    stats = {k: eng.kernel_stats(k) for k in range(6)}
    mstats = {k: pipe.eng2.kernel_stats(k) for k in (4, 5, 7)} if args.mode == "paired" else {}
    elapsed, n_aligned = combine_ranks(elapsed, n_aligned, dev, eng if world > 1 else None)
    total_reads = args.reads * args.chain_steps * world
    value = total_reads / elapsed

    # ---- roofline of the dominant kernel (per launch, rank 0's view) --------
    last = pipe.last
    names_k = ["exact_sweep", "seed_search", "one_mm", "get_offset", "sw_align", "sw_backtrace"]
    per_launch = {}
    n = pipe.n                                       # reads (paired: both mates)
    sweep_loads = int((pipe.sweep[:, 7].to(torch.int64) & 0xFFFFFFFF).sum())
    bytes_k = {
        # 64-B sides gathered + the read bytes each lane walks (2 strands)
        0: 64 * sweep_loads + 2 * n * args.read_len,
        1: 64 * int(pipe.sd_loads[:last["m"]].to(torch.int64).sum()) + int(pipe.nseeds[:last["m"]].sum()) * 2 * (pipe.pol.seedlen + 12),
        2: 64 * int(pipe.mm_loads.to(torch.int64).sum()) + 4 * n * args.read_len,
        3: 64 * int(last["loads_off"].to(torch.int64).sum()) + 12 * last["nrows"],
        4: None,
        5: None,
    }
    for k in range(6):
        launches, ms = stats[k]
        if launches:
            per_launch[k] = ms / launches
    sw_cells = last["npb"] * args.read_len * pipe.ncol
    sw_gcups = sw_cells / (per_launch.get(4, float("nan")) / 1e3) / 1e9
    # the dominant kernel: the longest per step among those with an algorithmic
    # work figure: FM kernels in bytes (HBM-bound), the SW fill
    # in integer ops, SW_OPS_PER_CELL per DP cell (VALU-bound)
    work_k = dict(bytes_k)
    work_k[4] = sw_cells * SW_OPS_PER_CELL if 4 in per_launch else None
    step_ms = {k: stats[k][1] / args.chain_steps for k in per_launch}
    dom = max((k for k in per_launch if work_k.get(k)), key=lambda k: step_ms[k])
    achieved = work_k[dom] / (per_launch[dom] / 1e3) / (1e12 if dom == 4 else 1e9)
    for k in per_launch:
        log(f"[rank {rank}] {names_k[k]:12s} {per_launch[k]:8.3f} ms/launch")
    mmprof = getattr(bt2g.lib(), "bt2g_mm_prof_waves", None) if "prof" in bt2g.LIB_PATH else None
    if mmprof is not None:
        # profiling build of the 1-mm far kernels (-DBT2G_MM_PROF): waves of the last launch
        import ctypes
        t0 = np.zeros(2 << 16, np.uint64); t1 = np.zeros(2 << 16, np.uint64); ws = np.zeros(2 << 16, np.uint32)
        if mmprof(t0.ctypes.data_as(ctypes.c_void_p), t1.ctypes.data_as(ctypes.c_void_p),
                  ws.ctypes.data_as(ctypes.c_void_p)) == 0:
            for h, nm in ((0, "far<true>"), (1, "far<false>")):
                a0, a1, st_ = t0[h << 16:(h + 1) << 16], t1[h << 16:(h + 1) << 16], ws[h << 16:(h + 1) << 16]
                ok = a1 > 0
                if not ok.any():
                    continue
                a0, a1, st_ = a0[ok].astype(np.float64), a1[ok].astype(np.float64), st_[ok]
                dur = (a1 - a0) / 100.0
                q = np.percentile(dur, [50, 90, 99, 100])
                qs = np.percentile(st_, [50, 90, 99, 100])
                log(f"[rank {rank}] mm_prof {nm}: {ok.sum()} waves, span {(a1.max() - a0.min()) / 100:.0f} us, "
                    f"start spread {(a0.max() - a0.min()) / 100:.0f} us; wave us p50/90/99/max "
                    f"{q[0]:.0f}/{q[1]:.0f}/{q[2]:.0f}/{q[3]:.0f}; max-lane LF steps p50/90/99/max "
                    f"{qs[0]:.0f}/{qs[1]:.0f}/{qs[2]:.0f}/{qs[3]:.0f}")
    prof = getattr(bt2g.lib(), "bt2g_bt_prof_read", None) if "prof" in bt2g.LIB_PATH else None
    if prof is not None and stats[5][0]:
        # profiling build of the backtrace (scripts/bt_bench.py): counters per launch
        import ctypes
        cnt = (ctypes.c_ulonglong * 16)()
        prof(cnt)
        nl = stats[5][0]
        names_p = ["walks", "steps", "colhit16_blocks", "escan_rounds", "candidates", "dom_tests", "replays",
                   "hget", "chunk_reloads", "tile_loads", "tile_writebacks", "colhit8_blocks", "dps_walked", "",
                   "", "wave_steps"]
        d = {k: int(v) // nl for k, v in zip(names_p, cnt) if k}
        d["lane_utilization"] = d["steps"] / max(1, d["wave_steps"])
        log(f"[rank {rank}] bt_prof per launch (all launches since start / {nl}): {d}")
    naln_np = pipe.naln[:last["npb"]].cpu().numpy()
    bt_stats = {"alignments": int(naln_np.clip(0).sum()), "dps_with_alignment": int((naln_np > 0).sum()),
                "dps_at_maxaln": int((naln_np >= pipe.maxaln).sum()), "maxaln": pipe.maxaln,
                "dps_cand_overflow": int((naln_np == -5).sum()),
                "cand_overflow_reruns_total": int(pipe.stats.get("cand_overflow_reruns", 0))}
    log(f"[rank {rank}] SW: {last['npb']} DPs/step, {sw_gcups:.0f} GCUPS; aligned {n_aligned/(args.chain_steps*world*args.reads):.4f}; backtrace {bt_stats}")
    mate_stats = None
    if args.mode == "paired":
        mk = {k: v[1] / args.chain_steps for k, v in mstats.items()}          # ms per step
        mcells = last["m_dps"] * args.read_len * pipe.mate_cols
        mate_stats = {"anchors": last["m_anchors"], "mate_dps": last["m_dps"], "pairs_mate_found": last["m_found"],
                      "frame_ms_per_step": mk[7], "fill_ms_per_step": mk[4], "backtrace_ms_per_step": mk[5],
                      "fill_gcups": mcells / (mk[4] / 1e3) / 1e9 if mk[4] else None,
                      "launches_per_step": mstats[4][0] / args.chain_steps}
        log(f"[rank {rank}] mate search: {mate_stats}")

    # ---- the repeat landscape the last step saw (rank 0's batch) -------------
    def hist(x):
        edges = [1, 2, 11, 101, 1001, 1 << 62]
        x = x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)
        return {f"{lo}-{hi - 1}" if hi - lo > 1 else str(lo): int(((x >= lo) & (x < hi)).sum())
                for lo, hi in zip(edges[:-1], edges[1:])}
    swl = pipe.sweep.to(torch.int64) & 0xFFFFFFFF
    exr = torch.minimum(swl[:, 0], swl[:, 1]) == 0
    ex_sz = torch.where(swl[:, 3] > swl[:, 2], swl[:, 3] - swl[:, 2], swl[:, 5] - swl[:, 4])[exr]
    sdl = pipe.seeds[:last["m"]].to(torch.int64) & 0xFFFFFFFF
    sd_sz = (sdl[..., 1] - sdl[..., 0]).flatten()
    sd_sz = sd_sz[sd_sz > 0]
    dpr = torch.bincount(last["probs"].view(torch.int32)[:, 0].to(torch.int64), minlength=pipe.n)
    landscape = {"exact_hit_range_sizes": hist(ex_sz), "seed_hit_range_sizes": hist(sd_sz),
                 "seed_hit_range_mean": float(sd_sz.double().mean()) if sd_sz.numel() else 0.0,
                 "dps_per_read": {str(k): int(v) for k, v in enumerate(torch.bincount(dpr).tolist())},
                 "hit_rows_per_read": float(last["nrows"] / pipe.n)}
    mmo = pipe.mm_ops.to(torch.int64)
    mmo = mmo[mmo > 0].double()
    if mmo.numel():
        q = torch.quantile(mmo[:1 << 24], torch.tensor([0.5, 0.9, 0.99, 0.999], dtype=torch.float64,
                                                       device=mmo.device)).tolist()
        landscape["one_mm_ops_per_read"] = {"reads": int(mmo.numel()), "mean": float(mmo.mean()), "p50": q[0],
                                            "p90": q[1], "p99": q[2], "p999": q[3], "max": float(mmo.max())}
    log(f"[rank {rank}] landscape {landscape}")

    # ---- optional: the reference's own chain on the host cores, rank 0, N=1 ---
    cpu = None
    parity = None
    if rank == 0 and world == 1 and args.chain_cpu_baseline:
        from oracle import ref_server as rs
        host = rs.host_cpus()
        threads = args.cpu_threads or host["usable"]
        sample = min(args.cpu_sample, pipe.npairs if args.mode == "paired" else pipe.n)
        try:
            dt, ref, mate, secs = cpu_baseline(idx, reads_np, quals_np, pipe, sample, threads, base=cache or None)
            paired = args.mode == "paired"
            cpu = {"value": sample / dt, "unit": "read pairs/s" if paired else "reads/s", "cores": threads,
                   "kind": "reference", "stage_seconds": secs,
                   "sample": f"first {sample} {'pairs (both mates)' if paired else 'reads'} of the batch through "
                             f"the reference's own chain (oracle/ref_chain.py) on {threads} threads"}
            parity = chain_parity(pipe, ref, mate)
            log(f"[rank 0] chain cpu baseline {sample/dt:.0f} {cpu['unit']} ({dt:.1f}s); parity {parity}")
        except Exception as e:  # the reference build is optional on the box
            import traceback
            traceback.print_exc()
            log(f"[rank 0] chain cpu baseline unavailable: {e!r}")
    for e in engs[::-1]:
        e.close()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return {
        "value": value, "unit": "read pairs/s" if args.mode == "paired" else "reads/s",
        "steps": args.chain_steps, "warmup": args.chain_warmup, "ms_per_step": elapsed / args.chain_steps * 1e3,
        "aligned_frac": n_aligned / total_reads, "aligned_per_s": n_aligned / elapsed,
        "workload": workload(args),
        "schedule": "fixed policy: exact sweep, gated 1-mm search, round-0 exact seeds, getOffset of each hit "
                    "range's top row, <= 2 seed-extension DPs per read, fill + nextAlignment loop; every read's "
                    "batch resident in HBM",
        "roofline": dict({"bound": "hbm", "kernel": names_k[dom], "achieved": achieved, "peak": HBM_PEAK_GBS,
                          "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "bytes_per_launch": bytes_k[dom]}
                         if dom != 4 else
                         {"bound": "valu", "kernel": "sw_align (systolic fill + decision plane, candidate sort)",
                          "achieved": achieved, "peak": VALU_PEAK_TOPS, "unit": "T int-ops/s",
                          "frac": achieved / VALU_PEAK_TOPS, "ops_per_cell": SW_OPS_PER_CELL,
                          "cells_per_launch": sw_cells, "gcups": sw_gcups,
                          "issued_valu_lane_ops_per_cell": VALU_OPS_PER_CELL},
                         ms_per_launch=per_launch[dom], ms_per_step=step_ms[dom],
                         traffic=pmc_traffic(args.pmc_fetch, args.pmc_write, PMC_KERNEL[dom])),
        "kernels_ms": {names_k[k]: per_launch[k] for k in per_launch},
        "kernels_gbs": {names_k[k]: bytes_k[k] / (per_launch[k] / 1e3) / 1e9 for k in per_launch if bytes_k.get(k)},
        "side_loads_per_step": {names_k[k]: (bytes_k[k] // 64) for k in (0, 1, 2, 3) if bytes_k.get(k)},
        "sw_gcups": sw_gcups,
        "sw_issue": {"issued_valu_lane_ops_per_cell": VALU_OPS_PER_CELL,
                     "issued_T_lane_ops_per_s": sw_gcups * VALU_OPS_PER_CELL / 1e3,
                     "of_valu_peak": sw_gcups * VALU_OPS_PER_CELL / 1e3 / VALU_PEAK_TOPS,
                     "of_packed_issue_ceiling": sw_gcups * VALU_OPS_PER_CELL / 1e3 / VALU_PACKED_TOPS}
        if args.mode == "ee" else None,
        "backtrace": bt_stats,
        "landscape": landscape,
        "mate_search": mate_stats,
        "cpu_baseline": cpu,
        "parity_sample": parity,
    }


if __name__ == "__main__":
    main()
