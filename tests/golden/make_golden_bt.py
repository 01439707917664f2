"""Backtrace golden fixtures from the REFERENCE itself (row A21).

Run here (needs /root/reference and the oracle/_ref build):
    make -C oracle/ref && python tests/golden/make_golden_bt.py

Inputs are the DP problems already committed in sw_{rand,log}_{ee,loc}.npz
(made by make_golden.py); each gets a seed-extension style rectangle (triml,
core diagonals [corel, corer] = [maxgap, 3*maxgap], dp_framer.cpp:116-125)
and is run through the reference's SwAligner::align followed by the
SwDriver nextAlignment loop (aligner_sw_driver.cpp:1157-1180) in
oracle/_ref/libbt2ref.so (bt2ref_sw_bt).  Written per source fixture:
  sw_bt_<src>.npz: triml, corel, corer (per problem); out (n x 7);
      aln (K x 10: cand, score, off, refoff, ns, gaps, refns, nedit, trim5p,
      trim3p) with aln_off (n+1); edits (E x 4: pos, type, chr, qchr) with
      edit_off (K+1); fates with fate_off (n+1).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.ref_harness import RefLib  # noqa: E402

SOURCES = ["sw_rand_ee", "sw_rand_loc", "sw_log_ee", "sw_log_loc"]


def strand_read(g, p):
    ri = int(g["rd_index"][p])
    L = int(g["lens"][ri])
    return g["reads"][ri][:L], g["quals"][ri][:L]


def main():
    lib = RefLib()
    for src in SOURCES:
        g = np.load(os.path.join(HERE, src + ".npz"))
        local = bool(g["local"])
        n = len(g["rd_index"])
        rng = np.random.default_rng(SOURCES.index(src) + 11)
        mg = rng.integers(0, 16, n)
        triml = np.where(rng.random(n) < 0.2, rng.integers(0, 4, n), 0).astype(np.int32)
        corel, corer = mg.astype(np.int32), (3 * mg).astype(np.int32)
        outs, alns, eds, fates = [], [], [], []
        aln_off, edit_off, fate_off = [0], [0], [0]
        for p in range(n):
            rd, q = strand_read(g, p)
            rf = g["rf"][g["rf_off"][p]:g["rf_off"][p + 1]]
            seq = "".join("ACGTN"[c] for c in rd).encode()
            o, a, e, f = lib.sw_bt(seq, bytes(q.tolist()), bool(g["fw"][p]), rf, int(g["minsc"][p]), local,
                                   int(triml[p]), int(corel[p]), int(corer[p]), maxaln=4096, maxedit=1024)
            outs.append(o)
            for k in range(len(a)):
                alns.append(a[k])
                eds.append(e[k])
                edit_off.append(edit_off[-1] + len(e[k]))
            aln_off.append(aln_off[-1] + len(a))
            fates.append(f)
            fate_off.append(fate_off[-1] + len(f))
        d = dict(triml=triml, corel=corel, corer=corer, out=np.array(outs, np.int64),
                 aln=np.array(alns, np.int64).reshape(-1, 10), aln_off=np.array(aln_off, np.int64),
                 edits=(np.concatenate(eds) if eds else np.zeros((0, 4))).astype(np.int32).reshape(-1, 4),
                 edit_off=np.array(edit_off, np.int64), fates=np.concatenate(fates).astype(np.int8),
                 fate_off=np.array(fate_off, np.int64))
        np.savez_compressed(os.path.join(HERE, "sw_bt_%s.npz" % src[3:]), **d)
        print(src, "problems", n, "alignments", len(alns), "edits", edit_off[-1])


if __name__ == "__main__":
    main()
