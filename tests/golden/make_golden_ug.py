"""Ungapped-alignment golden fixtures from the REFERENCE itself (row A22).

Run here (needs /root/reference and the oracle/_ref build):
    make -C oracle/ref && python tests/golden/make_golden_ug.py

Reads sampled from the lambda and the synthetic test genomes (substitutions,
Ns, both strands, positions off both reference ends, shifted diagonals and
random reads) run through the reference's SwAligner::ungappedAlign
(aligner_sw.cpp:286-494) via oracle/_ref/libbt2ref.so, end-to-end (minsc
-0.6-0.6L) and local (minsc 20+8 ln L).  Written: ug_<index>.npz with the
inputs (reads, quals, fw, refidx, off, minsc, local) and the outputs
(out n x 10: ret, score, refoff, ns, refns, nedit, trim5p, trim3p; edits
with edit_off).
"""
import math
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, HERE, os.path.join(ROOT, "bowtie2-server_amd", "tools"), os.path.join(ROOT, "tests")]

from oracle.ref_harness import RefLib  # noqa: E402
import bt2_index as bi  # noqa: E402
import synth  # noqa: E402
from conftest import get_index  # noqa: E402


def make_inputs(idx, seed, n):
    rng = np.random.default_rng(seed)
    refs = idx.ref_codes
    L = 150
    reads = np.zeros((n, L), np.uint8)
    quals = (rng.integers(2, 41, (n, L)) + 33).astype(np.uint8)
    fw = rng.random(n) < 0.5
    refidx = rng.integers(0, len(refs), n).astype(np.uint32)
    off = np.zeros(n, np.int64)
    for i in range(n):
        g = refs[refidx[i]]
        kind = rng.random()
        if kind < 0.08:
            o = int(rng.integers(-30, 1))                     # off the left end
        elif kind < 0.16:
            o = len(g) - L + int(rng.integers(0, 30))         # off the right end
        else:
            o = int(rng.integers(0, max(1, len(g) - L)))
        pos = np.arange(o, o + L)
        seq = np.where((pos >= 0) & (pos < len(g)), g[np.clip(pos, 0, len(g) - 1)], 4).astype(np.uint8)
        seq = np.where(seq > 3, rng.integers(0, 4, L), seq).astype(np.uint8)
        m = rng.random(L) < rng.choice([0.0, 0.005, 0.02, 0.08, 0.3])
        seq[m] = (seq[m] + rng.integers(1, 4, m.sum())) % 4
        seq[rng.random(L) < 0.003] = 4
        if rng.random() < 0.05:
            seq = rng.integers(0, 4, L).astype(np.uint8)       # random read
        elif rng.random() < 0.08:
            a = int(rng.integers(40, 80))                      # two good segments (local: sols > 1)
            seq[a:a + 30] = (seq[a:a + 30] + rng.integers(1, 4, 30)) % 4
        shift = int(rng.integers(-2, 3)) if rng.random() < 0.1 else 0
        off[i] = o + shift
        reads[i] = seq if fw[i] else np.where(seq > 3, 4, 3 - seq)[::-1]
    return reads, quals, fw, refidx, off


def main():
    lib = RefLib()
    for name in ("lambda", "synth"):
        idx = get_index(name)
        tmp = tempfile.mkdtemp(prefix="ug_")
        base = os.path.join(tmp, "g")
        bi.write_index(base, idx)
        R = lib.open(base)
        reads, quals, fw, refidx, off = make_inputs(idx, 5 if name == "lambda" else 6, 600)
        asc = synth.to_ascii(reads)
        seqs = [bytes(a) for a in asc]
        qs = [bytes(q) for q in quals]
        d = dict(reads=reads, quals=quals, fw=fw, refidx=refidx, off=off)
        for mode, local, minsc in (("ee", False, int(-0.6 - 0.6 * 150)), ("loc", True, int(20 + 8 * math.log(150)))):
            ms = np.full(len(seqs), minsc, np.int64)
            out, eds = R.ungapped(seqs, qs, fw, refidx, off, ms, local)
            d[mode + "_minsc"] = ms
            d[mode + "_out"] = out
            d[mode + "_edits"] = np.concatenate(eds) if eds else np.zeros((0, 4), np.int32)
            d[mode + "_edit_off"] = np.concatenate([[0], np.cumsum([len(e) for e in eds])]).astype(np.int64)
            print(name, mode, "ret counts", {r: int((out[:, 0] == r).sum()) for r in (-1, 0, 1)})
        R.close()
        np.savez_compressed(os.path.join(HERE, "ug_%s.npz" % name), **d)


if __name__ == "__main__":
    main()
