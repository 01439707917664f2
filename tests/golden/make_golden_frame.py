"""DP-framing golden fixtures from the REFERENCE itself (row A14).

Run here (needs /root/reference and the oracle/_ref build):
    make -C oracle/ref && python tests/golden/make_golden_frame.py

Seed-extension (DynProgFramer::frameSeedExtensionRect) and mate-search
(PairedEndPolicy::otherMate + DynProgFramer::frameFindMateRect) rectangles
computed by the reference's own objects through oracle/_ref/libbt2ref.so
(bt2ref_frame), as SwDriver::extendSeeds / extendSeedsPaired call them.
Cases: every PE policy x anchor mate x strand, the fragment-length settings
of the reference's own otherMate unit tests (pe.cpp main: -I 20 -X 30, mates
of 10 on a 200-long reference, anchor at 100, expand-to-fit, flipping,
dovetailing, containment and overlap toggled) and bowtie2's defaults
(-I 0 -X 500), anchors near both reference ends (trimming, with and without
--overhang), minsc from the end-to-end and local defaults and from perfect
scores (gap budgets 0), maxhalf 15 and wider.  Written: frame.npz with one
entry per setting: in_<k> (n x 8), out_<k> (n x 7), and its parameters.
"""
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT]

from oracle.ref_harness import RefLib  # noqa: E402

# (name, local, pe (policy, minfrag, maxfrag, flip, dovetail, olap, expand), maxhalf, trim_to_ref)
SETTINGS = [
    ("ee_default", False, (3, 0, 500, 0, 0, 1, 1), 15, True),
    ("loc_default", True, (3, 0, 500, 0, 0, 1, 1), 15, True),
    ("ee_overhang", False, (3, 0, 500, 0, 0, 1, 1), 15, False),
    ("ee_ff", False, (1, 0, 500, 0, 0, 1, 1), 15, True),
    ("ee_rr", False, (2, 0, 500, 0, 0, 1, 1), 15, True),
    ("ee_rf", False, (4, 50, 300, 0, 0, 1, 1), 15, True),
    ("unit_simple", False, (1, 20, 30, 1, 1, 1, 1), 15, True),
    ("unit_noolap", False, (3, 20, 30, 1, 1, 0, 1), 15, True),
    ("unit_nodove", False, (3, 20, 30, 1, 0, 1, 1), 15, True),
    ("unit_noflip", False, (3, 20, 30, 0, 1, 1, 1), 15, True),
    ("unit_noexpand", False, (3, 20, 30, 1, 1, 1, 0), 15, True),
    ("loc_wide", True, (3, 100, 800, 0, 0, 1, 1), 40, False),
]


def make_inputs(rng, local, n, short):
    x = np.zeros((n, 8), np.int64)
    x[:, 0] = rng.integers(0, 2, n)                       # kind
    if short:
        reflen = np.full(n, 200)
        rdlen = np.full(n, 10)
        alen = np.where(rng.random(n) < 0.7, 10, rng.integers(5, 40, n))
        off = np.where(rng.random(n) < 0.5, 100, rng.integers(-20, 220, n))
    else:
        reflen = rng.integers(400, 100000, n)
        rdlen = np.where(rng.random(n) < 0.6, 150, rng.integers(20, 300, n))
        alen = np.where(rng.random(n) < 0.6, 150, rng.integers(20, 300, n))
        # anywhere, near the left end, near the right end, off the ends
        where = rng.integers(0, 4, n)
        off = np.select([where == 0, where == 1, where == 2],
                        [rng.integers(0, reflen), rng.integers(-60, 60, n), reflen - rng.integers(-60, 400, n)],
                        rng.integers(-700, reflen + 700))
    L = rdlen.astype(np.float64)
    if local:
        minsc = (20 + 8 * np.log(L)).astype(np.int64)
        perfect = 2 * rdlen
    else:
        minsc = (-0.6 - 0.6 * L).astype(np.int64)
        perfect = np.zeros(n, np.int64)
    pick = rng.random(n)
    minsc = np.where(pick < 0.15, perfect, minsc)                           # gap budget 0
    minsc = np.where((pick >= 0.15) & (pick < 0.3), minsc - rng.integers(0, 200, n), minsc)
    x[:, 1], x[:, 2], x[:, 3], x[:, 4] = off, rdlen, reflen, minsc
    x[:, 5] = rng.integers(0, 2, n)                       # fw
    x[:, 6] = rng.integers(0, 2, n)                       # anchor1
    x[:, 7] = alen
    return x


def main():
    lib = RefLib()
    rng = np.random.default_rng(1414)
    out = {}
    for k, (name, local, pe, maxhalf, ttr) in enumerate(SETTINGS):
        x = make_inputs(rng, local, 1500 if name.startswith("unit") else 4000, name.startswith("unit"))
        if name.startswith("unit"):
            # the pe.cpp unit-test grid itself: every policy/anchor/strand at off 100
            grid = np.array([[1, 100, 10, 200, 0, fw, a1, 10] for a1 in (0, 1) for fw in (0, 1)], np.int64)
            x = np.concatenate([grid, x])
        y = lib.frame(x, local, pe=pe, maxhalf=maxhalf, trim_to_ref=ttr)
        out[f"in_{name}"], out[f"out_{name}"] = x, y
        out[f"par_{name}"] = np.array([int(local), *pe, maxhalf, int(ttr)], np.int64)
        print(name, "framed", int(y[:, 0].sum()), "of", len(y))
    np.savez_compressed(os.path.join(HERE, "frame.npz"), names=np.array([s[0] for s in SETTINGS]), **out)


if __name__ == "__main__":
    main()
