#!/usr/bin/env python3
"""Fixed cost of one host-pointer engine call (the drop-in's unit of work):
per-call wall time of small batches, from 1 thread and from T threads each on
its own shared context, next to the kernel time the context records.

  python scripts/call_overhead.py [--threads 1,8] [--calls 200]
"""
import argparse
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "bowtie2-server_amd"), os.path.join(ROOT, "bowtie2-server_amd", "tools"),
           os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,8")
    ap.add_argument("--calls", type=int, default=200)
    a = ap.parse_args()
    import bt2g
    import synth
    from conftest import get_index
    idx = get_index("synth")
    gen = np.concatenate(idx.ref_codes)
    reads, quals, pos, fw = synth.reads(5, gen, 256, 150)
    lens = np.full(len(reads), 150, np.uint32)
    probs = np.zeros(128, bt2g.SWPROB_DTYPE)
    probs["read"] = np.arange(128)
    probs["fw"] = fw[:128]
    probs["refl"] = pos[:128].astype(np.int64) - 30
    probs["win_off"] = -1
    probs["ncol"] = 210
    probs["minsc"] = -90
    rects = np.zeros(128, bt2g.SWRECT_DTYPE)
    rects["corel"], rects["corer"] = 15, 45
    rows = np.arange(1000, 1100, dtype=np.uint32)
    ms = np.full(64, -90, np.int32)
    work = {
        "exact_sweep(48)": lambda e: e.exact_sweep(reads[:48], lens[:48]),
        "seed_search(32)": lambda e: e.seed_search(reads[:32], lens[:32], 22, 15, 0, 16),
        "one_mm(48)": lambda e: e.one_mm(reads[:48], quals[:48], lens[:48], ms[:48], False),
        "get_offset(100)": lambda e: e.get_offset(rows),
        "sw_align_bt(128)": lambda e: e.sw_align_bt(reads, quals, lens, probs, rects=rects, maxaln=8, maxedit=64,
                                                     want_fates=False),
    }
    base = bt2g.Engine(index=idx)
    for T in [int(x) for x in a.threads.split(",")]:
        engs = [base.shared() for _ in range(T)]
        for name, fn in work.items():
            for e in engs:
                fn(e)                       # warm: scratch and staging sized
            per = [0.0] * T

            def run(t):
                t0 = time.perf_counter()
                for _ in range(a.calls):
                    fn(engs[t])
                per[t] = (time.perf_counter() - t0) / a.calls

            def timed():
                th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
                t0 = time.perf_counter()
                for x in th:
                    x.start()
                for x in th:
                    x.join()
                return time.perf_counter() - t0

            wall = timed()                        # call time: profiling off
            call = 1e3 * sum(per) / T
            for e in engs:
                e.reset_stats()
                e.set_profiling(True)
            timed()                               # kernel time: HIP events on
            kms = 0.0
            for e in engs:
                e.set_profiling(False)
                for k in range(8):
                    n, ms_ = e.kernel_stats(k)
                    kms += ms_
            kper = kms / (T * a.calls)
            print(f"T={T:2d} {name:18s} call {call:7.3f} ms  kernels {kper:7.3f} ms  "
                  f"calls/s {T * a.calls / wall:9.0f}", flush=True)
        for e in engs:
            e.close()
    base.close()


if __name__ == "__main__":
    main()
