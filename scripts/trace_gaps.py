#!/usr/bin/env python3
"""Timeline summary of a rocprofv3 --kernel-trace --memory-copy-trace run.

  python scripts/trace_gaps.py TRACE_DIR

Reads every *kernel_trace.csv and *memory_copy_trace.csv under TRACE_DIR and
prints: per kernel name, launches and mean / p50 / p99 duration; the copies by
direction and size bucket with their durations; per hardware queue, its
dispatches and busy fraction; the union of kernel time over the run (GPU busy)
and the mean number of kernels in flight while any is.  What it is for: where
an engine call's time goes besides its kernels (copy-engine waits, queues
shared between streams)."""
import collections
import csv
import glob
import os
import sys


def rows(d, pat):
    out = []
    for p in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def pct(v, q):
    if not v:
        return 0.0
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    d = sys.argv[1]
    ks = rows(d, "*kernel_trace.csv")
    cs = rows(d, "*memory_copy_trace.csv")
    if not ks:
        print("no kernel trace under", d)
        return
    print("kernel trace columns:", list(ks[0].keys()))
    if cs:
        print("copy trace columns:", list(cs[0].keys()))
    by = collections.defaultdict(list)
    iv, q = [], collections.defaultdict(list)
    for r in ks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()[:60]
        by[name].append((e - s) / 1e3)
        iv.append((s, e))
        q[r.get("Queue_Id", "?")].append((s, e))
    t0, t1 = min(s for s, _ in iv), max(e for _, e in iv)
    span = (t1 - t0) / 1e3
    busy = union(iv) / 1e3
    inflight = sum(e - s for s, e in iv) / 1e3 / max(busy, 1e-9)
    print(f"span {span / 1e3:.1f} ms, GPU busy (union of kernels) {busy / span:.3f}, kernels in flight while busy {inflight:.2f}")
    print("\nkernel, launches, mean us, p50, p99, total ms")
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {name:60s} {len(v):7d} {sum(v) / len(v):9.1f} {pct(v, .5):9.1f} {pct(v, .99):9.1f} {sum(v) / 1e3:9.1f}")
    print("\nqueue, dispatches, busy fraction of span")
    for k, v in sorted(q.items(), key=lambda kv: -len(kv[1])):
        print(f"  {k:>6s} {len(v):7d} {union(v) / 1e3 / span:.3f}")
    if cs:
        cb = collections.defaultdict(list)
        civ = []
        for r in cs:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            nb = int(r.get("Bytes") or r.get("Size") or 0)
            b = 0
            while (1 << (b + 1)) <= max(nb, 1) and b < 40:
                b += 1
            key = (r.get("Direction") or r.get("Kind") or "?", b)
            cb[key].append((e - s) / 1e3)
            civ.append((s, e))
        print(f"\ncopies {len(cs)}, copy engine busy (union) {union(civ) / 1e3 / span:.3f} of span")
        print("direction, size >= 2^b bytes, count, mean us, p50, p99")
        for (dr, b), v in sorted(cb.items()):
            print(f"  {dr:24s} 2^{b:<3d} {len(v):7d} {sum(v) / len(v):9.1f} {pct(v, .5):9.1f} {pct(v, .99):9.1f}")


if __name__ == "__main__":
    main()
