#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 --pmc passes (one pass per counter):

  python scripts/pmc_summary.py FETCH_DIR WRITE_DIR OUT.json [FETCH_BENCH.json WRITE_BENCH.json]

With the two passes' bench.py lines (run with BT2G_KWORK=1 in the server:
server.work_by_kernel, the algorithmic bytes the server counted per kernel
id), the summary also carries each pass's algorithmic work, so that bench.py
sets the counters' bytes against the work of the same dispatches
(bench.pmc_ratio).

Every *counter_collection.csv under each directory (one per profiled process)
is read; per kernel name (template arguments kept), the mean FETCH_SIZE and
WRITE_SIZE per dispatch in KiB and bytes.  FETCH_SIZE is also given doubled:
on gfx950 it counts 64 B per 128-B request for wide coalesced reads
(/opt/skills/guides/MI355X_MICROARCH.md, HBM section), uncalibrated for 64-B
gathers -- both figures are kept."""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(d, counter):
    vals = collections.defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name", counter) != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            vals[name].append(float(r["Counter_Value"]))
    return vals


def main():
    fd, wd, out = sys.argv[1:4]
    works = {}
    for key, path in zip(("fetch", "write"), sys.argv[4:6]):
        try:
            works[key] = json.load(open(path))["server"]["work_by_kernel"]
        except (OSError, ValueError, KeyError, TypeError):
            print(f"no work_by_kernel in {path}")
    f = per_kernel(fd, "FETCH_SIZE")
    w = per_kernel(wd, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        fk = sum(f[k]) / len(f[k]) if f.get(k) else None
        wk = sum(w[k]) / len(w[k]) if w.get(k) else None
        res[k] = {"dispatches": max(len(f.get(k, [])), len(w.get(k, []))),
                  "fetch_kib": fk, "write_kib": wk,
                  "fetch_bytes": fk * 1024 if fk is not None else None,
                  "fetch_bytes_x2": fk * 2048 if fk is not None else None,
                  "write_bytes": wk * 1024 if wk is not None else None}
    # the build the counters were taken on: bench.py flags a summary whose engine
    # library differs from the one it benchmarks (traffic_stale)
    import hashlib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    build = {}
    for rel in ("bowtie2-server_amd/libbt2g.so", "integration/bin/bowtie2-align-server-batch"):
        try:
            build[rel] = hashlib.sha256(open(os.path.join(root, rel), "rb").read()).hexdigest()
        except OSError:
            pass
    json.dump({"source": {"fetch": fd, "write": wd}, "build_sha256": build, "kernels": res,
               "work_by_kernel": works}, open(out, "w"), indent=1)
    for k, v in sorted(res.items(), key=lambda kv: -(kv[1]["dispatches"] or 0))[:20]:
        print(k[:80], v["dispatches"], v["fetch_kib"], v["write_kib"])


if __name__ == "__main__":
    main()
