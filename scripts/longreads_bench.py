#!/usr/bin/env python3
"""BASELINE configs[0] on the reference's real schedule: the lambda genome and the
reference's example/reads/longreads.fq (6 000 reads of 40-2 561 bp, committed as
tests/golden/longreads.fq.gz), stock server vs the drop-in, sorted SAM compared.

tests/test_integration.py::test_dropin_longreads_gpu runs the same comparison with
two workers (a parity test); here the drop-in gets the worker count it is meant to
run with, so its engine calls batch across reads.  Prints one JSON line.

  python scripts/longreads_bench.py [--workers 512] [--cpu-threads 0]
"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "bowtie2-server_amd", "tools")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import bt2_index as bi  # noqa: E402
from oracle import ref_server as rs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=512, help="drop-in server -p (fibers)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="stock server -p (0: usable host cores)")
    ap.add_argument("--dropin-binary", default=os.path.join(ROOT, "integration", "bin", "bowtie2-align-server-gpu"))
    ap.add_argument("--repeat", type=int, default=1, help="connections of the whole file, one at a time")
    ap.add_argument("--workdir", default="", help="index, server logs (default: a fresh temporary directory)")
    a = ap.parse_args()
    d = a.workdir or tempfile.mkdtemp(prefix="bt2lr_")
    os.makedirs(d, exist_ok=True)
    base = os.path.join(d, "lambda_virus")
    bi.write_index(base, bi.build_from_fasta(os.path.join(ROOT, "tests", "golden", "lambda_virus.fa")))
    reads = os.path.join(ROOT, "tests", "golden", "longreads.fq.gz")
    threads = a.cpu_threads or rs.host_cpus()["usable"]
    out = {"config": "configs[0]: lambda_virus, longreads.fq (6000 reads, 40-2561 bp)", "repeat": a.repeat}
    sams = {}
    for tag, binary, th in (("stock", rs.SERVER, threads),
                            ("dropin", a.dropin_binary, a.workers)):
        stats = os.path.join(d, f"stats_{tag}.json")
        with rs.Server(base, threads=th, binary=binary, env=rs.dropin_env(base, stats),
                       log_path=os.path.join(d, f"server_{tag}.log")) as s:
            dt, outs = s.run([["-U", reads]] * a.repeat, k=1)
        sams[tag] = rs.sorted_records(outs)
        out[tag] = {"seconds": dt, "reads_per_s": 6000 * a.repeat / dt, "threads": th,
                    "records": len(sams[tag]), "server_cpu_s": s.last_cpu_s}
        if os.path.exists(stats):
            out[tag]["engine_calls"] = json.load(open(stats))
        print(f"{tag}: {dt:.2f}s", file=sys.stderr, flush=True)
    out["sam_identical"] = sams["stock"] == sams["dropin"]
    out["dropin_vs_stock"] = out["stock"]["seconds"] / out["dropin"]["seconds"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
