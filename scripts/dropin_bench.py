#!/usr/bin/env python3
"""End-to-end timing on the reference's real schedule.

The stock reference server (oracle/_ref/bowtie2-align-server-s, CPU, -p <usable
cores>) and the same server with its seams bound to the MI355X engines
(integration/bin/bowtie2-align-server-gpu, integration/bt2g_seams.cpp, -p <many>
workers feeding the batching dispatcher) align the same reads against the same
index, each driven by k concurrent reference clients with <= 10 000 reads per
connection.  Prints one JSON line: both rates, the SAM comparison, the engine
call / batch counts and the CPU budget of the host.

  python scripts/dropin_bench.py --genome-mb 200 --reads 200000 [--mode paired] [--args --local]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "bowtie2-server_amd"), os.path.join(ROOT, "bowtie2-server_amd", "tools"),
           os.path.join(ROOT, "tests", "golden")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genome-mb", type=float, default=200.0)
    ap.add_argument("--reads", type=int, default=200_000, help="reads (paired: pairs)")
    ap.add_argument("--mode", choices=("unpaired", "paired"), default="unpaired")
    ap.add_argument("--args", nargs="*", default=[], help="server alignment options (e.g. --local)")
    ap.add_argument("--k", type=int, default=8, help="concurrent client connections")
    ap.add_argument("--gpu-workers", type=int, default=512)
    ap.add_argument("--cpu-threads", type=int, default=0, help="stock server -p (0: usable host cores)")
    ap.add_argument("--workdir", default="/tmp/dropin_bench")
    ap.add_argument("--skip-stock", action="store_true")
    ap.add_argument("--warmup-chunks", type=int, default=1, help="chunks sent untimed first (both servers)")
    ap.add_argument("--dropin-args", default="",
                    help="extra server options for the drop-in only, one string (throughput knobs that do not "
                         "change alignments, e.g. --dropin-args='--reads-per-batch 4')")
    ap.add_argument("--dropin-binary", default="", help="default integration/bin/bowtie2-align-server-gpu "
                                                       "(-stub: the binding over the CPU stand-in)")
    ap.add_argument("--dropin-prefix", default="", help="a launcher before the drop-in's command line, one string "
                    "(e.g. 'rocprofv3 --kernel-trace --stats -d DIR --'; the server gets BT2G_EXIT_CLEAN=1)")
    a = ap.parse_args()

    import bench
    import bt2_index as bi
    from oracle import ref_server as rs

    os.makedirs(a.workdir, exist_ok=True)
    base = os.path.join(a.workdir, "g")
    t0 = time.time()
    parts, names = bench.make_genome(a.genome_mb)
    if not os.path.exists(base + ".rev.2.bt2"):
        import torch
        dev = "cuda" if torch.cuda.is_available() else "cpu"
        idx = bi.build_index_device(parts, names=names, device=dev) if dev == "cuda" else \
            bi.build_index(parts, names=names)
        bi.write_index(base, idx)
        del idx
        if dev == "cuda":
            torch.cuda.empty_cache()
    log(f"genome + index {time.time() - t0:.1f}s")
    if a.mode == "paired":
        r, q = bench.make_pairs(parts, a.reads, 150, 42)
        n = a.reads
        chunks = rs.write_fastq_chunks(a.workdir, r[:n], q[:n], codes2=r[n:], quals2=q[n:])
    else:
        r, q = bench.make_reads(parts, a.reads, 150, 42)
        chunks = rs.write_fastq_chunks(a.workdir, r, q)
    cpus = rs.host_cpus()
    threads = a.cpu_threads or cpus["usable"]
    out = {"reads": a.reads, "mode": a.mode, "args": a.args, "dropin_args": a.dropin_args, "genome_mb": a.genome_mb,
           "k": a.k, "host": cpus}
    sams = {}
    runs = [] if a.skip_stock else [("stock", rs.SERVER, threads)]
    runs.append(("dropin", a.dropin_binary or os.path.join(os.path.dirname(rs.HERE), "integration", "bin", "bowtie2-align-server-gpu"), a.gpu_workers))
    for tag, binary, th in runs:
        stats = os.path.join(a.workdir, f"stats_{tag}.json")
        env = rs.dropin_env(base, stats)
        prefix = a.dropin_prefix.split() if tag == "dropin" else []
        if prefix:
            env["BT2G_EXIT_CLEAN"] = "1"
        with rs.Server(base, threads=th, args=a.args + (a.dropin_args.split() if tag == "dropin" else []), binary=binary, env=env,
                       log_path=os.path.join(a.workdir, f"server_{tag}.log"), prefix=prefix) as s:
            log(f"{tag}: server ready in {s.load_s:.1f}s (-p {th})")
            dt, outs = s.run(chunks, k=a.k, warmup=chunks[:a.warmup_chunks])
        sams[tag] = rs.sorted_records(outs)
        unit = "pairs/s" if a.mode == "paired" else "reads/s"
        out[tag] = {"seconds": dt, "rate": a.reads / dt, "unit": unit, "threads": th, "records": len(sams[tag]),
                    "server_cpu_s": s.last_cpu_s, "server_cores_busy": s.last_cpu_s / dt, "server_rss_gb": s.last_rss_gb,
                    "host_cpu_s": s.last_host_cpu_s, "throttled_s": s.last_throttled_s,
                    "server_threads_cpu": s.last_threads}
        time.sleep(0.5)
        if os.path.exists(stats):
            out[tag]["engine_calls"] = json.load(open(stats))
        log(f"{tag}: {a.reads / dt:.0f} {unit} ({dt:.2f}s)")
    if "stock" in sams:
        a_, b_ = sams["stock"], sams["dropin"]
        out["sam_identical"] = a_ == b_
        out["sam_records_differing"] = sum(1 for x, y in zip(a_, b_) if x != y) + abs(len(a_) - len(b_))
        out["speedup"] = out["dropin"]["rate"] / out["stock"]["rate"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
