#!/usr/bin/env python3
"""Summary of scripts/dropin_bench.py JSON lines: rates, CPU, per-seam engine calls.

  python scripts/dropin_summary.py gpurun_out/r03i/*.json
"""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.load(open(f))
    except (OSError, ValueError):
        continue
    for t in ("stock", "dropin"):
        if t not in d:
            continue
        x = d[t]
        print(f"{f} {t}: {x['rate']:.0f} {x['unit']}  cpu {x['server_cpu_s']:.1f}s  busy {x['server_cores_busy']:.2f}"
              f"  rss {x['server_rss_gb']:.1f} GB")
        th = x.get("server_threads_cpu") or {}
        print("   threads " + ", ".join(f"{k}:{v[1]:.1f}" for k, v in th.items()))
        ec = x.get("engine_calls")
        if not ec:
            continue
        names = [k for k in ec if isinstance(ec[k], list) and k not in ("queue_ms", "resume_ms", "spec")]
        for k, v in ec.items():
            if k == "spec":
                print(f"   spec prefetch: groups {v[0]}, DPs {v[1]}, hits {v[2]}, verify mismatches {v[3]}")
                continue
            if k in ("queue_ms", "resume_ms"):
                print(f"   {k} per call: " + ", ".join(f"{n}:{q / max(ec[n][0], 1):.2f}" for n, q in zip(names, v)))
                continue
            if k == "kernels":
                kk = {a: f"{b[1] / max(b[0], 1):.3f}ms x{b[0]}" for a, b in v.items() if b[0]}
                if kk:
                    print("   kernels", kk)
                continue
            print(f"   {k:12s} calls {v[0]:8d} cpu {v[1]:5d} batches {v[2]:6d} per-batch {v[0] / max(v[2], 1):6.1f}"
                  f"  call {v[3] / max(v[2], 1):5.2f} ms  wait/call {v[4] / max(v[0], 1):5.2f} ms")
    if "sam_identical" in d:
        print(f"   sam_identical {d['sam_identical']}  speedup {d.get('speedup', 0):.3f}")
