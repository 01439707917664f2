"""Latency of the FM walkers at the batch server's call sizes on an idle GPU:
k_exact_sweep / the one-mm family / k_seed_search on n reads of the bench's
hg38-like genome (ms per launch from the engine's own HIP-event timing), to
tell the walk's inherent step latency from what the server's concurrent calls
add (the server sees ~0.57 ms per exact-sweep launch of ~540 reads).

    python scripts/micro/sweep_latency.py [--mb 3100]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "bowtie2-server_amd"), os.path.join(ROOT, "bowtie2-server_amd", "tools"),
          os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=3100.0)
    a = ap.parse_args()
    import bench
    import bt2_index as bi
    import bt2g
    import tempfile
    t0 = time.time()
    parts, names = bench.make_genome(a.mb)
    # (bench.py's index cache: a bench run after this one in the same call reads it)
    cache = os.path.join(tempfile.gettempdir(), "bt2g_bench_index", f"hg38like_{a.mb:g}mb", "g")
    if os.path.exists(cache + ".rev.2.bt2"):
        idx = bi.read_index(cache)
    else:
        idx = bi.build_index_device(parts, names=names, device="cuda:0")
        os.makedirs(os.path.dirname(cache), exist_ok=True)
        bi.write_index(cache, idx)
    print(f"index {a.mb:.0f} Mbp in {time.time() - t0:.0f} s", flush=True)
    reads, quals = bench.make_reads(parts, 65536, 150, 3)
    lens = np.full(len(reads), 150, np.uint32)
    minsc = np.full(len(reads), -90, np.int32)
    with bt2g.Engine(index=idx, device=0) as eng:
        eng.set_profiling(True)
        for n in (256, 540, 1024, 4096, 16384, 65536):
            r, q, l, m = reads[:n], quals[:n], lens[:n], minsc[:n]
            eng.exact_sweep(r, l)                          # warm
            eng.reset_stats()
            for _ in range(5):
                eng.exact_sweep(r, l)
            la, ms = eng.kernel_stats(0)
            eng.reset_stats()
            for _ in range(5):
                eng.exact_sweep_1mm(r, q, l, m, False)
            l1, ms1 = eng.kernel_stats(2)
            eng.reset_stats()
            for _ in range(5):
                eng.seed_search(r, l, 22, 15, 0, 16)
            l2, ms2 = eng.kernel_stats(1)
            print(f"n {n:6d}: k_exact_sweep {ms / la:7.3f} ms ({ms / la * 1e3 / 150:5.2f} us per step)  "
                  f"one-mm family {ms1 / max(1, l1):7.3f} ms  k_seed_search {ms2 / max(1, l2):7.3f} ms", flush=True)


if __name__ == "__main__":
    main()
