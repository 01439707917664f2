"""SW-only benchmark: n seed-extension DP problems (150 x 210, end-to-end,
minsc -90) on the HBM-resident reference, timed with HIP events per launch."""
import argparse, ctypes as C, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bowtie2-server_amd"), os.path.join(ROOT, "bowtie2-server_amd", "tools"),
                os.path.join(ROOT, "tests", "golden")]
import torch
import bench, bt2g, bt2_index as bi

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--genome-mb", type=float, default=20)
a = ap.parse_args()
parts, names = bench.make_genome(a.genome_mb)
idx = bi.build_index_device(parts, names=names, device="cuda")
eng = bt2g.Engine(index=idx, device=0)
reads, quals = bench.make_reads(parts, a.n, 150, 42)
rng = np.random.default_rng(42)
sizes = np.array([len(p) for p in parts]); ref = rng.choice(len(parts), a.n, p=sizes / sizes.sum())
pos = (rng.random(a.n) * (sizes[ref] - 152)).astype(np.int64)
probs = np.zeros(a.n, bt2g.SWPROB_DTYPE)
probs["read"] = np.arange(a.n)
probs["fw"] = 1  # strand as generated is random; the score distribution is what matters
probs["refl"] = pos - 30
probs["win_off"] = -1
probs["refidx"] = ref
probs["ncol"] = 210
probs["minsc"] = -90
dev = torch.device("cuda")
tr, tq = torch.from_numpy(reads).to(dev), torch.from_numpy(quals).to(dev)
tl = torch.full((a.n,), 150, dtype=torch.int32, device=dev)
tp = torch.from_numpy(probs.view(np.uint8)).to(dev)
cap = 256
res = torch.empty((a.n, 8), dtype=torch.int32, device=dev)
cands = torch.empty((a.n, cap, 3), dtype=torch.int32, device=dev)
L = bt2g.lib()
bt2g._chk(L.bt2g_reserve_sw(eng.h, a.n, 210))
sc = bt2g.scoring(False)
P = lambda t: C.c_void_p(t.data_ptr())
S = C.c_void_p(torch.cuda.current_stream().cuda_stream)
def run():
    bt2g._chk(L.bt2g_sw_align_dev(eng.h, P(tr), P(tq), 150, P(tl), P(tp), a.n, None, C.byref(sc), 1, cap, P(res),
                                  P(cands), None, None, S))
run(); torch.cuda.synchronize()
eng.reset_stats(); eng.set_profiling(True)
for _ in range(a.iters):
    run()
torch.cuda.synchronize()
eng.set_profiling(False)
nl, ms = eng.kernel_stats(4)
cells = a.n * 150 * 210
print(f"sw_align {ms / nl:.3f} ms/launch, {cells / (ms / nl / 1e3) / 1e9:.0f} GCUPS, aligned "
      f"{float((res[:, 0] == 1).float().mean()):.3f}")
eng.close()
