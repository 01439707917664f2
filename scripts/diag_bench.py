"""Diagnostics for bench.py's pipeline on one GPU: index-builder agreement
(cuda vs cpu) and per-stage hit statistics against the reads' true origin."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "bowtie2-server_amd"), os.path.join(ROOT, "bowtie2-server_amd", "tools"),
          os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import torch
import bench, bt2g, bt2_index as bi

mb = float(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 20000
parts, names = bench.make_genome(mb)
t = time.time()
ig = bi.build_index_device(parts, names=names, device="cuda")
print("gpu build", time.time() - t, flush=True)
t = time.time()
ic = bi.build_index_device(parts, names=names, device="cpu")
print("cpu build", time.time() - t, flush=True)
for side in ("fw", "bw"):
    a, b = getattr(ig, side), getattr(ic, side)
    for f in ("ebwt", "ftab", "eftab", "offs", "fchr", "rstarts"):
        x, y = np.asarray(getattr(a, f)), np.asarray(getattr(b, f))
        print(side, f, x.shape == y.shape and np.array_equal(x, y), flush=True)
    print(side, "zoff", a.zoff, b.zoff)
reads, quals = bench.make_reads(parts, n, 150, 42)
rng = np.random.default_rng(42)
sizes = np.array([len(p) for p in parts]); ref = rng.choice(len(parts), n, p=sizes / sizes.sum())
pos = (rng.random(n) * (sizes[ref] - 152)).astype(np.int64)
eng = bt2g.Engine(index=ig, device=0)
pipe = bench.Pipeline(eng, ig, torch.from_numpy(reads).cuda(), torch.from_numpy(quals).cuda(), 150)
al = pipe.step(keep=True).cpu().numpy()
last = pipe.last
print("aligned", al.mean(), "exact", (np.minimum(pipe.sweep[:, 0].cpu().numpy(), pipe.sweep[:, 1].cpu().numpy()) == 0).mean())
pr = last["probs"].cpu().numpy()
pw = pr.view(np.int32)
res = pipe.res[:last["npb"]].cpu().numpy()
print("npb", last["npb"], "res aligned frac", (res[:, 0] == 1).mean(), "flags", np.unique(res[:, 7], return_counts=True))
rd = pw[:, 0]
print("problem on true ref", (pw[:, 6] == ref[rd]).mean(), "refl==pos-30", (pr[:, 1] == pos[rd] - 30).mean())
print(pr[:5], pos[rd[:5]], ref[rd[:5]])
eng.close()
