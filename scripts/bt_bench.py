"""Fill + backtrace benchmark: n seed-extension DP problems (150 x 210,
end-to-end, minsc -90, core diagonals [15, 45]) placed on the reads' true
positions in a synthetic genome, as bench.py's pipeline produces them.
Prints per-launch times of the fill (kernel id 4) and the backtrace (id 5).
BT2G_LIB selects an experimental build (make -C bowtie2-server_amd exp ...)."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bowtie2-server_amd"), os.path.join(ROOT, "bowtie2-server_amd", "tools"),
                os.path.join(ROOT, "tests", "golden")]
import torch  # noqa: E402
import bench  # noqa: E402
import bt2g  # noqa: E402
import bt2_index as bi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--genome-mb", type=float, default=20)
ap.add_argument("--maxaln", type=int, default=8)
ap.add_argument("--save", default="", help="write naln/alns/edits (npz) for an A/B comparison")
ap.add_argument("--compare", default="", help="compare with a --save file")
a = ap.parse_args()
parts, names = bench.make_genome(a.genome_mb)
g = parts[0]
idx = bi.build_index_device(parts, names=names, device="cuda")
eng = bt2g.Engine(index=idx, device=0)
import synth  # noqa: E402
rng = np.random.default_rng(7)
n, L, maxgap = a.n, 150, 15
pos = rng.integers(100, len(g) - 300, n)
fw = rng.random(n) < 0.5
win = g[pos[:, None] + np.arange(L + 1)[None, :]]
reads = win[:, :L].copy()
ind = np.nonzero(rng.random(n) < 0.05)[0]
for i in ind:
    k = rng.integers(1, L - 1)
    if rng.random() < 0.5:
        reads[i, k:] = win[i, k + 1:L + 1]
    else:
        reads[i, k + 1:] = win[i, k:L - 1]
reads[~fw] = np.where(reads[~fw] > 3, 4, 3 - reads[~fw])[:, ::-1]
m = rng.random((n, L)) < 0.004
reads[m] = (reads[m] + rng.integers(1, 4, m.sum(), dtype=np.uint8)) % 4
quals = (rng.integers(2, 41, (n, L), dtype=np.uint8) + 33).astype(np.uint8)
probs = np.zeros(n, bt2g.SWPROB_DTYPE)
probs["read"] = np.arange(n)
probs["fw"] = fw
probs["refl"] = pos - 2 * maxgap
probs["win_off"] = -1
probs["refidx"] = 0
probs["ncol"] = L + 4 * maxgap
probs["minsc"] = -90
dev = torch.device("cuda")
tr, tq = torch.from_numpy(reads.astype(np.uint8)).to(dev), torch.from_numpy(quals).to(dev)
tl = torch.full((n,), L, dtype=torch.int32, device=dev)
tp = torch.from_numpy(probs.view(np.uint8)).to(dev)
rects = torch.zeros((n, 4), dtype=torch.int32, device=dev)
rects[:, 1], rects[:, 2] = maxgap, 3 * maxgap
cap, maxaln, maxedit = 256, a.maxaln, 64
res = torch.empty((n, 8), dtype=torch.int32, device=dev)
cands = torch.empty((n, cap, 3), dtype=torch.int32, device=dev)
naln = torch.empty(n, dtype=torch.int32, device=dev)
alns = torch.empty((n, maxaln, 10), dtype=torch.int32, device=dev)
edits = torch.empty((n, maxaln, maxedit, 2), dtype=torch.int32, device=dev)
L_ = bt2g.lib()
bt2g._chk(L_.bt2g_reserve_sw_bt(eng.h, n, L, L + 4 * maxgap, 1))
sc = bt2g.scoring(False)
P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
S = C.c_void_p(torch.cuda.current_stream().cuda_stream)


def run():
    bt2g._chk(L_.bt2g_sw_align_bt_dev(eng.h, P(tr), P(tq), L, P(tl), P(tp), n, None, P(rects), C.byref(sc), 1, cap,
                                      P(res), P(cands), maxaln, maxedit, P(naln), P(alns), P(edits), None, S))


run()
torch.cuda.synchronize()
prof = getattr(bt2g.lib(), "bt2g_bt_prof_read", None) if "prof" in bt2g.LIB_PATH else None
if prof is not None:
    # profiling build (make -C bowtie2-server_amd exp V=btprof FLAGS=-DBT2G_BT_PROF=1): work counters of one launch
    cnt = (C.c_ulonglong * 16)()
    prof(cnt)
    run()
    torch.cuda.synchronize()
    nw = min((n + 63) // 64, 1 << 16)
    t0 = np.zeros(nw, np.uint64); t1 = np.zeros(nw, np.uint64); ws = np.zeros(nw, np.uint32)
    wok = bt2g.lib().bt2g_bt_prof_waves(t0.ctypes.data_as(C.c_void_p), t1.ctypes.data_as(C.c_void_p),
                                        ws.ctypes.data_as(C.c_void_p), C.c_uint32(nw)) == 0
    prof(cnt)
    names = ["walks", "steps", "colhit16_blocks", "escan_rounds", "candidates", "dom_tests", "replays", "hget",
             "chunk_reloads", "tile_loads", "tile_writebacks", "colhit8_blocks", "dps_walked", "", "", "wave_steps"]
    d = {k: int(v) for k, v in zip(names, cnt) if k}
    d["lane_utilization"] = d["steps"] / max(1, d["wave_steps"])
    print("bt_prof", d, flush=True)
    if wok:
        ok = t1 > 0
        t0, t1, ws = t0[ok].astype(np.float64), t1[ok].astype(np.float64), ws[ok]
        dur = (t1 - t0) / 100.0                      # us (100 MHz)
        span = (t1.max() - t0.min()) / 100.0
        q = np.percentile(dur, [50, 90, 99, 100])
        print(f"bt_waves n={ok.sum()} span {span:.0f} us; wave duration us p50 {q[0]:.0f} p90 {q[1]:.0f} "
              f"p99 {q[2]:.0f} max {q[3]:.0f}; sum {dur.sum()/1e6:.2f} wave-s; us per wave-step "
              f"{(dur / np.maximum(ws, 1)).mean():.2f}; concurrent waves ~{dur.sum() / max(span, 1):.0f}", flush=True)
        late = t0 > t0.min() + 0.5 * (t1.max() - t0.min())
        print(f"bt_waves started in the 2nd half of the span: {late.sum()}, their steps p50 {np.median(ws[late]) if late.any() else 0}", flush=True)
eng.reset_stats()
eng.set_profiling(True)
for _ in range(a.iters):
    run()
torch.cuda.synchronize()
eng.set_profiling(False)
f = eng.kernel_stats(4)
b = eng.kernel_stats(5)
nal = naln.cpu().numpy()
nc = res[:, 6].cpu().numpy()
print(f"lib={os.path.basename(bt2g.LIB_PATH)} n={n} fill {f[1]/f[0]:.3f} ms  backtrace {b[1]/b[0]:.3f} ms  "
      f"aligned {(nal > 0).mean():.4f} alns {nal.clip(0).sum()} mean ncand {nc.mean():.1f}", flush=True)
if a.save or a.compare:
    out = {"naln": nal, "alns": alns.cpu().numpy(), "edits": edits.cpu().numpy()}
    k = out["naln"].clip(0)
    mask = np.arange(maxaln)[None, :] < k[:, None]
    out["alns"] = np.where(mask[:, :, None], out["alns"], 0)
    ne = out["alns"][:, :, 6]
    emask = np.arange(maxedit)[None, None, :] < ne[:, :, None]
    out["edits"] = np.where(emask[:, :, :, None], out["edits"], 0)
    if a.save:
        np.savez_compressed(a.save, **out)
    if a.compare:
        ref = np.load(a.compare)
        bad = {key: int((ref[key] != out[key]).reshape(n, -1).any(1).sum()) for key in out}
        print("compare vs", a.compare, "problems differing:", bad, flush=True)
eng.close()
