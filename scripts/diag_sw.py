"""Compare the packed end-to-end SW path with the reference's recorded outputs
(tests/golden/sw_rand_ee.npz) problem by problem, in batch and alone."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bowtie2-server_amd"), os.path.join(ROOT, "tests")]
import bt2g
from conftest import get_index, load_golden
from test_gpu_sw import golden_batch
g = load_golden("sw_rand_ee")
probs = golden_batch(g)
eng = bt2g.Engine(index=get_index("lambda"))
res, c, _ = eng.sw_align(g["reads"], g["quals"], g["lens"], probs, windows=g["rf"])
out = g["out"]
bad = np.nonzero((res["aligned"] != out[:, 0]) | ((out[:, 0] == 1) & (res["best"] != out[:, 1])))[0]
print("mismatches", len(bad), bad[:20])
for p in bad[:8]:
    r1, _, _ = eng.sw_align(g["reads"], g["quals"], g["lens"], probs[p:p + 1], windows=g["rf"])
    ri = g["rd_index"][p]
    print(p, "batch", res["best"][p], "alone", r1["best"][0], "ref", out[p, 1], "L", g["lens"][ri],
          "ncol", probs["ncol"][p], "minsc", probs["minsc"][p])
eng.close()
# stride sweep on problem 17 (changes the number of dead rows / lanes)
eng = bt2g.Engine(index=get_index("lambda"))
p = 17
ri = g["rd_index"][p]
L = int(g["lens"][ri])
for stride in (37, 40, 48, 64, 100, 128, 150, 160, 200, 256):
    rd = np.full((1, stride), 4, np.uint8); qu = np.full((1, stride), 73, np.uint8)
    rd[0, :L] = g["reads"][ri, :L]; qu[0, :L] = g["quals"][ri, :L]
    pr = probs[p:p + 1].copy(); pr["read"] = 0
    r1, c1, _ = eng.sw_align(rd, qu, np.array([L], np.uint32), pr, windows=g["rf"])
    print("stride", stride, "S", (stride + 15) // 16, "best", r1["best"][0], "ncand", r1["ncand"][0], c1[0, :3])
eng.close()
