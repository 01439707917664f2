"""GPU DP framing (bt2g_frame, row A14): seed-extension and mate-search
rectangles for every PE policy and flag setting, bit-exact against the
oracle's restatement (itself pinned to the reference's own rectangles by
test_oracle_golden.py::test_frame).  Reference lengths come from the resident
index, so anchors are placed near both ends of its references."""
import numpy as np
import pytest

from conftest import get_index
from test_oracle_golden import orc  # noqa: F401  (session oracle fixture)

pytestmark = pytest.mark.gpu

SETTINGS = [
    (False, (3, 0, 500, 0, 0, 1, 1), 15, True),
    (True, (3, 0, 500, 0, 0, 1, 1), 15, True),
    (False, (1, 20, 300, 1, 1, 1, 1), 15, False),
    (False, (2, 0, 500, 0, 0, 0, 1), 15, True),
    (False, (4, 50, 300, 0, 1, 1, 0), 40, True),
    (True, (3, 100, 800, 1, 0, 1, 1), 40, False),
]


def _inputs(idx, rng, n, local):
    import bt2g
    reflens = np.array([len(c) for c in idx.ref_codes], np.int64)
    x = np.zeros(n, bt2g.FRAMEIN_DTYPE)
    x["kind"] = rng.integers(0, 2, n)
    x["refidx"] = rng.integers(0, len(reflens), n)
    tl = reflens[x["refidx"]]
    where = rng.integers(0, 4, n)
    x["off"] = np.select([where == 0, where == 1, where == 2],
                         [rng.integers(0, tl), rng.integers(-60, 60, n), tl - rng.integers(-60, 400, n)],
                         rng.integers(-700, tl + 700))
    lens = np.where(rng.random(n) < 0.6, 150, rng.integers(20, 300, n)).astype(np.uint32)
    x["read"] = np.arange(n)
    x["alen"] = np.where(rng.random(n) < 0.6, 150, rng.integers(20, 300, n))
    L = lens.astype(np.float64)
    minsc = (20 + 8 * np.log(L)) if local else (-0.6 - 0.6 * L)
    minsc = minsc.astype(np.int64)
    perfect = 2 * lens.astype(np.int64) if local else np.zeros(n, np.int64)
    pick = rng.random(n)
    minsc = np.where(pick < 0.15, perfect, np.where(pick < 0.3, minsc - rng.integers(0, 200, n), minsc))
    x["minsc"] = minsc
    x["fw"] = rng.integers(0, 2, n)
    x["anchor1"] = rng.integers(0, 2, n)
    return x, lens, tl


@pytest.mark.parametrize("k", range(len(SETTINGS)))
def test_frame_vs_oracle(orc, k):  # noqa: F811
    import bt2g
    local, pe, maxhalf, ttr = SETTINGS[k]
    idx = get_index("synth")
    rng = np.random.default_rng(100 + k)
    x, lens, tl = _inputs(idx, rng, 3000, local)
    pol = bt2g.pe_policy(policy=pe[0], minfrag=pe[1], maxfrag=pe[2], flip=bool(pe[3]), dovetail=bool(pe[4]),
                         olap=bool(pe[5]), expand=bool(pe[6]), local=local)
    with bt2g.Engine(index=idx) as eng:
        probs, rects, ok = eng.frame(x, lens, local=local, pe=pol, maxhalf=maxhalf, trim_to_ref=ttr)
    nok = 0
    for i in range(len(x)):
        e = orc.frame(int(x["kind"][i]), int(x["off"][i]), int(lens[i]), int(tl[i]), int(x["minsc"][i]),
                      int(x["fw"][i]), int(x["anchor1"][i]), int(x["alen"][i]), local=local, pe=pe,
                      maxhalf=maxhalf, trim_to_ref=ttr)
        assert ok[i] == e[0], (k, i)
        if not e[0]:
            continue
        nok += 1
        got = (1, int(probs["fw"][i]), int(probs["refl"][i]), int(probs["ncol"][i]), int(rects["triml"][i]),
               int(rects["corel"][i]), int(rects["corer"][i]))
        assert got == e, (k, i, got, e)
        assert probs["read"][i] == i and probs["refidx"][i] == x["refidx"][i] and probs["win_off"][i] == -1
        assert probs["minsc"][i] == x["minsc"][i]
    assert nok > 2500
