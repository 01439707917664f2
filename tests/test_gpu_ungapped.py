"""GPU ungapped alignment (bt2g_ungapped: SwAligner::ungappedAlign,
aligner_sw.cpp:286-494) against the reference's own results (ug_* golden
fixtures made by the reference build) and against the oracle on a larger
synthetic batch.  Bit-exact: return code, score, offset, N counts, trims,
every edit."""
import math

import numpy as np
import pytest

from conftest import get_index, load_golden

pytestmark = pytest.mark.gpu


def _probs(g, minsc):
    import bt2g
    n = len(g["fw"])
    probs = np.zeros(n, bt2g.UGPROB_DTYPE)
    probs["read"] = np.arange(n)
    probs["fw"], probs["off"], probs["refidx"], probs["minsc"] = g["fw"], g["off"], g["refidx"], minsc
    return probs


def _check(res, edits, exp, ee, tag):
    for i in range(len(res)):
        r = res[i]
        got = [r["ret"]] + ([r["score"], r["refoff"], r["ns"], r["refns"], r["nedit"], r["trim5p"], r["trim3p"]]
                            if r["ret"] == 1 else [0] * 7)
        assert got == list(exp[i][:8]), (tag, i, got, exp[i])
        if r["ret"] == 1:
            e = edits[i, :r["nedit"]]
            assert np.array_equal(np.stack([e["pos"], e["type"], e["chr"], e["qchr"]], 1), ee[i]), (tag, i)


@pytest.mark.parametrize("name", ["lambda", "synth"])
@pytest.mark.parametrize("mode", ["ee", "loc"])
def test_ungapped_golden(name, mode):
    import bt2g
    g = load_golden("ug_" + name)
    with bt2g.Engine(index=get_index(name)) as eng:
        lens = np.full(len(g["fw"]), g["reads"].shape[1], np.uint32)
        res, edits = eng.ungapped(g["reads"], g["quals"], lens, _probs(g, g[mode + "_minsc"]), local=mode == "loc")
    exp = g[mode + "_out"]
    ee = [g[mode + "_edits"][g[mode + "_edit_off"][i]:g[mode + "_edit_off"][i + 1]] for i in range(len(exp))]
    _check(res, edits, exp, ee, (name, mode))
    assert (res["ret"] == 1).sum() > 200


@pytest.mark.parametrize("mode", ["ee", "loc"])
def test_ungapped_vs_oracle(mode):
    """2000 reads of mixed quality on the lambda genome, incl. off-end offsets."""
    import bt2g
    import sys
    sys.path.insert(0, __file__.rsplit("/", 1)[0] + "/golden")
    from make_golden_ug import make_inputs
    from oracle.oracle import Oracle
    from test_oracle_golden import ug_cases
    idx = get_index("lambda")
    reads, quals, fw, refidx, off = make_inputs(idx, 77, 2000)
    minsc = int(-0.6 - 0.6 * 150) if mode == "ee" else int(20 + 8 * math.log(150))
    g = dict(reads=reads, quals=quals, fw=fw, refidx=refidx, off=off)
    with bt2g.Engine(index=idx) as eng:
        res, edits = eng.ungapped(reads, quals, np.full(len(fw), 150, np.uint32), _probs(g, minsc),
                                  local=mode == "loc")
    orc = Oracle()
    exp, ee = [], []
    g.update({mode + "_out": np.zeros((len(fw), 10), np.int64), mode + "_edits": np.zeros((0, 4), np.int32),
              mode + "_edit_off": np.zeros(len(fw) + 1, np.int64), mode + "_minsc": np.full(len(fw), minsc)})
    for i, rd, q, rf, o, reflen, ms, f, _, _ in ug_cases(idx, g, mode):
        out, ed = orc.ungapped(rd, q, rf, o, reflen, ms, mode == "loc", f)
        exp.append(out)
        ee.append(ed)
    _check(res, edits, exp, ee, mode)
