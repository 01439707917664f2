"""Pins the CPU oracle (oracle/oracle.c) to the reference's own outputs
(tests/golden/*.npz, generated from oracle/_ref by make_golden.py)."""
import numpy as np
import pytest

from conftest import get_index, load_golden


@pytest.fixture(scope="module")
def orc():
    from oracle.oracle import Oracle
    return Oracle()


def _ebwts(orc, name):
    idx = get_index(name)
    return orc.ebwt(idx.fw, True), orc.ebwt(idx.bw, False)


@pytest.mark.parametrize("name", ["lambda", "synth"])
def test_exact_sweep(orc, name):
    g = load_golden("fm_" + name)
    fe, _ = _ebwts(orc, name)
    out = orc.exact_sweep(fe, g["reads"], g["lens"])
    assert np.array_equal(out, g["exact"].astype(np.uint64))


@pytest.mark.parametrize("name", ["lambda", "synth"])
@pytest.mark.parametrize("pol", ["s22", "s20", "s10"])
def test_seed_search(orc, name, pol):
    g = load_golden("fm_" + name)
    fe, be = _ebwts(orc, name)
    L, iv, off = g["seedpol_" + pol]
    out, ns, ops = orc.seed_search(fe, be, g["reads"], g["lens"], int(L), int(iv), int(off), 64)
    assert np.array_equal(ns, g["seedn_" + pol])
    assert np.array_equal(out, g["seed_" + pol])
    assert np.array_equal(ops, g["seedops_" + pol])


def _mm_eq(ref, refn, out, cnt):
    assert np.array_equal(cnt, refn)
    for i in range(len(refn)):
        for k in range(refn[i]):
            x, y = ref[i, k], out[i, k]
            assert tuple(x[:5]) == tuple(y[:5]), (i, k)
            assert (x[5] & 0xff) == ord("ACGTN"[y[5]]) and (x[5] >> 8) == ord("ACGTN"[y[6]]), (i, k)


@pytest.mark.parametrize("name", ["lambda", "synth"])
@pytest.mark.parametrize("mode", ["ee", "loc"])
def test_one_mm(orc, name, mode):
    g = load_golden("fm_" + name)
    fe, be = _ebwts(orc, name)
    out, cnt, ops = orc.one_mm(fe, be, g["reads"], g["quals"], g["lens"], g["mmminsc_" + mode], mode == "loc")
    _mm_eq(g["mm_" + mode], g["mmn_" + mode], out, cnt)
    assert np.array_equal(ops, g["mmops_" + mode])


@pytest.mark.parametrize("name", ["lambda", "synth"])
def test_get_offset_and_bilf(orc, name):
    g = load_golden("fm_" + name)
    idx = get_index(name)
    fe, be = _ebwts(orc, name)
    got = [orc.get_offset(fe, int(r)) for r in g["off_rows"]]
    assert np.array_equal(np.array(got, np.uint32), g["off_vals"])
    for row in g["bilf"]:
        which, a, b, tp0 = (int(x) for x in row[:4])
        arrs = orc.bilf(be if which else fe, a, b, tp0)
        assert np.array_equal(np.concatenate(arrs), row[4:].astype(np.uint32)), row[:4]
    assert idx.fw.length > 0


@pytest.mark.parametrize("name", ["lambda", "synth"])
def test_extend(orc, name):
    """SwDriver::extend on every seed hit the reference's seed search found (ext_<name>.npz)."""
    g = load_golden("ext_" + name)
    fe, be = _ebwts(orc, name)
    bad = 0
    for k, (r, fw, off, ln, tf, bf, tb, bb) in enumerate(g["ranges"]):
        seq = g["reads"][r, :g["lens"][r]]
        got = orc.extend(fe, be, seq, int(fw), int(off), int(ln), int(tf), int(bf), int(tb), int(bb))
        bad += int(not np.array_equal(got, g["out"][k]))
    assert bad == 0


def sw_problems(g):
    """Yield (read codes as aligned, quals as aligned, rfmask, minsc, fw, expected out, expected cands)."""
    for p in range(len(g["rd_index"])):
        ri = g["rd_index"][p]
        L = int(g["lens"][ri])
        rd, q = g["reads"][ri, :L], g["quals"][ri, :L]
        fw = bool(g["fw"][p])
        if not fw:
            rd = np.where(rd > 3, 4, 3 - rd)[::-1]
            q = q[::-1]
        rf = g["rf"][g["rf_off"][p]:g["rf_off"][p + 1]]
        c = g["cands"][g["cand_off"][p]:g["cand_off"][p + 1]]
        yield p, rd, q, rf, int(g["minsc"][p]), fw, g["out"][p], c


@pytest.mark.parametrize("fx", ["sw_log_ee", "sw_log_loc", "sw_rand_ee", "sw_rand_loc"])
def test_sw(orc, fx):
    g = load_golden(fx)
    local = bool(g["local"])
    n = 0
    for p, rd, q, rf, minsc, fw, out, cands in sw_problems(g):
        o, c, _ = orc.sw(rd, q, rf, minsc, local)
        assert np.array_equal(o[:7], out), (fx, p, o[:7], out)
        assert np.array_equal(c, cands), (fx, p)
        n += 1
    assert n > 300


def bt_expected(b, p):
    """Reference alignments of problem p from a sw_bt_* fixture."""
    a = b["aln"][b["aln_off"][p]:b["aln_off"][p + 1]]
    eds = [b["edits"][b["edit_off"][k]:b["edit_off"][k + 1]] for k in range(b["aln_off"][p], b["aln_off"][p + 1])]
    return a, eds, b["fates"][b["fate_off"][p]:b["fate_off"][p + 1]]


@pytest.mark.parametrize("src", ["rand_ee", "rand_loc", "log_ee", "log_loc"])
def test_sw_backtrace(orc, src):
    """SwAligner::nextAlignment loop (aligner_sw.cpp:737-1146): every alignment,
    its candidate, score, offset, N/gap counts, soft trims, edits and every
    candidate's fate equal the reference's."""
    g, b = load_golden("sw_" + src), load_golden("sw_bt_" + src)
    local = bool(g["local"])
    nal = 0
    for p, rd, q, rf, minsc, fw, out, _ in sw_problems(g):
        o, a, eds, fates = orc.sw_bt(rd, q, rf, minsc, local, fw, int(b["triml"][p]), int(b["corel"][p]),
                                     int(b["corer"][p]), maxaln=4096, maxedit=1024)
        ea, eeds, efates = bt_expected(b, p)
        assert np.array_equal(o, b["out"][p]), (src, p)
        assert np.array_equal(a, ea), (src, p)
        assert all(np.array_equal(x, y) for x, y in zip(eds, eeds)), (src, p)
        assert np.array_equal(fates, efates), (src, p)
        nal += len(a)
    assert nal > 50


def ug_cases(idx, g, mode):
    """(read as aligned, quals as aligned, reference codes at off..off+L-1, ...) per fixture read."""
    for i in range(len(g["fw"])):
        rd, q = g["reads"][i], g["quals"][i]
        fw = bool(g["fw"][i])
        if not fw:
            rd, q = np.where(rd > 3, 4, 3 - rd)[::-1], q[::-1]
        ref = idx.ref_codes[int(g["refidx"][i])]
        o = int(g["off"][i])
        pos = np.arange(o, o + len(rd))
        rf = np.where((pos >= 0) & (pos < len(ref)), ref[np.clip(pos, 0, len(ref) - 1)], 4).astype(np.uint8)
        exp = g[mode + "_out"][i]
        ee = g[mode + "_edits"][g[mode + "_edit_off"][i]:g[mode + "_edit_off"][i + 1]]
        yield i, rd, q, rf, o, len(ref), int(g[mode + "_minsc"][i]), fw, exp, ee


@pytest.mark.parametrize("name", ["lambda", "synth"])
@pytest.mark.parametrize("mode", ["ee", "loc"])
def test_ungapped(orc, name, mode):
    """SwAligner::ungappedAlign (aligner_sw.cpp:286-494): return code, score,
    offset, N counts, trims and edits equal the reference's."""
    idx, g = get_index(name), load_golden("ug_" + name)
    for i, rd, q, rf, o, reflen, minsc, fw, exp, ee in ug_cases(idx, g, mode):
        out, ed = orc.ungapped(rd, q, rf, o, reflen, minsc, mode == "loc", fw)
        assert np.array_equal(out[:8], exp[:8]), (name, mode, i, out, exp)
        assert np.array_equal(ed, ee), (name, mode, i)


def test_frame(orc):
    """DP framing (row A14): the oracle's restatement of frameSeedExtensionRect,
    otherMate + frameFindMateRect and the gap budgets against the reference's
    own rectangles (frame.npz, tests/golden/make_golden_frame.py)."""
    g = load_golden("frame")
    nframed = 0
    for name in g["names"]:
        x, y, par = g[f"in_{name}"], g[f"out_{name}"], g[f"par_{name}"]
        local, pe, maxhalf, ttr = bool(par[0]), tuple(int(v) for v in par[1:8]), int(par[8]), bool(par[9])
        for i in range(len(x)):
            kind, off, rdlen, reflen, minsc, fw, a1, alen = (int(v) for v in x[i])
            got = orc.frame(kind, off, rdlen, reflen, minsc, fw, a1, alen, local=local, pe=pe, maxhalf=maxhalf,
                            trim_to_ref=ttr)
            exp = tuple(int(v) for v in y[i]) if y[i, 0] else (0,) * 7
            assert got == exp, (name, i, x[i].tolist(), got, exp)
            nframed += got[0]
    assert nframed > 30000
