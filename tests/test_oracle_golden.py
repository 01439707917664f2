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


# ---- the fused calls' reference fixtures (tests/golden/fused.npz, make_golden_fused.py) ----
def oracle_sweep_1mm(orc, fe, be, g, name, skip, off_cap=8, mm_cap=16):
    """The oracle composed as bt2g_exact_sweep_1mm composes the reference's calls
    (bt2_search.cpp:3453-3667): sweep, the gate, the gated 1-mm search, the small
    ranges' row offsets.  Returns (sweep, hits, counts (-1: gated off), bwops, offs)."""
    reads, quals, lens = g["reads"], g["quals"], g["lens"]
    ms = g["mmminsc_ee"]
    sw = orc.exact_sweep(fe, reads, lens)
    n = len(lens)
    hits = np.zeros((n, 64, 7), np.int64)
    cnt = np.full(n, -1, np.int32)
    ops = np.zeros(n, np.uint64)
    offs = np.full((n, 2 + mm_cap, off_cap), 0xFFFFFFFF, np.uint32)
    for i in range(n):
        mfw, mrc = int(sw[i, 0]), int(sw[i, 1])
        yfw, yrc = mfw <= 1, mrc <= 1
        rg = [(int(sw[i, 3]), int(sw[i, 4])) if mfw == 0 else (0, 0),
              (int(sw[i, 5]), int(sw[i, 6])) if mrc == 0 else (0, 0)]
        if not ((skip and min(mfw, mrc) == 0) or not (yfw or yrc)):
            h, c, bw = orc.one_mm(fe, be, reads[i:i + 1], quals[i:i + 1], lens[i:i + 1], ms[i:i + 1], False,
                                  nofw=not yfw, norc=not yrc)
            hits[i], cnt[i], ops[i] = h[0], c[0], bw[0]
            rg += [(int(h[0, k, 0]), int(h[0, k, 1])) for k in range(min(int(c[0]), mm_cap))]
        for slot, (t, b) in enumerate(rg):
            if 0 < b - t <= off_cap:
                for j in range(b - t):
                    offs[i, slot, j] = orc.get_offset(fe, t + j)
    return sw, hits, cnt, ops, offs


@pytest.mark.parametrize("name", ["lambda", "synth"])
@pytest.mark.parametrize("skip", [0, 1])
def test_fused_sweep_1mm(orc, name, skip):
    """The oracle, composed as bt2g_exact_sweep_1mm, against the reference's own
    composition (sweep, gated oneMmSearch, getOffset of the small ranges)."""
    f = load_golden("fused")
    g = load_golden("fm_" + name)
    fe, be = _ebwts(orc, name)
    sw, hits, cnt, ops, offs = oracle_sweep_1mm(orc, fe, be, g, name, skip)
    assert np.array_equal(sw, f[f"sweep_{name}"].astype(np.uint64))
    rc = f[f"mmn_{name}_{skip}"]
    assert np.array_equal(cnt, rc)
    _mm_eq(f[f"mm_{name}_{skip}"], rc.clip(0), hits, cnt.clip(0))
    assert np.array_equal(ops, f[f"mmops_{name}_{skip}"])
    assert np.array_equal(offs, f[f"offs_{name}_{skip}"])


@pytest.mark.parametrize("name", ["lambda", "synth"])
@pytest.mark.parametrize("pol", ["s22", "s10"])
def test_fused_seed_ext(orc, name, pol):
    """The oracle's seed round + SwDriver::extend of every range + row offsets
    against the reference's (bt2g_seed_search_ext's definition)."""
    f = load_golden("fused")
    g = load_golden("fm_" + name)
    fe, be = _ebwts(orc, name)
    L, iv, off0 = (int(x) for x in f[f"seedpol_{name}_{pol}"])
    maxs = f[f"sx_{name}_{pol}"].shape[2]
    out, ns, ops = orc.seed_search(fe, be, g["reads"], g["lens"], L, iv, off0, maxs)
    assert np.array_equal(out, f[f"seed_{name}_{pol}"]) and np.array_equal(ns, f[f"seedn_{name}_{pol}"])
    sx = np.zeros_like(f[f"sx_{name}_{pol}"])
    so = np.full_like(f[f"so_{name}_{pol}"], 0xFFFFFFFF)
    for i in range(len(ns)):
        ln = int(g["lens"][i])
        for s_ in range(2):
            for k in range(maxs):
                t, b, tb, bb = (int(x) for x in out[i, s_, k])
                depth, sl = off0 + k * iv, min(L, ln)
                if b > t and depth + sl <= ln:
                    sx[i, s_, k] = orc.extend(fe, be, g["reads"][i, :ln], 1 - s_, depth, sl, t, b, tb, bb)
                if 0 < b - t <= so.shape[3]:
                    for j in range(b - t):
                        so[i, s_, k, j] = orc.get_offset(fe, t + j)
    assert np.array_equal(sx, f[f"sx_{name}_{pol}"])
    assert np.array_equal(so, f[f"so_{name}_{pol}"])
