"""GPU backtrace (bt2g_sw_align_bt: SwAligner::align + the nextAlignment loop,
aligner_sw.cpp:737-1146) against the reference's own alignments (sw_bt_*
golden fixtures made by the reference build) and against the CPU oracle on
seed-extension problems that point into the HBM-resident reference.  Every
field of every alignment, every edit and every candidate fate is compared
bit-exactly (integer path, no tolerance)."""
import numpy as np
import pytest

from conftest import get_index, load_golden
from test_gpu_sw import golden_batch

pytestmark = pytest.mark.gpu

ALN_FIELDS = ("cand", "score", "off", "ns", "gaps", "refns", "nedit", "trim5p", "trim3p")
# reference fixture columns: cand, score, off, refoff, ns, gaps, refns, nedit, trim5p, trim3p
REF_COLS = (0, 1, 2, 4, 5, 6, 7, 8, 9)


@pytest.fixture(scope="module")
def eng():
    import bt2g
    e = bt2g.Engine(index=get_index("lambda"))
    yield e
    e.close()


def _aln_rows(alns, k):
    return np.stack([alns[f][:k] for f in ALN_FIELDS], 1).astype(np.int64)


def _edit_rows(ed):
    return np.stack([ed["pos"], ed["type"], ed["chr"], ed["qchr"]], 1).astype(np.int64)


def check_against(naln, alns, edits, fates, res, exp_out, exp_alns, exp_edits, exp_fates, tag):
    """exp_alns[p]: (k x 10) reference columns; exp_edits[p]: list of (e x 4)."""
    n = len(naln)
    for p in range(n):
        ea = exp_alns[p]
        assert naln[p] == len(ea), (tag, p, naln[p], len(ea))
        if len(ea):
            assert np.array_equal(_aln_rows(alns[p], len(ea)), ea[:, REF_COLS]), (tag, p)
            for k in range(len(ea)):
                ne = int(ea[k, 7])
                assert np.array_equal(_edit_rows(edits[p, k, :ne]), exp_edits[p][k]), (tag, p, k)
        if exp_fates is not None and res["aligned"][p]:
            ef = exp_fates[p]
            assert np.array_equal(fates[p, :len(ef)], ef), (tag, p)


@pytest.mark.parametrize("src", ["rand_ee", "rand_loc", "log_ee", "log_loc"])
def test_bt_golden(eng, src):
    """Reference fixtures: the reference server's logged DP problems and random
    ragged problems, each with its own rectangle trim / core diagonals."""
    import bt2g
    g, b = load_golden("sw_" + src), load_golden("sw_bt_" + src)
    local = bool(g["local"])
    probs = golden_batch(g)
    n = len(probs)
    rects = np.zeros(n, bt2g.SWRECT_DTYPE)
    rects["triml"], rects["corel"], rects["corer"] = b["triml"], b["corel"], b["corer"]
    res, cands, naln, alns, edits, fates = eng.sw_align_bt(g["reads"], g["quals"], g["lens"], probs,
                                                           windows=g["rf"], rects=rects, local=local, cap=4096,
                                                           maxaln=4096 if local else 256, maxedit=512)
    assert np.array_equal(res["aligned"], b["out"][:, 0])
    ea = [b["aln"][b["aln_off"][p]:b["aln_off"][p + 1]] for p in range(n)]
    ee = [[b["edits"][b["edit_off"][k]:b["edit_off"][k + 1]] for k in range(b["aln_off"][p], b["aln_off"][p + 1])]
          for p in range(n)]
    ef = [b["fates"][b["fate_off"][p]:b["fate_off"][p + 1]] for p in range(n)]
    check_against(naln, alns, edits, fates, res, b["out"], ea, ee, ef, src)
    assert naln.sum() > 50


def _synth_problems(gen, n, seed, length=150, maxgap=15, minsc=-90, sub=0.02, indel=0.3):
    import bt2g
    import synth
    codes, quals, pos, fw = synth.reads(seed, gen, n, length, sub=sub, indel=indel)
    rng = np.random.default_rng(seed)
    probs = np.zeros(n, bt2g.SWPROB_DTYPE)
    probs["read"] = np.arange(n)
    probs["fw"] = fw.astype(np.int32)
    refl = pos.astype(np.int64) - 2 * maxgap + rng.integers(-3, 4, n)
    refl[:4] = [-2 * maxgap, -7, len(gen) - length - 10, len(gen) - length + 5]
    probs["refl"] = refl
    probs["win_off"] = -1
    probs["ncol"] = length + 4 * maxgap
    probs["minsc"] = minsc
    rects = np.zeros(n, bt2g.SWRECT_DTYPE)
    rects["triml"] = 0
    rects["corel"], rects["corer"] = maxgap, 3 * maxgap
    return codes, quals, np.full(n, length, np.uint32), probs, rects


def _same_results_and_lists(a, b):
    """Two sw_align_bt outputs: the same results and alignment counts, and the same
    candidate lists up to each problem's ncand (the slots past it are never
    written: whatever the output buffer held, which differs between a call whose
    outputs fit the context's pinned block and one whose outputs did not)."""
    for f in a[0].dtype.names:
        assert np.array_equal(a[0][f], b[0][f]), f
    assert np.array_equal(a[2], b[2])
    nc = np.minimum(np.maximum(a[0]["ncand"], 0), a[1].shape[1])
    for p in range(len(nc)):
        for f in a[1].dtype.names:
            assert np.array_equal(a[1][f][p, :nc[p]], b[1][f][p, :nc[p]]), (p, f)


def _oracle_expect(orc, gen, codes, quals, probs, rects, local, sc=None, enable8=True):
    ea, ee, ef = [], [], []
    for p in range(len(probs)):
        rd, q = codes[p], quals[p]
        if not probs["fw"][p]:
            rd, q = np.where(rd > 3, 4, 3 - rd)[::-1], q[::-1]
        ncol = int(probs["ncol"][p])
        o = np.arange(probs["refl"][p], probs["refl"][p] + ncol + 1)
        cc = np.where((o >= 0) & (o < len(gen)), gen[np.clip(o, 0, len(gen) - 1)], 4).astype(np.int32)
        rf = np.where(cc > 3, 16, 1 << np.minimum(cc, 3)).astype(np.uint8)
        out, a, eds, fates = orc.sw_bt(rd, q, rf, int(probs["minsc"][p]), local, bool(probs["fw"][p]),
                                       int(rects["triml"][p]), int(rects["corel"][p]), int(rects["corer"][p]),
                                       enable8=enable8, maxaln=512, maxedit=512, sc=sc)
        ea.append(a)
        ee.append(eds)
        ef.append(fates)
    return ea, ee, ef


@pytest.mark.parametrize("case", ["u8", "i16", "custom_scoring"])
def test_bt_resident_vs_oracle(eng, case):
    """Seed-extension problems (150 x 210, dp_framer.cpp:95-125 geometry) over the
    resident reference, reads with substitutions, Ns and indels; windows off
    both reference ends.  u8: the systolic fill's byte score plane; i16:
    enable8 off (u16 plane); custom scoring: the generic fill's matrices."""
    import bt2g
    from oracle.oracle import Oracle, scoring as oscoring
    orc = Oracle()
    gen = get_index("lambda").ref_codes[0]
    codes, quals, lens, probs, rects = _synth_problems(gen, 600, 17)
    sc, osc, enable8 = None, None, True
    if case == "i16":
        enable8 = False
    elif case == "custom_scoring":
        sc = bt2g.scoring(False)
        sc.rdg_const, sc.rdg_lin, sc.rfg_const, sc.rfg_lin, sc.mmp_max = 4, 2, 6, 1, 5
        osc = oscoring(False)
        osc.rdg_const, osc.rdg_lin, osc.rfg_const, osc.rfg_lin, osc.mmp_max = 4, 2, 6, 1, 5
    res, cands, naln, alns, edits, fates = eng.sw_align_bt(codes, quals, lens, probs, rects=rects, cap=1024,
                                                           maxaln=512, maxedit=512, sc=sc, enable8=enable8)
    ea, ee, ef = _oracle_expect(orc, gen, codes, quals, probs, rects, False, sc=osc, enable8=enable8)
    check_against(naln, alns, edits, fates, res, None, ea, ee, ef, case)
    assert (naln > 0).sum() > 400
    assert (alns["gaps"][:, 0] > 0).sum() > 20          # indel alignments were walked


def test_bt_local_resident_vs_oracle(eng):
    """--local scoring on the resident reference (soft trimming, dominance)."""
    import bt2g
    from oracle.oracle import Oracle
    orc = Oracle()
    gen = get_index("lambda").ref_codes[0]
    # --score-min G,20,8 at 150 bp: (int)(20 + 8 ln 150) = 60
    codes, quals, lens, probs, rects = _synth_problems(gen, 300, 23, minsc=60)
    res, cands, naln, alns, edits, fates = eng.sw_align_bt(codes, quals, lens, probs, rects=rects, local=True,
                                                           cap=4096, maxaln=512, maxedit=512)
    ea, ee, ef = _oracle_expect(orc, gen, codes, quals, probs, rects, True)
    check_against(naln, alns, edits, fates, res, None, ea, ee, ef, "local")
    assert (naln > 0).sum() > 200


def test_bt_maxaln_truncates(eng):
    """maxaln bounds the loop: the first maxaln alignments equal the full run's."""
    gen = get_index("lambda").ref_codes[0]
    codes, quals, lens, probs, rects = _synth_problems(gen, 200, 31)
    full = eng.sw_align_bt(codes, quals, lens, probs, rects=rects, cap=1024, maxaln=64, maxedit=256)
    one = eng.sw_align_bt(codes, quals, lens, probs, rects=rects, cap=1024, maxaln=1, maxedit=256)
    assert np.array_equal(one[2], np.minimum(full[2], 1))
    has = full[2] > 0
    assert np.array_equal(one[3][has, 0], full[3][has, 0])
    for p in np.nonzero(has)[0]:
        ne = int(full[3]["nedit"][p, 0])
        assert np.array_equal(one[4][p, 0, :ne], full[4][p, 0, :ne]), p


@pytest.mark.parametrize("case", ["reserve_sw", "reserve_bt_u8_then_local", "reserve_narrow_stride"])
def test_bt_after_reservation(case):
    """Backtrace calls after bt2g_reserve_sw / bt2g_reserve_sw_bt whose
    reservation does not match the call: the score plane keeps the
    call's own pitch, so the results equal the unreserved run's and the oracle's."""
    import bt2g
    from oracle.oracle import Oracle
    orc = Oracle()
    gen = get_index("lambda").ref_codes[0]
    local = case == "reserve_bt_u8_then_local"
    codes, quals, lens, probs, rects = _synth_problems(gen, 256, 41, minsc=60 if local else -90)
    with bt2g.Engine(index=get_index("lambda")) as e:
        if case == "reserve_sw":
            e.reserve_sw(1024, 400)          # wider than the problems (210 columns)
        elif case == "reserve_bt_u8_then_local":
            e.reserve_sw_bt(1024, 150, 210, 1)
        else:
            e.reserve_sw_bt(1024, 100, 210, 1)   # stride 150 > reserved rows
        res, cands, naln, alns, edits, fates = e.sw_align_bt(codes, quals, lens, probs, rects=rects, local=local,
                                                             cap=4096, maxaln=512, maxedit=512)
    ea, ee, ef = _oracle_expect(orc, gen, codes, quals, probs, rects, local)
    check_against(naln, alns, edits, fates, res, None, ea, ee, ef, case)
    assert (naln > 0).sum() > 150


def test_close_frees_reserved_scratch():
    """bt2g_close releases the backtrace scratch of bt2g_reserve_sw_bt:
    repeated open / reserve / close cycles do not lose device memory."""
    import torch
    import bt2g
    idx = get_index("lambda")
    free = []
    for _ in range(4):
        with bt2g.Engine(index=idx) as e:
            e.reserve_sw_bt(200_000, 150, 210, 1)     # ~8 GB of plane + marks
        torch.cuda.synchronize()
        free.append(torch.cuda.mem_get_info()[0])
    assert max(free) - min(free) < (1 << 30), free


@pytest.mark.parametrize("local", [False, True], ids=["ee", "local"])
def test_bt_long_reads_vs_oracle(eng, local):
    """Reads of 1100..2048 bases (the two-wave systolic fill and its u16 plane):
    every alignment, edit and candidate fate of the nextAlignment loop equals
    the oracle's."""
    from oracle.oracle import Oracle
    orc = Oracle()
    gen = get_index("lambda").ref_codes[0]
    for L in (1100, 2048):
        # (local: a minsc near 1.8 x length keeps the candidate list under the cap of 8192)
        minsc = int(1.8 * L) if local else int(-(0.6 + 0.6 * L))
        codes, quals, lens, probs, rects = _synth_problems(gen, 16, 40 + L, length=L, maxgap=30, minsc=minsc,
                                                           sub=0.005 if local else 0.02)
        res, cands, naln, alns, edits, fates = eng.sw_align_bt(codes, quals, lens, probs, rects=rects, local=local,
                                                               cap=8192, maxaln=512, maxedit=2 * L + 8)
        ea, ee, ef = _oracle_expect(orc, gen, codes, quals, probs, rects, local)
        check_against(naln, alns, edits, fates, res, None, ea, ee, ef, f"long{L}")
        assert (naln > 0).sum() > 8


@pytest.mark.parametrize("shape", ["seedext", "mate"])
@pytest.mark.parametrize("variant", ["wg", "one_walker", "wg_lds64k"])
def test_bt_lds_resident_equals_lane_kernel(eng, monkeypatch, shape, variant):
    """Batches up to BT2G_BT_LDS_MAX problems walk LDS-resident: by default the
    workgroup walk (sw_backtrace_wg.hip; wide planes with the >64 KiB LDS opt-in),
    with BT2G_BT_WG=0 the one-walker LDS-resident kernel, with BT2G_BT_WG_LDS=0 the
    workgroup walk only where its layout fits 64 KiB (else the one-walker or the
    lane kernel).  BT2G_BT_LDS_MAX=0 forces the lane-per-problem kernel.  All give
    the same alignments, edits and fates on the same batch -- seed-extension
    shapes (150 x 210) and mate-search shapes (150 x ~700: the decision plane up to
    $BT2G_DEC_RATIO and the opt-in launch), the latter also against the oracle."""
    gen = get_index("lambda").ref_codes[0]
    maxgap, n = (15, 900) if shape == "seedext" else (137, 300)
    codes, quals, lens, probs, rects = _synth_problems(gen, n, 53, maxgap=maxgap)
    env = {"wg": {}, "one_walker": {"BT2G_BT_WG": "0"}, "wg_lds64k": {"BT2G_BT_WG_LDS": "0"}}[variant]
    outs = []
    for lim in ("65536", "0"):
        monkeypatch.setenv("BT2G_BT_LDS_MAX", lim)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        outs.append(eng.sw_align_bt(codes, quals, lens, probs, rects=rects, cap=1024, maxaln=64, maxedit=512))
        for k in env:
            monkeypatch.delenv(k)
    a, b = outs
    # results and counts: whole; candidate lists, alignments, edits and fates: the
    # valid parts (slots past them are not written)
    _same_results_and_lists(a, b)
    naln = a[2]
    for p in range(n):
        k = max(int(naln[p]), 0)
        for f in a[3].dtype.names:
            assert np.array_equal(a[3][f][p, :k], b[3][f][p, :k]), (p, f)
        for j in range(k):
            ne = min(int(a[3]["nedit"][p, j]), a[4].shape[2])
            for f in ("pos", "type", "chr", "qchr"):
                assert np.array_equal(a[4][f][p, j, :ne], b[4][f][p, j, :ne]), (p, j, f)
        nc = min(int(a[0]["ncand"][p]), a[5].shape[1])
        assert np.array_equal(a[5][p, :nc], b[5][p, :nc]), p
    assert (a[2] > 0).sum() > 0.6 * n
    if shape == "mate" and variant == "wg":
        from oracle.oracle import Oracle
        res, cands, naln, alns, edits, fates = a
        k = 64
        ea, ee, ef = _oracle_expect(Oracle(), gen, codes[:k], quals[:k], probs[:k], rects[:k], False)
        check_against(naln[:k], alns[:k], edits[:k], fates[:k], res[:k], None, ea, ee, ef, "mate")


@pytest.mark.parametrize("lds", ["marks", "marks_wpf1", "marks_cands", "marks_serial", "marks_flat", "plane",
                                 "plane64k"])
def test_bt_local_lds_resident_equals_lane_kernel(eng, monkeypatch, lds):
    """Local mode: batches up to BT2G_BT_LDS_MAX walk LDS-resident, one walker per
    workgroup, its candidates filtered and walked by the wave, up to 64 walks at a
    time resolved in the reference's order (default), filtered by the wave and
    walked one at a time (BT2G_BT_LOC_WPF=1), or filtered and walked by the walker
    one at a time (BT2G_BT_LOC_WPF=0, "marks_serial"), the wave reading the
    candidates from HBM (default) or from an LDS copy (BT2G_BT_LOC_CANDS=lds):
    both mark tile sets in LDS and the u16 plane read in place (default),
    or the plane and its block masks in LDS too (BT2G_BT_LOC_LDS=plane, past 64 KiB
    with the device's opt-in, else the lane kernel) -- the same alignments, edits and
    candidate fates as the lane-per-problem walk (BT2G_BT_LDS_MAX=0), and as the
    oracle on a sample."""
    from oracle.oracle import Oracle
    gen = get_index("lambda").ref_codes[0]
    n = 400
    codes, quals, lens, probs, rects = _synth_problems(gen, n, 61, minsc=60, sub=0.01)
    outs = []
    for lim in ("65536", "0"):
        monkeypatch.setenv("BT2G_BT_LDS_MAX", lim)
        if lds.startswith("plane"):
            monkeypatch.setenv("BT2G_BT_LOC_LDS", "plane")     # (default: the marks only)
        if lds == "plane64k":
            monkeypatch.setenv("BT2G_BT_WG_LDS", "0")
        if lds == "marks_flat":
            monkeypatch.setenv("BT2G_BT_LOC_FLAT", "1")
        if lds == "marks_serial":
            monkeypatch.setenv("BT2G_BT_LOC_WPF", "0")
        if lds == "marks_wpf1":
            monkeypatch.setenv("BT2G_BT_LOC_WPF", "1")
        if lds == "marks_cands":
            monkeypatch.setenv("BT2G_BT_LOC_CANDS", "lds")
        outs.append(eng.sw_align_bt(codes, quals, lens, probs, rects=rects, local=True, cap=4096, maxaln=64,
                                    maxedit=512))
        monkeypatch.delenv("BT2G_BT_LOC_WPF", raising=False)
        monkeypatch.delenv("BT2G_BT_LOC_CANDS", raising=False)
        monkeypatch.delenv("BT2G_BT_WG_LDS", raising=False)
        monkeypatch.delenv("BT2G_BT_LOC_LDS", raising=False)
        monkeypatch.delenv("BT2G_BT_LOC_FLAT", raising=False)
    a, b = outs
    _same_results_and_lists(a, b)
    naln = a[2]
    for p in range(n):
        k = max(int(naln[p]), 0)
        for f in a[3].dtype.names:
            assert np.array_equal(a[3][f][p, :k], b[3][f][p, :k]), (p, f)
        for j in range(k):
            ne = min(int(a[3]["nedit"][p, j]), a[4].shape[2])
            for f in ("pos", "type", "chr", "qchr"):
                assert np.array_equal(a[4][f][p, j, :ne], b[4][f][p, j, :ne]), (p, j, f)
        nc = min(int(a[0]["ncand"][p]), a[5].shape[1])
        assert np.array_equal(a[5][p, :nc], b[5][p, :nc]), p
    assert (naln > 0).sum() > 0.6 * n
    res, cands, naln, alns, edits, fates = a
    k = 48
    ea, ee, ef = _oracle_expect(Oracle(), gen, codes[:k], quals[:k], probs[:k], rects[:k], True)
    check_against(naln[:k], alns[:k], edits[:k], fates[:k], res[:k], None, ea, ee, ef, "local_lds")


@pytest.mark.parametrize("maxaln", [1, 2, 64])
def test_bt_local_maxaln_lds_equals_lane_kernel(eng, monkeypatch, maxaln):
    """Local DPs with several alignments each (windows holding three mutated
    copies of the read) and a maxaln that binds: the wave-parallel walk (the
    default LDS-resident form) stops where the serial walk does -- its in-order
    resolution of a batch of speculative walks ends at the maxaln-th success -- so
    the alignments, edits and candidate fates equal the lane-per-problem kernel's
    (BT2G_BT_LDS_MAX=0)."""
    gen = get_index("lambda").ref_codes[0]
    n = 200
    codes, quals, lens, probs, rects = _synth_problems(gen, n, 77, minsc=60, sub=0.01)
    rng = np.random.default_rng(78)
    wins, offs = [], []
    for p in range(n):
        parts = []
        for k in range(3):
            seg = codes[p].astype(np.int32).copy()
            flip = rng.random(seg.size) < 0.03
            seg[flip] = (seg[flip] + rng.integers(1, 4, int(flip.sum()))) % 4
            parts += [seg, rng.integers(0, 4, 20)]
        w = np.concatenate(parts)
        offs.append(sum(len(x) for x in wins))
        wins.append(np.where(w > 3, 16, 1 << np.minimum(w, 3)).astype(np.uint8))
    probs = probs.copy()
    probs["fw"] = 1
    probs["win_off"] = offs
    probs["ncol"] = [len(x) - 1 for x in wins]
    rects = rects.copy()
    rects["corel"], rects["corer"] = -200, 1000
    windows = np.concatenate(wins)
    outs = []
    for lim in ("65536", "0"):
        monkeypatch.setenv("BT2G_BT_LDS_MAX", lim)
        outs.append(eng.sw_align_bt(codes, quals, lens, probs, windows=windows, rects=rects, local=True, cap=4096,
                                    maxaln=maxaln, maxedit=512))
    monkeypatch.delenv("BT2G_BT_LDS_MAX", raising=False)
    a, b = outs
    _same_results_and_lists(a, b)
    for p in range(n):
        k = max(int(a[2][p]), 0)
        for f in a[3].dtype.names:
            assert np.array_equal(a[3][f][p, :k], b[3][f][p, :k]), (p, f)
        for j in range(k):
            ne = min(int(a[3]["nedit"][p, j]), a[4].shape[2])
            for f in ("pos", "type", "chr", "qchr"):
                assert np.array_equal(a[4][f][p, j, :ne], b[4][f][p, j, :ne]), (p, j, f)
        nc = min(int(a[0]["ncand"][p]), a[5].shape[1])
        assert np.array_equal(a[5][p, :nc], b[5][p, :nc]), p
    if maxaln < 64:
        assert (a[2] == maxaln).sum() > 0.5 * n          # the bound binds
    else:
        assert (a[2] >= 3).sum() > 0.5 * n               # three copies, three alignments
