"""SW engine on the GPU vs SwAligner::align's own outputs (golden fixtures from
the reference server's DP log and random problems) and vs the CPU oracle's full
H/E/F matrices.  Bit-exact for all four fills (u8/i16 x end-to-end/local)."""
import numpy as np
import pytest

from conftest import get_index, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import bt2g
    e = bt2g.Engine(index=get_index("lambda"))
    yield e
    e.close()


def golden_batch(g):
    import bt2g
    n = len(g["rd_index"])
    probs = np.zeros(n, bt2g.SWPROB_DTYPE)
    probs["read"] = g["rd_index"]
    probs["fw"] = g["fw"]
    probs["win_off"] = g["rf_off"][:-1]
    probs["ncol"] = np.diff(g["rf_off"]) - 1
    probs["minsc"] = g["minsc"]
    return probs


@pytest.mark.parametrize("fx", ["sw_log_ee", "sw_log_loc", "sw_rand_ee", "sw_rand_loc"])
def test_sw_golden(eng, fx):
    g = load_golden(fx)
    local = bool(g["local"])
    probs = golden_batch(g)
    res, cands, _ = eng.sw_align(g["reads"], g["quals"], g["lens"], probs, windows=g["rf"], local=local,
                                 cap=4096)
    out = g["out"]
    assert np.array_equal(res["aligned"], out[:, 0])
    al = out[:, 0] == 1
    assert np.array_equal(res["best"][al], out[al, 1])
    assert np.array_equal(res["u8succ"], out[:, 2]) and np.array_equal(res["i16succ"], out[:, 3])
    assert np.array_equal(res["colstop"], out[:, 4]) and np.array_equal(res["lastsolcol"], out[:, 5])
    assert np.array_equal(res["ncand"], out[:, 6])
    for p in range(len(probs)):
        ref = g["cands"][g["cand_off"][p]:g["cand_off"][p + 1]]
        got = cands[p, :len(ref)]
        assert np.array_equal(np.stack([got["row"], got["col"], got["score"]], 1), ref), (fx, p)


@pytest.mark.parametrize("local", [False, True])
def test_sw_matrices_vs_oracle(eng, local):
    """Full H/E/F of every cell (native value domain) against the oracle."""
    from oracle.oracle import Oracle
    orc = Oracle()
    g = load_golden("sw_rand_loc" if local else "sw_rand_ee")
    probs = golden_batch(g)[:120]
    res, cands, (mat, off) = eng.sw_align(g["reads"], g["quals"], g["lens"], probs, windows=g["rf"],
                                          local=local, want_mat=True)
    for p in range(len(probs)):
        ri = g["rd_index"][p]
        L = int(g["lens"][ri])
        rd, q = g["reads"][ri, :L], g["quals"][ri, :L]
        if not g["fw"][p]:
            rd, q = np.where(rd > 3, 4, 3 - rd)[::-1], q[::-1]
        rf = g["rf"][g["rf_off"][p]:g["rf_off"][p + 1]]
        o, c, m = orc.sw(rd, q, rf, int(probs["minsc"][p]), local, want_mat=True)
        if not (o[2] or o[3]):
            continue
        ncol = int(probs["ncol"][p])
        got = mat[off[p]:off[p] + L * ncol * 3].reshape(L, ncol, 3).astype(np.int32)
        cs = int(o[4]) if local else ncol
        assert np.array_equal(got[:, :cs], m[:, :cs]), p


def test_sw_resident_reference(eng):
    """Problems that point into the HBM-resident reference (incl. off-end N
    padding and the extra right column) == the same windows given explicitly."""
    import bt2g
    import synth
    idx = get_index("lambda")
    gen = idx.ref_codes[0]
    codes, quals, pos, fw = synth.reads(99, gen, 256, 150, sub=0.01)
    rng = np.random.default_rng(2)
    n = len(codes)
    probs = np.zeros(n, bt2g.SWPROB_DTYPE)
    probs["read"] = np.arange(n)
    probs["fw"] = fw.astype(np.int32)
    refl = pos.astype(np.int64) - 30 + rng.integers(-10, 10, n)
    refl[:8] = [-40, -5, len(gen) - 100, len(gen) - 150, len(gen) - 200, 0, -150, len(gen) - 60]
    probs["refl"] = refl
    probs["win_off"] = -1
    probs["ncol"] = 210
    probs["minsc"] = -90
    lens = np.full(n, 150, np.uint32)
    res1, c1, _ = eng.sw_align(codes, quals, lens, probs)
    wins = []
    for i in range(n):
        idxs = np.arange(refl[i], refl[i] + 211)
        cc = np.where((idxs >= 0) & (idxs < len(gen)), gen[np.clip(idxs, 0, len(gen) - 1)], 4)
        wins.append((1 << cc.astype(np.int32)).astype(np.uint8))
    p2 = probs.copy()
    p2["win_off"] = np.arange(n) * 211
    res2, c2, _ = eng.sw_align(codes, quals, lens, p2, windows=np.concatenate(wins))
    assert np.array_equal(res1, res2)
    assert np.array_equal(c1, c2)
    assert res1["aligned"].sum() > n // 2


@pytest.mark.parametrize("gaps", ["default", "rdg5,3_rfg4,2"])
def test_sw_packed_vs_per_lane(eng, gaps):
    """The packed two-problems-per-lane end-to-end fill (default path) against
    the one-problem-per-lane fill (taken when matrices are requested) on
    ragged problems: read lengths 1..400, widths 1..500, u8 and i16 minsc,
    Ns in reads and reference, windows off both reference ends."""
    import bt2g
    import synth
    idx = get_index("lambda")
    gen = idx.ref_codes[0]
    rng = np.random.default_rng(5)
    n = 700
    lens = rng.integers(1, 401, n).astype(np.uint32)
    lens[:5] = [1, 2, 4, 8, 400]
    stride = 400
    codes = np.full((n, stride), 4, np.uint8)
    quals = np.full((n, stride), 73, np.uint8)
    pos = rng.integers(-50, len(gen) + 50, n)
    fw = rng.random(n) < 0.5
    for i in range(n):
        L = int(lens[i])
        o = np.arange(pos[i], pos[i] + L)
        c = np.where((o >= 0) & (o < len(gen)), gen[np.clip(o, 0, len(gen) - 1)], 4)
        m = rng.random(L) < 0.03
        c[m] = rng.integers(0, 5, m.sum())
        if not fw[i]:
            c = np.where(c > 3, 4, 3 - c)[::-1]
        codes[i, :L] = c
        quals[i, :L] = rng.integers(33, 75, L)
    probs = np.zeros(n, bt2g.SWPROB_DTYPE)
    probs["read"] = np.arange(n)
    probs["fw"] = fw
    probs["ncol"] = np.clip(lens.astype(np.int64) + rng.integers(-20, 100, n), 1, 500)
    probs["refl"] = pos - rng.integers(0, 40, n)
    probs["win_off"] = -1
    probs["minsc"] = np.where(rng.random(n) < 0.3, -(0.6 + 2.5 * lens).astype(np.int64),
                              -(0.6 + 0.6 * lens).astype(np.int64))
    probs["minsc"][:3] = [0, -254, -255]
    sc = bt2g.scoring(False)
    if gaps != "default":          # unequal gap opens: the packed fill's general E/F form
        sc.rfg_const, sc.rfg_lin = 4, 2
    res_p, c_p, _ = eng.sw_align(codes, quals, lens, probs, cap=512, sc=sc)
    res_g, c_g, _ = eng.sw_align(codes, quals, lens, probs, cap=512, want_mat=True, sc=sc)
    assert np.array_equal(res_p, res_g)
    assert np.array_equal(c_p, c_g)
    assert 0 < res_p["aligned"].sum() < n
    assert (res_p["i16succ"] == 1).sum() > 0 and (res_p["u8succ"] == 1).sum() > 0


@pytest.mark.parametrize("gaps", ["default", "rdg5,3_rfg4,2"])
def test_sw_packed_vs_per_lane_local(eng, gaps):
    """The packed local fill (u8 and i16 local fills in one pass, column
    maxima for both padding-row layouts, block-wise candidate gather) against
    the one-problem-per-lane local fills on ragged problems: read lengths
    1..200 (every nrow mod 16, so both u8-only padding cases), widths 1..300,
    Ns, windows off both reference ends, low and high minsc (u8 saturation and
    not)."""
    import bt2g
    idx = get_index("lambda")
    gen = idx.ref_codes[0]
    rng = np.random.default_rng(6)
    n = 600
    lens = rng.integers(1, 201, n).astype(np.uint32)
    lens[:20] = np.arange(1, 21) + 140
    stride = 200
    codes = np.full((n, stride), 4, np.uint8)
    quals = np.full((n, stride), 73, np.uint8)
    pos = rng.integers(-50, len(gen) + 50, n)
    fw = rng.random(n) < 0.5
    for i in range(n):
        L = int(lens[i])
        o = np.arange(pos[i], pos[i] + L)
        c = np.where((o >= 0) & (o < len(gen)), gen[np.clip(o, 0, len(gen) - 1)], 4)
        m = rng.random(L) < 0.03
        c[m] = rng.integers(0, 5, m.sum())
        if not fw[i]:
            c = np.where(c > 3, 4, 3 - c)[::-1]
        codes[i, :L] = c
        quals[i, :L] = rng.integers(33, 75, L)
    probs = np.zeros(n, bt2g.SWPROB_DTYPE)
    probs["read"] = np.arange(n)
    probs["fw"] = fw
    probs["ncol"] = np.clip(lens.astype(np.int64) + rng.integers(-20, 100, n), 1, 300)
    probs["refl"] = pos - rng.integers(0, 40, n)
    probs["win_off"] = -1
    probs["minsc"] = np.where(rng.random(n) < 0.3, 10, (20 + 8 * np.log(np.maximum(lens, 2))).astype(np.int64))
    sc = bt2g.scoring(True)
    if gaps != "default":
        sc.rfg_const, sc.rfg_lin = 4, 2
    res_p, c_p, _ = eng.sw_align(codes, quals, lens, probs, cap=8192, sc=sc, local=True)
    res_g, c_g, _ = eng.sw_align(codes, quals, lens, probs, cap=8192, want_mat=True, sc=sc, local=True)
    for i in range(n):
        assert tuple(res_p[i]) == tuple(res_g[i]), (i, res_p[i], res_g[i])
    assert np.array_equal(c_p, c_g)
    assert 0 < res_p["aligned"].sum() < n
    assert (res_p["i16succ"] == 1).sum() > 0 and (res_p["u8succ"] == 1).sum() > 0


@pytest.mark.parametrize("local", [False, True], ids=["ee", "local"])
def test_sw_packed_wide_vs_per_lane(eng, local):
    """Reads of 1025..2048 bases: the two-wave systolic fill (WIDE, S = 65..128
    lanes per problem pair, lane 63 -> 64 through LDS) against the
    one-problem-per-lane fill on ragged long problems (configs[0]'s longreads.fq
    reach 2561 bp; the engines take up to BT2G_MAX_READ_LEN = 2048)."""
    import bt2g
    idx = get_index("lambda")
    gen = idx.ref_codes[0]
    rng = np.random.default_rng(8)
    n = 48
    stride = 2048
    lens = rng.integers(1025, 2049, n).astype(np.uint32)
    lens[:6] = [1025, 1040, 1500, 2047, 2048, 600]      # a short read in a wide batch too
    codes = np.full((n, stride), 4, np.uint8)
    quals = np.full((n, stride), 73, np.uint8)
    pos = rng.integers(-50, len(gen) - 1000, n)
    fw = rng.random(n) < 0.5
    for i in range(n):
        L = int(lens[i])
        o = np.arange(pos[i], pos[i] + L)
        c = np.where((o >= 0) & (o < len(gen)), gen[np.clip(o, 0, len(gen) - 1)], 4)
        m = rng.random(L) < (0.01 if local else 0.03)
        c[m] = rng.integers(0, 5, m.sum())
        if not fw[i]:
            c = np.where(c > 3, 4, 3 - c)[::-1]
        codes[i, :L] = c
        quals[i, :L] = rng.integers(33, 75, L)
    probs = np.zeros(n, bt2g.SWPROB_DTYPE)
    probs["read"] = np.arange(n)
    probs["fw"] = fw
    probs["ncol"] = np.clip(lens.astype(np.int64) + rng.integers(-20, 100, n), 1, 2200)
    probs["refl"] = pos - rng.integers(0, 40, n)
    probs["win_off"] = -1
    if local:
        # (local candidates: cells >= minsc that end a match run; over a 2 kb alignment a
        # minsc below ~1.8 x length leaves more than the engine's cap of 8192)
        probs["minsc"] = np.where(rng.random(n) < 0.3, 19 * lens // 10, 18 * lens // 10).astype(np.int64)
        sc = bt2g.scoring(True)
    else:
        probs["minsc"] = np.where(rng.random(n) < 0.3, -(0.6 + 2.5 * lens).astype(np.int64),
                                  -(0.6 + 0.6 * lens).astype(np.int64))
        probs["minsc"][:2] = [-200, -254]                # u8 fills of long reads
        sc = bt2g.scoring(False)
    cap = 8192
    res_p, c_p, _ = eng.sw_align(codes, quals, lens, probs, cap=cap, sc=sc, local=local)
    res_g, c_g, _ = eng.sw_align(codes, quals, lens, probs, cap=cap, want_mat=True, sc=sc, local=local)
    for i in range(n):
        assert tuple(res_p[i]) == tuple(res_g[i]), (i, res_p[i], res_g[i])
    assert np.array_equal(c_p, c_g)
    assert res_p["aligned"].sum() > n // 3
