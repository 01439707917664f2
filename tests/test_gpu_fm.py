"""FM engine on the GPU (libbt2g.so) vs the reference's golden vectors and the
CPU oracle.  Bit-exact: SA ranges, edit bounds, hit lists, FM-op counts."""
import numpy as np
import pytest

from conftest import get_index, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engines():
    import bt2g
    es = {name: bt2g.Engine(index=get_index(name)) for name in ("lambda", "synth")}
    yield es
    for e in es.values():
        e.close()


@pytest.fixture(scope="module")
def orc():
    from oracle.oracle import Oracle
    return Oracle()


def _gold_exact_to_gpu_layout(ex):
    # golden: mineFw, mineRc, nelt, fwtop, fwbot, rctop, rcbot, bwops
    return np.stack([ex[:, 0], ex[:, 1], ex[:, 3], ex[:, 4], ex[:, 5], ex[:, 6], ex[:, 7]], 1).astype(np.uint32)


@pytest.mark.parametrize("name", ["lambda", "synth"])
def test_exact_sweep_golden(engines, name):
    g = load_golden("fm_" + name)
    out = engines[name].exact_sweep(g["reads"], g["lens"])
    assert np.array_equal(out[:, :7], _gold_exact_to_gpu_layout(g["exact"]))
    assert (out[:, 7] <= out[:, 6]).all()          # one side load per FM op at most


@pytest.mark.parametrize("name", ["lambda", "synth"])
@pytest.mark.parametrize("pol", ["s22", "s20", "s10"])
def test_seed_search_golden(engines, name, pol):
    g = load_golden("fm_" + name)
    L, iv, off = (int(x) for x in g["seedpol_" + pol])
    out, ns, ops, loads = engines[name].seed_search(g["reads"], g["lens"], L, iv, off, 64)
    assert np.array_equal(ns, g["seedn_" + pol])
    assert np.array_equal(out, g["seed_" + pol])
    assert np.array_equal(ops, g["seedops_" + pol].astype(np.uint32))


@pytest.mark.parametrize("name", ["lambda", "synth"])
@pytest.mark.parametrize("mode", ["ee", "loc"])
def test_one_mm_golden(engines, name, mode):
    g = load_golden("fm_" + name)
    hits, cnt, ops, _ = engines[name].one_mm(g["reads"], g["quals"], g["lens"], g["mmminsc_" + mode],
                                             mode == "loc")
    ref, refn = g["mm_" + mode], g["mmn_" + mode]
    assert np.array_equal(cnt, refn)
    assert np.array_equal(ops, g["mmops_" + mode].astype(np.uint32))
    for i in range(len(refn)):
        for k in range(refn[i]):
            x, h = ref[i, k], hits[i, k]
            assert (h["top"], h["bot"], h["fw"], h["score"], h["pos"]) == tuple(int(v) for v in x[:5]), (i, k)
            assert (x[5] & 0xff) == ord("ACGTN"[h["chr"]]) and (x[5] >> 8) == ord("ACGTN"[h["qchr"]])


@pytest.mark.parametrize("name", ["lambda", "synth"])
def test_extend_golden(engines, name):
    """SwDriver::extend (k_extend) on every seed hit of the reference's seed search."""
    g = load_golden("ext_" + name)
    rg = g["ranges"]
    out = engines[name].extend(g["reads"], g["lens"], rg)
    assert np.array_equal(out[:, :3], g["out"])


@pytest.mark.parametrize("name", ["lambda", "synth"])
def test_get_offset_golden(engines, name):
    g = load_golden("fm_" + name)
    offs, loads = engines[name].get_offset(g["off_rows"])
    assert np.array_equal(offs, g["off_vals"])
    assert loads.mean() < 32          # geometric walk to a sampled row (offRate 4)


def test_large_batch_vs_oracle(engines, orc):
    """20k synthetic reads with errors, N's and ragged lengths; GPU == oracle."""
    import synth
    idx = get_index("synth")
    gen = np.concatenate(idx.ref_codes)
    n = 20000
    codes, quals, _, _ = synth.reads(4242, gen, n, 150, sub=0.01, nrate=0.002)
    lens = np.full(n, 150, np.uint32)
    rng = np.random.default_rng(1)
    short = rng.random(n) < 0.1
    lens[short] = rng.integers(1, 150, short.sum())
    for i in np.nonzero(short)[0]:
        codes[i, lens[i]:] = 4
    codes[5, :] = 4                                     # all-N read
    fe, be = orc.ebwt(idx.fw, True), orc.ebwt(idx.bw, False)
    e = engines["synth"]
    o_gpu = e.exact_sweep(codes, lens)
    o_cpu = orc.exact_sweep(fe, codes, lens)
    assert np.array_equal(o_gpu[:, :7], _gold_exact_to_gpu_layout(o_cpu))
    s_gpu, ns_gpu, ops_gpu, _ = e.seed_search(codes, lens, 22, 15, 0, 16)
    s_cpu, ns_cpu, ops_cpu = orc.seed_search(fe, be, codes, lens, 22, 15, 0, 16)
    assert np.array_equal(ns_gpu, ns_cpu) and np.array_equal(s_gpu, s_cpu)
    assert np.array_equal(ops_gpu, ops_cpu.astype(np.uint32))
    ms = np.array([int(-0.6 - 0.6 * L) for L in lens], np.int64)
    h_gpu, c_gpu, op_gpu, _ = e.one_mm(codes[:4000], quals[:4000], lens[:4000], ms[:4000], False)
    h_cpu, c_cpu, op_cpu = orc.one_mm(fe, be, codes[:4000], quals[:4000], lens[:4000], ms[:4000], False)
    assert np.array_equal(c_gpu, c_cpu) and np.array_equal(op_gpu, op_cpu.astype(np.uint32))
    for i in np.nonzero(c_cpu)[0]:
        for k in range(c_cpu[i]):
            h = h_gpu[i, k]
            assert (h["top"], h["bot"], h["fw"], h["score"], h["pos"], h["chr"], h["qchr"]) == \
                tuple(int(v) for v in h_cpu[i, k])


def _reads_with_errors(n, seed):
    import synth
    idx = get_index("synth")
    gen = np.concatenate(idx.ref_codes)
    codes, quals, _, _ = synth.reads(seed, gen, n, 150, sub=0.01, nrate=0.002)
    lens = np.full(n, 150, np.uint32)
    rng = np.random.default_rng(seed)
    short = rng.random(n) < 0.1
    lens[short] = rng.integers(1, 150, short.sum())
    for i in np.nonzero(short)[0]:
        codes[i, lens[i]:] = 4
    return codes, quals, lens


@pytest.mark.parametrize("n", [1, 7, 450, 20000])
def test_exact_sweep_quad_equals_lane(engines, n, monkeypatch):
    """The quad-cooperative exact sweep (k_exact_sweep_quad, fm_device.h: a side
    counted by four lanes, summed by DPP) against the one-lane kernel on the same
    reads, every output word (ranges, mine, bwops, side loads), nofw / norc too;
    and against the reference's golden sweep."""
    codes, _, lens = _reads_with_errors(max(n, 2), 77 + n)
    codes, lens = codes[:n], lens[:n]
    e = engines["synth"]
    for nofw, norc in ((0, 0), (1, 0), (0, 1)):
        monkeypatch.setenv("BT2G_FM_QUAD", "0")
        a = e.exact_sweep(codes, lens, nofw=nofw, norc=norc)
        monkeypatch.setenv("BT2G_FM_QUAD", "1")
        b = e.exact_sweep(codes, lens, nofw=nofw, norc=norc)
        assert np.array_equal(a, b), (nofw, norc, np.nonzero((a != b).any(1))[0][:5])
    for name in ("lambda", "synth"):
        g = load_golden("fm_" + name)
        out = engines[name].exact_sweep(g["reads"], g["lens"])
        assert np.array_equal(out[:, :7], _gold_exact_to_gpu_layout(g["exact"]))


def test_one_mm_merged_equals_split(engines, monkeypatch):
    """The 1-mm search with both index directions in one launch per stage
    (k_one_mm_*2, the default) against the two-stream form: hits, counts, bwops."""
    codes, quals, lens = _reads_with_errors(3000, 91)
    ms = np.array([int(-0.6 - 0.6 * L) for L in lens], np.int64)
    e = engines["synth"]
    monkeypatch.setenv("BT2G_MM_MERGED", "0")
    h0, c0, o0, l0 = e.one_mm(codes, quals, lens, ms, False)
    monkeypatch.setenv("BT2G_MM_MERGED", "1")
    h1, c1, o1, l1 = e.one_mm(codes, quals, lens, ms, False)
    assert np.array_equal(c0, c1) and np.array_equal(o0, o1)
    for i in np.nonzero(c0)[0]:
        assert np.array_equal(h0[i, :c0[i]], h1[i, :c0[i]]), i


@pytest.mark.parametrize("n", [3, 450, 3000])
def test_fm_quad_equals_lane(engines, n, monkeypatch):
    """Every kernel with a quad form (BT2G_FM_QUAD, default on: the 1-mm near half
    and branch walks, the seed ranges' extension) against its one-lane form on the
    same reads: 1-mm hits / counts / bwops, seed ranges, extensions, offsets."""
    codes, quals, lens = _reads_with_errors(max(n, 2), 500 + n)
    codes, quals, lens = codes[:n], quals[:n], lens[:n]
    ms = np.array([int(-0.6 - 0.6 * L) for L in lens], np.int64)
    e = engines["synth"]
    res = {}
    for v in ("0", "1"):
        monkeypatch.setenv("BT2G_FM_QUAD", v)
        res[v] = (e.one_mm(codes, quals, lens, ms, False), e.seed_search_ext(codes, lens, 20, 10, 0, 16, off_cap=8))
    (h0, c0, o0, _), x0 = res["0"]
    (h1, c1, o1, _), x1 = res["1"]
    assert np.array_equal(c0, c1) and np.array_equal(o0, o1)
    for i in np.nonzero(c0)[0]:
        assert np.array_equal(h0[i, :c0[i]], h1[i, :c0[i]]), i
    for a, b in zip(x0, x1):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("brq_cap", [1, 7, 64])
def test_one_mm_branch_queue_overflow(engines, brq_cap, monkeypatch):
    """A branch queue far too small for the batch ($BT2G_MM_BRQ_CAP): items whose
    branches do not fit go to the in-place state machine, each exactly once, so
    hits, counts and bwops equal the normal path's (a lane that met
    the full queue while its wave's flush also overflowed was queued twice)."""
    g = load_golden("fm_synth")
    e = engines["synth"]
    args = (g["reads"], g["quals"], g["lens"], g["mmminsc_ee"], False)
    h0, c0, o0, _ = e.one_mm(*args)
    monkeypatch.setenv("BT2G_MM_BRQ_CAP", str(brq_cap))
    h1, c1, o1, _ = e.one_mm(*args)
    assert np.array_equal(c0, c1) and np.array_equal(o0, o1)
    for i in np.nonzero(c0)[0]:
        assert np.array_equal(h0[i, :c0[i]], h1[i, :c0[i]]), i


def test_open_from_files_and_edge_cases(tmp_path):
    import bt2g
    import bt2_index as bi
    idx = get_index("lambda")
    base = str(tmp_path / "lam")
    bi.write_index(base, idx)
    with bt2g.Engine(index_base=base) as e:
        info = e.info()
        assert info[0] == idx.fw.length and info[1] == idx.fw.zoff and info[2] == idx.bw.zoff
        empty = e.exact_sweep(np.zeros((0, 150), np.uint8), np.zeros(0, np.uint32))
        assert empty.shape == (0, 8)
        # nofw / norc leave the skipped strand empty
        g = load_golden("fm_lambda")
        a = e.exact_sweep(g["reads"], g["lens"], nofw=True)
        assert (a[:, 0] == 0).all() and (a[:, 2] == 0).all()
        b = e.exact_sweep(g["reads"], g["lens"])
        assert np.array_equal(a[:, [1, 4, 5]], b[:, [1, 4, 5]])


@pytest.mark.parametrize("skip_exact", [False, True])
@pytest.mark.parametrize("strand", ["both", "norc"])
def test_exact_sweep_1mm_fused(engines, skip_exact, strand):
    """bt2g_exact_sweep_1mm (the batch driver's up-front searches in one call)
    equals bt2g_exact_sweep, then bt2g_one_mm on each read the gate lets through
    with nofw = !(mineFw <= 1), norc = !(mineRc <= 1) (bt2_search.cpp:3649-3667):
    sweep, hit lists in discovery order, counts and bwops."""
    g = load_golden("fm_synth")
    e = engines["synth"]
    norc = strand == "norc"
    reads, quals, lens, ms = g["reads"], g["quals"], g["lens"], g["mmminsc_ee"]
    sw, hits, cnt, ops, offs = e.exact_sweep_1mm(reads, quals, lens, ms, False, norc=norc, skip_exact=skip_exact,
                                                 cap=16, off_cap=8)
    assert np.array_equal(sw, e.exact_sweep(reads, lens, norc=norc))
    # the small ranges' rows: Ebwt::getOffset of each (bt2g_get_offset), BT2G_OFF_MASK elsewhere
    want = np.full(offs.shape, 0xFFFFFFFF, np.uint32)
    rows, where = [], []
    for i in range(len(lens)):
        rg = [(sw[i, 2], sw[i, 3]) if sw[i, 0] == 0 else (0, 0), (sw[i, 4], sw[i, 5]) if sw[i, 1] == 0 else (0, 0)]
        rg += [(int(hits[i, k]["top"]), int(hits[i, k]["bot"])) for k in range(min(cnt[i], 16))]
        for slot, (t, b) in enumerate(rg):
            if 0 < int(b) - int(t) <= 8:
                for j in range(int(b) - int(t)):
                    rows.append(int(t) + j)
                    where.append((i, slot, j))
    got_offs, _ = e.get_offset(np.array(rows, np.uint32))
    for (i, slot, j), o in zip(where, got_offs):
        want[i, slot, j] = o
    assert np.array_equal(offs, want) and len(rows) > 50
    ran = 0
    for i in range(len(lens)):
        yfw, yrc = sw[i, 0] <= 1, sw[i, 1] <= 1 and not norc
        if (skip_exact and min(sw[i, 0], sw[i, 1]) == 0) or not (yfw or yrc):
            assert cnt[i] == 0, i
            continue
        h1, c1, o1, _ = e.one_mm(reads[i:i + 1], quals[i:i + 1], lens[i:i + 1], ms[i:i + 1], False,
                                 nofw=not yfw, norc=not yrc, cap=1024)
        if cnt[i] > 16:
            # over the cap: the count says so (the batch driver then asks the search again)
            assert c1[0] > 16, i
            continue
        assert cnt[i] == c1[0] and ops[i] == o1[0], i
        assert np.array_equal(hits[i, :cnt[i]], h1[0, :c1[0]]), i
        ran += 1
    # (the bench rule with --norc: the skipped strand's mine is 0, so every read is skipped)
    assert ran > 20 or (norc and skip_exact)


@pytest.mark.parametrize("pol", ["s22", "s10"])
def test_seed_search_ext_fused(engines, pol):
    """bt2g_seed_search_ext (the batch driver's seed call) equals bt2g_seed_search,
    then bt2g_extend of every seed range as prioritizeSATups asks it (fw = strand
    0, off = the seed's depth, len = the seed length; aligner_sw_driver.cpp:574-589)
    and bt2g_get_offset of the rows of every range of at most off_cap rows."""
    import synth
    g = load_golden("fm_synth")
    L, iv, off = (int(x) for x in g["seedpol_" + pol])
    idx = get_index("synth")
    codes, _, _, _ = synth.reads(99, np.concatenate(idx.ref_codes), 600, 150, sub=0.01, nrate=0.002)
    lens = np.full(len(codes), 150, np.uint32)
    lens[::7] = 60
    for i in range(0, len(codes), 7):
        codes[i, 60:] = 4
    reads = np.concatenate([g["reads"], codes])            # (the golden reads are 150 wide)
    lens = np.concatenate([g["lens"].astype(np.uint32), lens])
    e = engines["synth"]
    maxs = 16
    out, ns, ops, ext, offs = e.seed_search_ext(reads, lens, L, iv, off, maxs, off_cap=8)
    o0, ns0, ops0, _ = e.seed_search(reads, lens, L, iv, off, maxs)
    assert np.array_equal(out, o0) and np.array_equal(ns, ns0) and np.array_equal(ops, ops0)
    rg, where, rows, rwhere = [], [], [], []
    for i in range(len(lens)):
        for f in range(2):
            for s in range(maxs):
                t, b, tb, bb = (int(v) for v in out[i, f, s])
                depth, sl = s * iv + off, min(L, int(lens[i]))
                if b > t and depth + sl <= lens[i]:
                    rg.append((i, 1 - f, depth, sl, t, b, tb, bb))
                    where.append((i, f, s))
                if 0 < b - t <= 8:
                    for j in range(b - t):
                        rows.append(t + j)
                        rwhere.append((i, f, s, j))
    want = np.zeros_like(ext)
    got = e.extend(reads, lens, np.array(rg, np.uint32))
    for (i, f, s), x in zip(where, got):
        want[i, f, s] = x
    assert np.array_equal(ext, want) and len(rg) > 500
    wo = np.full(offs.shape, 0xFFFFFFFF, np.uint32)
    ov, _ = e.get_offset(np.array(rows, np.uint32))
    for (i, f, s, j), o in zip(rwhere, ov):
        wo[i, f, s, j] = o
    assert np.array_equal(offs, wo) and len(rows) > 500


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["lambda", "synth"])
@pytest.mark.parametrize("skip", [0, 1])
def test_exact_sweep_1mm_reference(engines, name, skip):
    """bt2g_exact_sweep_1mm against the REFERENCE's composition of the same calls
    (tests/golden/fused.npz, make_golden_fused.py: exactSweep, the gate of
    bt2_search.cpp:3649-3650, oneMmSearch, getOffset of the small ranges' rows)."""
    f = load_golden("fused")
    g = load_golden("fm_" + name)
    e = engines[name]
    cap = 16
    sw, hits, cnt, ops, offs = e.exact_sweep_1mm(g["reads"], g["quals"], g["lens"], g["mmminsc_ee"], False,
                                                 skip_exact=bool(skip), cap=cap, off_cap=8)
    assert np.array_equal(sw[:, :7], _gold_exact_to_gpu_layout(f[f"sweep_{name}"]))
    rc = f[f"mmn_{name}_{skip}"]
    assert np.array_equal(cnt, rc.clip(0))
    assert np.array_equal(ops, f[f"mmops_{name}_{skip}"].astype(np.uint32))
    ref, roffs = f[f"mm_{name}_{skip}"], f[f"offs_{name}_{skip}"]
    assert np.array_equal(offs[:, :2], roffs[:, :2])           # the exact ranges' rows
    whole = 0
    for i in range(len(rc)):
        if rc[i] > cap:
            continue                                          # (over the cap: the caller asks again)
        whole += 1
        for k in range(rc[i]):
            x, h = ref[i, k], hits[i, k]
            assert (h["top"], h["bot"], h["fw"], h["score"], h["pos"]) == tuple(int(v) for v in x[:5]), (i, k)
            assert (x[5] & 0xff) == ord("ACGTN"[h["chr"]]) and (x[5] >> 8) == ord("ACGTN"[h["qchr"]])
        assert np.array_equal(offs[i], roffs[i]), i
    assert whole > 100 and (rc > 0).sum() > 50
    assert (e.last_mm_loads[rc < 0] == 0).all() and (e.last_mm_loads[rc > 0] > 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["lambda", "synth"])
@pytest.mark.parametrize("pol", ["s22", "s10"])
def test_seed_search_ext_reference(engines, name, pol):
    """bt2g_seed_search_ext against the REFERENCE: its seed round, SwDriver::extend
    of every range as prioritizeSATups asks it (aligner_sw_driver.cpp:574-589)
    and getOffset of the small ranges' rows (tests/golden/fused.npz)."""
    f = load_golden("fused")
    g = load_golden("fm_" + name)
    L, iv, off = (int(x) for x in f[f"seedpol_{name}_{pol}"])
    sx, so = f[f"sx_{name}_{pol}"], f[f"so_{name}_{pol}"]
    out, ns, ops, ext, offs = engines[name].seed_search_ext(g["reads"], g["lens"], L, iv, off, sx.shape[2],
                                                            off_cap=so.shape[3])
    assert np.array_equal(out, f[f"seed_{name}_{pol}"]) and np.array_equal(ns, f[f"seedn_{name}_{pol}"])
    assert np.array_equal(ops, f[f"seedops_{name}_{pol}"].astype(np.uint32))
    assert np.array_equal(ext[..., :3], sx)
    # side loads: one or two 64-B sides per LF step (the roofline's bytes)
    steps, loads = ext[..., 2].astype(np.int64), ext[..., 3].astype(np.int64)
    assert (loads <= 2 * steps).all() and loads.sum() >= 0.9 * steps.sum() > 0
    assert np.array_equal(offs, so)
