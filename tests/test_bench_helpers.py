"""CPU checks of bench.py's host helpers: the paired read generator's
geometry (fragments of 200..500, --fr mates) and the mate
rectangle width budget (gap_budget, checked against the oracle's framer,
itself pinned to the reference's rectangles by test_oracle_golden.py)."""
import numpy as np

import bench
from test_oracle_golden import orc  # noqa: F401  (session oracle fixture)


def test_gap_budget_matches_framer(orc):  # noqa: F811
    for minsc in (0, -1, -8, -9, -11, -50, -90, -91, -200, -600):
        # seed-extension rectangle with a huge maxhalf: corel = max(read gaps, ref gaps)
        ok, fw, refl, ncol, triml, corel, corer = orc.frame(0, 10_000, 150, 100_000, minsc, maxhalf=10_000)
        assert ok and corel == bench.gap_budget(minsc, 150), minsc


def test_make_pairs_geometry():
    parts, _ = bench.make_genome(0.5)
    n, L = 400, 150
    reads, quals = bench.make_pairs(parts, n, L, seed=3)
    assert reads.shape == (2 * n, L) and quals.shape == (2 * n, L)
    assert reads.max() <= 4 and quals.min() >= 33 + 2 and quals.max() <= 33 + 40
    g = np.concatenate(parts)
    # locate every mate exactly (ignoring mutated reads) and check the --fr fragment
    # a cheaper check: most mate-1 / mate-2 pairs map within 500 bp of each other on opposite strands
    def find(r):
        rc = np.where(r > 3, 4, 3 - r)[::-1]
        for strand, s in ((True, r), (False, rc)):
            key = s[:24].tobytes()
            hits = lookup_pos.get(key)
            if hits is not None:
                return strand, hits
        return None
    lookup_pos, seen = {}, set()
    for i in range(len(g) - 24):
        key = g[i:i + 24].tobytes()
        if key in lookup_pos:
            seen.add(key)                                # repeated 24-mer: ambiguous, skipped
        lookup_pos[key] = i
    for key in seen:
        del lookup_pos[key]
    good = 0
    for i in range(n):
        a, b = find(reads[i]), find(reads[n + i])
        if a is None or b is None:
            continue
        (sa, pa), (sb, pb) = a, b
        assert sa != sb                                  # --fr: opposite strands
        frag = max(pa, pb) + L - min(pa, pb)
        assert 150 <= frag <= 500 + 2, frag
        good += 1
    assert good > n // 2


def test_policy_seed_geometry():
    """Seed length / interval / count per strand at 150 bp (SURVEY.md 8a row A9:
    --sensitive 22/15 -> 9 seeds, --very-sensitive 20/7 -> 19, paired-end
    interval boost (int)(ival * 1.2 + 0.5), bt2_search.cpp:3392-3395)."""
    want = {("ee", "sensitive"): (22, 15, 9), ("ee", "very-sensitive"): (20, 7, 19),
            ("local", "sensitive"): (20, 10, 14), ("local", "very-sensitive"): (20, 7, 19),
            ("paired", "sensitive"): (22, 18, 8), ("paired", "very-sensitive"): (20, 8, 17)}
    for (mode, preset), (L, ival, nseeds) in want.items():
        p = bench.Policy(mode, 150, preset)
        assert (p.seedlen, p.interval, 1 + (150 - p.seedlen) // p.interval) == (L, ival, nseeds), (mode, preset)
        assert p.minsc == (60 if mode == "local" else -90)


def test_ref_chain_compare_cpu():
    """oracle/ref_chain: the reference's own seed-extension chain runs on a small
    synthetic index, and compare() reports zero for identical buffers and
    counts a planted difference at every stage."""
    import os
    import tempfile
    import pytest
    import numpy as np
    import bench
    import bt2_index as bi
    import synth
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not os.path.exists(os.path.join(root, "oracle", "_ref", "libbt2ref.so")):
        pytest.skip("oracle/_ref not built")
    from oracle.ref_chain import RefChain, compare
    g = synth.genome(5, 120_000, n_repeats=20, rep_len=2000, n_copies=3, n_runs=3)
    idx = bi.build_index([g[:60_000], g[60_000:]], names=[b"a", b"b"])
    base = os.path.join(tempfile.mkdtemp(), "g")
    bi.write_index(base, idx)
    r, q = bench.make_reads(idx.ref_codes, 400, 150, 3)
    seqs = [bytes(a) for a in synth.to_ascii(r)]
    pol = bench.Policy("ee", 150)
    ch = RefChain(base)
    ref = ch.run(seqs, [bytes(x) for x in q], np.full(400, 150), pol, 1 + (150 - pol.seedlen) // pol.interval, 16,
                 15, idx.ref_codes, 2)
    ch.close()
    assert ref["sw"][:, 2].sum() > 300                    # most reads align
    lut = np.full(256, 4)
    lut[[65, 67, 71, 84]] = [0, 1, 2, 3]
    h = ref["mm_hits"]
    mh = np.zeros(h.shape[:2] + (8,), np.int64)
    mh[:, :, :5] = h[:, :, :5]
    mh[:, :, 5], mh[:, :, 6] = lut[h[:, :, 5] & 255], lut[(h[:, :, 5] >> 8) & 255]
    gpu = {"sweep": ref["ex"][:, [0, 1, 3, 4, 5, 6, 7, 2]].astype(np.int64), "mm_cnt": ref["mm_cnt"].copy(),
           "mm_hits": mh, "seeds": ref["seeds"].copy(), "rows": ref["rows"]["row"].copy(), "offs": ref["offs"].copy(),
           "row_read": ref["rows"]["read"], "probs": {k: v.copy() for k, v in ref["probs"].items()}}
    c = compare(ref, gpu)
    assert all(c[k] == 0 for k in ("exact_sweep_mismatch", "one_mm_mismatch", "seed_mismatch", "row_mismatch",
                                   "offset_mismatch", "frame_mismatch")), c
    gpu["offs"][3] += 1
    gpu["probs"]["refl"][5] += 1
    gpu["sweep"][7, 0] += 1
    c = compare(ref, gpu)
    assert c["offset_mismatch"] == 1 and c["frame_mismatch"] == 1 and c["exact_sweep_mismatch"] == 1, c


def test_schedule_and_stock_baseline_cpu():
    """bench.schedule_run + bench.stock_baseline end to end on CPU: the batch
    server over the CPU stand-in of the engines (bowtie2-align-server-batch-stub)
    and the stock reference server on 2 500 reads of a small synthetic index
    (one chunk, k = 2):
    identical sorted SAM, the aligned count taken from the SAM, the server's
    engine statistics read back."""
    import os
    import tempfile
    import types
    import pytest
    import bench
    import bt2_index as bi
    import synth
    from oracle import ref_server as rs
    stub = os.path.join(rs.REF_DIR, "bowtie2-align-server-batch-stub")
    if not (os.path.exists(rs.SERVER) and os.path.exists(stub)):
        pytest.skip("oracle/_ref servers not built")
    g = synth.genome(7, 100_000, n_repeats=10, rep_len=1500, n_copies=3, n_runs=2)
    idx = bi.build_index([g], names=[b"chr"])
    d = tempfile.mkdtemp()
    base = os.path.join(d, "g")
    bi.write_index(base, idx)
    r, q = bench.make_reads(idx.ref_codes, 2500, 150, 5)
    args = types.SimpleNamespace(mode="ee", preset="sensitive", reads=2500, drivers=2, clients=2, warmup=1,
                                 warmup_chunks=1, steps=2, stock_sample=2500, cpu_threads=2, stock_runs=2)
    sc = bench.schedule_run(args, 0, 1, 0, base, r, q, d, binary=stub)
    # two timed passes: the first counted by the client alone, the last also from its SAM
    assert len(sc["pass_s"]) == 2
    assert sc["aligned"] == 2 * bench.count_aligned(sc["outs"], False) and 4000 < sc["aligned"] <= 5000
    assert sc["stats"]["driver"] == "batch" and sc["stats"]["reads"] >= 2500
    cpu, sam = bench.stock_baseline(args, base, sc["chunks"], sc["outs"], d)
    assert sam["identical"] and sam["records"] == 2500
    assert cpu["value"] > 0 and cpu["kind"] == "reference" and len(cpu["runs"]) == 2


def test_count_aligned_flags():
    sam = [b"r1\t0\tc\t1\n@CO x\nr2\t4\t*\t0\nr3\t256\tc\t5\nr4\t16\tc\t9\n",
           b"p1\t77\t*\t0\np1\t141\t*\t0\np2\t73\tc\t1\np2\t133\t*\t0\np3\t99\tc\t1\np3\t147\tc\t9\n"]
    assert bench.count_aligned(sam[:1], False) == 2
    assert bench.count_aligned(sam[1:], True) == 2


def test_line_roofline_names_largest_consumer():
    """The line's roofline is the largest consumer's; when that one has no bound
    (--local: the one-walker backtrace) it is the largest bounded kernel's, and the
    consumer is named in it."""
    def ids(**rows):
        v = [[0, 0.0, 0, 0] for _ in range(16)]
        for k, r in rows.items():
            v[int(k[1:])] = r
        return {"ids": v}
    st = {"kernels": {"exact_sweep": ids(i0=[100, 40.0, 10 ** 9, 4000], i2=[100, 90.0, 2 * 10 ** 9, 3000]),
                      "sw_dp": ids(i4=[100, 70.0, 10 ** 10, 5000], i5=[100, 500.0, 0, 0], i7=[100, 900.0, 0, 0])}}
    kern = bench.server_kernels(st)
    rl, rls = bench.line_rooflines(kern, "/nonexistent.json")
    assert rl["kernel"].startswith("k_one_mm") and rl["family"]
    assert rl["largest_consumer"]["id"] == "sw_dp:5"
    assert abs(rl["largest_consumer"]["share_of_kernel_time"] - 500 / 700) < 1e-9
    assert [e["id"] for e in rls] == ["exact_sweep:2", "sw_dp:4", "exact_sweep:0"]
    st["kernels"]["sw_dp"]["ids"][5] = [100, 5.0, 0, 0]
    rl, _ = bench.line_rooflines(bench.server_kernels(st), "/nonexistent.json")
    assert rl["kernel"].startswith("k_one_mm") and "largest_consumer" not in rl
