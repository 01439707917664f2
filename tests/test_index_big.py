"""The device index builder's >INT_MAX paths (bucketed suffix sort, chunked
nonzero / cummax), forced on a small genome by shrinking the chunk size, must
give the same index as the direct path (which test_index_build.py pins to
bowtie2-build's bytes)."""
import numpy as np

import bt2_index as bi
import synth


def test_chunked_builder_matches_direct():
    g = synth.genome(77, 60_000, n_repeats=6, rep_len=500, n_copies=3, n_runs=2)
    parts, names = [g[:25_000], g[25_000:]], [b"a", b"b"]
    ref = bi.build_index_device(parts, names=names, device="cpu")
    old = bi._CHUNK
    try:
        bi._CHUNK = 4096
        big = bi.build_index_device(parts, names=names, device="cpu")
    finally:
        bi._CHUNK = old
    for a, b in ((ref.fw, big.fw), (ref.bw, big.bw)):
        assert a.zoff == b.zoff
        for f in ("ebwt", "ftab", "eftab", "fchr", "offs"):
            assert np.array_equal(np.asarray(getattr(a, f)), np.asarray(getattr(b, f))), f
