"""The bench's whole per-read chain on the GPU -- exact sweep, gated 1-mm search,
seeds, hit rows (k_collect_rows), getOffset, joinedToTextOff + straddle filter +
frameSeedExtensionRect (k_frame, bt2g_frame), fill + the nextAlignment loop,
and in paired mode otherMate + frameFindMateRect + the mate DPs -- against the
reference's own chain on its own intermediates (oracle/ref_chain.py over the
reference build in oracle/_ref), on a 24 Mbp genome with hg38's repeat
landscape.  Every stage: 0 mismatches (bench.chain_parity)."""
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def genome_index():
    import torch
    import bench
    import bt2_index as bi
    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libbt2ref.so")):
        pytest.skip("oracle/_ref not built")
    parts, names = bench.make_genome(24)
    idx = bi.build_index_device(parts, names=names, device="cuda")
    torch.cuda.synchronize()
    return parts, idx


@pytest.mark.parametrize("mode", ["ee", "paired", "local"])
def test_chain_parity(genome_index, mode):
    import torch
    import bench
    import bt2g
    parts, idx = genome_index
    n = 8000
    if mode == "paired":
        r, q = bench.make_pairs(parts, n, 150, 11)
    else:
        r, q = bench.make_reads(parts, n, 150, 11)
    eng = bt2g.Engine(index=idx)
    pipe = None
    try:
        dev = torch.device("cuda")
        pipe = bench.Pipeline(eng, idx, torch.from_numpy(r).to(dev), torch.from_numpy(q).to(dev), 150, mode)
        pipe.step(keep=True)
        torch.cuda.synchronize()
        sample = 1500
        _, ref, mate, _ = bench.cpu_baseline(idx, r, q, pipe, sample, 8)
        parity = bench.chain_parity(pipe, ref, mate)
        bad = {k: v for k, v in parity.items() if k.endswith("mismatch") and v}
        npb = pipe.last["npb"]
        over = int((pipe.naln[:npb] == -5).sum())            # candidate lists longer than the cap
        assert not bad, (parity, "cand overflow", over)
        assert parity["dps"] > sample // 2 and parity.get("ref_alignments", 0) > 0, parity
        if mode == "paired":
            assert any(k.startswith("mate") for k in parity), parity
    finally:
        if pipe is not None and getattr(pipe, "eng2", None) is not None:
            pipe.eng2.close()
        eng.close()
