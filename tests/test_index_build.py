"""tools/bt2_index.py must write the same bytes as the reference bowtie2-build
(SHA-256 fixtures made by tests/golden/make_golden.py from oracle/_ref)."""
import hashlib
import json
import os

import pytest

from conftest import GOLD, get_index

EXTS = ["1.bt2", "2.bt2", "3.bt2", "4.bt2", "rev.1.bt2", "rev.2.bt2"]


@pytest.mark.parametrize("name", ["lambda", "multi", "synth"])
def test_index_bytes_match_reference(name, tmp_path):
    import bt2_index as bi
    ref = json.load(open(os.path.join(GOLD, "index_sha256.json")))[name]
    base = str(tmp_path / name)
    bi.write_index(base, get_index(name))
    for e in EXTS:
        h = hashlib.sha256(open(base + "." + e, "rb").read()).hexdigest()
        assert h == ref[e], f"{name}.{e} differs from bowtie2-build output"


def test_index_roundtrip(tmp_path):
    import numpy as np
    import bt2_index as bi
    idx = get_index("multi")
    base = str(tmp_path / "m")
    bi.write_index(base, idx)
    r = bi.read_index(base)
    assert (r.text == idx.text).all()
    assert all((a == b).all() for a, b in zip(r.ref_codes, idx.ref_codes))
    assert (r.fw.ftab == idx.fw.ftab).all() and (r.bw.ebwt == idx.bw.ebwt).all()
    assert r.fw.zoff == idx.fw.zoff and np.array_equal(r.fw.offs, idx.fw.offs)
