import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "bowtie2-server_amd")
GOLD = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG, os.path.join(PKG, "tools"), GOLD):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libbt2g.so)")


def synth_parts():
    import synth
    g = synth.genome(1234, 300_000, n_repeats=40, rep_len=1500, n_copies=3, n_runs=6)
    return [g[:100_000], g[100_000:220_000], g[220_000:]], [b"chrA", b"chrB", b"chrC"]


_IDX = {}


def get_index(name):
    """Indexes built by tools/bt2_index.py (byte-identical to bowtie2-build,
    see test_index_build.py)."""
    import bt2_index as bi
    if name not in _IDX:
        if name == "lambda":
            _IDX[name] = bi.build_from_fasta(os.path.join(GOLD, "lambda_virus.fa"))
        elif name == "multi":
            _IDX[name] = bi.build_from_fasta(os.path.join(GOLD, "multi.fa"))
        elif name == "synth":
            parts, names = synth_parts()
            _IDX[name] = bi.build_index(parts, names=names)
        else:
            raise KeyError(name)
    return _IDX[name]


@pytest.fixture(scope="session")
def idx_lambda():
    return get_index("lambda")


@pytest.fixture(scope="session")
def idx_synth():
    return get_index("synth")


def load_golden(name):
    return dict(np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False))
