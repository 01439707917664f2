"""libbt2g.so loads on the CPU host and exports every entry point of include/bt2g.h."""
import ctypes
import os
import re

from conftest import PKG, ROOT


def declared_symbols(header="bt2g.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"\b(bt2g_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_all_symbols():
    import bt2g
    bt2g.build()
    lib = ctypes.CDLL(bt2g.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 18
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # bench.py's glue lives in a library of its own (include/bt2g_bench.h), not the product's
    assert not any(hasattr(lib, s) for s in declared_symbols("bt2g_bench.h"))


def test_bench_library_exports_its_symbols():
    import bt2g
    bt2g.build()
    lib = ctypes.CDLL(bt2g.BENCH_LIB_PATH)
    syms = declared_symbols("bt2g_bench.h")
    assert syms == ["bt2g_bench_collect_rows_dev", "bt2g_bench_frame_dev"]
    assert all(hasattr(lib, s) for s in syms)


def test_library_is_gfx950_only():
    import bt2g
    blob = open(bt2g.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_no_oracle_in_product():
    """The product never loads or includes the oracle / reference build."""
    bad = re.compile(r"liboracle|libbt2ref|oracle/_ref|from oracle|import oracle|#include\s+\"\.\./\.\./oracle")
    for dp, _, fs in os.walk(PKG):
        for f in fs:
            if f.endswith((".hip", ".cpp", ".h", ".py", "Makefile")) or f == "Makefile":
                s = open(os.path.join(dp, f)).read()
                assert not bad.search(s), f
    blob = open(os.path.join(PKG, "libbt2g.so"), "rb").read()
    assert b"liboracle" not in blob and b"libbt2ref" not in blob
