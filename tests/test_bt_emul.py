"""The backtrace kernel source (bowtie2-server_amd/csrc/sw_backtrace.hip),
compiled for the host by tests/cpu_emul (stub HIP header, one kernel lane at a
time), against the reference's alignments (sw_bt_* golden fixtures).  The
fills are the oracle's (pinned to the reference by test_oracle_golden.py),
laid out as the GPU fills leave them: the systolic fill's u8 score plane
(kind 0), the one-problem-per-lane fills' top-aligned u16 plane (kind 1) and
the systolic local fill's u16 plane (kind 2: rows padded to a multiple of 16
at the stack bottom, only blocks holding a non-zero cell written).  CPU only:
catches indexing faults and logic errors before a GPU run."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, load_golden

EMUL = os.path.join(ROOT, "tests", "cpu_emul")
LIB = os.path.join(EMUL, "libbt_emul.so")
SRC = [os.path.join(EMUL, "bt_emul.cpp"), os.path.join(ROOT, "bowtie2-server_amd", "csrc", "sw_backtrace.hip"),
       os.path.join(ROOT, "bowtie2-server_amd", "csrc", "bt2g_kernels.h")]
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


class SwConst(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("match", "npen", "gapbar", "rdgo", "rdge", "rfgo", "rfge")] + \
               [("mmpen", C.c_int32 * 41)]


def build():
    if not os.path.exists(CLANG):
        pytest.skip("clang++ missing")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(s) for s in SRC):
        subprocess.check_call([CLANG, "-O1", "-g", "-std=c++17", "-fPIC", "-shared", "-Wno-unknown-attributes",
                               "-I", os.path.join(EMUL, "stub"), "-I", os.path.join(ROOT, "include"),
                               "-include", "vector", SRC[0], "-o", LIB])
    return C.CDLL(LIB)


def swconst(local):
    c = SwConst(match=2 if local else 0, npen=1, gapbar=4, rdgo=8, rdge=3, rfgo=8, rfge=3)
    for q in range(41):
        c.mmpen[q] = 2 + int(np.float32(q) / np.float32(40.0) * 4)
    return c


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


@pytest.fixture(scope="module")
def lib():
    return build()


def decision_nibbles(h, e, f, rd, q33, rf, sc):
    """The end-to-end u8 fill's decision plane (sw_ee_packed.hip DEC) from the
    oracle's H/E/F (u8 domain): bit 0 H != diag, bit 1 H != F, bit 2 F !=
    H(up) - rfgo, bit 3 E != H(left) - rdgo; row 0 / column 0 terms the
    reference never reads are left set."""
    L, ncol = h.shape
    h, e, f = (x.astype(np.int64) for x in (h, e, f))
    qq = np.clip(q33.astype(np.int64) - 33, 0, 40)
    mm = np.array([sc.mmpen[i] for i in range(41)], np.int64)
    rc = rd.astype(np.int64)[:, None]
    m = rf[:ncol].astype(np.int64)[None, :]
    n_ = (rc > 3) | (m > 15)
    sdiag = np.where(n_, -sc.npen, np.where((m >> np.minimum(rc, 3)) & 1, sc.match, -mm[qq][:, None]))
    up_left = np.full((L, ncol), -10 ** 6, np.int64)
    up_left[1:, 1:] = h[:-1, :-1]
    up = np.full((L, ncol), -10 ** 6, np.int64)
    up[1:, :] = h[:-1, :]
    left = np.full((L, ncol), -10 ** 6, np.int64)
    left[:, 1:] = h[:, :-1]
    nib = (h != up_left + sdiag).astype(np.uint8)
    nib |= (h != f).astype(np.uint8) << 1
    nib |= (f != up - sc.rfgo).astype(np.uint8) << 2
    nib |= (e != left - sc.rdgo).astype(np.uint8) << 3
    return nib


@pytest.mark.parametrize("src,kind", [("rand_ee", 0), ("log_ee", 0), ("rand_ee", 1), ("rand_loc", 1),
                                      ("log_loc", 1), ("rand_loc", 2), ("log_loc", 2), ("rand_ee", 3),
                                      ("log_ee", 3)])
def test_bt_kernel_source_on_cpu(lib, src, kind):
    x = _inputs(src, kind)
    lib.bt_emul_run(C.c_int({0: 0, 1: 1, 2: 1, 3: 2}[kind]), _p(x["probs"]), C.c_uint32(x["n"]), _p(x["reads"]),
                    _p(x["quals"]), C.c_uint32(x["stride"]), _p(x["lens"]), _p(x["rf"]), _p(x["rects"]),
                    _p(x["res"]), _p(x["cands"]), C.c_uint32(x["cap"]), _p(x["plane"]), C.c_uint64(x["slot"]),
                    C.c_uint32(x["S16"]), C.c_int(x["plane_top"]), C.c_uint32(x["maxrow"]), C.c_uint32(x["maxcol"]),
                    C.byref(swconst(x["local"])), C.c_int(int(x["local"])), C.c_double(0.0), C.c_double(0.15),
                    C.c_uint32(x["maxaln"]), C.c_uint32(x["maxedit"]), _p(x["naln"]), _p(x["alns"]), _p(x["edits"]),
                    _p(x["fates"]))
    _check(x, src, kind)


WG_SRC = [os.path.join(EMUL, "wg_emul.cpp"), os.path.join(ROOT, "bowtie2-server_amd", "csrc", "sw_backtrace_wg.hip"),
          os.path.join(ROOT, "bowtie2-server_amd", "csrc", "bt2g_kernels.h"),
          os.path.join(EMUL, "stub_wg", "hip", "hip_runtime.h")]
WG_LIB = os.path.join(EMUL, "libwg_emul.so")


@pytest.fixture(scope="module")
def wglib():
    if not os.path.exists(CLANG):
        pytest.skip("clang++ missing")
    if not os.path.exists(WG_LIB) or os.path.getmtime(WG_LIB) < max(os.path.getmtime(s) for s in WG_SRC):
        subprocess.check_call([CLANG, "-O1", "-g", "-std=c++17", "-fPIC", "-shared", "-Wno-unknown-attributes",
                               "-pthread", "-I", os.path.join(EMUL, "stub_wg"), "-I", os.path.join(ROOT, "include"),
                               WG_SRC[0], "-o", WG_LIB])
    return C.CDLL(WG_LIB)


@pytest.mark.parametrize("src,maxaln", [("rand_ee", 256), ("log_ee", 256), ("log_ee", 2)])
def test_bt_wg_kernel_source_on_cpu(wglib, src, maxaln):
    """sw_backtrace_wg.hip (a workgroup per DP, candidates walked in parallel, the
    reportedThrough resolution by the wave) run as 64 host threads per workgroup:
    every alignment, edit and candidate fate equals the reference's (maxaln 2:
    the loop's stop after the second alignment)."""
    x = _inputs(src, 3, maxaln=maxaln)
    x["n"] = min(x["n"], 120)           # (64 host threads per workgroup: a subset keeps the CPU suite short)
    wglib.wg_emul_run(_p(x["probs"]), C.c_uint32(x["n"]), _p(x["reads"]), _p(x["quals"]), C.c_uint32(x["stride"]),
                      _p(x["lens"]), _p(x["rf"]), _p(x["rects"]), _p(x["res"]), _p(x["cands"]), C.c_uint32(x["cap"]),
                      _p(x["plane"]), C.c_uint64(x["slot"]), C.c_uint32(x["S16"]), C.c_uint32(x["maxcol"]),
                      C.byref(swconst(False)), C.c_double(0.0), C.c_double(0.15), C.c_uint32(x["maxaln"]),
                      C.c_uint32(x["maxedit"]), _p(x["naln"]), _p(x["alns"]), _p(x["edits"]), _p(x["fates"]))
    _check(x, src, 3, maxaln=maxaln)


def _inputs(src, kind, maxaln=None):
    import bt2g
    from oracle.oracle import Oracle
    from test_oracle_golden import sw_problems
    orc = Oracle()
    g, b = load_golden("sw_" + src), load_golden("sw_bt_" + src)
    local = bool(g["local"])
    probs = np.zeros(len(g["rd_index"]), bt2g.SWPROB_DTYPE)
    probs["read"], probs["fw"], probs["minsc"] = g["rd_index"], g["fw"], g["minsc"]
    probs["win_off"] = g["rf_off"][:-1]
    probs["ncol"] = np.diff(g["rf_off"]) - 1
    n, cap = len(probs), 4096
    res = np.zeros(n, bt2g.SWRES_DTYPE)
    cands = np.zeros((n, cap), bt2g.SWCAND_DTYPE)
    stride = g["reads"].shape[1]
    S16 = 16 * ((stride + 15) // 16)
    maxcol = int(probs["ncol"].max())
    maxrow = int(g["lens"].max())
    es = 1 if kind in (0, 3) else 2
    plane_top = {0: 0, 1: 1, 2: 2, 3: 0}[kind]
    slot = S16 * maxcol * es + ((maxcol * 2 + 15) & ~15)   # plane + per-column block masks
    plane = np.zeros(slot * n, np.uint8)
    keep = np.ones(n, bool)
    for p, rd, q, rf, minsc, fw, out, cref in sw_problems(g):
        o, c, m = orc.sw(rd, q, rf, minsc, local, want_mat=True, cap=cap)
        res[p] = (o[0], max(o[1], -2**31), o[2], o[3], o[4], o[5], o[6], 0)
        cands[p, :len(c)] = [tuple(x) for x in c]
        L, ncol = len(rd), len(rf) - 1
        if kind == 2:
            # systolic local layout: score domain, padded rows end at the stack
            # bottom, blocks without a non-zero cell unwritten (garbage) + masks
            top = S16 - ((L + 15) // 16) * 16
            stack = np.zeros((S16, maxcol), np.uint16)
            stack[top:top + L, :ncol] = ((m[:, :, 0].astype(np.int64) + (0 if o[2] else 0x8000)) & 0xffff)
            blocks = stack.reshape(S16 // 16, 16, maxcol)
            live = blocks.max(1) > 0
            if S16 > 256:
                live[:] = True
            blocks = np.where(live[:, None, :], blocks, 0x5a5a).astype(np.uint16)
            plane[p * slot:p * slot + S16 * maxcol * 2] = blocks.transpose(0, 2, 1).ravel().view(np.uint8)
            if S16 <= 256:
                masks = (live.astype(np.uint32) << np.arange(S16 // 16)[:, None].astype(np.uint32)).sum(0)
                plane[p * slot + S16 * maxcol * 2:p * slot + S16 * maxcol * 2 + 2 * maxcol] = \
                    masks.astype(np.uint16).view(np.uint8)
        if kind == 1:
            # one-problem-per-lane fill layout: u16 (score + 0x8000 for i16
            # fills), rows top-aligned, all blocks written, no masks
            h = m[:, :, 0].astype(np.int64) + (0 if o[2] else 0x8000)
            stack = np.zeros((S16, maxcol), np.uint16)
            stack[:L, :ncol] = (h & 0xffff).astype(np.uint16)
            plane[p * slot:p * slot + S16 * maxcol * 2] = \
                stack.reshape(S16 // 16, 16, maxcol).transpose(0, 2, 1).ravel().view(np.uint8)
        if kind == 3:
            # decision bits (kernel kind 2): block-major [stack row // 16][column][2 words],
            # same block masks as kind 0
            if o[0] and not o[2]:
                keep[p] = False
                continue
            nib = decision_nibbles(m[:, :, 0], m[:, :, 1], m[:, :, 2], rd, q, rf, swconst(False))
            stack = np.full((S16, maxcol), 0xf, np.uint8)
            stack[S16 - L:, :ncol] = nib
            hs = np.full((S16, maxcol), 0xff, np.uint8)
            hs[S16 - L:, :ncol] = m[:, :, 0]
            live = hs.reshape(S16 // 16, 16, maxcol).max(1) >= 255 + minsc
            if S16 > 256:
                live[:] = True
            # word w of a block column: row 8w+i's bits 0/1/2 at 3(7-i)+2/+1/+0, bit 3 at 24+7-i
            st = stack.astype(np.uint32).reshape(S16 // 16, 2, 8, maxcol)            # (blk, w, i, col)
            sh = (3 * (7 - np.arange(8)))[None, None, :, None].astype(np.uint32)
            b0, b1, b2, b3 = st & 1, (st >> 1) & 1, (st >> 2) & 1, (st >> 3) & 1
            words = ((b0 << (sh + 2)) | (b1 << (sh + 1)) | (b2 << sh) |
                     (b3 << (24 + 7 - np.arange(8)).astype(np.uint32)[None, None, :, None])).sum(2).astype(np.uint32)
            words = np.where(live[:, None, :], words, 0xa5a5a5a5).astype(np.uint32)   # (blk, w, col)
            plane[p * slot:p * slot + S16 * maxcol // 2] = words.transpose(0, 2, 1).ravel().view(np.uint8)
            if S16 <= 256:
                masks = (live.astype(np.uint32) << np.arange(S16 // 16)[:, None].astype(np.uint32)).sum(0)
                plane[p * slot + S16 * maxcol:p * slot + S16 * maxcol + 2 * maxcol] = \
                    masks.astype(np.uint16).view(np.uint8)
        if kind == 0:
            if o[0] and not o[2]:
                keep[p] = False          # i16 fill: not in a u8 plane (naln -4)
                continue
            # block-major: [stack row // 16][column][stack row % 16]; as the fill,
            # only blocks holding a cell >= minsc are written (others garbage)
            stack = np.full((S16, maxcol), 0xff, np.uint8)
            stack[S16 - L:, :ncol] = m[:, :, 0]
            blocks = stack.reshape(S16 // 16, 16, maxcol)
            live = blocks.max(1) >= 255 + minsc                      # (blocks, cols)
            if S16 > 256:
                live[:] = True                                       # no masks: all written
            blocks = np.where(live[:, None, :], blocks, 0x5a)        # dead: garbage
            plane[p * slot:p * slot + S16 * maxcol] = blocks.transpose(0, 2, 1).ravel()
            if S16 <= 256:
                masks = (live.astype(np.uint32) << np.arange(S16 // 16)[:, None].astype(np.uint32)).sum(0)
                plane[p * slot + S16 * maxcol:p * slot + S16 * maxcol + 2 * maxcol] = \
                    masks.astype(np.uint16).view(np.uint8)
    rects = np.zeros(n, bt2g.SWRECT_DTYPE)
    rects["triml"], rects["corel"], rects["corer"] = b["triml"], b["corel"], b["corer"]
    if maxaln is None:
        maxaln = 4096 if local else 256
    maxedit = 512
    naln = np.zeros(n, np.int32)
    alns = np.zeros((n, maxaln), bt2g.SWALN_DTYPE)
    edits = np.zeros((n, maxaln, maxedit), bt2g.EDIT_DTYPE)
    fates = np.zeros((n, cap), np.int8)
    lens = np.ascontiguousarray(g["lens"], np.uint32)
    return dict(probs=probs, n=n, reads=g["reads"], quals=g["quals"], stride=stride, lens=lens, rf=g["rf"],
                rects=rects, res=res, cands=cands, cap=cap, plane=plane, slot=slot, S16=S16, plane_top=plane_top,
                maxrow=maxrow, maxcol=maxcol, local=local, maxaln=maxaln, maxedit=maxedit, naln=naln, alns=alns,
                edits=edits, fates=fates, keep=keep, b=b)


def _check(x, src, kind, maxaln=None):
    from test_oracle_golden import bt_expected
    n, keep, naln, alns, edits, fates, b = (x[k] for k in ("n", "keep", "naln", "alns", "edits", "fates", "b"))
    nal = 0
    for p in range(n):
        if not keep[p]:
            assert naln[p] == -4
            continue
        ea, eeds, efates = bt_expected(b, p)
        if maxaln is not None and len(ea) > maxaln:
            # the loop stops at maxaln: the first maxaln alignments, the fates up to the last of them
            last = int(ea[maxaln - 1, 0])
            ea, eeds, efates = ea[:maxaln], eeds[:maxaln], efates[:last + 1]
        assert naln[p] == len(ea), (src, kind, p)
        for k in range(len(ea)):
            got = alns[p, k]
            assert [got[f] for f in ("cand", "score", "off", "ns", "gaps", "refns", "nedit", "trim5p", "trim3p")] \
                == [ea[k, i] for i in (0, 1, 2, 4, 5, 6, 7, 8, 9)], (src, kind, p, k)
            e = edits[p, k, :int(ea[k, 7])]
            assert np.array_equal(np.stack([e["pos"], e["type"], e["chr"], e["qchr"]], 1), eeds[k]), (src, p, k)
        if len(efates):
            assert np.array_equal(fates[p, :len(efates)], efates), (src, kind, p)
        nal += len(ea)
    assert nal > (8 if maxaln is not None else 40)
