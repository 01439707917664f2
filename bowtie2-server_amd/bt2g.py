"""Python binding of the C ABI in include/bt2g.h (libbt2g.so, built in-tree).

Thin ctypes layer used by the tests, bench.py and __graft_entry__; the product
is the C ABI itself (a C++ host such as bt2_search.cpp would call it
directly).  Raises if the HIP library is missing: there is
no CPU fallback anywhere on this path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# BT2G_LIB selects an alternative in-tree build (kernel experiments)
LIB_PATH = os.environ.get("BT2G_LIB", os.path.join(HERE, "libbt2g.so"))

BT2G_OK = 0
BT2G_ERR_OVERFLOW = -6
K_EXACT_SWEEP, K_SEED_SEARCH, K_ONE_MM, K_GET_OFFSET, K_SW_ALIGN, K_SW_BACKTRACE, K_UNGAPPED, K_FRAME = range(8)


class Scoring(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("match", "mmp_max", "mmp_min", "npen", "rdg_const", "rdg_lin",
                                          "rfg_const", "rfg_lin", "gapbar", "local")] + \
               [("ncl_const", C.c_double), ("ncl_lin", C.c_double)]


def scoring(local=False):
    """bowtie2 defaults (scoring.h:28-83, bt2_search.cpp:452)."""
    return Scoring(match=2 if local else 0, mmp_max=6, mmp_min=2, npen=1, rdg_const=5, rdg_lin=3,
                   rfg_const=5, rfg_lin=3, gapbar=4, local=1 if local else 0, ncl_const=0.0, ncl_lin=0.15)


MM1_DTYPE = np.dtype([("top", "<u4"), ("bot", "<u4"), ("fw", "<i4"), ("score", "<i4"), ("pos", "<i4"),
                      ("chr", "<i4"), ("qchr", "<i4"), ("pad", "<i4")])
SWPROB_DTYPE = np.dtype([("read", "<u4"), ("fw", "<i4"), ("refl", "<i8"), ("win_off", "<i8"), ("refidx", "<u4"),
                         ("ncol", "<u4"), ("minsc", "<i4"), ("pad", "<u4")])
SWRES_DTYPE = np.dtype([("aligned", "<i4"), ("best", "<i4"), ("u8succ", "<i4"), ("i16succ", "<i4"),
                        ("colstop", "<i4"), ("lastsolcol", "<i4"), ("ncand", "<i4"), ("flag", "<i4")])
SWCAND_DTYPE = np.dtype([("row", "<i4"), ("col", "<i4"), ("score", "<i4")])
SWRECT_DTYPE = np.dtype([("triml", "<i4"), ("corel", "<i4"), ("corer", "<i4"), ("pad", "<i4")])
SWALN_DTYPE = np.dtype([(n, "<i4") for n in ("cand", "score", "off", "ns", "gaps", "refns", "nedit", "trim5p",
                                             "trim3p", "pad")])
UGPROB_DTYPE = np.dtype([("read", "<u4"), ("fw", "<i4"), ("off", "<i8"), ("refidx", "<u4"), ("minsc", "<i4")])
UGRES_DTYPE = np.dtype([("ret", "<i4"), ("score", "<i4"), ("refoff", "<i8")] +
                       [(n, "<i4") for n in ("ns", "refns", "nedit", "trim5p", "trim3p", "pad")])
EDIT_DTYPE = np.dtype([("pos", "<u4"), ("type", "u1"), ("chr", "u1"), ("qchr", "u1"), ("pad", "u1")])
FRAMEIN_DTYPE = np.dtype([("off", "<i8"), ("read", "<u4"), ("refidx", "<u4"), ("minsc", "<i4"), ("fw", "<i4"),
                          ("kind", "<i4"), ("anchor1", "<i4"), ("alen", "<u4"), ("pad", "<u4")])
PE_FF, PE_RR, PE_FR, PE_RF = 1, 2, 3, 4   # pe.h PE_POLICY_*


class PePolicy(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("policy", "minfrag", "maxfrag", "local", "flip", "dovetail", "contain",
                                          "olap", "expand", "pad")]


def pe_policy(policy=PE_FR, minfrag=0, maxfrag=500, local=False, flip=False, dovetail=False, contain=True,
              olap=True, expand=True):
    """PairedEndPolicy defaults of bowtie2 (--fr -I 0 -X 500, no dovetail,
    containment and overlap allowed, bt2_search.cpp)."""
    return PePolicy(policy=policy, minfrag=minfrag, maxfrag=maxfrag, local=int(local), flip=int(flip),
                    dovetail=int(dovetail), contain=int(contain), olap=int(olap), expand=int(expand))


class EbwtMem(C.Structure):
    _fields_ = [("len", C.c_uint32), ("zoff", C.c_uint32), ("ftab_chars", C.c_uint32), ("off_rate", C.c_uint32),
                ("line_rate", C.c_uint32), ("fchr", C.c_void_p), ("sides", C.c_void_p), ("sides_bytes", C.c_uint64),
                ("ftab", C.c_void_p), ("eftab", C.c_void_p), ("offs", C.c_void_p), ("offs_len", C.c_uint64),
                ("rstarts", C.c_void_p), ("nfrag", C.c_uint32)]


class IndexMem(C.Structure):
    _fields_ = [("fw", EbwtMem), ("bw", EbwtMem), ("ref_codes", C.c_void_p), ("ref_starts", C.c_void_p),
                ("nref", C.c_uint32)]


def build(force=False):
    """Compile libbt2g.so for gfx950 (make -C bowtie2-server_amd)."""
    if force or not os.path.exists(LIB_PATH) or not os.path.exists(BENCH_LIB_PATH):
        subprocess.check_call(["make", "-C", HERE, "-j8"], stdout=subprocess.DEVNULL)
    return LIB_PATH


_lib = None
_bench_lib = None
BENCH_LIB_PATH = os.path.join(HERE, "libbt2g_bench.so")


def bench_lib():
    """libbt2g_bench.so (include/bt2g_bench.h): bench.py's kernel-chain glue,
    kept out of the product library."""
    global _bench_lib
    if _bench_lib is None:
        if not os.path.exists(BENCH_LIB_PATH):
            raise RuntimeError(f"{BENCH_LIB_PATH} is missing: build it with `make -C bowtie2-server_amd`")
        L = C.CDLL(BENCH_LIB_PATH)
        vp, u32 = C.c_void_p, C.c_uint32
        L.bt2g_bench_collect_rows_dev.argtypes = [u32, vp, vp, vp, vp, u32, vp, vp, u32, u32, u32, vp, vp, vp, vp, vp,
                                                  u32, vp]
        L.bt2g_bench_frame_dev.argtypes = [u32, vp, vp, vp, vp, vp, vp, vp, vp, vp, u32, C.c_int32, vp, vp,
                                           u32, vp]
        _bench_lib = L
    return _bench_lib


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C bowtie2-server_amd` "
                               "(there is no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        vp, u32, i32, u64 = C.c_void_p, C.c_uint32, C.c_int32, C.c_uint64
        L.bt2g_last_error.restype = C.c_char_p
        L.bt2g_open.argtypes = [C.c_char_p, C.c_int, C.POINTER(vp)]
        L.bt2g_open_mem.argtypes = [C.POINTER(IndexMem), C.c_int, C.POINTER(vp)]
        L.bt2g_close.argtypes = [vp]
        L.bt2g_open_shared.argtypes = [vp, C.POINTER(vp)]
        L.bt2g_info.argtypes = [vp, vp, C.c_int]
        L.bt2g_exact_sweep.argtypes = [vp, vp, u32, vp, u32, u32, C.c_int, C.c_int, vp]
        L.bt2g_exact_sweep_dev.argtypes = [vp, vp, u32, vp, u32, u32, C.c_int, C.c_int, vp, vp]
        L.bt2g_seed_search.argtypes = [vp, vp, u32, vp, u32, u32, u32, u32, u32, vp, vp, vp, vp]
        L.bt2g_seed_search_ext.argtypes = [vp, vp, u32, vp, u32, u32, u32, u32, u32, vp, vp, vp, vp, vp, u32, vp]
        L.bt2g_seed_search_dev.argtypes = [vp, vp, u32, vp, u32, u32, u32, u32, u32, vp, vp, vp, vp, vp]
        L.bt2g_one_mm.argtypes = [vp, vp, vp, u32, vp, u32, vp, C.POINTER(Scoring), C.c_int, C.c_int, u32, vp, vp,
                                  vp, vp]
        L.bt2g_one_mm_dev.argtypes = [vp, vp, vp, u32, vp, u32, vp, C.POINTER(Scoring), C.c_int, C.c_int, u32, vp,
                                      vp, vp, vp, vp]
        L.bt2g_one_mm_gated_dev.argtypes = [vp, vp, vp, u32, vp, u32, vp, C.POINTER(Scoring), vp, u32, vp, vp, vp,
                                            vp, vp]
        L.bt2g_exact_sweep_1mm.argtypes = [vp, vp, vp, u32, vp, u32, u32, C.c_int, C.c_int, C.c_int, vp,
                                           C.POINTER(Scoring), u32, vp, vp, vp, vp, vp, u32, vp]
        L.bt2g_reserve_sw.argtypes = [vp, u32, u32]
        L.bt2g_get_offset.argtypes = [vp, vp, u32, vp, vp]
        L.bt2g_extend.argtypes = [vp, vp, u32, vp, u32, vp, u32, vp]
        L.bt2g_extend_dev.argtypes = [vp, vp, u32, vp, vp, u32, vp, vp]
        L.bt2g_sw_align_bt_packed.argtypes = [vp, vp, vp, u32, vp, vp, u32, vp, u64, vp, C.POINTER(Scoring), C.c_int,
                                              u32, vp, u32, u32, vp, vp, vp, vp, vp, vp]
        L.bt2g_get_offset_dev.argtypes = [vp, vp, u32, vp, vp, vp]
        L.bt2g_sw_align.argtypes = [vp, vp, vp, u32, vp, vp, u32, vp, u64, C.POINTER(Scoring), C.c_int, u32, vp, vp,
                                    vp, vp]
        L.bt2g_sw_align_dev.argtypes = [vp, vp, vp, u32, vp, vp, u32, vp, C.POINTER(Scoring), C.c_int, u32, vp, vp,
                                        vp, vp, vp]
        L.bt2g_sw_align_bt.argtypes = [vp, vp, vp, u32, vp, vp, u32, vp, u64, vp, C.POINTER(Scoring), C.c_int, u32,
                                       vp, vp, u32, u32, vp, vp, vp, vp]
        L.bt2g_sw_align_bt_dev.argtypes = [vp, vp, vp, u32, vp, vp, u32, vp, vp, C.POINTER(Scoring), C.c_int, u32,
                                           vp, vp, u32, u32, vp, vp, vp, vp, vp]
        L.bt2g_reserve_sw_bt.argtypes = [vp, u32, u32, u32, C.c_int]
        L.bt2g_ungapped.argtypes = [vp, vp, vp, u32, vp, vp, u32, C.POINTER(Scoring), C.c_int, u32, vp, vp]
        L.bt2g_ungapped_dev.argtypes = [vp, vp, vp, u32, vp, vp, u32, C.POINTER(Scoring), C.c_int, u32, vp, vp, vp]
        L.bt2g_frame.argtypes = [vp, vp, u32, vp, u32, C.POINTER(Scoring), C.POINTER(PePolicy), C.c_int32, C.c_int,
                                 vp, vp, vp]
        L.bt2g_frame_dev.argtypes = [vp, vp, u32, vp, C.POINTER(Scoring), C.POINTER(PePolicy), C.c_int32, C.c_int,
                                     vp, vp, vp, vp]
        L.bt2g_set_profiling.argtypes = [vp, C.c_int]
        L.bt2g_kernel_stats.argtypes = [vp, C.c_int, C.POINTER(u64), C.POINTER(C.c_double)]
        L.bt2g_reset_stats.argtypes = [vp]
        L.bt2g_comm_unique_id.argtypes = [vp]
        L.bt2g_comm_init.argtypes = [vp, C.c_int, C.c_int, vp]
        L.bt2g_allreduce_counts.argtypes = [vp, vp, u32]
        _lib = L
    return _lib


class Bt2gError(RuntimeError):
    def __init__(self, rc, msg):
        super().__init__(f"bt2g error {rc}: {msg}")
        self.rc = rc


def _chk(rc, allow=()):
    if rc != BT2G_OK and rc not in allow:
        raise Bt2gError(rc, lib().bt2g_last_error().decode(errors="replace"))
    return rc


def _ptr(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


class Engine:
    """An index resident in HBM of one GPU (bt2g_open / bt2g_open_mem)."""

    def __init__(self, index_base=None, device=0, index=None):
        self.h = C.c_void_p()
        if index is not None:
            self._keep = []
            m = IndexMem()
            for dst, e, fw in ((m.fw, index.fw, True), (m.bw, index.bw, False)):
                arrs = dict(fchr=_c(e.fchr, np.uint32), sides=_c(e.ebwt, np.uint8), ftab=_c(e.ftab, np.uint32),
                            eftab=_c(e.eftab, np.uint32), rstarts=_c(e.rstarts, np.uint32))
                if fw and e.offs is not None:
                    arrs["offs"] = _c(e.offs, np.uint32)
                self._keep.append(arrs)
                dst.len, dst.zoff, dst.ftab_chars = e.length, e.zoff, e.ftab_chars
                dst.off_rate, dst.line_rate = e.off_rate, e.line_rate
                dst.fchr, dst.sides = arrs["fchr"].ctypes.data, arrs["sides"].ctypes.data
                dst.sides_bytes = arrs["sides"].nbytes
                dst.ftab, dst.eftab = arrs["ftab"].ctypes.data, arrs["eftab"].ctypes.data
                if "offs" in arrs:
                    dst.offs, dst.offs_len = arrs["offs"].ctypes.data, len(arrs["offs"])
                dst.rstarts, dst.nfrag = arrs["rstarts"].ctypes.data, len(arrs["rstarts"]) // 3
            codes = np.concatenate(index.ref_codes).astype(np.uint8)
            starts = np.zeros(len(index.ref_codes) + 1, np.uint64)
            starts[1:] = np.cumsum([len(c) for c in index.ref_codes])
            self._keep.append((codes, starts))
            m.ref_codes, m.ref_starts, m.nref = codes.ctypes.data, starts.ctypes.data, len(index.ref_codes)
            _chk(lib().bt2g_open_mem(C.byref(m), device, C.byref(self.h)))
            self._keep = None
        else:
            _chk(lib().bt2g_open(index_base.encode(), device, C.byref(self.h)))

    def shared(self):
        """A second Engine on this one's index and device (bt2g_open_shared): its
        own stream and scratch, for another thread.  Close it before this one."""
        e = Engine.__new__(Engine)
        e.h = C.c_void_p()
        _chk(lib().bt2g_open_shared(self.h, C.byref(e.h)))
        return e

    # ---- multi-GPU: the ranks' one collective (RCCL) -----------------------
    @staticmethod
    def comm_unique_id():
        """A communicator id (bytes) for comm_init; made by one rank, sent to the others."""
        buf = (C.c_uint8 * 128)()
        _chk(lib().bt2g_comm_unique_id(C.cast(buf, C.c_void_p)))
        return bytes(buf)

    def comm_init(self, nranks, rank, uid):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        _chk(lib().bt2g_comm_init(self.h, nranks, rank, C.cast(buf, C.c_void_p)))

    def allreduce_counts(self, counts):
        """Sum of a u64 counter vector over the ranks of comm_init (collective)."""
        a = np.ascontiguousarray(np.asarray(counts, dtype=np.uint64)).copy()
        _chk(lib().bt2g_allreduce_counts(self.h, _ptr(a), len(a)))
        return a

    def close(self):
        if self.h:
            _chk(lib().bt2g_close(self.h))     # fails while shared() contexts are open
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def info(self):
        o = np.zeros(13, np.uint64)
        _chk(lib().bt2g_info(self.h, _ptr(o), 13))
        return o

    # ---- FM ----------------------------------------------------------------
    def exact_sweep(self, reads, lens, mine_max=2, nofw=False, norc=False):
        reads, lens = _c(reads, np.uint8), _c(lens, np.uint32)
        out = np.zeros((len(lens), 8), np.uint32)
        _chk(lib().bt2g_exact_sweep(self.h, _ptr(reads), reads.shape[1], _ptr(lens), len(lens), mine_max,
                                    int(nofw), int(norc), _ptr(out)))
        return out

    def seed_search(self, reads, lens, seedlen, interval, offset, maxseeds=64):
        reads, lens = _c(reads, np.uint8), _c(lens, np.uint32)
        n = len(lens)
        out = np.zeros((n, 2, maxseeds, 4), np.uint32)
        ns = np.zeros(n, np.int32)
        ops = np.zeros(n, np.uint32)
        loads = np.zeros(n, np.uint32)
        _chk(lib().bt2g_seed_search(self.h, _ptr(reads), reads.shape[1], _ptr(lens), n, seedlen, interval, offset,
                                    maxseeds, _ptr(out), _ptr(ns), _ptr(ops), _ptr(loads)))
        return out, ns, ops, loads

    def seed_search_ext(self, reads, lens, seedlen, interval, offset, maxseeds=64, off_cap=8):
        """bt2g_seed_search_ext: seed_search plus, per seed range, SwDriver::extend
        (ext n x 2 x maxseeds x 4) and the offsets of its rows when it has at most
        off_cap of them (offs n x 2 x maxseeds x off_cap)."""
        reads, lens = _c(reads, np.uint8), _c(lens, np.uint32)
        n = len(lens)
        out = np.zeros((n, 2, maxseeds, 4), np.uint32)
        ns = np.zeros(n, np.int32)
        ops = np.zeros(n, np.uint32)
        ext = np.zeros((n, 2, maxseeds, 4), np.uint32)
        offs = np.zeros((n, 2, maxseeds, max(off_cap, 1)), np.uint32)
        _chk(lib().bt2g_seed_search_ext(self.h, _ptr(reads), reads.shape[1], _ptr(lens), n, seedlen, interval, offset,
                                        maxseeds, _ptr(out), _ptr(ns), _ptr(ops), None, _ptr(ext), off_cap,
                                        _ptr(offs) if off_cap else None))
        return out, ns, ops, ext, offs

    def one_mm(self, reads, quals, lens, minsc, local, nofw=False, norc=False, cap=64):
        reads, quals, lens = _c(reads, np.uint8), _c(quals, np.uint8), _c(lens, np.uint32)
        ms = _c(minsc, np.int32)
        n = len(lens)
        hits = np.zeros((n, cap), MM1_DTYPE)
        cnt = np.zeros(n, np.int32)
        ops = np.zeros(n, np.uint32)
        loads = np.zeros(n, np.uint32)
        sc = scoring(local)
        rc = lib().bt2g_one_mm(self.h, _ptr(reads), _ptr(quals), reads.shape[1], _ptr(lens), n, _ptr(ms),
                               C.byref(sc), int(nofw), int(norc), cap, _ptr(hits), _ptr(cnt), _ptr(ops), _ptr(loads))
        _chk(rc)
        return hits, cnt, ops, loads

    def exact_sweep_1mm(self, reads, quals, lens, minsc, local, nofw=False, norc=False, skip_exact=False, cap=64,
                        off_cap=0):
        """bt2g_exact_sweep_1mm: the sweep and the sweep-gated 1-mm search in one call
        (off_cap > 0: also the offsets of the small ranges' rows, returned fifth)."""
        reads, quals, lens = _c(reads, np.uint8), _c(quals, np.uint8), _c(lens, np.uint32)
        ms = _c(minsc, np.int32)
        n = len(lens)
        sweep = np.zeros((n, 8), np.uint32)
        hits = np.zeros((n, cap), MM1_DTYPE)
        cnt = np.zeros(n, np.int32)
        ops = np.zeros(n, np.uint32)
        sc = scoring(local)
        offs = np.zeros((n, 2 + cap, off_cap), np.uint32) if off_cap else None
        self.last_mm_loads = np.zeros(n, np.uint32)
        _chk(lib().bt2g_exact_sweep_1mm(self.h, _ptr(reads), _ptr(quals), reads.shape[1], _ptr(lens), n, 2, int(nofw),
                                        int(norc), int(skip_exact), _ptr(ms), C.byref(sc), cap, _ptr(sweep),
                                        _ptr(hits), _ptr(cnt), _ptr(ops), _ptr(self.last_mm_loads), off_cap,
                                        _ptr(offs) if off_cap else None))
        return (sweep, hits, cnt, ops, offs) if off_cap else (sweep, hits, cnt, ops)

    def extend(self, reads, lens, ranges):
        """SwDriver::extend per seed-hit range; ranges n x 8 = (read, fw, off, len,
        topf, botf, topb, botb).  Returns n x 4 (nlex, nrex, LF steps, 64-B sides gathered)."""
        reads, lens = _c(reads, np.uint8), _c(lens, np.uint32)
        rg = _c(ranges, np.uint32)
        out = np.zeros((len(rg), 4), np.uint32)
        _chk(lib().bt2g_extend(self.h, _ptr(reads), reads.shape[1], _ptr(lens), len(lens), _ptr(rg), len(rg),
                               _ptr(out)))
        return out

    def get_offset(self, rows):
        rows = _c(rows, np.uint32)
        offs = np.zeros(len(rows), np.uint32)
        loads = np.zeros(len(rows), np.uint32)
        _chk(lib().bt2g_get_offset(self.h, _ptr(rows), len(rows), _ptr(offs), _ptr(loads)))
        return offs, loads

    # ---- SW ----------------------------------------------------------------
    def sw_align(self, reads, quals, lens, probs, windows=None, local=False, enable8=True, cap=4096,
                 want_mat=False, sc=None):
        reads, quals, lens = _c(reads, np.uint8), _c(quals, np.uint8), _c(lens, np.uint32)
        probs = _c(probs, SWPROB_DTYPE)
        n = len(probs)
        res = np.zeros(n, SWRES_DTYPE)
        cands = np.zeros((n, cap), SWCAND_DTYPE)
        win = _c(windows, np.uint8) if windows is not None else None
        mat = mat_off = None
        if want_mat:
            sizes = lens[probs["read"]].astype(np.uint64) * probs["ncol"].astype(np.uint64) * 3
            mat_off = np.zeros(n, np.uint64)
            mat_off[1:] = np.cumsum(sizes)[:-1]
            mat = np.zeros(int(sizes.sum()), np.int16)
        sc = scoring(local) if sc is None else sc
        _chk(lib().bt2g_sw_align(self.h, _ptr(reads), _ptr(quals), reads.shape[1], _ptr(lens), _ptr(probs), n,
                                 _ptr(win), 0 if win is None else win.nbytes, C.byref(sc), int(enable8), cap,
                                 _ptr(res), _ptr(cands), _ptr(mat), _ptr(mat_off)))
        return res, cands, (mat, mat_off)

    def sw_align_bt(self, reads, quals, lens, probs, windows=None, rects=None, local=False, enable8=True,
                    cap=4096, maxaln=64, maxedit=256, sc=None, want_fates=True):
        """Fill + the nextAlignment loop (bt2g_sw_align_bt).  Returns res, cands,
        naln (n), alns (n x maxaln SWALN_DTYPE), edits (n x maxaln x maxedit
        EDIT_DTYPE), fates (n x cap int8 or None)."""
        reads, quals, lens = _c(reads, np.uint8), _c(quals, np.uint8), _c(lens, np.uint32)
        probs = _c(probs, SWPROB_DTYPE)
        n = len(probs)
        res = np.zeros(n, SWRES_DTYPE)
        cands = np.zeros((n, cap), SWCAND_DTYPE)
        naln = np.zeros(n, np.int32)
        alns = np.zeros((n, maxaln), SWALN_DTYPE)
        edits = np.zeros((n, maxaln, maxedit), EDIT_DTYPE)
        fates = np.zeros((n, cap), np.int8) if want_fates else None
        win = _c(windows, np.uint8) if windows is not None else None
        rects = _c(rects, SWRECT_DTYPE) if rects is not None else None
        sc = scoring(local) if sc is None else sc
        _chk(lib().bt2g_sw_align_bt(self.h, _ptr(reads), _ptr(quals), reads.shape[1], _ptr(lens), _ptr(probs), n,
                                    _ptr(win), 0 if win is None else win.nbytes, _ptr(rects), C.byref(sc),
                                    int(enable8), cap, _ptr(res), _ptr(cands), maxaln, maxedit, _ptr(naln),
                                    _ptr(alns), _ptr(edits), _ptr(fates)))
        return res, cands, naln, alns, edits, fates

    def ungapped(self, reads, quals, lens, probs, local=False, ohang=False, maxedit=256, sc=None):
        """SwAligner::ungappedAlign per problem (bt2g_ungapped): res (UGRES_DTYPE),
        edits (n x maxedit EDIT_DTYPE)."""
        reads, quals, lens = _c(reads, np.uint8), _c(quals, np.uint8), _c(lens, np.uint32)
        probs = _c(probs, UGPROB_DTYPE)
        n = len(probs)
        res = np.zeros(n, UGRES_DTYPE)
        edits = np.zeros((n, maxedit), EDIT_DTYPE)
        sc = scoring(local) if sc is None else sc
        _chk(lib().bt2g_ungapped(self.h, _ptr(reads), _ptr(quals), reads.shape[1], _ptr(lens), _ptr(probs), n,
                                 C.byref(sc), int(ohang), maxedit, _ptr(res), _ptr(edits)))
        return res, edits

    def frame(self, inputs, lens, local=False, pe=None, maxhalf=15, trim_to_ref=True, sc=None):
        """DP rectangles (bt2g_frame): seed extensions (kind 0) and mate searches
        (kind 1).  Returns probs (SWPROB_DTYPE), rects (SWRECT_DTYPE), ok (int32)."""
        inputs, lens = _c(inputs, FRAMEIN_DTYPE), _c(lens, np.uint32)
        n = len(inputs)
        probs = np.zeros(n, SWPROB_DTYPE)
        rects = np.zeros(n, SWRECT_DTYPE)
        ok = np.zeros(n, np.int32)
        sc = scoring(local) if sc is None else sc
        _chk(lib().bt2g_frame(self.h, _ptr(inputs), n, _ptr(lens), len(lens), C.byref(sc),
                              None if pe is None else C.byref(pe), maxhalf, int(trim_to_ref), _ptr(probs),
                              _ptr(rects), _ptr(ok)))
        return probs, rects, ok

    # ---- measurement -------------------------------------------------------
    def reserve_sw(self, max_problems, max_cols):
        """Persistent fill scratch (bt2g_reserve_sw)."""
        _chk(lib().bt2g_reserve_sw(self.h, max_problems, max_cols))

    def reserve_sw_bt(self, max_problems, max_rows, max_cols, hbytes):
        """Persistent fill + backtrace scratch (bt2g_reserve_sw_bt)."""
        _chk(lib().bt2g_reserve_sw_bt(self.h, max_problems, max_rows, max_cols, hbytes))

    def set_profiling(self, on=True):
        _chk(lib().bt2g_set_profiling(self.h, int(on)))

    def kernel_stats(self, k):
        n, ms = C.c_uint64(0), C.c_double(0)
        _chk(lib().bt2g_kernel_stats(self.h, k, C.byref(n), C.byref(ms)))
        return n.value, ms.value

    def reset_stats(self):
        _chk(lib().bt2g_reset_stats(self.h))
