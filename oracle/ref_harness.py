"""ctypes binding for oracle/_ref/libbt2ref.so (the REFERENCE built from
/root/reference by oracle/ref/Makefile).  TEST INFRASTRUCTURE ONLY: used by
tests/golden/make_golden.py to produce golden vectors and by bench.py's
cpu_baseline leg ("kind": "reference").  Never imported by the product."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_ref", "libbt2ref.so")


class ScoreParams(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("match", "mmp_max", "mmp_min", "npen", "rdg_const", "rdg_lin",
                                          "rfg_const", "rfg_lin", "gapbar", "local")] + \
               [("ncl_const", C.c_double), ("ncl_lin", C.c_double)]


def score_params(local=False, **kw):
    d = dict(match=2 if local else 0, mmp_max=6, mmp_min=2, npen=1, rdg_const=5, rdg_lin=3,
             rfg_const=5, rfg_lin=3, gapbar=4, local=1 if local else 0, ncl_const=0.0, ncl_lin=0.15)
    d.update(kw)
    return ScoreParams(**d)


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


class RefLib:
    def __init__(self, path=LIB):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle/ref`")
        self.lib = L = C.CDLL(path)
        L.bt2ref_open.restype = C.c_void_p
        L.bt2ref_open.argtypes = [C.c_char_p]
        L.bt2ref_close.argtypes = [C.c_void_p]
        L.bt2ref_info.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.bt2ref_contains.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_uint32)]
        L.bt2ref_bilf.argtypes = [C.c_void_p, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32] + [C.POINTER(C.c_uint32)] * 4
        L.bt2ref_ftab_lohi.restype = C.c_uint32
        L.bt2ref_ftab_lohi.argtypes = [C.c_void_p, C.c_int, C.c_uint32, C.POINTER(C.c_uint32)]
        L.bt2ref_get_offset.restype = C.c_uint32
        L.bt2ref_get_offset.argtypes = [C.c_void_p, C.c_uint32]
        L.bt2ref_get_stretch.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint8)]
        L.bt2ref_exact_sweep.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                         C.c_int, C.POINTER(C.c_uint64)]
        L.bt2ref_one_mm.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                    C.POINTER(C.c_int64), C.c_int, C.c_int, C.c_int, C.c_int,
                                    C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.POINTER(C.c_uint64)]
        L.bt2ref_seed_search.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                         C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint32),
                                         C.POINTER(C.c_int32), C.POINTER(C.c_uint64)]
        L.bt2ref_sw.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.POINTER(C.c_uint8), C.c_int, C.c_int64,
                                C.POINTER(ScoreParams), C.c_int, C.c_int, C.POINTER(C.c_int64),
                                C.POINTER(C.c_int64), C.POINTER(C.c_int32)]

    def frame(self, inputs, local, pe=(3, 0, 500, 0, 0, 1, 1), maxhalf=15, trim_to_ref=True, sp=None):
        """DynProgFramer / PairedEndPolicy::otherMate as SwDriver calls them
        (bt2ref_frame).  inputs: n x 8 int64 {kind, off, rdlen, reflen, minsc,
        fw, anchor1, alen}.  Returns n x 7 {ok, fw, refl, ncol, triml, corel, corer}."""
        x = np.ascontiguousarray(inputs, np.int64)
        n = len(x)
        out = np.zeros((n, 7), np.int64)
        pev = np.ascontiguousarray(pe, np.int32)
        sp = sp if sp is not None else score_params(local)
        self.lib.bt2ref_frame(C.c_int(n), _p(x, C.c_int64), C.byref(sp), _p(pev, C.c_int32), C.c_int(maxhalf),
                              C.c_int(int(trim_to_ref)), _p(out, C.c_int64))
        return out

    def sw_bt(self, seq, qual, fw, rfmask, minsc, local, triml=0, corel=0, corer=0, enable8=True,
              maxaln=64, maxedit=256, sp=None):
        """SwAligner::align + the SwDriver nextAlignment loop.  Returns (out[7],
        alns (k x 10: cand, score, off, refoff, ns, gaps, refns, nedit, trim5, trim3),
        edits (list of k arrays (nedit x 4: pos, type, chr, qchr)), fates)."""
        L = self.lib
        if not hasattr(self, "_bt_init"):
            L.bt2ref_sw_bt.restype = C.c_int
            L.bt2ref_sw_bt.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.POINTER(C.c_uint8), C.c_int, C.c_int64,
                                       C.POINTER(ScoreParams), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                       C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_int]
            self._bt_init = True
        rf = np.ascontiguousarray(rfmask, np.uint8)
        ncol = len(rf) - 1
        out = np.zeros(8, np.int64)
        aln = np.zeros(10 * maxaln, np.int64)
        edits = np.zeros(4 * maxaln * maxedit, np.int32)
        fates = np.zeros(8192, np.int32)
        sp = sp if sp is not None else score_params(local)
        na = L.bt2ref_sw_bt(seq, qual, 1 if fw else 0, _p(rf, C.c_uint8), ncol, int(minsc), C.byref(sp),
                            1 if enable8 else 0, triml, corel, corer, maxaln, maxedit, _p(out, C.c_int64),
                            _p(aln, C.c_int64), _p(edits, C.c_int32), _p(fates, C.c_int32), len(fates))
        k = min(na, maxaln)
        aln = aln[:10 * k].reshape(k, 10)
        ed = edits.reshape(maxaln, maxedit, 4)
        eds = [ed[i, :min(int(aln[i, 7]), maxedit)].copy() for i in range(k)]
        nc = int(out[6])
        return out[:7], aln, eds, fates[:min(nc, len(fates))].copy()

    def open(self, base):
        return RefIndex(self, base)

    def sw(self, seq, qual, fw, rfmask, minsc, local, enable8=True, cap=4096, want_mat=False):
        rf = np.ascontiguousarray(rfmask, np.uint8)
        ncol = len(rf) - 1
        out = np.zeros(8, np.int64)
        cands = np.zeros(3 * cap, np.int64)
        mat = np.zeros(3 * len(seq) * ncol, np.int32) if want_mat else None
        sp = score_params(local)
        self.lib.bt2ref_sw(seq, qual, 1 if fw else 0, _p(rf, C.c_uint8), ncol, int(minsc), C.byref(sp),
                           1 if enable8 else 0, cap, _p(out, C.c_int64), _p(cands, C.c_int64),
                           _p(mat, C.c_int32) if want_mat else None)
        nc = int(out[6])
        return out, cands[: 3 * min(nc, cap)].reshape(-1, 3), (mat.reshape(len(seq), ncol, 3) if want_mat else None)


def _cstrs(lst):
    arr = (C.c_char_p * len(lst))()
    arr[:] = lst
    return arr


class RefIndex:
    def __init__(self, lib, base):
        self.L = lib.lib
        self.h = self.L.bt2ref_open(base.encode())

    def close(self):
        if self.h:
            self.L.bt2ref_close(self.h)
            self.h = None

    def info(self):
        o = np.zeros(13, np.uint64)
        self.L.bt2ref_info(self.h, _p(o, C.c_uint64))
        return o

    def contains(self, seq):
        o = np.zeros(4, np.uint32)
        ok = self.L.bt2ref_contains(self.h, seq, _p(o, C.c_uint32))
        return ok, o

    def bilf(self, which, top, bot, topp):
        arrs = [np.zeros(4, np.uint32) for _ in range(4)]
        self.L.bt2ref_bilf(self.h, which, top, bot, topp, *[_p(a, C.c_uint32) for a in arrs])
        return arrs

    def ftab_lohi(self, which, i):
        b = C.c_uint32(0)
        t = self.L.bt2ref_ftab_lohi(self.h, which, i, C.byref(b))
        return t, b.value

    def get_offset(self, row):
        return self.L.bt2ref_get_offset(self.h, row)

    def stretch(self, refidx, off, n):
        d = np.zeros(n, np.uint8)
        self.L.bt2ref_get_stretch(self.h, refidx, off, n, _p(d, C.c_uint8))
        return d

    def exact_sweep(self, seqs, quals, mine_max=2):
        out = np.zeros(8 * len(seqs), np.uint64)
        self.L.bt2ref_exact_sweep(self.h, len(seqs), _cstrs(seqs), _cstrs(quals), mine_max, _p(out, C.c_uint64))
        return out.reshape(-1, 8)

    def one_mm(self, seqs, quals, minsc, local, nofw=False, norc=False, cap=64):
        n = len(seqs)
        out = np.zeros(n * cap * 6, np.int64)
        counts = np.zeros(n, np.int32)
        bw = np.zeros(n, np.uint64)
        ms = np.ascontiguousarray(minsc, np.int64)
        self.L.bt2ref_one_mm(self.h, n, _cstrs(seqs), _cstrs(quals), _p(ms, C.c_int64), int(local), int(nofw),
                             int(norc), cap, _p(out, C.c_int64), _p(counts, C.c_int32), _p(bw, C.c_uint64))
        return out.reshape(n, cap, 6), counts, bw

    def ungapped(self, seqs, quals, fws, refidx, offs, minsc, local, ohang=False, maxedit=256):
        """SwAligner::ungappedAlign per read.  Returns (out n x 10, edits list)."""
        L = self.L
        L.bt2ref_ungapped.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(ScoreParams),
                                      C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        n = len(seqs)
        fws = np.ascontiguousarray(fws, np.uint8)
        refidx = np.ascontiguousarray(refidx, np.uint32)
        offs = np.ascontiguousarray(offs, np.int64)
        minsc = np.ascontiguousarray(minsc, np.int64)
        out = np.zeros((n, 10), np.int64)
        ed = np.zeros((n, maxedit, 4), np.int32)
        sp = score_params(local)
        L.bt2ref_ungapped(self.h, n, _cstrs(seqs), _cstrs(quals), fws.ctypes.data, refidx.ctypes.data,
                          offs.ctypes.data, minsc.ctypes.data, C.byref(sp), 1 if ohang else 0, maxedit,
                          out.ctypes.data, ed.ctypes.data)
        return out, [ed[i, :int(out[i, 5])].copy() for i in range(n)]

    def extend(self, seqs, quals, fw, off, ln, tb):
        """SwDriver::extend per range (seqs[i] the read of range i): tb n x 4 =
        (topf, botf, topb, botb).  Returns n x 3 (nlex, nrex, nSdFmops)."""
        L = self.L
        L.bt2ref_extend.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p)] + [C.c_void_p] * 5
        n = len(seqs)
        fw = np.ascontiguousarray(fw, np.int32)
        off = np.ascontiguousarray(off, np.uint32)
        ln = np.ascontiguousarray(ln, np.uint32)
        tb = np.ascontiguousarray(tb, np.uint32)
        out = np.zeros((n, 3), np.uint32)
        L.bt2ref_extend(self.h, n, _cstrs(seqs), _cstrs(quals), fw.ctypes.data, off.ctypes.data, ln.ctypes.data,
                        tb.ctypes.data, out.ctypes.data)
        return out

    def seed_search(self, seqs, quals, seedlen, interval, offset, maxseeds=64):
        n = len(seqs)
        out = np.zeros(n * 2 * maxseeds * 4, np.uint32)
        ns = np.zeros(n, np.int32)
        bw = np.zeros(n, np.uint64)
        self.L.bt2ref_seed_search(self.h, n, _cstrs(seqs), _cstrs(quals), seedlen, interval, offset, maxseeds,
                                  _p(out, C.c_uint32), _p(ns, C.c_int32), _p(bw, C.c_uint64))
        return out.reshape(n, 2, maxseeds, 4), ns, bw
