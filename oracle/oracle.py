"""ctypes binding for oracle/liboracle.so (the C restatement in oracle.c).

TEST INFRASTRUCTURE ONLY -- see oracle.c header.  Index arrays come from
bowtie2-server_amd/tools/bt2_index.py (read_ebwt)."""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


def build(force=False):
    src = os.path.join(HERE, "oracle.c")
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-o", LIB, src])
    return LIB


class OrcEbwt(C.Structure):
    _fields_ = [("ebwt", C.c_void_p), ("fchr", C.c_void_p), ("ftab", C.c_void_p), ("eftab", C.c_void_p),
                ("offs", C.c_void_p), ("len", C.c_uint32), ("zoff", C.c_uint32), ("ftab_chars", C.c_uint32),
                ("off_rate", C.c_uint32), ("fw", C.c_int)]


class OrcScoring(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("match", "mmp_max", "mmp_min", "npen", "rdg_const", "rdg_lin",
                                          "rfg_const", "rfg_lin", "gapbar", "local")] + \
               [("ncl_const", C.c_double), ("ncl_lin", C.c_double)]


def scoring(local=False):
    return OrcScoring(match=2 if local else 0, mmp_max=6, mmp_min=2, npen=1, rdg_const=5, rdg_lin=3,
                      rfg_const=5, rfg_lin=3, gapbar=4, local=1 if local else 0, ncl_const=0.0, ncl_lin=0.15)


def _p(a, t=C.c_void_p):
    return a.ctypes.data_as(C.POINTER(t)) if t is not C.c_void_p else C.c_void_p(a.ctypes.data)


class Oracle:
    def __init__(self):
        build()
        L = self.lib = C.CDLL(LIB)
        L.orc_exact_sweep.argtypes = [C.POINTER(OrcEbwt), C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32,
                                      C.c_uint32, C.c_void_p]
        L.orc_seed_search.argtypes = [C.POINTER(OrcEbwt), C.POINTER(OrcEbwt), C.c_void_p, C.c_uint32, C.c_void_p,
                                      C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                                      C.c_void_p, C.c_void_p]
        L.orc_one_mm.argtypes = [C.POINTER(OrcEbwt), C.POINTER(OrcEbwt), C.c_void_p, C.c_void_p, C.c_uint32,
                                 C.c_void_p, C.c_uint32, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                 C.POINTER(OrcScoring), C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_get_offset.restype = C.c_uint32
        L.orc_get_offset.argtypes = [C.POINTER(OrcEbwt), C.c_uint32]
        L.orc_bilf.argtypes = [C.POINTER(OrcEbwt), C.c_uint32, C.c_uint32, C.c_uint32] + [C.c_void_p] * 4
        L.orc_extend.argtypes = [C.POINTER(OrcEbwt), C.POINTER(OrcEbwt), C.c_void_p, C.c_uint32, C.c_int,
                                 C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
        L.orc_sw.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int64,
                             C.POINTER(OrcScoring), C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_ungapped.restype = C.c_int
        L.orc_ungapped.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int64, C.c_int64, C.c_int64,
                                   C.POINTER(OrcScoring), C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.orc_sw_bt.restype = C.c_int
        L.orc_sw_bt.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int64,
                                C.POINTER(OrcScoring), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]

    def ebwt(self, e, fw=True):
        """Wrap a bt2_index.Ebwt; keeps references alive on the returned struct."""
        s = OrcEbwt(ebwt=e.ebwt.ctypes.data, fchr=e.fchr.ctypes.data, ftab=e.ftab.ctypes.data,
                    eftab=e.eftab.ctypes.data, offs=e.offs.ctypes.data if e.offs is not None else None,
                    len=e.length, zoff=e.zoff, ftab_chars=e.ftab_chars, off_rate=e.off_rate, fw=1 if fw else 0)
        s._keep = e
        return s

    def exact_sweep(self, fe, reads, lens, mine_max=2):
        reads = np.ascontiguousarray(reads, np.uint8)
        lens = np.ascontiguousarray(lens, np.uint32)
        out = np.zeros((len(lens), 8), np.uint64)
        self.lib.orc_exact_sweep(C.byref(fe), _p(reads), reads.shape[1], _p(lens), len(lens), mine_max, _p(out))
        return out

    def seed_search(self, fe, be, reads, lens, seedlen, interval, offset, maxseeds=64):
        reads = np.ascontiguousarray(reads, np.uint8)
        lens = np.ascontiguousarray(lens, np.uint32)
        n = len(lens)
        out = np.zeros((n, 2, maxseeds, 4), np.uint32)
        ns = np.zeros(n, np.int32)
        bw = np.zeros(n, np.uint64)
        self.lib.orc_seed_search(C.byref(fe), C.byref(be), _p(reads), reads.shape[1], _p(lens), n, seedlen,
                                 interval, offset, maxseeds, _p(out), _p(ns), _p(bw))
        return out, ns, bw

    def one_mm(self, fe, be, reads, quals, lens, minsc, local, nofw=False, norc=False, cap=64):
        reads = np.ascontiguousarray(reads, np.uint8)
        quals = np.ascontiguousarray(quals, np.uint8)
        lens = np.ascontiguousarray(lens, np.uint32)
        ms = np.ascontiguousarray(minsc, np.int64)
        n = len(lens)
        out = np.zeros((n, cap, 7), np.int64)
        cnt = np.zeros(n, np.int32)
        bw = np.zeros(n, np.uint64)
        sc = scoring(local)
        self.lib.orc_one_mm(C.byref(fe), C.byref(be), _p(reads), _p(quals), reads.shape[1], _p(lens), n, _p(ms),
                            int(local), int(nofw), int(norc), C.byref(sc), cap, _p(out), _p(cnt), _p(bw))
        return out, cnt, bw

    def get_offset(self, fe, row):
        return self.lib.orc_get_offset(C.byref(fe), row)

    def extend(self, fe, be, seq, fw, off, ln, topf, botf, topb, botb):
        """SwDriver::extend of one seed-hit range -> (nlex, nrex, LF steps)."""
        seq = np.ascontiguousarray(seq, np.uint8)
        out = np.zeros(3, np.uint32)
        self.lib.orc_extend(C.byref(fe), C.byref(be) if be is not None else None, seq.ctypes.data, len(seq),
                            int(fw), off, ln, topf, botf, topb, botb, out.ctypes.data)
        return out

    def bilf(self, e, top, bot, topp):
        arrs = [np.zeros(4, np.uint32) for _ in range(4)]
        self.lib.orc_bilf(C.byref(e), top, bot, topp, *[_p(a) for a in arrs])
        return arrs

    def sw(self, rd, q33, rfmask, minsc, local, enable8=True, cap=4096, want_mat=False):
        rd = np.ascontiguousarray(rd, np.uint8)
        q33 = np.ascontiguousarray(q33, np.uint8)
        rf = np.ascontiguousarray(rfmask, np.uint8)
        ncol = len(rf) - 1
        out = np.zeros(8, np.int64)
        cands = np.zeros(3 * cap, np.int64)
        mat = np.zeros(3 * len(rd) * ncol, np.int32) if want_mat else None
        sc = scoring(local)
        self.lib.orc_sw(_p(rd), _p(q33), len(rd), _p(rf), ncol, int(minsc), C.byref(sc), 1 if enable8 else 0, cap,
                        _p(out), _p(cands), _p(mat) if want_mat else None)
        nc = int(out[6])
        return out, cands[: 3 * min(nc, cap)].reshape(-1, 3), (mat.reshape(len(rd), ncol, 3) if want_mat else None)

    def sw_bt(self, rd, q33, rfmask, minsc, local, fw=True, triml=0, corel=0, corer=0, enable8=True,
              maxaln=64, maxedit=256, sc=None):
        """SwAligner::align + the nextAlignment loop; rd/q33 already oriented (rc
        when not fw).  Returns (out[7], alns k x 10, [edits k_i x 4], fates) as
        oracle.ref_harness.RefLib.sw_bt."""
        rd = np.ascontiguousarray(rd, np.uint8)
        q33 = np.ascontiguousarray(q33, np.uint8)
        rf = np.ascontiguousarray(rfmask, np.uint8)
        ncol = len(rf) - 1
        out = np.zeros(8, np.int64)
        aln = np.zeros(10 * maxaln, np.int64)
        edits = np.zeros(4 * maxaln * maxedit, np.int32)
        fates = np.zeros(8192, np.int32)
        sc = sc if sc is not None else scoring(local)
        na = self.lib.orc_sw_bt(_p(rd), _p(q33), len(rd), _p(rf), ncol, int(minsc), C.byref(sc),
                                1 if enable8 else 0, 1 if fw else 0, triml, corel, corer, maxaln, maxedit,
                                _p(out), _p(aln), _p(edits), _p(fates), len(fates))
        k = min(na, maxaln)
        aln = aln[:10 * k].reshape(k, 10)
        ed = edits.reshape(maxaln, maxedit, 4)
        eds = [ed[i, :min(int(aln[i, 7]), maxedit)].copy() for i in range(k)]
        return out[:7], aln, eds, fates[:min(int(out[6]), len(fates))].copy()

    def ungapped(self, rd, q33, rf, rfi, reflen, minsc, local, fw=True, ohang=False, sc=None):
        """SwAligner::ungappedAlign: rd/q33 as aligned, rf = reference codes at
        rfi..rfi+len-1 (4 off the reference).  Returns (out[10], edits k x 4)."""
        rd = np.ascontiguousarray(rd, np.uint8)
        q33 = np.ascontiguousarray(q33, np.uint8)
        rf = np.ascontiguousarray(rf, np.uint8)
        out = np.zeros(10, np.int64)
        ed = np.zeros(4 * (len(rd) + 1), np.int32)
        sc = sc if sc is not None else scoring(local)
        self.lib.orc_ungapped(_p(rd), _p(q33), len(rd), _p(rf), int(rfi), int(reflen), int(minsc), C.byref(sc),
                              1 if ohang else 0, 1 if fw else 0, _p(out), _p(ed))
        return out, ed[:4 * int(out[5])].reshape(-1, 4)

    def frame(self, kind, off, rdlen, reflen, minsc, fw=True, anchor1=True, alen=0, local=False, pe=None,
              maxhalf=15, trim_to_ref=True, sc=None):
        """DP rectangle of one seed extension (kind 0) or mate search (kind 1).
        pe = (policy, minfrag, maxfrag, flip, dovetail, olap, expand).  Returns
        (ok, fw, refl, ncol, triml, corel, corer)."""
        out = np.zeros(7, np.int64)
        pev = np.array(pe if pe is not None else (3, 0, 500, 0, 0, 1, 1), np.int32)
        sc = sc if sc is not None else scoring(local)
        self.lib.orc_frame(int(kind), C.c_int64(int(off)), C.c_uint64(int(rdlen)), C.c_int64(int(reflen)),
                           C.c_int64(int(minsc)), int(bool(fw)), int(bool(anchor1)), C.c_uint64(int(alen)),
                           C.byref(sc), _p(pev), C.c_int64(int(maxhalf)), int(bool(trim_to_ref)), _p(out))
        return tuple(int(x) for x in out)

