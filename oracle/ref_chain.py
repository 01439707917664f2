"""oracle/ref_chain.py -- TEST INFRASTRUCTURE ONLY (never part of the product).

The reference's own code (oracle/_ref/libbt2ref.so, built from /root/reference
by oracle/ref/Makefile) run over bench.py's whole per-step chain,
independently of every GPU intermediate: for each read

  SeedAligner::exactSweep                       aligner_seed.cpp:854-968
  SeedAligner::oneMmSearch, gated as bt2_search.cpp:3640-3667 (hits kept)
  instantiateSeeds + searchAllSeeds, round 0     aligner_seed.cpp:498-718
  -> the bench's hit rows (same order as bench_frame.hip k_collect_rows)
  Ebwt::getOffset                               bt2_idx.cpp:150-171
  Ebwt::joinedToTextOff (straddlers rejected)   bt2_idx.cpp:54
  -> the bench's two smallest diagonals per read (k_frame's policy)
  DynProgFramer::frameSeedExtensionRect         dp_framer.cpp:81-129
  SwAligner::align + the nextAlignment loop     aligner_sw.cpp:500-1146

`run()` times only the reference calls (split over host threads); the numpy
glue between them restates the bench's own policy and is not timed.  bench.py
compares every stage with the GPU's buffers (`compare()`).
"""
import concurrent.futures as cf
import ctypes as C
import time

import numpy as np

from oracle.ref_harness import RefLib, score_params

U32 = 0xFFFFFFFF


def _cs(lst):
    return (C.c_char_p * len(lst))(*lst)


def _split(total, threads):
    b = np.linspace(0, total, threads + 1).astype(int)
    return [(int(b[i]), int(b[i + 1])) for i in range(threads) if b[i + 1] > b[i]]


class RefChain:
    def __init__(self, base):
        self.lib = RefLib()
        L = self.L = self.lib.lib
        vp = C.c_void_p
        L.bt2ref_one_mm_gated_hits.argtypes = [vp, C.c_int, vp, vp, vp, vp, vp, C.c_int, C.c_int, vp]
        L.bt2ref_get_offsets.argtypes = [vp, C.c_int, vp, vp]
        L.bt2ref_joined_to_text_off.argtypes = [vp, C.c_int, vp, vp, C.c_int, vp]
        L.bt2ref_frame.argtypes = [C.c_int, vp, vp, vp, C.c_int, C.c_int, vp]
        L.bt2ref_sw_bt_batch_rects.argtypes = [C.c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        self.R = self.lib.open(base)
        self.secs = {}

    def close(self):
        self.R.close()

    def _timed(self, name, threads, total, fn):
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(threads) as ex:
            parts = list(ex.map(lambda a: fn(*a), _split(total, threads)))
        self.secs[name] = self.secs.get(name, 0.0) + time.perf_counter() - t0
        return parts

    def run(self, seqs, quals, lens, pol, maxseeds, mm_cap, maxhalf, gen_codes, threads):
        """seqs/quals: lists of ASCII bytes (the sampled reads).  Returns a dict of
        every stage's outputs (numpy)."""
        L, R = self.L, self.R
        n = len(seqs)
        minsc = np.full(n, pol.minsc, np.int64)

        # -- exact sweep, gated 1-mm search (with hits), exact seeds of the reads without an exact hit
        def seed_phase(lo, hi):
            s, q = seqs[lo:hi], quals[lo:hi]
            ex = R.exact_sweep(s, q, 2)
            cnt = np.zeros(hi - lo, np.int32)
            hits = np.zeros((hi - lo) * mm_cap * 6, np.int64)
            exu = np.ascontiguousarray(ex, np.uint64)
            L.bt2ref_one_mm_gated_hits(R.h, hi - lo, _cs(s), _cs(q), minsc[lo:hi].ctypes.data, exu.ctypes.data,
                                       cnt.ctypes.data, int(pol.local), mm_cap, hits.ctypes.data)
            need = np.nonzero(np.minimum(ex[:, 0], ex[:, 1]) != 0)[0]
            sd = np.zeros((hi - lo, 2, maxseeds, 4), np.uint32)
            ns = np.zeros(hi - lo, np.int32)
            if len(need):
                o, nsd, _ = R.seed_search([s[i] for i in need], [q[i] for i in need], pol.seedlen, pol.interval, 0,
                                          maxseeds)
                sd[need], ns[need] = o, nsd
            return ex, cnt, hits.reshape(hi - lo, mm_cap, 6), sd, ns

        parts = self._timed("seed_phase", threads, n, seed_phase)
        ex = np.concatenate([p[0] for p in parts])
        mm_cnt = np.concatenate([p[1] for p in parts])
        mm_hits = np.concatenate([p[2] for p in parts])
        seeds = np.concatenate([p[3] for p in parts])
        nseeds = np.concatenate([p[4] for p in parts])

        # -- hit rows in k_collect_rows's order: exact, 1-mm hits, seeds (strand-major)
        exact = np.minimum(ex[:, 0], ex[:, 1]) == 0
        r_read, r_ord, r_row, r_fw, r_dep, r_hl = [], [], [], [], [], []
        ei = np.nonzero(exact)[0]
        efw = ex[ei, 4] > ex[ei, 3]
        r_read.append(ei); r_ord.append(np.zeros(len(ei), np.int64))
        r_row.append(np.where(efw, ex[ei, 3], ex[ei, 5]).astype(np.int64)); r_fw.append(efw)
        r_dep.append(np.zeros(len(ei), np.int64)); r_hl.append(lens[ei].astype(np.int64))
        nm = np.clip(mm_cnt, 0, mm_cap)
        mi, mk = np.nonzero(np.arange(mm_cap)[None, :] < nm[:, None])
        r_read.append(mi); r_ord.append(1 + mk)
        r_row.append(mm_hits[mi, mk, 0]); r_fw.append(mm_hits[mi, mk, 2] != 0)
        r_dep.append(np.zeros(len(mi), np.int64)); r_hl.append(lens[mi].astype(np.int64))
        si, sf, ss = np.nonzero(seeds[:, :, :, 1] > seeds[:, :, :, 0])
        r_read.append(si); r_ord.append(1 + mm_cap + sf * maxseeds + ss)
        r_row.append(seeds[si, sf, ss, 0].astype(np.int64)); r_fw.append(sf == 0)
        r_dep.append(ss.astype(np.int64) * pol.interval); r_hl.append(np.full(len(si), pol.seedlen, np.int64))
        cat = [np.concatenate(x) for x in (r_read, r_ord, r_row, r_fw, r_dep, r_hl)]
        o = np.lexsort((cat[1], cat[0]))
        rows = {k: v[o] for k, v in zip(("read", "ord", "row", "fw", "dep", "hitlen"), cat)}

        # -- SA rows -> joined offsets -> (reference, offset)
        rr = np.ascontiguousarray(rows["row"].astype(np.uint32))
        offs = np.zeros(len(rr), np.uint32)

        def get_offsets(lo, hi):
            L.bt2ref_get_offsets(R.h, hi - lo, rr[lo:hi].ctypes.data, offs[lo:hi].ctypes.data)

        self._timed("get_offset", threads, len(rr), get_offsets)
        hl = np.ascontiguousarray(rows["hitlen"].astype(np.uint32))
        jt = np.zeros((len(rr), 3), np.int64)

        def joined(lo, hi):
            out = np.zeros((hi - lo, 3), np.int64)
            L.bt2ref_joined_to_text_off(R.h, hi - lo, offs[lo:hi].ctypes.data, hl[lo:hi].ctypes.data, 1,
                                        out.ctypes.data)
            jt[lo:hi] = out

        self._timed("joined_to_text_off", threads, len(rr), joined)

        # -- two smallest distinct (strand, reference, start) per read (k_frame's policy)
        ok = jt[:, 0] >= 0
        rd, fw, tid, toff = rows["read"][ok], rows["fw"][ok], jt[ok, 0], jt[ok, 1]
        dep, hitl = rows["dep"][ok], rows["hitlen"][ok]
        start = np.where(fw, toff - dep, toff - (lens[rd].astype(np.int64) - dep - hitl))
        key = (fw.astype(np.uint64) << np.uint64(62)) | (tid.astype(np.uint64) << np.uint64(40)) | \
              (start + (1 << 39)).astype(np.uint64)
        o = np.lexsort((key, rd))
        rd, key = rd[o], key[o]
        first = np.ones(len(rd), bool)
        first[1:] = (rd[1:] != rd[:-1]) | (key[1:] != key[:-1])
        rd, key = rd[first], key[first]
        rank = np.arange(len(rd)) - np.searchsorted(rd, rd, side="left")
        sel = rank < 2
        rd, key = rd[sel], key[sel]
        p_fw = (key >> np.uint64(62)).astype(np.int64)
        p_tid = ((key >> np.uint64(40)) & np.uint64(0x3FFFFF)).astype(np.int64)
        p_start = (key & np.uint64((1 << 40) - 1)).astype(np.int64) - (1 << 39)

        # -- DynProgFramer::frameSeedExtensionRect
        tlen = np.array([len(gen_codes[t]) for t in range(len(gen_codes))], np.int64)
        fx = np.zeros((len(rd), 8), np.int64)
        fx[:, 0] = 0
        fx[:, 1] = p_start
        fx[:, 2] = lens[rd]
        fx[:, 3] = tlen[p_tid]
        fx[:, 4] = pol.minsc
        fx[:, 5] = p_fw
        fr = np.zeros((len(rd), 7), np.int64)
        sp = score_params(pol.local)
        pev = np.array([3, 0, 500, 0, 0, 1, 1], np.int32)

        def frame(lo, hi):
            out = np.zeros((hi - lo, 7), np.int64)
            x = np.ascontiguousarray(fx[lo:hi])
            L.bt2ref_frame(hi - lo, x.ctypes.data, C.byref(sp), pev.ctypes.data, maxhalf, 1, out.ctypes.data)
            fr[lo:hi] = out

        self._timed("frame", threads, len(rd), frame)
        keep = fr[:, 0] == 1
        probs = dict(read=rd[keep], fw=fr[keep, 1], refl=fr[keep, 2], ncol=fr[keep, 3], refidx=p_tid[keep],
                     triml=fr[keep, 4], corel=fr[keep, 5], corer=fr[keep, 6])

        # -- SwAligner::align + nextAlignment loop on the reference's own rectangles
        npb = len(probs["read"])
        rf_off = np.zeros(npb + 1, np.int64)
        rf_off[1:] = np.cumsum(probs["ncol"] + 1)
        # reference masks of each window (N = 16 off the reference ends), gathered at once
        starts = np.zeros(len(gen_codes) + 1, np.int64)
        starts[1:] = np.cumsum([len(g) for g in gen_codes])
        gall = np.concatenate(gen_codes)
        w = probs["ncol"] + 1
        pos = np.repeat(probs["refl"], w) + (np.arange(int(rf_off[-1])) - np.repeat(rf_off[:-1], w))
        rlen = np.repeat(tlen[probs["refidx"]], w)
        inside = (pos >= 0) & (pos < rlen)
        gpos = np.repeat(starts[probs["refidx"]], w) + np.clip(pos, 0, None)
        cc = np.where(inside, gall[np.minimum(gpos, len(gall) - 1)], 4)
        rf = np.ascontiguousarray((1 << cc.astype(np.int64)).astype(np.uint8))
        rects = np.ascontiguousarray(np.stack([probs["triml"], probs["corel"], probs["corer"],
                                               np.zeros(npb, np.int64)], 1).astype(np.int32))
        sw = np.zeros((npb, 8), np.int64)
        fwv = np.ascontiguousarray(probs["fw"].astype(np.uint8))
        ncv = np.ascontiguousarray(probs["ncol"].astype(np.int32))
        msv = np.full(npb, pol.minsc, np.int64)

        def dps(lo, hi):
            k = hi - lo
            out = np.zeros((k, 8), np.int64)
            L.bt2ref_sw_bt_batch_rects(k, _cs([seqs[r] for r in probs["read"][lo:hi]]),
                                       _cs([quals[r] for r in probs["read"][lo:hi]]), fwv[lo:].ctypes.data,
                                       rf.ctypes.data, np.ascontiguousarray(rf_off[lo:hi + 1]).ctypes.data,
                                       ncv[lo:].ctypes.data, msv[lo:].ctypes.data, C.byref(sp),
                                       rects[lo:].ctypes.data, out.ctypes.data)
            sw[lo:hi] = out

        self._timed("sw", threads, npb, dps)
        return dict(ex=ex, mm_cnt=mm_cnt, mm_hits=mm_hits, seeds=seeds, nseeds=nseeds, rows=rows, offs=offs, jt=jt,
                    probs=probs, sw=sw)


def compare(ref, gpu):
    """Stage-by-stage mismatch counts between the reference chain (RefChain.run)
    and the GPU's buffers of the same reads (numpy, already restricted to the
    sample: see bench.py)."""
    out = {}
    ex, gs = ref["ex"], gpu["sweep"].astype(np.int64) & U32
    out["exact_sweep_mismatch"] = int((gs[:, [0, 1, 2, 3, 4, 5]] != ex[:, [0, 1, 3, 4, 5, 6]].astype(np.int64))
                                      .any(1).sum())
    # 1-mm hits in discovery order: {top, bot, fw, score, pos, chr, qchr}
    cap = ref["mm_hits"].shape[1]
    gc, rc = gpu["mm_cnt"], ref["mm_cnt"]
    bad = gc != rc
    h = ref["mm_hits"]
    lut = np.full(256, 4, np.int64)                           # ASCII edit characters -> codes
    lut[[65, 67, 71, 84]] = [0, 1, 2, 3]
    rchr, rq = lut[h[:, :, 5] & 0xFF], lut[(h[:, :, 5] >> 8) & 0xFF]
    gh = gpu["mm_hits"].astype(np.int64)
    # a read with more hits than the slots: the count must agree, the stored subset is unspecified
    live = (np.arange(cap)[None, :] < np.minimum(rc, cap)[:, None]) & (rc <= cap)[:, None]
    diff = (gh[:, :, 0] & U32) != h[:, :, 0]
    diff |= (gh[:, :, 1] & U32) != h[:, :, 1]
    diff |= gh[:, :, 2] != h[:, :, 2]
    diff |= gh[:, :, 3] != h[:, :, 3]
    diff |= gh[:, :, 4] != h[:, :, 4]
    diff |= gh[:, :, 5] != rchr
    diff |= gh[:, :, 6] != rq
    bad |= (diff & live).any(1)
    out["one_mm_mismatch"] = int(bad.sum())
    out["one_mm_hits"] = int(rc.sum())
    # exact seeds (reads searched on either side)
    gsd = gpu["seeds"].astype(np.int64) & U32
    out["seed_mismatch"] = int((gsd != ref["seeds"].astype(np.int64)).any((1, 2, 3)).sum())
    out["seed_hits"] = int((ref["seeds"][:, :, :, 1] > ref["seeds"][:, :, :, 0]).sum())
    # hit rows, their offsets
    rr = ref["rows"]
    g_rows, g_offs, g_read = gpu["rows"], gpu["offs"], gpu["row_read"]
    same = len(g_rows) == len(rr["row"])
    if same:
        o = np.lexsort((np.arange(len(g_read)), g_read))      # GPU rows are contiguous per read, reads in any order
        same_rows = (g_rows[o].astype(np.int64) & U32) == (rr["row"] & U32)
        out["row_mismatch"] = int((~same_rows).sum())
        out["offset_mismatch"] = int(((g_offs[o].astype(np.int64) & U32) != ref["offs"].astype(np.int64)).sum())
    else:
        out["row_mismatch"] = abs(len(g_rows) - len(rr["row"])) or -1
        out["offset_mismatch"] = -1
    out["rows"] = int(len(rr["row"]))
    # DP rectangles: same set per read
    rp = ref["probs"]
    gp = gpu["probs"]
    rk = np.stack([rp["read"], rp["fw"], rp["refidx"], rp["refl"], rp["ncol"], rp["triml"], rp["corel"],
                   rp["corer"]], 1).astype(np.int64)
    gk = np.stack([gp["read"], gp["fw"], gp["refidx"], gp["refl"], gp["ncol"], gp["triml"], gp["corel"],
                   gp["corer"]], 1).astype(np.int64)
    rk_s = rk[np.lexsort(rk.T[::-1])]
    gk_s = gk[np.lexsort(gk.T[::-1])]
    if len(rk_s) == len(gk_s):
        out["frame_mismatch"] = int((rk_s != gk_s).any(1).sum())
    else:
        out["frame_mismatch"] = abs(len(rk_s) - len(gk_s))
    out["dps"] = int(len(rk_s))
    return out
