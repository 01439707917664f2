"""Bowtie 2 index (.bt2) builder / reader used by the tests and bench.py.

This is NOT the hot path: the product loads finished .bt2 files through the
C-ABI (``bt2g_open``, csrc/bt2_index.cpp).  It exists because hg38 cannot be
fetched here, so tests and the bench synthesise genomes and need byte-exact
bowtie2 indexes for them.  Output is byte-identical to the reference's
``bowtie2-build`` (checked in tests/test_index_build.py against SHA-256 fixtures
of indexes built by the reference here, see tests/golden/make_golden.py).

Format followed (reference file:line):
  * header / array order .......... bt2_io.cpp:134-174, 241-312, 388-464, 513-595
  * EbwtParams geometry ........... bt2_idx.h:133-167
  * side layout, occ, fchr, ftab,
    eftab, offs sampling .......... bt2_idx.h:2829-3168 (Ebwt::buildToDisk)
  * '$' sorts AFTER every base ..... implied by fchr[0]=0 / fchr[4]=len
                                      (bt2_idx.h:3104-3113) and ftab absorb logic
  * fragments / RefRecords ........ ref_read.cpp:28-160, bt2_idx.h:2695-2804
  * .3/.4 reference files ......... reference.cpp:100-235, ref_read.h:73-92
  * mirror index = whole joined text reversed, flags -5 (EBWT_ENTIRE_REV),
    rstarts listed in reversed order (bt2_build.cpp:532-533, 679-695)

Suffix sorting is prefix doubling on torch tensors so it runs on the GPU for
the bench's large synthetic genomes and on the CPU for small test genomes.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass, field

import numpy as np

OFF_MASK = 0xFFFFFFFF

_ASC = np.full(256, 4, dtype=np.uint8)
for _c, _v in zip(b"ACGTacgt", [0, 1, 2, 3, 0, 1, 2, 3]):
    _ASC[_c] = _v


@dataclass
class RefRecord:
    off: int
    len: int
    first: bool


@dataclass
class Ebwt:
    """In-memory image of one .1.bt2 (+ .2.bt2) file."""
    length: int
    line_rate: int
    off_rate: int
    ftab_chars: int
    flags: int
    plen: np.ndarray
    rstarts: np.ndarray          # (nFrag*3,) uint32
    ebwt: np.ndarray             # sides, uint8, numSides*64
    zoff: int
    fchr: np.ndarray             # (5,) uint32
    ftab: np.ndarray             # uint32
    eftab: np.ndarray            # uint32
    names: bytes = b""
    offs: np.ndarray | None = None   # uint32 SA sample (.2.bt2)

    @property
    def side_sz(self):
        return 1 << self.line_rate

    @property
    def num_sides(self):
        bwt_sz = self.length // 4 + 1
        side_bwt_sz = self.side_sz - 16
        return (bwt_sz + side_bwt_sz - 1) // side_bwt_sz


@dataclass
class Bt2Index:
    fw: Ebwt
    bw: Ebwt
    recs: list = field(default_factory=list)
    text: np.ndarray | None = None      # joined unambiguous text (codes 0..3)
    ref_codes: list | None = None       # per reference: uint8 codes incl. N=4


# --------------------------------------------------------------------------
# FASTA -> records / joined text
# --------------------------------------------------------------------------
def parse_fasta(path):
    """Return [(name, bytes)] in file order (one entry per '>' line)."""
    seqs, name, chunks = [], None, []
    with open(path, "rb") as f:
        for line in f:
            line = line.rstrip(b"\r\n")
            if line.startswith(b">"):
                if name is not None:
                    seqs.append((name, b"".join(chunks)))
                name, chunks = line[1:], []
            else:
                chunks.append(line.strip())
    if name is not None:
        seqs.append((name, b"".join(chunks)))
    return seqs


def records_for(seqs_codes):
    """RefRecords as BitPairReference::szsFromFasta emits them.

    One record per maximal run of unambiguous bases: off = ambiguous bases
    since the previous run (or the sequence start), first = first record of
    the sequence.  Trailing ambiguous bases give (off, 0, False); an
    all-ambiguous sequence gives (n, 0, True)."""
    recs = []
    for codes in seqs_codes:
        amb = codes > 3
        n = len(codes)
        if n == 0:
            continue
        d = np.diff(np.concatenate([[1], amb.astype(np.int8), [1]]))
        starts = np.nonzero(d == -1)[0]
        ends = np.nonzero(d == 1)[0]
        if len(starts) == 0:
            recs.append(RefRecord(n, 0, True))
            continue
        prev = 0
        for k, (s, e) in enumerate(zip(starts, ends)):
            recs.append(RefRecord(int(s - prev), int(e - s), k == 0))
            prev = e
        if prev < n:
            recs.append(RefRecord(int(n - prev), 0, False))
    return recs


def joined_text(seqs_codes):
    parts = [c[c <= 3] for c in seqs_codes]
    return np.concatenate(parts).astype(np.uint8) if parts else np.zeros(0, np.uint8)


# --------------------------------------------------------------------------
# Suffix array ($ sorts after every base), prefix doubling on torch
# --------------------------------------------------------------------------
def suffix_array(text: np.ndarray, device="cpu"):
    """SA of text+'$' (n+1 entries) with '$' the LARGEST symbol.  int64 numpy."""
    import torch
    n = int(len(text))
    K = 21  # 3 bits per symbol in an int64 key
    dev = torch.device(device)
    t = torch.from_numpy(text.astype(np.int64)).to(dev)
    # symbol value: base+1 (1..4), '$' at position n -> 5, beyond -> 5
    sym = torch.full((n + K,), 5, dtype=torch.int64, device=dev)
    sym[:n] = t + 1
    key = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    for k in range(K):
        key = key * 8 + sym[k:k + n + 1]
    key, sa = torch.sort(key)
    # rank = index of first element of its group in sorted order
    newgrp = torch.ones(n + 1, dtype=torch.bool, device=dev)
    newgrp[1:] = key[1:] != key[:-1]
    del key
    h = K
    while True:
        idx = torch.arange(n + 1, device=dev)
        grpstart = torch.where(newgrp, idx, torch.zeros_like(idx))
        grpstart = torch.cummax(grpstart, 0).values
        rank = torch.empty(n + 1 + h, dtype=torch.int64, device=dev)
        rank[sa] = grpstart
        rank[n + 1:] = -1
        # unresolved = members of groups with size > 1
        single = newgrp.clone()
        single[:-1] &= newgrp[1:]
        unresolved = torch.nonzero(~single).squeeze(1)
        if unresolved.numel() == 0:
            break
        pos = sa[unresolved]
        k2 = rank[pos + h]
        k1 = grpstart[unresolved]
        # stable LSD: secondary then primary
        o = torch.sort(k2, stable=True).indices
        pos, k1, k2 = pos[o], k1[o], k2[o]
        o = torch.sort(k1, stable=True).indices
        pos, k1, k2 = pos[o], k1[o], k2[o]
        sa[unresolved] = pos
        # new group boundaries among the unresolved block
        ng = torch.ones_like(k1, dtype=torch.bool)
        ng[1:] = (k1[1:] != k1[:-1]) | (k2[1:] != k2[:-1])
        newgrp[unresolved] = ng
        h *= 2
        del rank, k1, k2, pos, o, ng
    return sa.cpu().numpy()


# --------------------------------------------------------------------------
# Ebwt construction (Ebwt::buildToDisk semantics)
# --------------------------------------------------------------------------
def build_ebwt(text, sa, recs, flags, rstarts, plen, off_rate=4, ftab_chars=10, line_rate=6):
    n = int(len(text))
    assert len(sa) == n + 1
    side_sz = 1 << line_rate
    side_bwt_sz = side_sz - 16
    side_bwt_len = side_bwt_sz * 4
    bwt_sz = n // 4 + 1
    num_sides = (bwt_sz + side_bwt_sz - 1) // side_bwt_sz
    tot = num_sides * side_bwt_len
    sa = np.asarray(sa, dtype=np.int64)
    bwt = np.zeros(tot, dtype=np.uint8)                   # padding = 'A'
    prev = sa - 1
    zoff = int(np.nonzero(sa == 0)[0][0])
    bwt[: n + 1] = text[np.where(prev < 0, 0, prev)]
    bwt[zoff] = 0
    counted = np.ones(tot, dtype=bool)
    counted[zoff] = False
    # fchr (exclusive prefix over counts excluding '$')
    cnt = np.bincount(bwt[: n + 1][counted[: n + 1]], minlength=4).astype(np.int64)
    fchr = np.zeros(5, dtype=np.uint32)
    fchr[1:] = np.cumsum(cnt)
    # occ before each side (padding counted, '$' not)
    side_counts = np.zeros((num_sides, 4), dtype=np.int64)
    b2 = bwt.reshape(num_sides, side_bwt_len)
    c2 = counted.reshape(num_sides, side_bwt_len)
    for c in range(4):
        side_counts[:, c] = ((b2 == c) & c2).sum(axis=1)
    occ_before = np.zeros_like(side_counts)
    occ_before[1:] = np.cumsum(side_counts, axis=0)[:-1]
    packed = (b2.reshape(num_sides, side_bwt_sz, 4).astype(np.uint8)
              << np.array([0, 2, 4, 6], dtype=np.uint8)).sum(axis=2).astype(np.uint8)
    sides = np.zeros((num_sides, side_sz), dtype=np.uint8)
    sides[:, :side_bwt_sz] = packed
    sides[:, side_bwt_sz:] = occ_before.astype(np.uint32).view(np.uint8).reshape(num_sides, 16)
    # ftab / eftab
    ftab_len = (1 << (2 * ftab_chars)) + 1
    eftab_len = ftab_chars * 2
    long_ = (n - sa) >= ftab_chars
    pos = sa[long_]
    sufint = np.zeros(len(pos), dtype=np.int64)
    for i in range(ftab_chars):
        sufint = (sufint << 2) | text[pos + i].astype(np.int64)
    ftab = np.zeros(ftab_len, dtype=np.int64)
    np.add.at(ftab, sufint + 1, 1)
    absorb = np.zeros(ftab_len, dtype=np.int64)
    # short suffixes are absorbed into the next long suffix's bucket, trailing ones into the last
    is_long = long_.astype(np.int64)
    short_rows = np.nonzero(~long_)[0]
    if len(short_rows):
        long_rows = np.nonzero(long_)[0]
        nxt = np.searchsorted(long_rows, short_rows)
        sufint_by_row = np.full(n + 1, -1, dtype=np.int64)
        sufint_by_row[long_rows] = sufint
        tgt = np.where(nxt < len(long_rows), sufint_by_row[long_rows[np.minimum(nxt, len(long_rows) - 1)]],
                       ftab_len - 1)
        np.add.at(absorb, tgt, 1)
    # Ebwt::buildToDisk prefix pass (bt2_idx.h:3145-3159), vectorised:
    # lo[i] = ftab[i] + ftabHi(i-1), ftabHi(i) = lo[i] + absorb[i]
    cnt = ftab.copy()
    cnt[0] = 0
    ab = absorb.copy()
    ab[0] = 0
    lo = np.cumsum(cnt) + np.concatenate([[0], np.cumsum(ab)[:-1]])
    out = lo.copy()
    eftab = np.zeros(eftab_len, dtype=np.int64)
    for ecur, i in enumerate(np.nonzero(ab > 0)[0]):
        eftab[ecur * 2] = lo[i]
        eftab[ecur * 2 + 1] = lo[i] + ab[i]
        out[i] = ecur ^ OFF_MASK
    out[0] = 0
    offs = sa[:: 1 << off_rate].astype(np.uint32)
    return Ebwt(length=n, line_rate=line_rate, off_rate=off_rate, ftab_chars=ftab_chars, flags=flags,
                plen=np.asarray(plen, np.uint32), rstarts=np.asarray(rstarts, np.uint32),
                ebwt=sides.reshape(-1), zoff=zoff, fchr=fchr, ftab=out.astype(np.uint32),
                eftab=eftab.astype(np.uint32), offs=offs)


def _plen_rstarts(recs, reverse, n):
    plen = []
    for r in recs:
        if r.first:
            plen.append(r.off + r.len)
        else:
            plen[-1] += r.off + r.len
    frags = []  # (joined off, text id, text off, len)
    joff, tid, toff = 0, -1, 0
    for r in recs:
        if r.first:
            tid += 1
            toff = 0
        toff += r.off
        if r.len > 0:
            frags.append((joff, tid, toff, r.len))
        joff += r.len
        toff += r.len
    if reverse:
        rs = []
        for (jo, t, to, ln) in reversed(frags):
            rs.append((n - jo - ln, t, to))
    else:
        rs = [(jo, t, to) for (jo, t, to, ln) in frags]
    return plen, np.asarray(rs, dtype=np.uint32).reshape(-1)


def build_index(seqs_codes, names=None, off_rate=4, ftab_chars=10, device="cpu"):
    """Build fw + mirror Ebwt for a list of per-reference code arrays (0..3, N=4)."""
    seqs_codes = [np.asarray(c, dtype=np.uint8) for c in seqs_codes]
    recs = records_for(seqs_codes)
    text = joined_text(seqs_codes)
    n = len(text)
    names_blob = b""
    if names is not None:
        names_blob = b"\n".join(names) + b"\n\0"
    out = {}
    for rev in (False, True):
        t = text[::-1].copy() if rev else text
        sa = suffix_array(t, device=device)
        plen, rs = _plen_rstarts(recs, rev, n)
        e = build_ebwt(t, sa, recs, -5 if rev else -1, rs, plen, off_rate, ftab_chars)
        e.names = names_blob
        out[rev] = e
    return Bt2Index(fw=out[False], bw=out[True], recs=recs, text=text, ref_codes=seqs_codes)


def build_from_fasta(path, **kw):
    seqs = parse_fasta(path)
    codes = [_ASC[np.frombuffer(s, dtype=np.uint8)] for _, s in seqs]
    names = [nm for nm, _ in seqs]
    return build_index(codes, names=names, **kw)


# --------------------------------------------------------------------------
# Writers / readers
# --------------------------------------------------------------------------
def _write_ebwt(path1, path2, e: Ebwt):
    with open(path1, "wb") as f:
        f.write(struct.pack("<IIiiiii", 1, e.length, e.line_rate, 2, e.off_rate, e.ftab_chars, e.flags))
        f.write(struct.pack("<I", len(e.plen)))
        f.write(e.plen.astype("<u4").tobytes())
        f.write(struct.pack("<I", len(e.rstarts) // 3))
        f.write(e.rstarts.astype("<u4").tobytes())
        f.write(e.ebwt.tobytes())
        f.write(struct.pack("<I", e.zoff))
        f.write(e.fchr.astype("<u4").tobytes())
        f.write(e.ftab.astype("<u4").tobytes())
        f.write(e.eftab.astype("<u4").tobytes())
        f.write(e.names)
    if path2 is not None and e.offs is not None:
        with open(path2, "wb") as f:
            f.write(struct.pack("<I", 1))
            f.write(e.offs.astype("<u4").tobytes())


def write_index(base, idx: Bt2Index):
    _write_ebwt(base + ".1.bt2", base + ".2.bt2", idx.fw)
    _write_ebwt(base + ".rev.1.bt2", base + ".rev.2.bt2", idx.bw)
    with open(base + ".3.bt2", "wb") as f:
        f.write(struct.pack("<II", 1, len(idx.recs)))
        for r in idx.recs:
            f.write(struct.pack("<IIB", r.off, r.len, 1 if r.first else 0))
    t = idx.text
    pad = (-len(t)) % 4
    tp = np.concatenate([t, np.zeros(pad, np.uint8)]).reshape(-1, 4)
    packed = (tp << np.array([0, 2, 4, 6], np.uint8)).sum(axis=1).astype(np.uint8)
    with open(base + ".4.bt2", "wb") as f:
        f.write(packed.tobytes())


def read_ebwt(path1, path2=None) -> Ebwt:
    d = open(path1, "rb").read()
    one, ln, lr, _lps, orate, fc, flags = struct.unpack_from("<IIiiiii", d, 0)
    assert one == 1, "big-endian index not supported"
    p = 28
    npat = struct.unpack_from("<I", d, p)[0]; p += 4
    plen = np.frombuffer(d, "<u4", npat, p).copy(); p += 4 * npat
    nfrag = struct.unpack_from("<I", d, p)[0]; p += 4
    rst = np.frombuffer(d, "<u4", 3 * nfrag, p).copy(); p += 12 * nfrag
    e = Ebwt(ln, lr, orate, fc, flags, plen, rst, None, 0, None, None, None)
    tot = e.num_sides * e.side_sz
    e.ebwt = np.frombuffer(d, np.uint8, tot, p).copy(); p += tot
    e.zoff = struct.unpack_from("<I", d, p)[0]; p += 4
    e.fchr = np.frombuffer(d, "<u4", 5, p).copy(); p += 20
    flen = (1 << (2 * fc)) + 1
    e.ftab = np.frombuffer(d, "<u4", flen, p).copy(); p += 4 * flen
    e.eftab = np.frombuffer(d, "<u4", 2 * fc, p).copy(); p += 8 * fc
    e.names = d[p:]
    if path2 is not None and os.path.exists(path2):
        d2 = open(path2, "rb").read()
        e.offs = np.frombuffer(d2, "<u4", (len(d2) - 4) // 4, 4).copy()
    return e


def read_index(base) -> Bt2Index:
    fw = read_ebwt(base + ".1.bt2", base + ".2.bt2")
    bw = read_ebwt(base + ".rev.1.bt2", base + ".rev.2.bt2")
    d = open(base + ".3.bt2", "rb").read()
    _, nrec = struct.unpack_from("<II", d, 0)
    recs = []
    for i in range(nrec):
        off, ln, first = struct.unpack_from("<IIB", d, 8 + 9 * i)
        recs.append(RefRecord(off, ln, bool(first)))
    n = fw.length
    raw = np.frombuffer(open(base + ".4.bt2", "rb").read(), np.uint8)
    text = ((raw[:, None] >> np.array([0, 2, 4, 6], np.uint8)) & 3).reshape(-1)[:n].astype(np.uint8)
    ref_codes, jo = [], 0
    for r in recs:
        if r.first:
            ref_codes.append([])
        ref_codes[-1].append(np.full(r.off, 4, np.uint8))
        ref_codes[-1].append(text[jo:jo + r.len])
        jo += r.len
    ref_codes = [np.concatenate(x) for x in ref_codes]
    return Bt2Index(fw=fw, bw=bw, recs=recs, text=text, ref_codes=ref_codes)


# --------------------------------------------------------------------------
# Device-side construction for large synthetic genomes (bench.py).  Same bytes
# as build_ebwt(); every O(n) pass is a torch op so it runs on the GPU.
# --------------------------------------------------------------------------
def _build_ebwt_torch(t, sa, flags, rstarts, plen, off_rate=4, ftab_chars=10, line_rate=6):
    import torch
    dev = t.device
    n = int(t.numel())
    side_sz = 1 << line_rate
    side_bwt_sz = side_sz - 16
    side_bwt_len = side_bwt_sz * 4
    num_sides = (n // 4 + 1 + side_bwt_sz - 1) // side_bwt_sz
    tot = num_sides * side_bwt_len
    zoff = int(_nonzero_big(sa == 0)[0])
    bwt = torch.zeros(tot, dtype=torch.uint8, device=dev)
    prev = (sa - 1).clamp_(min=0)
    bwt[: n + 1] = t[prev]
    del prev
    bwt[zoff] = 0
    b2 = bwt.view(num_sides, side_bwt_len)
    cnt = torch.empty((num_sides, 4), dtype=torch.int64, device=dev)
    for c in range(4):
        cnt[:, c] = (b2 == c).sum(dim=1)
    # '$' (at zoff) must not be counted as an 'A'
    cnt[zoff // side_bwt_len, 0] -= 1
    occ = torch.zeros_like(cnt)
    occ[1:] = torch.cumsum(cnt, 0)[:-1]
    tot_cnt = cnt.sum(0)
    # bases beyond n (padding 'A') are counted in occ but not in fchr
    pad = tot - (n + 1)
    fcnt = tot_cnt.clone()
    fcnt[0] -= pad
    fchr = torch.zeros(5, dtype=torch.int64, device=dev)
    fchr[1:] = torch.cumsum(fcnt, 0)
    sh = torch.tensor([0, 2, 4, 6], dtype=torch.uint8, device=dev)
    packed = (b2.view(num_sides, side_bwt_sz, 4) << sh).sum(dim=2, dtype=torch.uint8)
    sides = torch.empty((num_sides, side_sz), dtype=torch.uint8, device=dev)
    sides[:, :side_bwt_sz] = packed
    sides[:, side_bwt_sz:] = occ.to(torch.int32).contiguous().view(torch.uint8).view(num_sides, 16)
    del bwt, b2, packed
    # ftab: bucket counts of every length-ftab_chars k-mer of the text (= long suffixes)
    ftab_len = (1 << (2 * ftab_chars)) + 1
    m = n - ftab_chars + 1
    key = torch.zeros(max(m, 0), dtype=torch.int64, device=dev)
    for i in range(ftab_chars):
        key = (key << 2) | t[i:i + m].to(torch.int64)
    ftab = torch.zeros(ftab_len, dtype=torch.int64, device=dev)
    ftab[1:] += torch.bincount(key, minlength=ftab_len - 1)[: ftab_len - 1]
    # short suffixes (n - sa < ftab_chars): absorbed by the next long suffix's bucket
    short_rows = _nonzero_big((n - sa) < ftab_chars).cpu().numpy()
    absorb = np.zeros(ftab_len, dtype=np.int64)
    short_set = set(int(r) for r in short_rows)
    for r in short_rows:
        nx = int(r) + 1
        while nx in short_set:
            nx += 1
        if nx > n:
            absorb[ftab_len - 1] += 1
        else:
            absorb[int(key[int(sa[nx])])] += 1
    ftab = ftab.cpu().numpy()
    cnt_ = ftab.copy()
    cnt_[0] = 0
    ab = absorb.copy()
    ab[0] = 0
    lo = np.cumsum(cnt_) + np.concatenate([[0], np.cumsum(ab)[:-1]])
    out = lo.copy()
    eftab = np.zeros(ftab_chars * 2, dtype=np.int64)
    for ecur, i in enumerate(np.nonzero(ab > 0)[0]):
        eftab[ecur * 2] = lo[i]
        eftab[ecur * 2 + 1] = lo[i] + ab[i]
        out[i] = ecur ^ OFF_MASK
    out[0] = 0
    offs = sa[:: 1 << off_rate].to(torch.int64).cpu().numpy().astype(np.uint32)
    return Ebwt(length=n, line_rate=line_rate, off_rate=off_rate, ftab_chars=ftab_chars, flags=flags,
                plen=np.asarray(plen, np.uint32), rstarts=np.asarray(rstarts, np.uint32),
                ebwt=sides.view(-1).cpu().numpy(), zoff=zoff, fchr=fchr.cpu().numpy().astype(np.uint32),
                ftab=out.astype(np.uint32), eftab=eftab.astype(np.uint32), offs=offs)


_CHUNK = 1 << 30      # torch sort / nonzero take at most INT_MAX elements


def _nonzero_big(mask):
    """torch.nonzero(mask).squeeze(1) for masks longer than INT_MAX."""
    import torch
    n = int(mask.numel())
    if n <= _CHUNK:
        return torch.nonzero(mask).squeeze(1)
    parts = [torch.nonzero(mask[i:i + _CHUNK]).squeeze(1) + i for i in range(0, n, _CHUNK)]
    return torch.cat(parts)


def _cummax_big(x):
    """torch.cummax(x, 0).values in chunks, carrying the running maximum."""
    import torch
    n = int(x.numel())
    if n <= _CHUNK:
        return torch.cummax(x, 0).values
    out = torch.empty_like(x)
    carry = None
    for i in range(0, n, _CHUNK):
        c = torch.cummax(x[i:i + _CHUNK], 0).values
        if carry is not None:
            c = torch.maximum(c, carry)
        out[i:i + _CHUNK] = c
        carry = c[-1]
    return out


def _sort_big(key, top_shift):
    """torch.sort(key) for more than INT_MAX non-negative keys: bucket by the
    bits above top_shift (key order), sort every bucket on its own."""
    import torch
    n = int(key.numel())
    if n <= _CHUNK:
        return torch.sort(key)
    b = (key >> top_shift).to(torch.uint8)          # < 64 buckets
    nb = int(b.max()) + 1
    keys, perms = [], []
    for v in range(nb):
        idx = _nonzero_big(b == v)
        if idx.numel() == 0:
            continue
        k, o = torch.sort(key[idx])
        keys.append(k)
        perms.append(idx[o])
        del idx, k, o
    return torch.cat(keys), torch.cat(perms)


def _suffix_array_torch(t):
    """suffix_array() on a device tensor; returns an int64 device tensor."""
    import torch
    n = int(t.numel())
    K = 21
    dev = t.device
    sym = torch.full((n + K,), 5, dtype=torch.int64, device=dev)
    sym[:n] = t.to(torch.int64) + 1
    key = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    for k in range(K):
        key.mul_(8).add_(sym[k:k + n + 1])
    del sym
    # 21 symbols x 3 bits = 63 bits; beyond INT_MAX keys the first two symbols bucket the sort
    key, sa = _sort_big(key, 3 * (K - 2))
    newgrp = torch.ones(n + 1, dtype=torch.bool, device=dev)
    newgrp[1:] = key[1:] != key[:-1]
    del key
    h = K
    while True:
        single = newgrp.clone()
        single[:-1] &= newgrp[1:]
        unresolved = _nonzero_big(~single)
        del single
        if unresolved.numel() == 0:
            break
        idx = torch.arange(n + 1, device=dev)
        grpstart = torch.where(newgrp, idx, torch.zeros_like(idx))
        del idx
        grpstart = _cummax_big(grpstart)
        rank = torch.full((n + 1 + h,), -1, dtype=torch.int64, device=dev)
        rank[sa] = grpstart
        pos = sa[unresolved]
        k2 = rank[pos + h]
        k1 = grpstart[unresolved]
        del rank, grpstart
        o = torch.sort(k2, stable=True).indices
        pos, k1, k2 = pos[o], k1[o], k2[o]
        o = torch.sort(k1, stable=True).indices
        pos, k1, k2 = pos[o], k1[o], k2[o]
        sa[unresolved] = pos
        ng = torch.ones_like(k1, dtype=torch.bool)
        ng[1:] = (k1[1:] != k1[:-1]) | (k2[1:] != k2[:-1])
        newgrp[unresolved] = ng
        h *= 2
        del k1, k2, pos, o, ng, unresolved
    return sa


def build_index_device(seqs_codes, names=None, off_rate=4, ftab_chars=10, device="cuda"):
    """build_index() with every large pass on `device` (for bench-sized genomes)."""
    import torch
    seqs_codes = [np.asarray(c, dtype=np.uint8) for c in seqs_codes]
    recs = records_for(seqs_codes)
    text = joined_text(seqs_codes)
    n = len(text)
    names_blob = (b"\n".join(names) + b"\n\0") if names is not None else b""
    out = {}
    tt = torch.from_numpy(text).to(device)
    for rev in (False, True):
        t = torch.flip(tt, [0]).contiguous() if rev else tt
        sa = _suffix_array_torch(t)
        plen, rs = _plen_rstarts(recs, rev, n)
        e = _build_ebwt_torch(t, sa, -5 if rev else -1, rs, plen, off_rate, ftab_chars)
        e.names = names_blob
        out[rev] = e
        del sa, t
        torch.cuda.empty_cache() if str(device).startswith("cuda") else None
    return Bt2Index(fw=out[False], bw=out[True], recs=recs, text=text, ref_codes=seqs_codes)
