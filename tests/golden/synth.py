"""Deterministic synthetic genomes and reads (numpy PCG64; stable across runs).

Used by tests/golden/make_golden.py (to make reference fixtures here) and by
the tests / bench (to regenerate the same inputs on the GPU box).  Read model
follows BASELINE.md section 3: substitutions 0.4 %/base, read-N 0.05 %/base,
a 1-bp indel in 5 % of reads, Phred qualities uniform in [2, 40].
"""
import numpy as np

ACGT = np.frombuffer(b"ACGT", np.uint8)


def genome(seed, n, n_repeats=0, rep_len=2000, n_copies=4, n_runs=0):
    """Random genome codes (0..3) with planted near-duplicate repeats and N runs (4)."""
    rng = np.random.default_rng(seed)
    g = rng.integers(0, 4, n, dtype=np.uint8)
    for _ in range(n_repeats):
        src = rng.integers(0, n - rep_len)
        unit = g[src:src + rep_len].copy()
        for _ in range(n_copies):
            dst = rng.integers(0, n - rep_len)
            cp = unit.copy()
            nm = rng.integers(0, max(1, rep_len // 100))
            pos = rng.integers(0, rep_len, nm)
            cp[pos] = rng.integers(0, 4, nm, dtype=np.uint8)
            g[dst:dst + rep_len] = cp
    for _ in range(n_runs):
        s = rng.integers(0, n - 100)
        g[s:s + rng.integers(1, 60)] = 4
    return g


def _scatter_copies(rng, g, source, lens, rates, chunk=1_000_000):
    """Write len(lens) diverged copies into g at random positions (either
    strand).  source(ci, w) gives base w of copy ci (vectors); copy i gets a
    per-copy substitution rate rates[i]."""
    n = len(g)
    for c0 in range(0, len(lens), chunk):
        L = np.asarray(lens[c0:c0 + chunk], np.int64)
        off = np.concatenate([[0], np.cumsum(L)])
        ci = np.repeat(np.arange(c0, c0 + len(L)), L)
        w = np.arange(int(off[-1])) - np.repeat(off[:-1], L)
        rc = np.repeat(rng.random(len(L)) < 0.5, L)
        w = np.where(rc, np.repeat(L, L) - 1 - w, w)          # reverse strand: read the copy backwards ...
        cat = source(ci, w).astype(np.uint8)
        cat[rc] = 3 - cat[rc]                                   # ... complemented
        m = rng.random(len(cat)) < np.repeat(np.asarray(rates[c0:c0 + chunk]), L)
        cat[m] = (cat[m] + rng.integers(1, 4, int(m.sum()), dtype=np.uint8)) % 4
        dst = rng.integers(0, n - int(L.max()) - 1, len(L))
        g[np.repeat(dst, L) + (np.arange(int(off[-1])) - np.repeat(off[:-1], L))] = cat


def genome_hg38like(seed, n):
    """A synthetic genome with hg38's repeat landscape at scale n (codes 0..4):
    41 % GC background; Alu-like SINEs (3 subfamilies of ~300 bp, 10 % of the
    genome, 5-20 % divergence from consensus); L1-like LINEs (one 6 kb
    consensus, 5'-truncated copies of 0.3-6 kb, 17 %, 3-20 %); segmental
    duplications (10-50 kb copies of the genome itself, 5 %, 1-4 %);
    microsatellites (1-6 bp units in 20-200 bp runs, 2 %); N gaps (~2 %, runs
    of 1-50 kb).  Repeats fragment exact matches into many-element SA ranges
    and give reads several competing DP windows, as in the human genome."""
    rng = np.random.default_rng(seed)
    lut = np.repeat(np.arange(4, dtype=np.uint8), [295, 205, 205, 295])       # 41 % GC
    g = lut[rng.integers(0, 1000, n, dtype=np.uint16)]
    alus = rng.integers(0, 4, (3, 310)).astype(np.uint8)
    k = int(0.10 * n / 300)
    fam, aln = rng.integers(0, 3, k), rng.integers(250, 311, k)
    _scatter_copies(rng, g, lambda ci, w: alus[fam[ci], 310 - aln[ci] + w], aln, rng.uniform(0.05, 0.20, k))
    l1 = rng.integers(0, 4, 6000).astype(np.uint8)
    ln = np.minimum(6000, (rng.pareto(1.2, int(0.17 * n / 1400)) * 300 + 300).astype(np.int64))
    _scatter_copies(rng, g, lambda ci, w: l1[6000 - ln[ci] + w], ln, rng.uniform(0.03, 0.20, len(ln)))
    sd_len = rng.integers(10_000, 50_001, max(1, int(0.05 * n / 30_000)))
    sd_len = sd_len[sd_len < n // 4]
    if len(sd_len):
        src = rng.integers(0, n - int(sd_len.max()) - 1, len(sd_len))
        snap = g.copy() if n <= 50_000_000 else g          # large genomes: copy from the live sequence
        _scatter_copies(rng, g, lambda ci, w: snap[src[ci] + w] % 4, sd_len, rng.uniform(0.01, 0.04, len(sd_len)),
                        chunk=256)
    ms = int(0.02 * n / 100)
    ul = rng.integers(1, 7, ms)
    units = rng.integers(0, 4, (ms, 6)).astype(np.uint8)
    _scatter_copies(rng, g, lambda ci, w: units[ci, w % ul[ci]], rng.integers(20, 201, ms), rng.uniform(0.0, 0.05, ms))
    gaps = max(1, int(0.02 * n / 25_000))
    gl = rng.integers(1_000, 50_001, gaps)
    gl = gl[gl < n // 50]
    for s0, l_ in zip(rng.integers(0, n - 50_001, len(gl)), gl):
        g[s0:s0 + l_] = 4
    return g


def reads(seed, gen, n, length=150, sub=0.004, nrate=0.0005, indel=0.05, rc_frac=0.5):
    """Sample reads from `gen` (codes, may contain 4).  Returns (codes[n,length] u8,
    quals[n,length] u8 Phred+33, true_pos[n], true_fw[n])."""
    rng = np.random.default_rng(seed)
    G = len(gen)
    out = np.zeros((n, length), np.uint8)
    pos = rng.integers(0, G - length - 2, n)
    fw = rng.random(n) >= rc_frac
    for i in range(n):
        p = pos[i]
        frag = gen[p:p + length + 1].copy()
        if rng.random() < indel:
            k = rng.integers(1, length - 1)
            if rng.random() < 0.5:
                frag = np.concatenate([frag[:k], frag[k + 1:]])          # deletion from read
            else:
                frag = np.concatenate([frag[:k], rng.integers(0, 4, 1, dtype=np.uint8), frag[k:]])
        frag = frag[:length]
        if not fw[i]:
            frag = np.where(frag > 3, 4, 3 - frag)[::-1].astype(np.uint8)
        m = rng.random(length) < sub
        frag[m] = (frag[m] + rng.integers(1, 4, m.sum(), dtype=np.uint8)) % 4
        frag[rng.random(length) < nrate] = 4
        out[i] = frag
    quals = rng.integers(2, 41, (n, length), dtype=np.uint8) + 33
    return out, quals, pos, fw


def to_ascii(codes):
    return np.frombuffer(b"ACGTN", np.uint8)[codes]


def write_fastq(path, codes, quals, prefix="r"):
    with open(path, "wb") as f:
        for i in range(len(codes)):
            f.write(b"@%s%d\n" % (prefix.encode(), i))
            f.write(to_ascii(codes[i]).tobytes() + b"\n+\n" + quals[i].tobytes() + b"\n")


def write_fasta(path, seqs, names):
    with open(path, "wb") as f:
        for nm, s in zip(names, seqs):
            f.write(b">" + nm + b"\n")
            a = to_ascii(s).tobytes()
            for j in range(0, len(a), 60):
                f.write(a[j:j + 60] + b"\n")
