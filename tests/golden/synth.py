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
