"""Generate the committed golden fixtures from the REFERENCE itself.

Run here (needs /root/reference and the oracle/_ref build):
    make -C oracle/ref && python tests/golden/make_golden.py

Everything it writes is data (inputs + the reference's outputs):
  * index_sha256.json  SHA-256 of every .bt2 file the reference's bowtie2-build
                       writes for lambda_virus.fa, multi.fa and the synthetic
                       genome -> pins tools/bt2_index.py byte-for-byte.
  * multi.fa           small multi-sequence FASTA (N runs, IUPAC, lowercase).
  * fm_<name>.npz      reads + reference outputs of SeedAligner::exactSweep,
                       exact-seed searchAllSeeds (two policies), oneMmSearch
                       (end-to-end and local), Ebwt::getOffset and single
                       bidirectional LF steps (oracle/_ref/libbt2ref.so).
  * sw_<name>.npz      DP problems logged by the reference server itself
                       (--log-dp, bt2_search.cpp:3117-3126) plus random problems,
                       with SwAligner::align's outputs (aligned, best, u8/i16
                       success, colstop_, lastsolcol_, sorted btncand_).
"""
import hashlib
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "bowtie2-server_amd", "tools"))

import synth  # noqa: E402
import bt2_index as bi  # noqa: E402
from oracle.ref_harness import RefLib  # noqa: E402

REFDIR = "/root/reference"
REFBIN = os.path.join(ROOT, "oracle", "_ref")
EXTS = ["1.bt2", "2.bt2", "3.bt2", "4.bt2", "rev.1.bt2", "rev.2.bt2"]
MAXSEEDS = 64


def sha(path):
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def ref_build(fa, base):
    subprocess.check_call([os.path.join(REFBIN, "bowtie2-build-s"), "-q", fa, base],
                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return {e: sha(base + "." + e) for e in EXTS}


def make_multi_fa(path):
    rng = np.random.default_rng(7)

    def rs(n):
        return "".join("ACGT"[i] for i in rng.integers(0, 4, n))
    rep = rs(120)
    seqs = ["NN" + rs(300) + "NNNNN" + rs(250) + "N" + rs(40), rs(500),
            rs(100) + rep + rs(30) + rep + rs(50) + rep.lower() + "NNNN", "N" * 10,
            rs(70) + "RYK" + rs(80)]
    with open(path, "w") as f:
        for i, s in enumerate(seqs):
            f.write(">seq%d desc\n" % i)
            for j in range(0, len(s), 60):
                f.write(s[j:j + 60] + "\n")


def synth_genome():
    return synth.genome(1234, 300_000, n_repeats=40, rep_len=1500, n_copies=3, n_runs=6)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_server_logdp(base, fq, extra, workdir):
    """Start the reference server (-p 1, --log-dp) and push fq through the client."""
    port = free_port()
    log = os.path.join(workdir, "dp.log")
    srv = subprocess.Popen([os.path.join(REFBIN, "bowtie2-align-server-s"), "-x", base, "-p", "1",
                            "--log-dp", log, "--server-port", str(port)] + extra,
                           stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    try:
        t0 = time.time()
        while True:
            line = srv.stderr.readline().decode()
            if "Server ready" in line:
                break
            if srv.poll() is not None or time.time() - t0 > 120:
                raise RuntimeError("server did not start")
        env = dict(os.environ, BT2CLT_SERVER_PORT=str(port), BT2CLT_SERVER_HOST="127.0.0.1")
        subprocess.check_call([os.path.join(REFBIN, "bowtie2-align-l"), "-x", os.path.basename(base),
                               "-U", fq, "-S", os.path.join(workdir, "out.sam")], env=env,
                              stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    finally:
        srv.kill()
        srv.wait()
    return log


def parse_dplog(path, maxprob):
    probs = []
    with open(path) as f:
        for line in f:
            parts = line.rstrip("\n").split("\t")
            if len(parts) <= 2:
                continue
            seq, qual = parts[0], parts[1]
            for p in parts[2:]:
                fs = p.split(",")
                if len(fs) < 16 or fs[15] == "":
                    continue  # last record can be cut short when the server is stopped
                refidx, reflen, minsc = int(fs[0]), int(fs[1]), int(fs[2])
                fw = fs[3] == "+"
                refl, refr = int(fs[4]), int(fs[5])
                refstr = fs[13]
                aligned, score = int(fs[14]), int(fs[15])
                probs.append((seq, qual, refidx, reflen, minsc, fw, refl, refr, refstr, aligned, score))
                if len(probs) >= maxprob:
                    return probs
    return probs


MASK = {"A": 1, "C": 2, "G": 4, "T": 8, "N": 16}
CODE = {"A": 0, "C": 1, "G": 2, "T": 3, "N": 4}


def sw_fixture(lib, ref, probs, local, rng_extra=None):
    """Re-run each logged problem through SwAligner (extra right column from the
    reference, aligner_sw.cpp:174-176) and record outputs."""
    reads, quals, rd_index, fws, minscs, rf_off, rf_all, outs, cand_all, cand_off = [], [], [], [], [], [0], [], [], [], [0]
    seen = {}
    for (seq, qual, refidx, reflen, minsc, fw, refl, refr, refstr, aligned, score) in probs:
        ncol = len(refstr)
        nxt = refr + 1
        extra = int(ref.stretch(refidx, nxt, 1)[0]) if 0 <= nxt < reflen else 4
        rfm = np.array([MASK[c] for c in refstr] + [1 << extra], np.uint8)
        out, cands, _ = lib.sw(seq.encode(), qual.encode(), fw, rfm, minsc, local)
        assert out[0] == aligned, "harness disagrees with the server's own DP log"
        assert not aligned or out[1] == score
        key = (seq, qual)
        if key not in seen:
            seen[key] = len(reads)
            reads.append(np.array([CODE[c] for c in seq], np.uint8))
            quals.append(np.frombuffer(qual.encode(), np.uint8))
        rd_index.append(seen[key])
        fws.append(fw)
        minscs.append(minsc)
        rf_all.append(rfm)
        rf_off.append(rf_off[-1] + len(rfm))
        outs.append(out[:7])
        cand_all.append(cands)
        cand_off.append(cand_off[-1] + len(cands))
        _ = ncol
    lens = np.array([len(r) for r in reads], np.uint32)
    mx = int(lens.max())
    R = np.full((len(reads), mx), 4, np.uint8)
    Q = np.full((len(reads), mx), 33, np.uint8)
    for i, (r, q) in enumerate(zip(reads, quals)):
        R[i, :len(r)] = r
        Q[i, :len(q)] = q
    return dict(reads=R, quals=Q, lens=lens, rd_index=np.array(rd_index, np.int32), fw=np.array(fws, np.uint8),
                minsc=np.array(minscs, np.int64), rf=np.concatenate(rf_all), rf_off=np.array(rf_off, np.int64),
                out=np.array(outs, np.int64), cands=np.concatenate(cand_all).astype(np.int64).reshape(-1, 3),
                cand_off=np.array(cand_off, np.int64), local=np.array(local))


def random_sw_problems(gen, n, seed, local):
    """Random problems around true read positions, with off-end N padding."""
    rng = np.random.default_rng(seed)
    codes, quals, pos, fw = synth.reads(seed, gen, n, 150, sub=0.02, indel=0.3)
    probs = []
    for i in range(n):
        L = int(rng.choice([150, 150, 150, 37, 101, 77]))
        rd = codes[i][:L]
        q = quals[i][:L]
        w = int(L + 60 + rng.integers(-5, 500))
        start = int(pos[i]) - 30 + int(rng.integers(-40, 40))
        if rng.random() < 0.2:
            start = int(rng.integers(-50, len(gen) - w))
        minsc = int(20 + 8 * np.log(L)) if local else int(-0.6 - 0.6 * L)
        if rng.random() < 0.1:
            minsc = 5 if local else minsc - 150       # forces EE i16 / easy local
        isfw = bool(fw[i])
        rdfw = rd if isfw else np.where(rd > 3, 4, 3 - rd)[::-1]
        qfw = q if isfw else q[::-1]
        idxs = np.arange(start, start + w + 1)
        win = np.where((idxs >= 0) & (idxs < len(gen)), gen[np.clip(idxs, 0, len(gen) - 1)], 4)
        refstr = "".join("ACGTN"[c] for c in win[:-1])
        probs.append(("".join("ACGTN"[c] for c in rdfw), bytes(qfw).decode(), -1, -1, minsc, isfw,
                      start, start + w - 1, refstr, None, None, int(win[-1])))
    return probs


def sw_fixture_random(lib, probs, local):
    fake = []
    extras = []
    for p in probs:
        out, _, _ = lib.sw(p[0].encode(), p[1].encode(), p[5],
                           np.array([MASK[c] for c in p[8]] + [1 << p[11]], np.uint8), p[4], local)
        fake.append(p[:9] + (int(out[0]), int(out[1])))
        extras.append(p[11])

    class _R:
        def __init__(self, ex):
            self.ex = ex
            self.i = 0

        def stretch(self, refidx, nxt, n):
            v = self.ex[self.i]
            self.i += 1
            return np.array([v], np.uint8)
    fake2 = [(f[0], f[1], 0, 10 ** 12) + f[4:] for f in fake]
    return sw_fixture(lib, _R(extras), fake2, local)


def fm_fixture(R, codes, quals, lens, local_minsc, ee_minsc):
    asc = synth.to_ascii(codes)
    seqs = [bytes(asc[i, :lens[i]]) for i in range(len(codes))]
    qs = [bytes(quals[i, :lens[i]]) for i in range(len(codes))]
    d = dict(reads=codes, quals=quals, lens=lens)
    d["exact"] = R.exact_sweep(seqs, qs, 2)
    for tag, (L, iv, off) in {"s22": (22, 15, 0), "s20": (20, 7, 3), "s10": (10, 9, 0)}.items():
        o, ns, bw = R.seed_search(seqs, qs, L, iv, off, MAXSEEDS)
        d["seed_" + tag] = o
        d["seedn_" + tag] = ns
        d["seedops_" + tag] = bw
        d["seedpol_" + tag] = np.array([L, iv, off])
    for tag, local, ms in (("ee", 0, ee_minsc), ("loc", 1, local_minsc)):
        o, c, bw = R.one_mm(seqs, qs, ms, local, cap=64)
        d["mm_" + tag] = o
        d["mmn_" + tag] = c
        d["mmops_" + tag] = bw
        d["mmminsc_" + tag] = ms
    info = R.info()
    n = int(info[0])
    rng = np.random.default_rng(3)
    rows = np.unique(np.concatenate([rng.integers(0, n + 1, 400), [0, n, int(info[1])],
                                     np.arange(0, min(n, 400))]))
    d["off_rows"] = rows.astype(np.uint32)
    d["off_vals"] = np.array([R.get_offset(int(r)) for r in rows], np.uint32)
    # single bidirectional steps: random ranges incl. ones straddling sides / '$'
    steps = []
    for which in (0, 1):
        zo = int(info[1 + which])
        cand = [(zo, zo + 1), (max(0, zo - 3), zo + 5), (191, 193), (0, n), (190, 384)]
        for _ in range(300):
            a = int(rng.integers(0, n))
            b = a + int(rng.choice([1, 1, 2, 7, 50, 400]))
            cand.append((a, min(b, n)))
        for (a, b) in cand:
            if b <= a:
                continue
            t, bo, tp, bp = R.bilf(which, a, b, 1000)
            steps.append([which, a, b, 1000] + list(t) + list(bo) + list(tp) + list(bp))
    d["bilf"] = np.array(steps, np.int64)
    return d


def main():
    lib = RefLib()
    out = {}
    tmp = tempfile.mkdtemp(prefix="bt2gold_")
    try:
        # ---- indexes -------------------------------------------------------
        multi_fa = os.path.join(HERE, "multi.fa")
        make_multi_fa(multi_fa)
        synth_fa = os.path.join(tmp, "synth.fa")
        g = synth_genome()
        # split into 3 references to exercise rstarts
        parts = [g[:100_000], g[100_000:220_000], g[220_000:]]
        synth.write_fasta(synth_fa, parts, [b"chrA", b"chrB", b"chrC"])
        bases = {}
        for name, fa in (("lambda", os.path.join(REFDIR, "example/reference/lambda_virus.fa")),
                         ("multi", multi_fa), ("synth", synth_fa)):
            base = os.path.join(tmp, name)
            out[name] = ref_build(fa, base)
            bases[name] = base
        with open(os.path.join(HERE, "index_sha256.json"), "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
        # ---- FM fixtures ---------------------------------------------------
        for name, n in (("lambda", 400), ("synth", 600)):
            R = lib.open(bases[name])
            idx = bi.read_index(bases[name])
            gen = np.concatenate(idx.ref_codes)
            codes, quals, _, _ = synth.reads(100 + len(name), gen, n, 150, sub=0.006, nrate=0.002)
            lens = np.full(n, 150, np.uint32)
            # ragged tail: a few short / odd-length reads (len < ftabChars too)
            for i, L in enumerate([7, 10, 11, 21, 22, 23, 64, 99, 149]):
                lens[i] = L
                codes[i, L:] = 4
            ee = np.array([int(-0.6 - 0.6 * L) for L in lens], np.int64)
            loc = np.array([int(20 + 8 * np.log(L)) for L in lens], np.int64)
            d = fm_fixture(R, codes, quals, lens, loc, ee)
            np.savez_compressed(os.path.join(HERE, "fm_%s.npz" % name), **d)
            R.close()
        # ---- SW fixtures from the server's own DP logs ---------------------
        R = lib.open(bases["synth"])
        idx = bi.read_index(bases["synth"])
        gen = np.concatenate(idx.ref_codes)
        codes, quals, _, _ = synth.reads(77, gen, 1500, 150)
        fq = os.path.join(tmp, "r.fq")
        synth.write_fastq(fq, codes, quals)
        for tag, extra, local in (("ee", ["--sensitive"], 0), ("loc", ["--local"], 1)):
            wd = os.path.join(tmp, "srv_" + tag)
            os.makedirs(wd)
            log = run_server_logdp(bases["synth"], fq, extra, wd)
            probs = parse_dplog(log, 1200)
            d = sw_fixture(lib, R, probs, local)
            np.savez_compressed(os.path.join(HERE, "sw_log_%s.npz" % tag), **d)
            print(tag, "logged problems", len(probs), "aligned", int(d["out"][:, 0].sum()))
        R.close()
        for tag, local in (("ee", 0), ("loc", 1)):
            probs = random_sw_problems(gen, 400, 900 + local, local)
            d = sw_fixture_random(lib, probs, local)
            np.savez_compressed(os.path.join(HERE, "sw_rand_%s.npz" % tag), **d)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
