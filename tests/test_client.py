"""Row (f)-4: the multi-connection client (integration/bin/bt2g-client) against
the reference's own client (oracle/_ref/bowtie2-align-l, PatternSourceWebClient,
pat.cpp:2219-2789) on the same server and the same reads.

The SAM a connection returns depends on the read, its slot id on the wire (the
server seeds each read's random source from the name it sees, and the name is
the 4-hex slot of LockedOrigBufMap, pat.h:2464-2550) and nothing else; so with
the same slots the two clients must print the same lines (sorted: the server's
output order is arbitrary, pat.cpp:2024-2034).  Connections of <= 10 000 reads
hand out slots 0..n-1 in read order in both clients; past 20 000 reads the
reuse of the first map depends on when its END READ lines arrive, in the
reference as here, so that case is checked for names and counts only.

The server is the stock reference server (oracle/_ref/bowtie2-align-server-s)
on CPU: the client side is what is under test.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "bowtie2-server_amd", "tools"), os.path.join(ROOT, "tests", "golden")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import bt2_index as bi  # noqa: E402
import synth  # noqa: E402
from oracle import ref_server as rs  # noqa: E402

CLIENT = os.path.join(ROOT, "integration", "bin", "bt2g-client")
LONGREADS = os.path.join(ROOT, "tests", "golden", "longreads.fq.gz")
LAMBDA_PE = [os.path.join(ROOT, "tests", "golden", f"reads_{m}.fq.gz") for m in (1, 2)]


def _need(*paths):
    for p in paths:
        if not os.path.exists(p):
            pytest.skip(f"{os.path.relpath(p, ROOT)} not built (python -c 'import __graft_entry__ as g; g.build()')")


@pytest.fixture(scope="module")
def server(tmp_path_factory):
    _need(rs.SERVER, rs.CLIENT, CLIENT)
    d = tmp_path_factory.mktemp("clt")
    g = synth.genome(11, 400_000, n_repeats=60, rep_len=2000, n_copies=3, n_runs=5)
    base = str(d / "syn")
    idx = bi.build_index([g[:200_000], g[200_000:]], names=[b"c1", b"c2"])
    bi.write_index(base, idx)
    lam = str(d / "lambda_virus")
    bi.write_index(lam, bi.build_from_fasta(os.path.join(ROOT, "tests", "golden", "lambda_virus.fa")))
    srv = {}
    with rs.Server(base, threads=4) as s1, rs.Server(lam, threads=4) as s2:
        srv["synth"] = (s1, base, idx)
        srv["lambda"] = (s2, lam, None)
        yield srv


def _env(s):
    return dict(os.environ, BT2CLT_SERVER_PORT=str(s.port), BT2CLT_SERVER_HOST="127.0.0.1")


def _ref(s, base, args):
    r = subprocess.run([rs.CLIENT, "-x", base, "--no-hd"] + args, env=_env(s), capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def _ours(s, base, args):
    r = subprocess.run([CLIENT, "-x", base, "--no-hd"] + args, env=_env(s), capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def _lines(*texts):
    out = []
    for t in texts:
        out += [ln for ln in t.split(b"\n") if ln]
    return sorted(out)


def _same(a, b):
    la, lb = _lines(a), _lines(b)
    assert len(la) == len(lb) and len(la) > 0, (len(la), len(lb))
    bad = [(x, y) for x, y in zip(la, lb) if x != y]
    assert not bad, f"{len(bad)} lines differ, first:\nref  {bad[0][0][:300]}\nours {bad[0][1][:300]}"


def _reads(s_idx, n, seed, paired=False):
    import bench
    if paired:
        r, q = bench.make_pairs(s_idx.ref_codes, n, 150, seed)
        return r[:n], q[:n], r[n:], q[n:]
    r, q = bench.make_reads(s_idx.ref_codes, n, 150, seed)
    return r, q, None, None


def test_unpaired_same_sam(server, tmp_path):
    s, base, idx = server["synth"]
    r, q, _, _ = _reads(idx, 1500, 3)
    ch = rs.write_fastq_chunks(str(tmp_path), r, q)
    _same(_ref(s, base, ch[0]), _ours(s, base, ch[0]))


def test_paired_same_sam(server, tmp_path):
    s, base, idx = server["synth"]
    r, q, r2, q2 = _reads(idx, 600, 4, paired=True)
    ch = rs.write_fastq_chunks(str(tmp_path), r, q, codes2=r2, quals2=q2)
    _same(_ref(s, base, ch[0]), _ours(s, base, ch[0]))


def test_fastq_edge_cases(server, tmp_path):
    """The light parser and parse() of FastqPatternSource (pat.cpp:1066-1258):
    names ending /1 (dropped in the SAM) or with spaces, CRLF line ends, blank
    lines between and inside records, lower case, IUPAC letters and '.' as N,
    an empty name (named by its read number), a last record without a final
    newline; and the two sides of --trim5/--trim3."""
    s, base, idx = server["synth"]
    import bench
    r, q = bench.make_reads(idx.ref_codes, 40, 150, 9)
    acgt = b"ACGTN"
    recs = []
    for i in range(len(r)):
        seq = bytes(acgt[c] for c in r[i])
        qual = bytes(q[i])
        name = [b"e%d/1" % i, b"e%d with space" % i, b"e%d" % i, b""][i % 4]
        if i % 5 == 1:
            seq = seq[:20].lower() + seq[20:]
        if i % 7 == 2:
            seq = seq[:30] + b"R.Y" + seq[33:]
        nl = b"\r\n" if i % 3 == 0 else b"\n"
        gap = b"\n\n" if i % 6 == 4 else b""
        recs.append(b"@" + name + nl + seq + nl + b"+" + nl + qual + nl + gap)
    data = b"\n" + b"".join(recs)
    data = data.rstrip(b"\n")               # no newline after the last quality line
    f = tmp_path / "edge.fq"
    f.write_bytes(data)
    _same(_ref(s, base, ["-U", str(f)]), _ours(s, base, ["-U", str(f)]))
    _same(_ref(s, base, ["-U", str(f), "-3", "7", "-5", "4"]), _ours(s, base, ["-U", str(f), "-3", "7", "-5", "4"]))


def test_passthrough(server, tmp_path):
    """--passthrough (sam_print_xr): the read's FASTQ record, %-escaped, after its SAM line."""
    s, base, idx = server["synth"]
    r, q, r2, q2 = _reads(idx, 200, 5, paired=True)
    ch = rs.write_fastq_chunks(str(tmp_path), r, q, codes2=r2, quals2=q2)
    _same(_ref(s, base, ch[0] + ["--passthrough"]), _ours(s, base, ch[0] + ["--passthrough"]))


def test_longreads_gz(server):
    """configs[0]'s input, gzip-compressed (example/reads/longreads.fq)."""
    _need(LONGREADS)
    s, base, _ = server["lambda"]
    _same(_ref(s, base, ["-U", LONGREADS]), _ours(s, base, ["-U", LONGREADS]))


def test_lambda_pairs_upto(server):
    """example/reads/reads_{1,2}.fq (gzip), -u 2000 and -s 100 -u 900 (skipReads / qUpto)."""
    _need(*LAMBDA_PE)
    s, base, _ = server["lambda"]
    a = ["-1", LAMBDA_PE[0], "-2", LAMBDA_PE[1], "-u", "2000"]
    _same(_ref(s, base, a), _ours(s, base, a))
    a = ["-1", LAMBDA_PE[0], "-2", LAMBDA_PE[1], "-s", "100", "-u", "900"]
    _same(_ref(s, base, a), _ours(s, base, a))


def test_many_connections_equal_chunked_reference(server, tmp_path):
    """One input split over connections of <= 1 000 reads (-R), 3 open at a time
    (-k), 2 threads: the SAM of the reference client run once per 1 000-read
    chunk file -- and --chunks/--out-dir with the same chunk files, per chunk."""
    s, base, idx = server["synth"]
    r, q, _, _ = _reads(idx, 3500, 6)
    os.makedirs(tmp_path / "w")
    whole = rs.write_fastq_chunks(str(tmp_path / "w"), r, q, chunk=10_000)[0]
    chs = rs.write_fastq_chunks(str(tmp_path), r, q, chunk=1000)
    ref = [_ref(s, base, c) for c in chs]
    _same(b"".join(ref), _ours(s, base, whole + ["-k", "3", "-R", "1000", "-p", "2"]))
    lst = tmp_path / "chunks.txt"
    lst.write_text("".join(f"U {c[1]}\n" for c in chs))
    out = tmp_path / "out"
    _ours(s, base, ["--chunks", str(lst), "-k", "4", "--out-dir", str(out)])
    for i, t in enumerate(ref):
        _same(t, (out / f"chunk{i:05d}.sam").read_bytes())


def test_more_than_two_maps_of_reads(server, tmp_path):
    """25 000 short reads over one connection: slots 10 000.. come from the second
    map and the first is reused once emptied (LockedOrigBufMap); which reads
    reuse it depends on timing in both clients, so names and counts only."""
    s, base, _ = server["lambda"]
    g = open(os.path.join(ROOT, "tests", "golden", "lambda_virus.fa"), "rb").read().split(b"\n", 1)[1].replace(b"\n", b"")
    import random
    rnd = random.Random(1)
    fq = []
    for i in range(25_000):
        p = rnd.randrange(0, len(g) - 60)
        fq.append(b"@q%d\n%s\n+\n%s\n" % (i, g[p:p + 50], b"I" * 50))
    f = tmp_path / "many.fq"
    f.write_bytes(b"".join(fq))
    a, b = _ref(s, base, ["-U", str(f)]), _ours(s, base, ["-U", str(f)])
    na = sorted(ln.split(b"\t", 1)[0] for ln in a.split(b"\n") if ln and not ln.startswith(b"@"))
    nb = sorted(ln.split(b"\t", 1)[0] for ln in b.split(b"\n") if ln and not ln.startswith(b"@"))
    assert na == nb and len(na) >= 25_000


def test_errors_like_reference(server, tmp_path):
    """Malformed input fails as the reference client does (non-zero exit, its message)."""
    s, base, _ = server["synth"]
    bad = tmp_path / "bad.fq"
    bad.write_bytes(b"@x\nACGT\n+\nII\n")
    r = subprocess.run([CLIENT, "-x", base, "-U", str(bad)], env=_env(s), capture_output=True, timeout=60)
    assert r.returncode != 0 and b"more read characters than quality values" in r.stderr
    bad.write_bytes(b"ACGT\n")
    r = subprocess.run([CLIENT, "-x", base, "-U", str(bad)], env=_env(s), capture_output=True, timeout=60)
    assert r.returncode != 0 and b"does not look like a FASTQ file" in r.stderr
    r = subprocess.run([CLIENT, "-x", base, "-U", str(bad), "--server-port", "1"], capture_output=True, timeout=60)
    assert r.returncode != 0


def _seqs(idx, n, seed):
    import bench
    r, q = bench.make_reads(idx.ref_codes, n, 150, seed)
    acgt = b"ACGTN"
    return [bytes(acgt[c] for c in r[i]) for i in range(n)], [bytes(q[i]) for i in range(n)]


def test_fasta_same_sam(server, tmp_path):
    """-f: FastaPatternSource (pat.cpp:790-912) -- multi-line records, lower case,
    '.' and IUPAC letters, CRLF, an empty name (its read number), blank lines,
    no newline after the last record (whose last base the reference drops);
    unpaired, trimmed, and -1/-2 pairs."""
    s, base, idx = server["synth"]
    seqs, _ = _seqs(idx, 60, 21)
    recs = []
    for i, sq in enumerate(seqs):
        name = [b"f%d/1" % i, b"f%d desc" % i, b"", b"f%d" % i][i % 4]
        if i % 5 == 2:
            sq = sq[:40].lower() + sq[40:]
        if i % 7 == 3:
            sq = sq[:50] + b"R.Y" + sq[53:]
        nl = b"\r\n" if i % 3 == 0 else b"\n"
        body = nl.join(sq[k:k + 60] for k in range(0, len(sq), 60))
        recs.append(b">" + name + nl + body + nl + (b"\n" if i % 6 == 5 else b""))
    f = tmp_path / "r.fa"
    f.write_bytes(b"\n" + b"".join(recs).rstrip(b"\n"))
    for extra in ([], ["-5", "3", "-3", "6"]):
        a = ["-f", "-U", str(f)] + extra
        _same(_ref(s, base, a), _ours(s, base, a))
    r, q, r2, q2 = _reads(idx, 300, 22, paired=True)
    acgt = b"ACGTN"
    f1, f2 = tmp_path / "p1.fa", tmp_path / "p2.fa"
    f1.write_bytes(b"".join(b">p%d/1\n%s\n" % (i, bytes(acgt[c] for c in r[i])) for i in range(len(r))))
    f2.write_bytes(b"".join(b">p%d/2\n%s\n" % (i, bytes(acgt[c] for c in r2[i])) for i in range(len(r2))))
    a = ["-f", "-1", str(f1), "-2", str(f2)]
    _same(_ref(s, base, a), _ours(s, base, a))
    a += ["--passthrough"]
    _same(_ref(s, base, a), _ours(s, base, a))


def test_tabbed_same_sam(server, tmp_path):
    """--tab5 / --12 / --tab6: TabbedPatternSource (pat.cpp:1524-1661) -- unpaired
    and paired lines mixed in one file, blank lines, CRLF; --passthrough."""
    s, base, idx = server["synth"]
    r, q, r2, q2 = _reads(idx, 200, 23, paired=True)
    acgt = b"ACGTN"
    l5, l6 = [], []
    for i in range(len(r)):
        s1, q1 = bytes(acgt[c] for c in r[i]), bytes(q[i])
        s2, qq2 = bytes(acgt[c] for c in r2[i]), bytes(q2[i])
        nl = b"\r\n" if i % 4 == 0 else b"\n"
        if i % 3 == 0:
            l5.append(b"u%d\t%s\t%s%s" % (i, s1, q1, nl))
            l6.append(b"u%d\t%s\t%s%s" % (i, s1, q1, nl))
        else:
            l5.append(b"t%d\t%s\t%s\t%s\t%s%s" % (i, s1, q1, s2, qq2, nl))
            l6.append(b"t%d/1\t%s\t%s\tt%d/2\t%s\t%s%s" % (i, s1, q1, i, s2, qq2, nl))
        if i % 17 == 5:
            l5.append(b"\n")
    f5, f6 = tmp_path / "r.tab5", tmp_path / "r.tab6"
    f5.write_bytes(b"".join(l5))
    f6.write_bytes(b"".join(l6))
    for a in (["--tab5", str(f5)], ["--12", str(f5)], ["--tab6", str(f6)], ["--tab6", str(f6), "--passthrough"],
              ["--tab5", str(f5), "-3", "5"]):
        _same(_ref(s, base, a), _ours(s, base, a))


def test_raw_and_cmdline_same_sam(server, tmp_path):
    """-r (RawPatternSource, pat.cpp:1743-1817) and -c (VectorPatternSource,
    pat.cpp:614-700: SEQ[:QUALS] arguments)."""
    s, base, idx = server["synth"]
    seqs, quals = _seqs(idx, 80, 24)
    f = tmp_path / "r.raw"
    f.write_bytes(b"".join(sq + (b"\r\n" if i % 5 == 0 else b"\n") + (b"\n" if i % 9 == 2 else b"")
                           for i, sq in enumerate(seqs)))
    _same(_ref(s, base, ["-r", "-U", str(f)]), _ours(s, base, ["-r", "-U", str(f)]))
    # (qualities without ',' or ':', the argument's separators)
    qs = [bytes(65 + c % 9 for c in qv).decode() for qv in quals]
    cl = ",".join(sq.decode() + (":" + qs[i] if i % 2 else "") for i, sq in enumerate(seqs[:12]))
    _same(_ref(s, base, ["-c", "-U", cl]), _ours(s, base, ["-c", "-U", cl]))
