"""SAM parity of the batch-first driver (integration/bt2g_batch.cpp).

The reference's alignment server with its search workers replaced by batch
driver threads: every read's worker logic (multiseedSearchWorker's per-read
body, SwDriver::extendSeeds) runs as a resumable state machine and the
engines take one call per stage for all reads in flight.  Its SAM must equal
the stock server's on the same reads (sorted records, <= 10 000 reads per
connection):

  * -stub (CPU tests): oracle/_ref/bowtie2-align-server-batch-stub, the driver
    over the CPU stand-in of the ABI (the reference answers every engine call),
    which checks the driver's own logic -- the restated control flow, RNG
    order, DP table reuse across minimum scores, CPU fallbacks;
  * GPU: integration/bin/bowtie2-align-server-batch on libbt2g.so.
"""
import json
import os
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "bowtie2-server_amd", "tools"), os.path.join(ROOT, "tests", "golden")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import bt2_index as bi  # noqa: E402
import synth  # noqa: E402
from oracle import ref_server as rs  # noqa: E402

SRV_BATCH = os.path.join(ROOT, "integration", "bin", "bowtie2-align-server-batch")
SRV_BATCH_STUB = os.path.join(rs.REF_DIR, "bowtie2-align-server-batch-stub")
LONGREADS = os.path.join(ROOT, "tests", "golden", "longreads.fq.gz")     # example/reads/longreads.fq
LAMBDA_PE = [os.path.join(ROOT, "tests", "golden", f"reads_{m}.fq.gz") for m in (1, 2)]  # example/reads/reads_{1,2}.fq


def _need(*paths):
    for p in paths:
        if not os.path.exists(p):
            pytest.skip(f"{os.path.relpath(p, ROOT)} not built (python -c 'import __graft_entry__ as g; g.build()')")


@pytest.fixture(scope="module")
def indexes(tmp_path_factory):
    d = tmp_path_factory.mktemp("idx")
    lam = bi.build_from_fasta(os.path.join(ROOT, "tests", "golden", "lambda_virus.fa"))
    bi.write_index(str(d / "lambda_virus"), lam)
    # 400 kb, two references, planted 2 kb near-repeats (multi-mappers, XS:i) and N runs
    g = synth.genome(11, 400_000, n_repeats=60, rep_len=2000, n_copies=3, n_runs=5)
    syn = bi.build_index([g[:200_000], g[200_000:]], names=[b"c1", b"c2"])
    bi.write_index(str(d / "syn"), syn)
    return {"lambda": str(d / "lambda_virus"), "synth": (str(d / "syn"), syn)}


def _reads(idx, n, seed, dirpath, read_len=150, paired=False):
    import bench
    if paired:
        r, q = bench.make_pairs(idx.ref_codes, n, read_len, seed)
        return rs.write_fastq_chunks(dirpath, r[:n], q[:n], codes2=r[n:], quals2=q[n:])
    r, q = bench.make_reads(idx.ref_codes, n, read_len, seed)
    return rs.write_fastq_chunks(dirpath, r, q)


def _run(binary, base, chunks, args, dirpath, tag, threads=2, env_extra=None, client=None):
    stats = os.path.join(dirpath, f"stats_{tag}.json")
    env = dict(rs.dropin_env(base, stats), **(env_extra or {}))
    with rs.Server(base, threads=threads, args=args, binary=binary, env=env,
                   log_path=os.path.join(dirpath, f"server_{tag}.log")) as s:
        dt, outs = s.run(chunks, k=2, client=client or rs.CLIENT)
    st = None
    for _ in range(50):                      # written by the driver's SIGTERM handler
        if os.path.exists(stats):
            st = json.load(open(stats))
            break
        time.sleep(0.1)
    return dt, rs.sorted_records(outs), st


def compare(binary, base, chunks, args, dirpath, threads=2, env_extra=None, cpu_ok=(), client=None):
    """The stock server through the reference client against `binary` through
    `client` (default: the reference client too; rs.NATIVE_CLIENT: bt2g-client,
    as bench.py sends its reads): sorted SAM identical, no CPU fallback."""
    t_ref, a, _ = _run(rs.SERVER, base, chunks, args, dirpath, "ref")
    t_new, b, st = _run(binary, base, chunks, args, dirpath, "batch", threads, env_extra, client)
    assert len(a) == len(b) and len(a) > 0
    bad = [(x, y) for x, y in zip(a, b) if x != y]
    assert not bad, f"{len(bad)} SAM records differ, first:\nref   {bad[0][0][:400]}\nbatch {bad[0][1][:400]}"
    assert st is not None and st.get("driver") == "batch", "driver wrote no counts"
    assert st["reads"] > 0 and st["exact_sweep"][0] > 0
    for k in ("exact_sweep", "one_mm", "seed_search", "extend", "get_offset", "ungapped", "sw_dp"):
        if k not in cpu_ok:
            assert st[k][1] == 0, f"{k}: {st[k][1]} CPU fallbacks"
    return t_ref, t_new, len(a), st


CASES = [
    ("sensitive", [], 1500),                       # configs[1] policy
    ("local", ["--local"], 1000),                  # configs[3]
    ("very_sensitive", ["--very-sensitive"], 800),
    ("k5", ["-k", "5"], 800),                      # -k mode (no -M tightening)
    ("mp_rdg", ["--mp", "4,2", "--rdg", "4,2", "--score-min", "L,-0.8,-0.8"], 800),
    ("norc", ["--norc"], 600),
]


@pytest.mark.parametrize("name,args,n", CASES, ids=[c[0] for c in CASES])
def test_batch_sam_parity_cpu(indexes, tmp_path, name, args, n):
    _need(rs.SERVER, rs.CLIENT, SRV_BATCH_STUB)
    base, idx = indexes["synth"]
    chunks = _reads(idx, n, 7, str(tmp_path))
    _, _, nrec, st = compare(SRV_BATCH_STUB, base, chunks, args, str(tmp_path))
    assert st["sw_dp"][0] > 0


PAIRED_CASES = [
    ("paired", [], 800),                           # configs[2] policy, --end-to-end
    ("paired_vs", ["--very-sensitive"], 500),      # configs[4] policy
    ("paired_local", ["--local"], 400),
    ("paired_nomixed", ["-I", "100", "-X", "300", "--no-mixed"], 400),
    ("paired_ff_nodisc", ["--ff", "--no-discordant"], 300),
    ("paired_k3", ["-k", "3"], 300),
]


@pytest.mark.parametrize("name,args,n", PAIRED_CASES, ids=[c[0] for c in PAIRED_CASES])
def test_batch_sam_parity_paired_cpu(indexes, tmp_path, name, args, n):
    """extendSeedsPaired restated (anchor + mate-search DPs): SAM equals the stock server's."""
    _need(rs.SERVER, rs.CLIENT, SRV_BATCH_STUB)
    base, idx = indexes["synth"]
    chunks = _reads(idx, n, 29, str(tmp_path), paired=True)
    _, _, _, st = compare(SRV_BATCH_STUB, base, chunks, args, str(tmp_path))
    assert st["sw_dp"][0] > 0


def test_batch_lambda_pairs_cpu(indexes, tmp_path):
    """lambda example pairs (example/reads/reads_{1,2}.fq), the first 2 000."""
    _need(rs.SERVER, rs.CLIENT, SRV_BATCH_STUB, *LAMBDA_PE)
    compare(SRV_BATCH_STUB, indexes["lambda"], [["-1", LAMBDA_PE[0], "-2", LAMBDA_PE[1], "-u", "2000"]], [],
            str(tmp_path))


def test_batch_no_speculation_cpu(indexes, tmp_path):
    """BT2G_SPEC_DPS=1: every DP asked when the loop reaches it (no table reuse)."""
    _need(rs.SERVER, rs.CLIENT, SRV_BATCH_STUB)
    base, idx = indexes["synth"]
    chunks = _reads(idx, 800, 17, str(tmp_path))
    _, _, _, st = compare(SRV_BATCH_STUB, base, chunks, [], str(tmp_path), env_extra={"BT2G_SPEC_DPS": "1"})
    assert st["dp"][0] == 0


def test_batch_dp_reruns_cpu(indexes, tmp_path):
    """Tiny first-pass room (BT2G_DP_MAXEDIT=2 edits per alignment; two lanes per
    driver): DPs whose alignments have more edits run again with room for all,
    and the SAM is the same."""
    _need(rs.SERVER, rs.CLIENT, SRV_BATCH_STUB)
    base, idx = indexes["synth"]
    chunks = _reads(idx, 800, 19, str(tmp_path))
    _, _, _, st = compare(SRV_BATCH_STUB, base, chunks, [], str(tmp_path),
                          env_extra={"BT2G_DP_MAXEDIT": "2", "BT2G_LANES": "2"})
    assert st["dp_again"] > 0


def test_batch_no_services_cpu(indexes, tmp_path):
    """BT2G_SERVICES=0: every driver makes its own engine calls, one kind after another."""
    _need(rs.SERVER, rs.CLIENT, SRV_BATCH_STUB)
    base, idx = indexes["synth"]
    chunks = _reads(idx, 800, 13, str(tmp_path))
    compare(SRV_BATCH_STUB, base, chunks, [], str(tmp_path), threads=3, env_extra={"BT2G_SERVICES": "0"})


def test_batch_cpu_fallback_cpu(indexes, tmp_path):
    """-N 1 seeds (the engine's seed search is exact-only) and --ignore-quals (a
    mismatch model the engines do not implement): the driver runs the
    reference's own code for those stages; SAM unchanged."""
    _need(rs.SERVER, rs.CLIENT, SRV_BATCH_STUB)
    base, idx = indexes["synth"]
    chunks = _reads(idx, 500, 19, str(tmp_path))
    compare(SRV_BATCH_STUB, base, chunks, ["-N", "1", "--ignore-quals"], str(tmp_path),
            cpu_ok=("seed_search", "one_mm", "ungapped", "sw_dp"))


def test_batch_longreads_cpu(indexes, tmp_path):
    """configs[0]: lambda, example/reads/longreads.fq (6 000 reads of 40-2 561 bp)."""
    _need(rs.SERVER, rs.CLIENT, SRV_BATCH_STUB, LONGREADS)
    compare(SRV_BATCH_STUB, indexes["lambda"], [["-U", LONGREADS]], [], str(tmp_path),
            cpu_ok=("exact_sweep", "seed_search", "extend", "sw_dp"))


def test_batch_many_drivers_cpu(indexes, tmp_path):
    """-p 6 drivers, two devices (BT2G_DEVICES=0,1: an index replica each)."""
    _need(rs.SERVER, rs.CLIENT, SRV_BATCH_STUB)
    base, idx = indexes["synth"]
    chunks = _reads(idx, 3000, 23, str(tmp_path))
    compare(SRV_BATCH_STUB, base, chunks, [], str(tmp_path), threads=6, env_extra={"BT2G_DEVICES": "0,1"})


GPU_CASES = [
    ("sensitive", [], 20000, False),
    ("local", ["--local"], 10000, False),
    ("very_sensitive", ["--very-sensitive"], 5000, False),
    ("paired", [], 8000, True),
    ("paired_vs", ["--very-sensitive"], 4000, True),
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,args,n,paired", GPU_CASES, ids=[c[0] for c in GPU_CASES])
def test_batch_sam_parity_gpu(indexes, tmp_path, name, args, n, paired):
    _need(rs.SERVER, rs.CLIENT, SRV_BATCH)
    base, idx = indexes["synth"]
    chunks = _reads(idx, n, 7, str(tmp_path), paired=paired)
    t_ref, t_new, nrec, st = compare(SRV_BATCH, base, chunks, args, str(tmp_path), threads=8)
    print(f"\n[{name}] {nrec} records identical; stock {t_ref:.2f}s, batch {t_new:.2f}s; {st}")


@pytest.mark.gpu
def test_batch_lambda_pairs_gpu(indexes, tmp_path):
    _need(rs.SERVER, rs.CLIENT, SRV_BATCH, *LAMBDA_PE)
    compare(SRV_BATCH, indexes["lambda"], [["-1", LAMBDA_PE[0], "-2", LAMBDA_PE[1]]], [], str(tmp_path), threads=8)


@pytest.mark.gpu
def test_batch_longreads_gpu(indexes, tmp_path):
    _need(rs.SERVER, rs.CLIENT, SRV_BATCH, LONGREADS)
    t_ref, t_new, nrec, st = compare(SRV_BATCH, indexes["lambda"], [["-U", LONGREADS]], [], str(tmp_path),
                                     cpu_ok=("exact_sweep", "seed_search", "extend", "sw_dp"))
    print(f"\n[longreads] {nrec} records identical; stock {t_ref:.2f}s, batch {t_new:.2f}s; {st}")


def _client_inputs(idx, dirpath):
    """Reads for the client checks: FASTQ chunks, and the same reads as FASTA and tab6."""
    import bench
    r, q = bench.make_pairs(idx.ref_codes, 3000, 150, 31)
    n = 3000
    acgt = b"ACGTN"
    fa = os.path.join(dirpath, "r.fa")
    t6 = os.path.join(dirpath, "r.tab6")
    with open(fa, "wb") as f:
        f.write(b"".join(b">f%d\n%s\n" % (i, bytes(acgt[c] for c in r[i])) for i in range(n)))
    with open(t6, "wb") as f:
        f.write(b"".join(b"t%d/1\t%s\t%s\tt%d/2\t%s\t%s\n" % (i, bytes(acgt[c] for c in r[i]), bytes(q[i]), i,
                                                               bytes(acgt[c] for c in r[n + i]), bytes(q[n + i]))
                         for i in range(n)))
    return [["-f", "-U", fa], ["--tab6", t6]]


@pytest.mark.parametrize("fmt", [0, 1], ids=["fasta", "tab6"])
def test_batch_native_client_cpu(indexes, tmp_path, fmt):
    """Row (f)-4 on the stand-in: bt2g-client into the batch server, the reference
    client into the stock server -- same SAM (FASTA and paired/unpaired-mixed
    tab6 inputs; FASTQ in the GPU case and bench.py's sam_parity)."""
    _need(rs.SERVER, rs.CLIENT, SRV_BATCH_STUB, rs.NATIVE_CLIENT)
    base, idx = indexes["synth"]
    compare(SRV_BATCH_STUB, base, [_client_inputs(idx, str(tmp_path))[fmt]], [], str(tmp_path),
            client=rs.NATIVE_CLIENT)


@pytest.mark.gpu
def test_batch_native_client_gpu(indexes, tmp_path):
    """Row (f)-4 on the GPU box: the batch server on the engines fed by bt2g-client
    (FASTQ chunks of unpaired reads and pairs, FASTA, tab6) against the stock
    server fed by the reference client (bowtie2-align-l)."""
    _need(rs.SERVER, rs.CLIENT, SRV_BATCH, rs.NATIVE_CLIENT)
    base, idx = indexes["synth"]
    chunks = _reads(idx, 12000, 37, str(tmp_path)) + _reads(idx, 3000, 41, str(tmp_path), paired=True)
    compare(SRV_BATCH, base, chunks, [], str(tmp_path), threads=8, client=rs.NATIVE_CLIENT)
    for inp in _client_inputs(idx, str(tmp_path)):
        compare(SRV_BATCH, base, [inp], [], str(tmp_path), threads=8, client=rs.NATIVE_CLIENT)
