"""Multi-rank path of bench.py on CPU (gloo, world size 2): per-rank read
shards are distinct and deterministic, and the one collective (max time, sum
of aligned reads) combines them as the GPU run does over RCCL."""
import os
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    parts, _ = bench.make_genome(0.2, seed=7)
    reads, _ = bench.make_reads(parts, 64, 50, bench.shard_seed(rank))
    elapsed, n = bench.combine_ranks(1.0 + rank, 10 + rank, torch.device("cpu"))
    q.put((rank, elapsed, n, reads.sum(), int(reads[0, :8].tolist()[0])))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_and_reduction():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, e0, n0, s0, _), (r1, e1, n1, s1, _) = out
    assert e0 == e1 == 2.0            # max over ranks
    assert n0 == n1 == 21             # sum over ranks
    assert s0 != s1                   # distinct shards


def test_single_rank_is_identity():
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
    import torch
    import bench
    assert bench.combine_ranks(3.5, 7, torch.device("cpu")) == (3.5, 7)
    parts, _ = bench.make_genome(0.2, seed=7)
    a, _ = bench.make_reads(parts, 16, 50, bench.shard_seed(0))
    b, _ = bench.make_reads(parts, 16, 50, bench.shard_seed(0))
    assert np.array_equal(a, b)


def _sched_worker(rank, world, port, base, q):
    """One rank of bench.py's north-star path: its own read shard through its own
    batch server (the CPU stand-in of the engines), then the one reduction."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "bowtie2-server_amd", "tools")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import tempfile
    import types
    import torch
    import torch.distributed as dist
    import bench
    import bt2_index as bi
    from oracle import ref_server as rs
    dist.init_process_group("gloo", rank=rank, world_size=world)
    idx = bi.read_index(base)
    r, qq = bench.make_reads(idx.ref_codes, 1500, 150, bench.shard_seed(rank))
    args = types.SimpleNamespace(mode="ee", preset="sensitive", reads=1500, drivers=2, clients=2, warmup=1,
                                 warmup_chunks=1, steps=1, rank_mem_gb=0.0)
    stub = os.path.join(rs.REF_DIR, "bowtie2-align-server-batch-stub")
    sc = bench.schedule_run(args, rank, world, 0, base, r, qq, tempfile.mkdtemp(), binary=stub)
    el, n = bench.combine_ranks(sc["elapsed"], sc["aligned"], torch.device("cpu"))
    q.put((rank, sc["elapsed"], sc["aligned"], el, n, sc["slots_per_driver"], sc["stats"]["slots"],
           bench.count_aligned(sc["outs"], False)))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_batch_servers_reduce():
    """World size 2 over gloo through bench.schedule_run: each rank runs its own
    batch server (bowtie2-align-server-batch-stub) on its own shard within the
    per-rank host-memory budget (slots per driver from bench.slots_per_driver),
    and the aligned counts sum / the times max over ranks."""
    import tempfile
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "bowtie2-server_amd", "tools")]
    import bench
    import bt2_index as bi
    import synth
    from oracle import ref_server as rs
    if not os.path.exists(os.path.join(rs.REF_DIR, "bowtie2-align-server-batch-stub")):
        pytest.skip("oracle/_ref servers not built")
    g = synth.genome(9, 100_000, n_repeats=10, rep_len=1500, n_copies=3, n_runs=2)
    base = os.path.join(tempfile.mkdtemp(), "g")
    bi.write_index(base, bi.build_index([g], names=[b"chr"]))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + os.getpid() % 1000
    procs = [ctx.Process(target=_sched_worker, args=(r, 2, port, base, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, e0, a0, el0, n0, sp0, sl0, c0), (_, e1, a1, el1, n1, sp1, sl1, c1) = out
    assert n0 == n1 == a0 + a1 and 2 * 1200 < a0 + a1 <= 3000
    assert el0 == el1 == max(e0, e1)
    assert a0 == c0 and a1 == c1
    assert sp0 == sp1 == bench.slots_per_driver(2, 2) and sl0 <= 2 * sp0 and sl1 <= 2 * sp1
