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
