"""The engines' one collective (bt2g_comm_* / bt2g_allreduce_counts, RCCL) on
the GPU box's one device: a single-rank communicator, whose all-reduce is the
identity.  The multi-rank reduction is covered on CPU (tests/test_multi.py,
gloo) and at round end by the driver's 8-GPU bench, which sums its counters
through this call (bench.combine_ranks)."""
import numpy as np
import pytest

from conftest import get_index

pytestmark = pytest.mark.gpu


def test_single_rank_allreduce_is_identity():
    import bt2g
    with bt2g.Engine(index=get_index("lambda")) as e:
        with pytest.raises(bt2g.Bt2gError):
            e.allreduce_counts([1, 2])                     # no communicator yet
        uid = bt2g.Engine.comm_unique_id()
        assert len(uid) == 128
        e.comm_init(1, 0, uid)
        v = np.array([0, 1, 2 ** 40 + 7, 2 ** 63 - 1], np.uint64)
        assert np.array_equal(e.allreduce_counts(v), v)
        with pytest.raises(bt2g.Bt2gError):
            e.comm_init(1, 0, uid)                         # one communicator per context
