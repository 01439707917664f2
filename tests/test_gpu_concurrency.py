"""Several threads, each driving its own context on one index (bt2g_open_shared),
as the drop-in binding's dispatchers do (integration/bt2g_seams.cpp): every
host-pointer call must return exactly what the same call returns alone.

This pins the wrappers' scratch: a device memory pool shared by threads handed
overlapping blocks to concurrent calls (wrong hits, then illegal addresses, in
the 1024-worker drop-in run); the wrappers now use a per-context arena."""
import threading

import numpy as np
import pytest

from conftest import get_index

pytestmark = pytest.mark.gpu


def _work(e, reads, quals, lens, minsc, sl):
    """One round of FM calls over the reads in slice `sl`."""
    r, q, ln = reads[sl], quals[sl], lens[sl]
    ex = e.exact_sweep(r, ln)
    seeds = e.seed_search(r, ln, 22, 15, 0, 16)
    hits, cnt, ops, _ = e.one_mm(r, q, ln, minsc[sl], False, cap=64)
    hits = hits.copy()
    hits[np.arange(hits.shape[1])[None, :] >= cnt[:, None]] = 0   # slots past a read's count are unspecified
    return ex, seeds[0], seeds[1], hits, cnt, ops


def test_shared_contexts_threads_match_serial():
    import bt2g
    import synth
    idx = get_index("synth")
    gen = np.concatenate(idx.ref_codes)
    n = 6000
    reads, quals, _, _ = synth.reads(777, gen, n, 150, sub=0.01, nrate=0.002)
    lens = np.full(n, 150, np.uint32)
    minsc = np.full(n, -60, np.int32)
    base = bt2g.Engine(index=idx)
    engines = []
    try:
        # batches of ragged sizes, as the dispatchers form them
        rng = np.random.default_rng(5)
        cuts = np.unique(np.concatenate([[0, n], rng.integers(1, n, 40)]))
        slices = [slice(int(a), int(b)) for a, b in zip(cuts[:-1], cuts[1:])]
        want = [_work(base, reads, quals, lens, minsc, sl) for sl in slices]
        engines += [base.shared() for _ in range(6)]
        got = [None] * (len(slices) * len(engines))
        errs = []

        def run(t):
            try:
                for rep in range(len(slices)):
                    k = (rep + 7 * t) % len(slices)        # threads on different batches at once
                    got[t * len(slices) + k] = _work(engines[t], reads, quals, lens, minsc, slices[k])
            except Exception as ex:                       # noqa: BLE001
                errs.append(repr(ex))

        th = [threading.Thread(target=run, args=(t,)) for t in range(len(engines))]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=240)
        assert not errs, errs[:3]
        for t in range(len(engines)):
            for k in range(len(slices)):
                g, w = got[t * len(slices) + k], want[k]
                assert g is not None, (t, k)
                for a, b in zip(g, w):
                    assert np.array_equal(a, b), (t, k)
    finally:
        for e in engines:
            e.close()
        base.close()


def test_shared_context_close_order():
    """A shared context reports the index's HBM bytes, and the index owner cannot
    be closed while a shared context still uses its index."""
    import bt2g
    base = bt2g.Engine(index=get_index("lambda"))
    sh = base.shared()
    try:
        assert sh.info()[12] == base.info()[12] > 0
        with pytest.raises(bt2g.Bt2gError):
            base.close()
        assert base.h                               # still open and usable
        assert base.info()[0] == sh.info()[0]
    finally:
        sh.close()
        base.close()
    assert not base.h
