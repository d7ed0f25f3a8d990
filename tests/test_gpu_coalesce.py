"""Batch-1 request coalescing (gvdb_coalescer_*, csrc/gvdb_coalesce.cpp):
many threads each search ONE query -- the reference's concurrent readers of
Arc<RwLock<dyn VectorIndex>> (src/lib.rs:238) running HnswVectorIndex::search
(src/index.rs:212-231) -- and concurrent queries share batched searches.
Every caller's ids and score bits equal its own serial search, which equals
the oracle's multi_stage_search."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g(gvdb_mod):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return gvdb_mod


@pytest.mark.parametrize("threads,mode", [(1, 0), (8, 0), (32, 0), (16, 1)])
def test_coalesced_equals_serial(g, oracle_mod, threads, mode):
    N, D, k, R = 60_000, 256, 10, 100
    r = np.random.default_rng(7)
    x = r.standard_normal((N, D)).astype(np.float32)
    x[100:140] = x[3]  # ties
    Q = r.standard_normal((threads * 6, D)).astype(np.float32)
    Q[0] = x[3]
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    sp = g.SearchParams(mode=mode, rescore_count=R)
    ser = [ix.search_batch(Q[i:i + 1], k, sp) for i in range(len(Q))]
    co = g.RequestCoalescer(ix, D, k, sp)
    got = [None] * len(Q)
    barrier = threading.Barrier(threads)

    def worker(t):
        barrier.wait()
        for i in range(t, len(Q), threads):
            got[i] = co.search(Q[i])

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    batches, queries, largest = co.stats()
    co.close()
    assert queries == len(Q)
    if threads >= 8:
        assert batches < len(Q), "no query was coalesced"
    for i in range(len(Q)):
        ids, sc, n = got[i]
        si, ss, sn = ser[i]
        assert n == sn[0] == k
        assert (ids == si[0]).all() and sc.tobytes() == ss[0].tobytes(), i
    if mode == 0:  # and the reference restatement
        ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R)
        for i in range(len(Q)):
            assert (got[i][0] == ri[i, :k]).all() and got[i][1].tobytes() == rs[i, :k].tobytes()


def test_coalescer_errors(g):
    D = 64
    ix = g.GpuVectorIndex(dimension=D)
    co = g.RequestCoalescer(ix, D, 5)
    with pytest.raises(g.IndexNotBuilt):  # empty index: the reference's IndexNotBuilt (index.rs:213)
        co.search(np.zeros(D, np.float32))
    with pytest.raises(g.DimensionMismatch):
        co.search(np.zeros(D + 1, np.float32))
    co.close()


@pytest.mark.parametrize("ratio", [None, 0.1])
def test_nan_query_fails_only_its_caller(g, ratio):
    """A query with a NaN poisons only its own result: the other callers batched
    with it still get exactly their serial results (one
    QuantizationError used to fail the whole coalesced batch).  ratio=0.1 is the
    reference's default depth (the certified path, sent to the B x R rerank by the
    poisoned query)."""
    N, D, k = 100_000, 256, 10  # R = 0.1 N = 10000 > 8192: the certified default depth
    r = np.random.default_rng(11)
    x = r.standard_normal((N, D)).astype(np.float32)
    Q = r.standard_normal((48, D)).astype(np.float32)
    bad = {5, 17, 40}
    for i in bad:
        Q[i, 3] = np.nan
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    sp = g.SearchParams(rescore_count=100) if ratio is None else g.SearchParams(rescore_ratio=ratio)
    ser = {}
    for i in range(len(Q)):
        if i in bad:
            with pytest.raises(g.QuantizationError):
                ix.search_batch(Q[i:i + 1], k, sp)
        else:
            ser[i] = ix.search_batch(Q[i:i + 1], k, sp)
    co = g.RequestCoalescer(ix, D, k, sp)
    got, errs = [None] * len(Q), [None] * len(Q)
    threads = 16
    barrier = threading.Barrier(threads)

    def worker(t):
        barrier.wait()
        for i in range(t, len(Q), threads):
            try:
                got[i] = co.search(Q[i])
            except g.VectorDbError as e:
                errs[i] = e

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    batches, queries, _ = co.stats()
    co.close()
    assert batches < len(Q), "no query was coalesced"
    for i in range(len(Q)):
        if i in bad:
            assert isinstance(errs[i], g.QuantizationError), i
        else:
            assert errs[i] is None, (i, errs[i])
            ids, sc, n = got[i]
            si, ss, sn = ser[i]
            assert n == sn[0] == k
            assert (ids == si[0]).all() and sc.tobytes() == ss[0].tobytes(), i
