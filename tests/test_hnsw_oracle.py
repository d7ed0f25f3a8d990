"""CPU: the instant-distance HNSW restatement (oracle/hnsw_oracle.cpp), the
CPU-HNSW baseline of HnswVectorIndex (index.rs:140-154, 212-231).

Graph identity is parity-unpinned (the crate builds with rayon in parallel
from an OS-random seed); what is pinned here is the reference's own HNSW test
(query.rs:428-483: a 3-d corpus {test1: [1,0,0]} queried with [1,0.1,0] ->
top-1 test1), the distance definition (index.rs:64-79) and recall@10 against
exact ground truth."""
import numpy as np
import pytest


def _truth(q, x, k):
    d2 = ((q[:, None, :].astype(np.float64) - x[None, :, :]) ** 2).sum(-1)
    return np.argsort(d2, axis=1, kind="stable")[:, :k]


def _recall(ids, gt):
    return float(np.mean([len(set(a.tolist()) & set(b.tolist())) / gt.shape[1] for a, b in zip(ids, gt)]))


def test_reference_query_engine_kat(oracle_mod):
    x = np.array([[1.0, 0.0, 0.0]], np.float32)
    h = oracle_mod.Hnsw(x, threads=1)
    ids, dist, n = h.search(np.array([1.0, 0.1, 0.0], np.float32), k=5)
    assert n[0] == 1 and ids[0, 0] == 0
    assert dist[0, 0] == np.float32(np.sqrt(np.float32(0.01)))


def test_distance_is_sequential_l2(oracle_mod):
    rng = np.random.default_rng(3)
    x = rng.standard_normal((64, 100)).astype(np.float32)
    q = rng.standard_normal(100).astype(np.float32)
    h = oracle_mod.Hnsw(x, threads=1)
    ids, dist, n = h.search(q, k=64, ef_search=200)
    assert n[0] == 64  # a 64-point graph is fully reachable at ef=200
    for i, dv in zip(ids[0], dist[0]):
        assert dv == np.float32(oracle_mod.l2_distance(q, x[int(i)]))
    assert np.all(np.diff(dist[0]) >= 0)


@pytest.mark.parametrize("n,d,threads", [(3000, 16, 1), (6000, 64, 4)])
def test_recall_vs_exact(oracle_mod, n, d, threads):
    rng = np.random.default_rng(n)
    x = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((50, d)).astype(np.float32)
    h = oracle_mod.Hnsw(x, threads=threads)
    ids, _, cnt = h.search(q, k=10, threads=2)
    assert np.all(cnt == 10)
    assert _recall(ids.astype(np.int64), _truth(q, x, 10)) >= 0.9


def test_ef_search_bounds_results(oracle_mod):
    rng = np.random.default_rng(5)
    x = rng.standard_normal((500, 8)).astype(np.float32)
    h = oracle_mod.Hnsw(x, threads=2)
    _, _, cnt = h.search(rng.standard_normal((4, 8)), k=50, ef_search=20)
    assert np.all(cnt == 20)  # take(k) of an ef-sized result list
