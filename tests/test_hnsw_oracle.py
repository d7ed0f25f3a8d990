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


def test_recall_curve_converges_at_d768(oracle_mod):
    """Pins the restatement at the north-star width (Missing 1): on
    50K x 768 unit rows (i.i.d. N(0,1), L2-normalised: the bench's data, the
    hardest case for a graph search) recall@10 rises with ef_search and reaches
    >= 0.95 at ef = N/10, so the low recall at 1M-10M rows is the data, not a
    restatement bug.  The same curve (and one for un-normalised rows) is
    recorded by scripts/hnsw_recall_curve.py in profiles/r06/."""
    n, d = 50_000, 768
    rng = np.random.default_rng(50_000)
    x = rng.standard_normal((n, d)).astype(np.float32)
    x /= np.linalg.norm(x.astype(np.float64), axis=1, keepdims=True).astype(np.float32)
    q = rng.standard_normal((64, d)).astype(np.float32)
    q /= np.linalg.norm(q.astype(np.float64), axis=1, keepdims=True).astype(np.float32)
    gt = np.argsort(-(q.astype(np.float64) @ x.T.astype(np.float64)), axis=1, kind="stable")[:, :10]
    h = oracle_mod.Hnsw(x, threads=8)
    curve = []
    for ef in (10, 100, 400, 1000, n // 10):
        ids, _, cnt = h.search(q, k=10, ef_search=ef, threads=8)
        assert np.all(cnt == 10)
        curve.append(_recall(ids.astype(np.int64), gt))
    assert all(b >= a - 0.01 for a, b in zip(curve, curve[1:])), curve
    assert curve[0] < 0.5 and curve[-1] >= 0.95, curve
