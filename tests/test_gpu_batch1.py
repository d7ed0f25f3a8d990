"""GPU: the batch-1 fast path (k_b1_sample -> k_b1_scan -> k_b1_tail: three
launches, self-cleaning state, no host round trip) against the oracle's
multi_stage_search (quantization.rs:151-193) and HnswVectorIndex semantics
(index.rs:212-231: k hits, orphans dropped after take(k)).

Every case runs single queries one after another through the SAME pooled
workspace, so a state left dirty by one call would corrupt the next.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g(gvdb_mod):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return gvdb_mod


def rows(seed, n, d, dup=0):
    r = np.random.default_rng(seed)
    x = r.standard_normal((n, d)).astype(np.float32)
    for i in range(dup):
        x[(7 * i + 11) % n] = x[(13 * i + 3) % n]
    return x


def same_f32(a, b):
    return np.asarray(a, np.float32).tobytes() == np.asarray(b, np.float32).tobytes()


@pytest.mark.parametrize("N,D,R,k,metric", [
    (1_000, 64, 100, 10, 0),        # whole shard as the "sample" (exact threshold)
    (300_000, 768, 100, 10, 0),     # sampled threshold (N > 262144)
    (300_000, 768, 100, 10, 1),     # L2 scores (VectorPoint::distance)
    (300_000, 768, 100, 10, 2),     # 1 - cosine
    (270_000, 1000, 1000, 50, 0),   # D not a multiple of 64 / 128, larger R
    (100_000, 1024, 4096, 10, 0),   # the largest R / D of the fused tail
    (5_000, 100, 17, 40, 0),        # k > R: R becomes k
    (262_144, 32, 64, 64, 0),       # boundary of the exact-threshold regime, k = R
])
def test_batch1_matches_oracle(g, oracle_mod, N, D, R, k, metric):
    x = rows(N + D + R, N, D, dup=40)
    Q = rows(D + 11, 6, D)
    Q[2] = x[N // 3]            # exact hit
    Q[3] = x[(13 * 5 + 3) % N]  # a duplicated row: two equal candidates
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64) * 5 + 1, x)
    sp = g.SearchParams(metric=metric, rescore_count=R)
    Reff = max(R, k)
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, Reff,
                                                   kind=metric)
    for b in range(len(Q)):
        ids, sc, n = ix.search_batch(Q[b:b + 1], k, sp)
        kk = min(k, Reff, N)
        assert n[0] == kk
        assert (ids[0, :kk] == ri[b, :kk] * 5 + 1).all(), b
        assert same_f32(sc[0, :kk], rs[b, :kk]), b


def test_batch1_equals_general_path(g, monkeypatch):
    """GVDB_B1=0 (the general multi-kernel path, read once per process) is not
    switchable here, so compare batch-1 against the same query inside a
    batch of 2 (which always takes the general path)."""
    N, D, R, k = 400_000, 768, 100, 10
    x = rows(91, N, D, dup=30)
    Q = rows(92, 8, D)
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    sp = g.SearchParams(rescore_count=R)
    for b in range(0, 8, 2):
        i2, s2, n2 = ix.search_batch(Q[b:b + 2], k, sp)
        for j in range(2):
            i1, s1, n1 = ix.search_batch(Q[b + j:b + j + 1], k, sp)
            assert (i1[0] == i2[j]).all() and same_f32(s1[0], s2[j]) and n1[0] == n2[j]


def test_batch1_orphans_and_nan(g):
    """Re-added ids shadow their old rows (dropped after take(k)); a NaN
    query poisons the device result and raises on the host form."""
    import torch

    N, D = 300_000, 128
    x = rows(93, N, D)
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    q = x[1234].copy()
    ix.add_batch(np.array([1234], np.uint64), (x[1234:1235] * 0.5).astype(np.float32))  # shadows row 1234
    ids, sc, n = ix.search_batch(q[None], 5, g.SearchParams(rescore_count=50))
    assert 1234 in ids[0, :n[0]].tolist()  # the new row (same direction, cosine 1)
    assert n[0] <= 5
    bad = q.copy()
    bad[3] = np.nan
    with pytest.raises(g.QuantizationError):
        ix.search_batch(bad[None], 5, g.SearchParams(rescore_count=50))
    qd = torch.from_numpy(bad[None].copy()).cuda()
    oi = torch.zeros((1, 5), dtype=torch.int64, device="cuda")
    osc = torch.zeros((1, 5), dtype=torch.float32, device="cuda")
    on = torch.zeros(1, dtype=torch.int32, device="cuda")
    ix.search_device(qd, 5, oi, osc, on, g.SearchParams(rescore_count=50))
    torch.cuda.synchronize()
    assert int(on.cpu().numpy().view(np.uint32)[0]) == g._ffi.GVDB_N_POISONED
    # the next (clean) query still works on the same pooled state
    ids2, sc2, n2 = ix.search_batch(x[77][None], 5, g.SearchParams(rescore_count=50))
    assert ids2[0, 0] == 77 and n2[0] == 5


def test_batch1_forced_rescan(g, oracle_mod, monkeypatch):
    N, D, R, k = 50_000, 256, 100, 10
    x = rows(94, N, D, dup=20)
    Q = rows(95, 3, D)
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    monkeypatch.setenv("GVDB_FORCE_RESCAN", "1")
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R, kind=0)
    for b in range(3):
        ids, sc, n = ix.search_batch(Q[b:b + 1], k, g.SearchParams(rescore_count=R))
        assert (ids[0] == ri[b, :k]).all() and same_f32(sc[0], rs[b, :k])


def test_batch1_device_pipelined_200_queries(g):
    """200 device searches back to back, no sync in between (the bench's
    batch-1 loop); results equal the host-synchronous ones."""
    import torch

    N, D, k = 500_000, 768, 10
    x = rows(96, N, D)
    Q = rows(97, 200, D)
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    sp = g.SearchParams(rescore_count=100)
    qd = torch.from_numpy(Q).cuda()
    outs = []
    for i in range(200):
        oi = torch.empty((1, k), dtype=torch.int64, device="cuda")
        osc = torch.empty((1, k), dtype=torch.float32, device="cuda")
        ix.search_device(qd[i:i + 1], k, oi, osc, None, sp)
        outs.append((oi, osc))
    torch.cuda.synchronize()
    ids, sc, n = ix.search_batch(Q[:20], k, sp)  # general path for 20 of them
    for i in range(20):
        assert (outs[i][0].cpu().numpy().view(np.uint64)[0] == ids[i]).all()
        assert same_f32(outs[i][1].cpu().numpy()[0], sc[i])
