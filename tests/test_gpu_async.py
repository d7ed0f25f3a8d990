"""GPU: the host-sync-free BQ search (gvdb_index_search_device returns after
enqueueing; every fallback runs on the device).

* k_select's tie path: more than 8192 rows tied at the R-th distance inside the
  candidate buffer -> radix select over the row index keeps the reference's
  stable order (quantization.rs:165-179).
* k_select's device-side rescan: candidate-buffer overflow (and, forced, every
  query) -> exact all-rows top-R in the select block.
* NaN scores: the _device form marks the query GVDB_N_POISONED, the host form
  raises QuantizationError (the reference's sort panics).
* Pooled workspaces reused across streams with no host sync in between.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g(gvdb_mod):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return gvdb_mod


def same_f32(a, b):
    return np.asarray(a, np.float32).tobytes() == np.asarray(b, np.float32).tobytes()


def prototype_rows(seed, n, d, groups):
    """Rows sharing their sign pattern (hence their BQ code) within a group;
    small positive jitter keeps the cosines distinct."""
    r = np.random.default_rng(seed)
    proto = np.sign(r.standard_normal((groups, d))).astype(np.float32)
    proto[proto == 0] = 1.0
    x = proto[r.integers(0, groups, n)] * (1.0 + 0.2 * r.random((n, d), dtype=np.float32))
    return x.astype(np.float32)


def check_vs_oracle(g, oracle_mod, x, Q, R, k):
    ix = g.GpuVectorIndex(dimension=x.shape[1])
    ix.add_batch(np.arange(x.shape[0], dtype=np.uint64), x)
    ids, sc, n = ix.search_batch(Q, k, g.SearchParams(rescore_count=R))
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R, kind=0)
    assert (n == k).all()
    assert (ids == ri[:, :k]).all()
    assert same_f32(sc, rs[:, :k])
    return ix


def test_select_ties_beyond_lds_radix_path(g, oracle_mod):
    """200K rows in 22 code groups (~9.1K identical codes each), R = 1000: the
    candidate buffer (exact threshold, capacity 8R + 2048) holds the whole tied
    group, more than the 8192-key LDS sort -> radix select of the first
    R tied rows in row order."""
    x = prototype_rows(501, 200_000, 64, 22)
    Q = np.random.default_rng(502).standard_normal((4, 64)).astype(np.float32)
    Q[0], Q[1] = x[0], x[5]  # their own group is the only one at distance 0
    check_vs_oracle(g, oracle_mod, x, Q, 1000, 10)


def test_select_buffer_overflow_rescans_on_device(g, oracle_mod):
    """Same data, R = 100: the tied group overflows the 2848-entry buffer, so the
    select block answers with the exact all-rows rescan."""
    x = prototype_rows(503, 200_000, 64, 22)
    Q = np.random.default_rng(504).standard_normal((3, 64)).astype(np.float32)
    check_vs_oracle(g, oracle_mod, x, Q, 100, 10)


@pytest.mark.parametrize("N,D,B", [(50_000, 768, 3), (300_001, 128, 2)])
def test_forced_rescan_matches_oracle(g, oracle_mod, monkeypatch, N, D, B):
    r = np.random.default_rng(505 + N)
    x = r.standard_normal((N, D)).astype(np.float32)
    x[17] = x[4242]  # an exact duplicate pair: tie in Hamming and cosine
    Q = r.standard_normal((B, D)).astype(np.float32)
    Q[0] = x[4242]
    monkeypatch.setenv("GVDB_FORCE_RESCAN", "1")
    check_vs_oracle(g, oracle_mod, x, Q, 100, 10)


def test_nan_query_poisons_device_result(g):
    import torch

    N, D, k = 20_000, 64, 5
    x = np.random.default_rng(506).standard_normal((N, D)).astype(np.float32)
    Q = np.random.default_rng(507).standard_normal((3, D)).astype(np.float32)
    Q[1, 7] = np.nan
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    q = torch.from_numpy(Q).cuda()
    oi = torch.zeros((3, k), dtype=torch.int64, device="cuda")
    osc = torch.zeros((3, k), dtype=torch.float32, device="cuda")
    on = torch.zeros(3, dtype=torch.int32, device="cuda")
    ix.search_device(q, k, oi, osc, on, g.SearchParams(rescore_count=100))
    torch.cuda.synchronize()
    n = on.cpu().numpy().view(np.uint32)
    assert n[1] == g._ffi.GVDB_N_POISONED and n[0] == k and n[2] == k
    with pytest.raises(g.QuantizationError):
        ix.search_batch(Q, k, g.SearchParams(rescore_count=100))


def test_device_search_interleaved_streams_no_sync(g):
    """Alternate batch-1 and batch-256 device searches over two streams with no
    host sync between them; every result equals its synchronous twin."""
    import torch

    N, D, k, R = 400_000, 768, 10, 100
    r = np.random.default_rng(508)
    x = r.standard_normal((N, D)).astype(np.float32)
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    sp = g.SearchParams(rescore_count=R)
    batches = [torch.from_numpy(r.standard_normal((b, D)).astype(np.float32)).cuda() for b in (1, 256, 1, 7, 256, 1)]
    want = []
    for q in batches:
        ids, sc, n = ix.search_batch(q.cpu().numpy(), k, sp)
        want.append((ids, sc, n))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    torch.cuda.synchronize()
    for rep in range(3):
        for i, q in enumerate(batches):
            st = streams[(i + rep) % 2]
            with torch.cuda.stream(st):
                oi = torch.empty((q.shape[0], k), dtype=torch.int64, device="cuda")
                osc = torch.empty((q.shape[0], k), dtype=torch.float32, device="cuda")
                on = torch.empty(q.shape[0], dtype=torch.int32, device="cuda")
                ix.search_device(q, k, oi, osc, on, sp, stream=st.cuda_stream)
                outs.append((i, oi, osc, on))
    torch.cuda.synchronize()
    for i, oi, osc, on in outs:
        ids, sc, n = want[i]
        assert (oi.cpu().numpy().view(np.uint64) == ids).all()
        assert same_f32(osc.cpu().numpy(), sc)
        assert (on.cpu().numpy() == n).all()
