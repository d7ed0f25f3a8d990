"""GPU: the sharded search path (ShardManager::search_vectors, shard.rs:760-786,
within one node) through the C ABI.

* G = 8 shard indices on ONE GPU (config 4's split at reduced N, D = 3072):
  per-shard candidates written into the blocks one all-gather would deliver,
  then the packed merge with G = 8 -- equal to one index over the whole
  corpus and to the oracle's multi_stage_search over the concatenation.
* The RCCL communicator inside libgvdb (gvdb_comm_* +
  gvdb_index_search_sharded_device) with one rank: equal to the single-device
  search, including a shard with fewer rows than R.  More ranks need more
  GPUs (one RCCL rank per device); the driver's multi-GPU bench runs them.
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


def single_device(g, x, Q, R, k):
    import torch

    ix = g.GpuVectorIndex(dimension=x.shape[1])
    ix.add_batch(np.arange(x.shape[0], dtype=np.uint64), x)
    q = torch.from_numpy(Q).cuda()
    oi = torch.zeros((len(Q), k), dtype=torch.int64, device="cuda")
    osc = torch.zeros((len(Q), k), dtype=torch.float32, device="cuda")
    on = torch.zeros(len(Q), dtype=torch.int32, device="cuda")
    ix.search_device(q, k, oi, osc, on, g.SearchParams(rescore_count=R))
    torch.cuda.synchronize()
    return oi.cpu().numpy().view(np.uint64), osc.cpu().numpy(), on.cpu().numpy()


def test_g8_packed_merge_d3072_equals_single_index_and_oracle(g, oracle_mod):
    """Config 4 (10M x 3072 over 8 GPUs) at 80K rows: 8 contiguous shards of
    10K rows with global-row ids, merged by gvdb_bq_shard_merge_packed_device."""
    import torch

    G, n_per, D, B, R, k = 8, 10_000, 3072, 16, 100, 10
    N = G * n_per
    x = rows(401, N, D, dup=60)
    Q = rows(402, B, D)
    Q[3] = x[12_345]           # an exact hit in shard 1
    Q[9] = x[N - 1]            # the last row of the last shard
    q = torch.from_numpy(Q).cuda()
    BR = B * R
    gathered = torch.zeros((G, 4 * BR), dtype=torch.int32, device="cuda")
    counts = torch.full((G, B), R, dtype=torch.int32, device="cuda")
    L = g.lib()
    shards = []
    for s in range(G):
        ix = g.GpuVectorIndex(dimension=D)
        ix.add_batch(np.arange(s * n_per, (s + 1) * n_per, dtype=np.uint64), x[s * n_per:(s + 1) * n_per])
        p = gathered[s].data_ptr()
        assert L.gvdb_index_bq_candidates_device(ix._h, q.data_ptr(), B, D, R, p, p + 8 * BR, p + 12 * BR, None) == 0
        shards.append(ix)
    mi = torch.zeros((B, k), dtype=torch.int64, device="cuda")
    ms = torch.zeros((B, k), dtype=torch.float32, device="cuda")
    mn = torch.zeros(B, dtype=torch.int32, device="cuda")
    assert L.gvdb_bq_shard_merge_packed_device(gathered.data_ptr(), counts.data_ptr(), G, B, R, k, mi.data_ptr(),
                                               ms.data_ptr(), mn.data_ptr(), None) == 0
    torch.cuda.synchronize()
    got_i, got_s = mi.cpu().numpy().view(np.uint64), ms.cpu().numpy()
    si, ss, sn = single_device(g, x, Q, R, k)
    assert (got_i == si).all() and same_f32(got_s, ss) and (mn.cpu().numpy() == k).all()
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R, kind=0)
    assert (got_i == ri[:, :k]).all()
    assert same_f32(got_s, rs[:, :k])
    assert got_i[3, 0] == 12_345 and got_i[9, 0] == N - 1


@pytest.mark.parametrize("N,B", [(120_000, 64), (50, 5)])
def test_rccl_world1_equals_single_device(g, N, B):
    """gvdb_index_search_sharded_device over a 1-rank RCCL communicator (the
    all-gather is skipped, the merge reads the send block): same ids, scores
    and counts as gvdb_index_search_device; N=50 < R exercises the clamped
    shard R (stride-R block rows, counts = 50)."""
    import torch

    from gvdb.sharded import RcclShardedSearch

    D, R, k = 768, 100, 10
    x = rows(403 + N, N, D, dup=min(N // 4, 30))
    Q = rows(404, B, D)
    Q[1] = x[N // 2]
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    sh = RcclShardedSearch(ix, R, k)
    q = torch.from_numpy(Q).cuda()
    oi = torch.zeros((B, k), dtype=torch.int64, device="cuda")
    osc = torch.zeros((B, k), dtype=torch.float32, device="cuda")
    on = torch.zeros(B, dtype=torch.int32, device="cuda")
    for _ in range(2):  # the second call reuses the communicator's buffers
        sh.search_into(q, oi, osc, on)
    torch.cuda.synchronize()
    si, ss, sn = single_device(g, x, Q, R, k)
    assert (oi.cpu().numpy().view(np.uint64) == si).all()
    assert same_f32(osc.cpu().numpy(), ss)
    assert (on.cpu().numpy() == sn).all()
    sh.close()


def test_rccl_sharded_argument_checks(g):
    import ctypes as C

    import torch

    from gvdb.sharded import RcclShardedSearch

    D = 64
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(100, dtype=np.uint64), rows(405, 100, D))
    sh = RcclShardedSearch(ix, 100, 10)
    q = torch.zeros((2, D), device="cuda")
    oi = torch.zeros((2, 10), dtype=torch.int64, device="cuda")
    osc = torch.zeros((2, 10), dtype=torch.float32, device="cuda")
    L = g.lib()
    for sp in (g.SearchParams(rescore_count=0), g.SearchParams(rescore_count=5000),
               g.SearchParams(rescore_count=100, mode=1)):
        c = sp.to_c()
        st = L.gvdb_index_search_sharded_device(ix._h, sh._h, q.data_ptr(), 2, D, 10, C.byref(c), oi.data_ptr(),
                                                osc.data_ptr(), None, None)
        assert st == g._ffi.GVDB_ERR_INVALID_ARGUMENT
    w, r = C.c_int32(), C.c_int32()
    assert L.gvdb_comm_info(sh._h, C.byref(w), C.byref(r)) == 0 and (w.value, r.value) == (1, 0)
    sh.close()
