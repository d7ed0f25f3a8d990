"""GPU: the sharded search path (ShardManager::search_vectors, shard.rs:760-786,
within one node) through the C ABI.

* The two-exchange protocol (gvdb_shard_stage1_device -> gather ->
  gvdb_shard_rerank_device -> gather -> gvdb_shard_final_device) with G = 8
  ranks emulated on ONE GPU (each rank's blocks written where an all-gather
  would put them): equal to one index over the concatenated corpus and to the
  oracle, for R = 100 and R = 1000 (G*R = 8000 > the old 4096 merge cap),
  batch 256 (FP4-MFMA stage 1), uneven shards and an EMPTY shard, D = 768 and
  the config-4 width D = 3072.
* Sharded FLAT with G = 8 at D = 3072: the ranks' exact top-k merged by
  gvdb_shard_flat_final_device == the single index's exact flat search ==
  the oracle.

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


def emulate_two_exchange(g, shards, q, D, R, k, rerank_twice=False):
    """Run the three phases for every rank on one GPU; returns the merged
    results of every rank (they must all agree).  rerank_twice: phase 2 runs
    twice on the same phase-1 scratch (it must only read it)."""
    import ctypes as C

    import torch

    L = g.lib()
    G, B = len(shards), q.shape[0]
    w1, w2, scr = C.c_uint64(), C.c_uint64(), C.c_uint64()
    L.gvdb_shard_sizes(B, R, k, D, C.byref(w1), C.byref(w2), C.byref(scr))
    g1 = torch.zeros((G, w1.value), dtype=torch.int32, device="cuda")
    g2 = torch.zeros((G, w2.value), dtype=torch.int32, device="cuda")
    scratch = torch.zeros((G, scr.value), dtype=torch.uint8, device="cuda")  # per rank (deep: members kept)
    for r, ix in enumerate(shards):
        g.check(L.gvdb_shard_stage1_device(ix._h, q.data_ptr(), B, D, R, g1[r].data_ptr(), scratch[r].data_ptr(),
                                           None))
    for _ in range(2 if rerank_twice else 1):
        for r, ix in enumerate(shards):
            g.check(L.gvdb_shard_rerank_device(ix._h, q.data_ptr(), B, D, R, k, g1.data_ptr(), G, r,
                                               scratch[r].data_ptr(), g2[r].data_ptr(), None))
    outs = []
    for _ in range(2):  # every rank runs the same final merge
        oi = torch.zeros((B, k), dtype=torch.int64, device="cuda")
        osc = torch.zeros((B, k), dtype=torch.float32, device="cuda")
        on = torch.zeros(B, dtype=torch.int32, device="cuda")
        g.check(L.gvdb_shard_final_device(g2.data_ptr(), G, B, k, oi.data_ptr(), osc.data_ptr(), on.data_ptr(), None))
        outs.append((oi, osc, on))
    torch.cuda.synchronize()
    (a, b, c), (a2, b2, c2) = outs
    assert torch.equal(a, a2) and torch.equal(b, b2) and torch.equal(c, c2)
    return a.cpu().numpy().view(np.uint64), b.cpu().numpy(), c.cpu().numpy()


@pytest.mark.parametrize("sizes,D,B,R", [
    ((9000, 11000, 0, 10000, 12500, 7000, 10000, 10500), 768, 256, 100),
    ((9000, 11000, 0, 10000, 12500, 7000, 10000, 10500), 768, 96, 1000),
    ((5000,) * 8, 3072, 32, 100),
    ((2000, 3, 2000, 2000, 1, 2000, 2000, 2000), 256, 20, 50),
    # a skewed split: rank 0 owns most of the global top-3000 (> 1024 owned
    # entries: the sorted local top-k; R > 2048: the own arrays in scratch),
    # D % 4 != 0 (the scalar row loads and folds of the rerank)
    ((30000, 500, 500, 0, 500, 500, 500, 500), 130, 8, 3000),
])
def test_two_exchange_g8_equals_single_index_and_oracle(g, oracle_mod, sizes, D, B, R):
    import torch

    k = 10
    N = sum(sizes)
    x = rows(500 + D + R, N, D, dup=80)
    bounds = np.cumsum((0,) + sizes)
    # ties across shard boundaries: equal rows in different shards
    for j in range(1, 8):
        if sizes[j] and bounds[j] > 0:
            x[bounds[j]] = x[0]
    Q = rows(501 + D, B, D)
    Q[0] = x[0]
    Q[1] = x[N - 1]
    Q[2] = x[bounds[4]]
    q = torch.from_numpy(Q).cuda()
    shards = []
    for r in range(8):
        ix = g.GpuVectorIndex(dimension=D)
        if sizes[r]:
            ix.add_batch(np.arange(bounds[r], bounds[r + 1], dtype=np.uint64), x[bounds[r]:bounds[r + 1]])
        shards.append(ix)
    got_i, got_s, got_n = emulate_two_exchange(g, shards, q, D, R, k)
    si, ss, sn = single_device(g, x, Q, R, k)
    assert (got_n == sn).all() and (got_i == si).all() and same_f32(got_s, ss)
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R, kind=0)
    assert (got_i == ri[:, :k]).all() and same_f32(got_s, rs[:, :k])


@pytest.mark.parametrize("sizes,D,B,R", [
    # the reference's default depth at shard scale (R > 8192: the deep form,
    # histogram exchange): uneven shards, an empty one, a shard smaller than the
    # LDS select (k_select's sorted list), one of 15000 rows < R (every row a
    # member through k_select_big), batch 128 (FP4-MFMA stage 1)
    ((60000, 5000, 0, 15000, 80000, 40000, 60000, 60000), 768, 128, 20000),
    ((9000, 11000, 0, 10000, 12500, 7000, 10000, 10500), 130, 8, 12000),
])
def test_deep_two_exchange_g8_equals_single_index_and_oracle(g, oracle_mod, sizes, D, B, R):
    """The deep two-exchange protocol (R > 8192) with G = 8 ranks emulated on
    one GPU: bit-identical to one index over the concatenated corpus (the
    single-device large-R path) and to the oracle's multi_stage_search."""
    import torch

    k = 10
    N = sum(sizes)
    x = rows(700 + D, N, D, dup=120)
    bounds = np.cumsum((0,) + sizes)
    for j in range(1, 8):  # equal rows across shard boundaries: cosine ties broken by corpus row
        if sizes[j] and bounds[j] > 0:
            x[bounds[j]] = x[3]
    Q = rows(701 + D, B, D)
    Q[0] = x[3]
    Q[1] = x[N - 1]
    Q[2] = x[bounds[4] + 7]
    q = torch.from_numpy(Q).cuda()
    shards = []
    for r in range(8):
        ix = g.GpuVectorIndex(dimension=D)
        if sizes[r]:
            ix.add_batch(np.arange(bounds[r], bounds[r + 1], dtype=np.uint64), x[bounds[r]:bounds[r + 1]])
        shards.append(ix)
    got_i, got_s, got_n = emulate_two_exchange(g, shards, q, D, R, k, rerank_twice=True)
    si, ss, sn = single_device(g, x, Q, R, k)
    assert (got_n == sn).all() and (got_i == si).all() and same_f32(got_s, ss)
    assert got_i[0, 0] == 3 and got_i[1, 0] == N - 1
    nq = min(B, 12)  # the oracle's stage 1 sorts the whole corpus per query
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q[:nq]), oracle_mod.quantize(x), Q[:nq], x, R,
                                                   kind=0)
    assert (got_i[:nq] == ri[:, :k]).all() and same_f32(got_s[:nq], rs[:, :k])


def deep_cert_counts(g):
    import ctypes as C

    L = g.lib()
    L.gvdb_debug_deep_cert.argtypes = [C.POINTER(C.c_uint64)]
    out = (C.c_uint64 * 2)()
    assert L.gvdb_debug_deep_cert(out) == 0
    return int(out[0]), int(out[1])


@pytest.mark.parametrize("plant,R", [(False, 16_000), (True, 16_000), (False, 24_000), (True, 24_000)])
def test_deep_certified_phase2_equals_single_index_and_oracle(g, oracle_mod, plant, R):
    """The certified deep phase 2 (shards of >= 65536 rows, k <= 32): each rank's
    local top-k comes from its exact cosine top-32 filtered by the owned-row rule
    k_shard_deep_own writes, not from reranking its ~R / G owned rows.  Equal rows
    across the shard boundary make cross-shard cosine ties.  plant: 70 rows of
    cosine ~0.85 but Hamming 400 (> T) in shard 1 for query 0 fill that rank's list,
    so rank 1 cannot certify and reranks its owned rows while rank 0 certifies;
    the merged results are the same either way.  R = 16000: the member-list form
    (a 90K-row shard's dense block exceeds the scratch's list regions); R = 24000:
    stage 1 keeps the dense block and its segment histograms in the scratch, ties at
    T are counted from them and the fallback compacts from the block (k_dense_own)."""
    import torch

    sizes, D, B, k = (70_000, 90_000), 768, 48, 10
    N = sum(sizes)
    x = rows(733, N, D, dup=100)
    x[sizes[0]] = x[5]
    x[sizes[0] + 9] = x[N - 3]
    Q = rows(734, B, D)
    Q[1] = x[5]
    Q[2] = x[N - 3]
    if plant:
        r = np.random.default_rng(92)
        base = Q[0].copy()
        small = np.argsort(np.abs(Q[0]))[:400]
        base[small] = -Q[0][small]
        for j in range(70):
            x[sizes[0] + 100 + 13 * j] = base + 0.01 * r.standard_normal(D).astype(np.float32)
    q = torch.from_numpy(Q).cuda()
    bounds = np.cumsum((0,) + sizes)
    shards = []
    for j in range(2):
        ix = g.GpuVectorIndex(dimension=D)
        ix.add_batch(np.arange(bounds[j], bounds[j + 1], dtype=np.uint64), x[bounds[j]:bounds[j + 1]])
        shards.append(ix)
    c0 = deep_cert_counts(g)
    got_i, got_s, got_n = emulate_two_exchange(g, shards, q, D, R, k, rerank_twice=True)
    c1 = deep_cert_counts(g)
    # phase 2 ran twice per rank: (certified, reranked) batches
    assert (c1[0] - c0[0], c1[1] - c0[1]) == ((2, 2) if plant else (4, 0))
    si, ss, sn = single_device(g, x, Q, R, k)
    assert (got_n == sn).all() and (got_i == si).all() and same_f32(got_s, ss)
    assert got_i[1, 0] in (5, sizes[0]) and got_i[2, 0] in (N - 3, sizes[0] + 9)
    nq = 8
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q[:nq]), oracle_mod.quantize(x), Q[:nq], x, R,
                                                   kind=0)
    assert (got_i[:nq] == ri[:, :k]).all() and same_f32(got_s[:nq], rs[:, :k])


def test_sharded_flat_g8_d3072_equals_single_index_and_oracle(g, oracle_mod):
    """Sharded FLAT (the recall-1.0 mode) at the config-4 width: 8 shards of
    9K rows (> the 65536-row MFMA floor on no shard: exact scans) and 2 shards
    of 70K (MFMA-certified tiers), ranks' exact top-k merged on the device."""
    import ctypes as C

    import torch

    D, B, k = 3072, 12, 10
    sizes = (9000, 70000, 9000, 9000, 70000, 9000, 9000, 9000)
    N = sum(sizes)
    bounds = np.cumsum((0,) + sizes)
    x = rows(601, N, D, dup=20)
    x[bounds[3]] = x[5]  # a tie across shards
    Q = rows(602, B, D)
    Q[0] = x[5]
    q = torch.from_numpy(Q).cuda()
    L = g.lib()
    wf = L.gvdb_shard_flat_words(B, k)
    gathered = torch.zeros((8, wf), dtype=torch.int32, device="cuda")
    sp = g.SearchParams(mode=1, metric=0).to_c()
    shards = []
    for r in range(8):
        ix = g.GpuVectorIndex(dimension=D)
        ix.add_batch(np.arange(bounds[r], bounds[r + 1], dtype=np.uint64), x[bounds[r]:bounds[r + 1]])
        p = gathered[r].data_ptr()
        g.check(L.gvdb_index_search_device(ix._h, q.data_ptr(), B, D, k, C.byref(sp), p, p + 8 * B * k,
                                           p + 12 * B * k, None))
        shards.append(ix)
    oi = torch.zeros((B, k), dtype=torch.int64, device="cuda")
    osc = torch.zeros((B, k), dtype=torch.float32, device="cuda")
    on = torch.zeros(B, dtype=torch.int32, device="cuda")
    g.check(L.gvdb_shard_flat_final_device(gathered.data_ptr(), 8, B, k, 0, oi.data_ptr(), osc.data_ptr(),
                                           on.data_ptr(), None))
    torch.cuda.synchronize()
    got_i, got_s, got_n = oi.cpu().numpy().view(np.uint64), osc.cpu().numpy(), on.cpu().numpy()
    full = g.GpuVectorIndex(dimension=D)
    full.add_batch(np.arange(N, dtype=np.uint64), x)
    si, ss, sn = full.search_batch(Q, k, g.SearchParams(mode=1, metric=0))
    assert (got_n == sn).all() and (got_i == si).all() and same_f32(got_s, ss)
    for b in range(B):
        ri, rs = oracle_mod.storage_vector_search(Q[b], x, k)
        assert list(got_i[b]) == list(ri) and same_f32(got_s[b], rs)


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
    side = torch.cuda.Stream()
    for it in range(3):  # later calls reuse the communicator's buffers; the last on another stream
        if it == 2:
            with torch.cuda.stream(side):
                sh.search_into(q, oi, osc, on)
            side.synchronize()
        else:
            sh.search_into(q, oi, osc, on)
    torch.cuda.synchronize()
    si, ss, sn = single_device(g, x, Q, R, k)
    assert (oi.cpu().numpy().view(np.uint64) == si).all()
    assert same_f32(osc.cpu().numpy(), ss)
    assert (on.cpu().numpy() == sn).all()
    sh.close()
    # FLAT through the same communicator path: the exact top-k
    shf = RcclShardedSearch(ix, R, k, params=g.SearchParams(mode=1, metric=0))
    shf.search_into(q, oi, osc, on)
    torch.cuda.synchronize()
    fi, fs, fn = ix.search_batch(Q, k, g.SearchParams(mode=1, metric=0))
    assert (oi.cpu().numpy().view(np.uint64) == fi).all() and same_f32(osc.cpu().numpy(), fs)
    assert (on.cpu().numpy() == fn.astype(np.int32)).all()
    shf.close()


def test_rccl_world1_deep_form_equals_single_device(g):
    """gvdb_index_search_sharded_device at R = 20000 > 8192 (the deep form:
    histogram exchange) over a 1-rank communicator: equal to the single-device
    large-R search."""
    import torch

    from gvdb.sharded import RcclShardedSearch

    N, D, B, R, k = 150_000, 768, 40, 20_000, 10
    x = rows(407, N, D, dup=40)
    Q = rows(408, B, D)
    Q[2] = x[N // 3]
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    sh = RcclShardedSearch(ix, R, k)
    q = torch.from_numpy(Q).cuda()
    oi = torch.zeros((B, k), dtype=torch.int64, device="cuda")
    osc = torch.zeros((B, k), dtype=torch.float32, device="cuda")
    on = torch.zeros(B, dtype=torch.int32, device="cuda")
    sh.search_into(q, oi, osc, on)
    sh.search_into(q, oi, osc, on)  # the communicator's buffers reused
    torch.cuda.synchronize()
    si, ss, sn = single_device(g, x, Q, R, k)
    assert (oi.cpu().numpy().view(np.uint64) == si).all()
    assert same_f32(osc.cpu().numpy(), ss)
    assert (on.cpu().numpy() == sn).all()
    assert si[2, 0] == N // 3
    sh.close()


def test_rccl_world1_empty_shard_joins_and_returns_nothing(g):
    """An empty shard still runs the protocol (no early return that would
    leave other ranks in the collective): every query gets 0 results."""
    import torch

    from gvdb.sharded import RcclShardedSearch

    D, B, k = 64, 4, 10
    ix = g.GpuVectorIndex(dimension=D)
    sh = RcclShardedSearch(ix, 100, k)
    q = torch.from_numpy(rows(406, B, D)).cuda()
    oi = torch.zeros((B, k), dtype=torch.int64, device="cuda")
    osc = torch.zeros((B, k), dtype=torch.float32, device="cuda")
    on = torch.full((B,), 7, dtype=torch.int32, device="cuda")
    sh.search_into(q, oi, osc, on)
    torch.cuda.synchronize()
    assert (on.cpu().numpy() == 0).all()
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
    for sp in (g.SearchParams(rescore_count=0), g.SearchParams(rescore_count=(1 << 20) + 1),
               g.SearchParams(rescore_count=100, metric=1)):
        c = sp.to_c()
        st = L.gvdb_index_search_sharded_device(ix._h, sh._h, q.data_ptr(), 2, D, 10, C.byref(c), oi.data_ptr(),
                                                osc.data_ptr(), None, None)
        assert st == g._ffi.GVDB_ERR_INVALID_ARGUMENT
    w, r = C.c_int32(), C.c_int32()
    assert L.gvdb_comm_info(sh._h, C.byref(w), C.byref(r)) == 0 and (w.value, r.value) == (1, 0)
    sh.close()
