"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar: bit-exact bytes / ids / Hamming distances, and bit-exact f32 scores
(the rerank folds each row in the reference's sequential order, so cosine
scores match to the last bit; the north-star tolerance 1e-5 is asserted as
well for documentation).  Sizes stay where the oracle finishes in seconds.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

COS_TOL = 1e-5  # north_star: "cosine scores within 1e-5"


@pytest.fixture(scope="module")
def g(gvdb_mod):
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return gvdb_mod


def rng_rows(seed, n, d, dup=0):
    r = np.random.default_rng(seed)
    x = r.standard_normal((n, d)).astype(np.float32)
    for i in range(dup):  # duplicate rows -> equal Hamming AND equal cosine ties
        x[(7 * i + 11) % n] = x[(13 * i + 3) % n]
    return x


def same_f32(a, b):
    return np.array(a, np.float32).tobytes() == np.array(b, np.float32).tobytes()


# --------------------------------------------------------------------------- K1
def test_quantize_kat(g):
    q = g.BinaryQuantizer()
    assert q.quantize([0.5, -0.3, 0.8, -0.1, 0.2]).data == bytes([0xA8])  # quantization.rs:361-372
    a = q.quantize([1.0, -1.0, 1.0, -1.0])
    b = q.quantize([1.0, 1.0, -1.0, -1.0])
    assert (a.data, b.data) == (bytes([0xA0]), bytes([0xC0]))
    assert q.hamming_distance(a, b) == 2.0 and q.similarity(a, b) == 0.5  # quantization.rs:375-386


@pytest.mark.parametrize("D", [1, 5, 8, 31, 63, 64, 65, 100, 128, 129, 768, 1000, 3072])
def test_quantize_matches_oracle(g, oracle_mod, D):
    x = rng_rows(D, 257, D)
    x[0, 0] = np.nan
    x[1, : min(D, 4)] = -0.0
    x[2, : min(D, 4)] = 0.0
    for thr in (0.0, 0.25):
        got = g.BinaryQuantizer(g.BinaryQuantizationConfig(threshold=thr)).quantize_batch(x)
        ref = oracle_mod.quantize(x, thr)
        assert all(got[i].data == ref[i].tobytes() for i in range(len(x)))


def test_hamming_matches_oracle(g, oracle_mod):
    q = g.BinaryQuantizer()
    for D in (3, 64, 768):
        x = rng_rows(D + 1, 20, D)
        bv = q.quantize_batch(x)
        ref = oracle_mod.quantize(x)
        for i in range(0, 20, 2):
            assert q.hamming_distance(bv[i], bv[i + 1]) == oracle_mod.hamming(ref[i], ref[i + 1])
    with pytest.raises(g.InvalidVectorDimension):
        q.hamming_distance(q.quantize([1.0, 2.0]), q.quantize([1.0]))


# --------------------------------------------------------------------------- K2+K3 (multi_stage_search)
@pytest.mark.parametrize("N,D,ratio", [(1, 8, 1.0), (2, 8, 1.0), (10, 16, 0.5), (1000, 100, 0.1), (5000, 128, 0.02),
                                       (3000, 768, 0.05), (2000, 3072, 0.01), (4000, 64, 1.0)])
def test_multi_stage_matches_oracle(g, oracle_mod, N, D, ratio):
    x = rng_rows(N * 7 + D, N, D, dup=min(N // 4, 40))
    qv = rng_rows(D, 1, D)[0]
    bq = g.BinaryQuantizer(g.BinaryQuantizationConfig(rescore_ratio=ratio))
    cb = bq.quantize_batch(x)
    qb = bq.quantize(qv)
    got = bq.multi_stage_search(qb, cb, qv, x)
    ri, rc = oracle_mod.multi_stage_search(oracle_mod.quantize(qv)[0], D, oracle_mod.quantize(x), D, qv, x, ratio)
    assert [i for i, _ in got] == [int(i) for i in ri]
    assert same_f32([c for _, c in got], rc)  # bit-exact cosine
    assert np.max(np.abs(np.array([c for _, c in got]) - rc), initial=0.0) <= COS_TOL


def test_multi_stage_dimension_mismatch(g, oracle_mod):
    x = rng_rows(1, 50, 16)
    qv = rng_rows(2, 1, 8)[0]
    bq = g.BinaryQuantizer(g.BinaryQuantizationConfig(rescore_ratio=0.5))
    got = bq.multi_stage_search(bq.quantize(qv), bq.quantize_batch(x), qv, x)
    ri, rc = oracle_mod.multi_stage_search(oracle_mod.quantize(qv)[0], 8, oracle_mod.quantize(x), 16, qv, x, 0.5)
    assert [i for i, _ in got] == [int(i) for i in ri] and same_f32([c for _, c in got], rc)


def test_multi_stage_errors(g):
    bq = g.BinaryQuantizer()
    with pytest.raises(g.QuantizationError):  # quantization.rs:158-162
        bq.multi_stage_search(bq.quantize([1.0]), [bq.quantize([1.0])], [1.0], [[1.0], [2.0]])
    assert bq.multi_stage_search(bq.quantize([1.0]), [], [1.0], []) == []


# --------------------------------------------------------------------------- stage 1 at scale (sampling path)
def topr(g, ix, Q, R):
    import torch

    q = torch.from_numpy(Q).cuda()
    rows = torch.zeros((Q.shape[0], R), dtype=torch.int64, device="cuda")
    dist = torch.zeros((Q.shape[0], R), dtype=torch.int32, device="cuda")
    ix.bq_topr_device(q, R, rows, dist)
    torch.cuda.synchronize()
    return rows.cpu().numpy().astype(np.uint64), dist.cpu().numpy().astype(np.uint32)


@pytest.mark.parametrize("N,D,B,R,dup", [(600_000, 128, 6, 100, 0), (300_000, 768, 4, 64, 0),
                                          (100_000, 64, 5, 1000, 2000), (50_000, 128, 3, 5000, 0),
                                          (40_000, 32, 3, 9000, 0)])
def test_stage1_topr_matches_oracle(g, oracle_mod, N, D, B, R, dup):
    x = rng_rows(N + D, N, D)
    if dup:  # a block of identical rows: massive ties at one distance
        x[1000:1000 + dup] = x[5]
    Q = rng_rows(D + 99, B, D)
    Q[0] = x[5]
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    gi, gd = topr(g, ix, Q, R)
    ri, rd = oracle_mod.bq_topr_batch(oracle_mod.quantize(Q), oracle_mod.quantize(x), D, R)
    assert (gd == rd).all()
    assert (gi == ri).all()


@pytest.mark.parametrize("N,D,B,R", [(200_000, 768, 160, 100), (100_000, 256, 96, 64), (120_000, 384, 128, 200),
                                     (90_000, 512, 300, 50), (80_000, 1024, 100, 100), (70_000, 768, 256, 1000),
                                     (50_000, 1536, 200, 100), (40_000, 2048, 200, 300), (60_000, 3072, 256, 100),
                                     (50_000, 3000, 130, 100), (40_000, 4096, 100, 100),
                                     (60_000, 200, 128, 100), (50_000, 700, 97, 100), (30_001, 330, 256, 40)])
def test_stage1_mfma_batches_match_oracle(g, oracle_mod, N, D, B, R):
    """Large batches (B >= 96) take the FP4-MFMA scan: k_scan_mx5 for W4 in
    {2,3,4,6} (padded dims included: D = 200, 330, 700), k_scan_mx4 (query tiles per launch bounded by LDS, partial
    last launch) for W4 in {8,12,16,24,32}; distances must equal the popcount
    path (GVDB_SCAN=valu) and the oracle bit for bit."""
    import os

    x = rng_rows(N + 3 * D, N, D, dup=200)
    Q = rng_rows(D + 77, B, D)
    Q[3] = x[11]
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    gi, gd = topr(g, ix, Q, R)
    for variant in ("valu",):
        os.environ["GVDB_SCAN"] = variant
        try:
            vi, vd = topr(g, ix, Q, R)
        finally:
            del os.environ["GVDB_SCAN"]
        assert (gi == vi).all() and (gd == vd).all(), variant
    ri, rd = oracle_mod.bq_topr_batch(oracle_mod.quantize(Q), oracle_mod.quantize(x), D, R)
    assert (gd == rd).all() and (gi == ri).all()


def test_stage1_massive_ties_fallback(g, oracle_mod):
    # 12k identical nearest rows > the 8192-key LDS select: exact slow path
    N, D, R = 30_000, 64, 500
    x = rng_rows(3, N, D)
    x[100:12_100] = x[1]
    Q = x[1:2].copy()
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    gi, gd = topr(g, ix, Q, R)
    ri, rd = oracle_mod.bq_topr_batch(oracle_mod.quantize(Q), oracle_mod.quantize(x), D, R)
    assert (gi == ri).all() and (gd == rd).all()


def test_index_search_after_fallback(g, oracle_mod):
    # a batch where one query leaves the fast path (12k ties) and the others do not
    N, D, R, k = 30_000, 64, 500, 10
    x = rng_rows(4, N, D)
    x[100:12_100] = x[1]
    Q = np.concatenate([x[1:2], rng_rows(5, 3, D)])
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    ids, sc, n = ix.search_batch(Q, k, g.SearchParams(rescore_count=R))
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R)
    assert (ids == ri[:, :k]).all() and same_f32(sc, rs[:, :k])


# --------------------------------------------------------------------------- index search (VectorIndex)
@pytest.mark.parametrize("N,D,B,R,k,metric", [(20_000, 128, 16, 100, 10, 0), (20_000, 128, 8, 100, 10, 1),
                                               (20_000, 96, 8, 64, 64, 2), (300_000, 768, 4, 100, 10, 0),
                                               (5_000, 256, 4, 4500, 20, 0)])
def test_index_search_matches_oracle(g, oracle_mod, N, D, B, R, k, metric):
    x = rng_rows(N + 1, N, D, dup=50)
    Q = rng_rows(D + 5, B, D)
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64) * 3 + 7, x)
    ids, sc, n = ix.search_batch(Q, k, g.SearchParams(metric=metric, rescore_count=R))
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R, kind=metric)
    kk = min(k, R, N)
    assert (n == kk).all()
    assert (ids[:, :kk] == ri[:, :kk] * 3 + 7).all()
    assert same_f32(sc[:, :kk], rs[:, :kk])


@pytest.mark.parametrize("N,D,B,ratio,k,force", [(200_000, 768, 8, 0.1, 10, False), (200_000, 768, 128, 0.1, 10, False),
                                                  (400_000, 256, 96, 0.05, 25, False), (60_000, 200, 4, 0.3, 300, False),
                                                  (50_000, 128, 3, 0.2, 10, True)])
def test_default_rescore_ratio_large_r_matches_oracle(g, oracle_mod, monkeypatch, N, D, B, ratio, k, force):
    """The reference's DEFAULT depth R = (N as f32 * 0.1) as usize
    (quantization.rs:27,178) -- R = 20K at 200K rows, beyond the LDS select --
    on the batched large-R path (gvdb_bigr.hip: k_select_big's exact top-R
    membership, rerank, k_topk_big): ids and cosine bits equal the oracle's
    multi_stage_search; B = 128 / 96 take the FP4-MFMA scan, 400K rows a
    sampled threshold, k = 300 > the tie LDS window's usual size, and a forced
    device-side rescan (GVDB_FORCE_RESCAN) the all-rows fallback."""
    if force:
        monkeypatch.setenv("GVDB_FORCE_RESCAN", "1")
    x = rng_rows(N + D, N, D, dup=200)
    Q = rng_rows(D + 17, B, D)
    Q[0] = x[123]
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    ids, sc, n = ix.search_batch(Q, k, g.SearchParams(rescore_ratio=ratio))
    R = int(np.float32(N) * np.float32(ratio))
    assert R > 8192
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R)
    assert (n == k).all()
    assert (ids == ri[:, :k]).all()
    assert same_f32(sc, rs[:, :k])


@pytest.mark.parametrize("dense", ["0", "1"])
def test_large_r_emit_and_dense_selects_match_oracle(g, oracle_mod, monkeypatch, dense):
    """Both large-R stage-1 forms at the reference's default ratio on one corpus:
    GVDB_DENSE_SEL=0 keeps the threshold scan + candidate buffer + k_select_big;
    the default at R/N >= 1/64 writes every distance (k_scan_mx7<DENSE>, f16 dots)
    and k_select_dense picks the members.  Duplicate rows make ties at the
    threshold; a row count that is not a multiple of 8 or 32 leaves a ragged last row block (100001 rows)."""
    if dense == "0":
        monkeypatch.setenv("GVDB_DENSE_SEL", "0")
    N, D, B, k = 100_001, 768, 20, 10
    x = rng_rows(N + 3, N, D, dup=300)
    Q = rng_rows(D + 41, B, D)
    Q[0] = x[N - 1]
    Q[1] = x[5]
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    c0 = deep_cert_counts(g)
    ids, sc, n = ix.search_batch(Q, k, g.SearchParams(rescore_ratio=0.1))
    c1 = deep_cert_counts(g)
    R = int(np.float32(N) * np.float32(0.1))
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R)
    assert (n == k).all()
    assert (ids == ri[:, :k]).all()
    assert same_f32(sc, rs[:, :k])
    assert ids[0, 0] == N - 1
    # the dense form answers through the certified default-depth search (no B x R rerank)
    assert c1[0] - c0[0] == (1 if dense == "1" else 0) and c1[1] == c0[1]


def deep_cert_counts(g):
    """(certified batches, batches sent to the B x R rerank) of the certified
    default-depth search (gvdb_capi.hip: deep_cert_search)."""
    import ctypes as C

    L = g.lib()
    L.gvdb_debug_deep_cert.argtypes = [C.POINTER(C.c_uint64)]
    out = (C.c_uint64 * 2)()
    assert L.gvdb_debug_deep_cert(out) == 0
    return int(out[0]), int(out[1])


def test_default_depth_certified_over_query_groups(g, oracle_mod):
    """The certified default-depth search over more than one 256-query group
    (B = 300: stage 1, the flat list and the certify pass all run per group or
    over the whole batch), D = 256, duplicate rows (cosine AND Hamming ties)."""
    N, D, B, ratio, k = 70_003, 256, 300, 0.2, 10
    x = rng_rows(N + 13, N, D, dup=150)
    Q = rng_rows(D + 59, B, D)
    Q[0] = x[19]
    Q[299] = x[N - 1]
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    c0 = deep_cert_counts(g)
    ids, sc, n = ix.search_batch(Q, k, g.SearchParams(rescore_ratio=ratio))
    c1 = deep_cert_counts(g)
    R = int(np.float32(N) * np.float32(ratio))
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R)
    assert (n == k).all() and (ids == ri[:, :k]).all() and same_f32(sc, rs[:, :k])
    assert ids[299, 0] == N - 1
    assert (c1[0] - c0[0], c1[1] - c0[1]) == (1, 0)


def test_default_depth_certificate_falls_back_to_rerank(g, oracle_mod):
    """Rows whose cosine with a query is high (~0.84) but whose Hamming distance
    is beyond the query's top 10 % (400 of 768 signs flipped on the query's
    smallest components): 70 of them fill the exact cosine top-64, so fewer than
    k members remain in the list and the certificate must fail.  The batch then
    takes the B x R rerank, and the results still equal the oracle's."""
    N, D, B, k = 100_000, 768, 6, 10
    r = np.random.default_rng(91)
    x = rng_rows(N + 21, N, D)
    Q = rng_rows(D + 23, B, D)
    for qi in range(2):
        q = Q[qi]
        base = q.copy()
        small = np.argsort(np.abs(q))[:400]
        base[small] = -q[small]
        for j in range(70):
            x[5000 * qi + 11 * j] = base + 0.01 * r.standard_normal(D).astype(np.float32)
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    c0 = deep_cert_counts(g)
    ids, sc, n = ix.search_batch(Q, k, g.SearchParams(rescore_ratio=0.1))
    c1 = deep_cert_counts(g)
    R = int(np.float32(N) * np.float32(0.1))
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R)
    assert (n == k).all() and (ids == ri[:, :k]).all() and same_f32(sc, rs[:, :k])
    assert (c1[0] - c0[0], c1[1] - c0[1]) == (0, 1)
    # the planted rows are not members: the answer holds none of them
    planted = {5000 * qi + 11 * j for qi in range(2) for j in range(70)}
    assert not planted & set(ids[:2].ravel().tolist())


@pytest.mark.parametrize("form,shift,D", [("8", 0, 768), ("0", 0, 768), ("8", 0, 256), ("8", 300, 768),
                                          ("8", -300, 768), ("8", 0, 200)])
def test_default_depth_byte_rule_matches_oracle(g, oracle_mod, monkeypatch, form, shift, D):
    """The certified default depth's dense rule in its byte form (round 6,
    GVDB_DENSE8, default on: one byte per pair around a per-query window from
    k_dense_base) and in the f16 form (GVDB_DENSE8=0): ids and cosine bits equal
    the oracle, the batch certifies, duplicate rows make ties at T (the tie cut
    comes from the bytes).  D = 256 / 200: the window starts at 0 (exact bytes).
    A window shifted off T (GVDB_DENSE8_SHIFT = +-300: T below base, or above the
    counted range) must not certify: the rule reports no rule, the batch takes
    the B x R rerank, and the answer is still the oracle's."""
    monkeypatch.setenv("GVDB_DENSE8", form)
    if shift:
        monkeypatch.setenv("GVDB_DENSE8_SHIFT", str(shift))
    N, B, k = 131_077, 40, 10
    x = rng_rows(N + D + 5, N, D, dup=400)
    Q = rng_rows(D + 61, B, D)
    Q[0] = x[N - 3]
    Q[1] = x[(7 * 5 + 11) % N]  # a duplicated row: Hamming and cosine ties
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    c0 = deep_cert_counts(g)
    ids, sc, n = ix.search_batch(Q, k, g.SearchParams(rescore_ratio=0.1))
    c1 = deep_cert_counts(g)
    R = int(np.float32(N) * np.float32(0.1))
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R)
    assert (n == k).all() and (ids == ri[:, :k]).all() and same_f32(sc, rs[:, :k])
    assert ids[0, 0] == N - 3
    assert (c1[0] - c0[0], c1[1] - c0[1]) == ((0, 1) if shift else (1, 0))


def test_dense_select_query_groups_match_oracle(g, oracle_mod):
    """Dense large-R stage 1 over more than one 256-query group (B = 300: the
    dense block is reused by the second group of 44 queries), D = 256."""
    N, D, B, ratio, k = 60_000, 256, 300, 0.2, 10
    x = rng_rows(N + 9, N, D, dup=150)
    Q = rng_rows(D + 53, B, D)
    Q[0] = x[17]
    Q[299] = x[N - 2]
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    ids, sc, n = ix.search_batch(Q, k, g.SearchParams(rescore_ratio=ratio))
    R = int(np.float32(N) * np.float32(ratio))
    assert R > 8192
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R)
    assert (n == k).all()
    assert (ids == ri[:, :k]).all()
    assert same_f32(sc, rs[:, :k])
    assert ids[299, 0] == N - 2


def test_default_ratio_sampled_mfma_takes_no_rescan(g, oracle_mod, monkeypatch):
    """R/N = 0.1 on a SAMPLED shard (400K rows > the 262144-row exact window)
    with an FP4-MFMA batch (B = 128): the dense FP4 sample keeps one minimum
    per 16 rows and cannot reach a target of ~R*S/N, so stage1_plan must pick
    the FP4 histogram instead.  Results equal the oracle and no
    query took k_select_big's all-rows rescan."""
    import ctypes as C

    N, D, B, ratio, k = 400_000, 256, 128, 0.1, 10
    x = rng_rows(N + 5, N, D, dup=100)
    Q = rng_rows(D + 29, B, D)
    Q[1] = x[77]
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    monkeypatch.setenv("GVDB_DEBUG_THR", "1")
    monkeypatch.setenv("GVDB_DEEP_CERT", "0")  # the B x R rerank path, whose stage 1 this test inspects
    ids, sc, n = ix.search_batch(Q, k, g.SearchParams(rescore_ratio=ratio))
    L = g.lib()
    L.gvdb_debug_stage1_rescanned.argtypes = [C.POINTER(C.c_uint32)]
    flag = C.c_uint32(7)
    assert L.gvdb_debug_stage1_rescanned(C.byref(flag)) == 0
    assert flag.value == 0, "a query fell back to the all-rows rescan"
    R = int(np.float32(N) * np.float32(ratio))
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R)
    assert (n == k).all() and (ids == ri[:, :k]).all() and same_f32(sc, rs[:, :k])


def test_index_semantics(g):
    ix = g.GpuVectorIndex()
    with pytest.raises(g.IndexNotBuilt):  # index.rs:213
        ix.search([1.0, 0.0, 0.0], 5)
    ix.add_vector("test1", [1.0, 0.0, 0.0])  # query.rs:428-483 KAT
    assert ix.search([1.0, 0.1, 0.0], 5)[0][0] == "test1"
    with pytest.raises(g.DimensionMismatch) as e:  # index.rs:160-168
        ix.add_vector("bad", [1.0, 2.0])
    assert (e.value.expected, e.value.actual) == (3, 2)
    ix.add_vectors([("a", [0.0, 1.0, 0.0]), ("b", [0.0, 0.0, 1.0])])
    assert ix.len() == 3 and not ix.is_empty()
    # re-adding an id shadows the old row (HashMap insert, index.rs:175-176)
    ix.add_vector("a", [0.9, 0.1, 0.0])
    assert ix.len() == 3 and ix.get_stats().memory_usage == 4 * 3 * 4
    res = ix.search_batch(np.array([[1.0, 0, 0]], np.float32), 10, g.SearchParams(rescore_count=4))
    ids = [int(i) for i in res[0][0, :res[2][0]]]
    assert len(ids) == 3  # the orphaned row is dropped after take(k)
    assert ix.remove_vector("b") is True and ix.remove_vector("zzz") is False
    assert ix.len() == 2 and ix.get_stats().memory_usage == 2 * 3 * 4  # orphans compacted away
    hits = ix.search([1.0, 0.0, 0.0], 5)
    assert [h[0] for h in hits] == ["test1", "a"]
    ix.clear()
    assert ix.is_empty() and ix.get_stats().dimension == 0
    with pytest.raises(g.IndexNotBuilt):
        ix.search([1.0], 1)


def test_index_flat_mode_matches_oracle(g, oracle_mod):
    N, D = 3000, 64
    x = rng_rows(9, N, D, dup=30)
    x[17] = 0.0  # zero-norm row
    Q = rng_rows(10, 5, D)
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    ids, sc, n = ix.search_batch(Q, 25, g.SearchParams(mode=1, metric=0))
    for b in range(5):
        ri, rs = oracle_mod.storage_vector_search(Q[b], x, 25)
        assert list(ids[b, :n[b]]) == list(ri) and same_f32(sc[b, :n[b]], rs)
    ids, sc, n = ix.search_batch(Q, 25, g.SearchParams(mode=1, metric=2))
    for b in range(5):
        ri, rs = oracle_mod.flat_cosine_distance_search(Q[b], x, 25)
        assert list(ids[b, :n[b]]) == list(ri) and same_f32(sc[b, :n[b]], rs)


@pytest.mark.parametrize("kind", ["i8", "bf16"])
@pytest.mark.parametrize("N,D,B,k,metric", [(200_000, 768, 48, 10, 0), (200_000, 768, 256, 10, 0),
                                             (160_000, 704, 256, 10, 2), (150_000, 100, 300, 25, 0),
                                             (100_000, 200, 17, 100, 2), (70_000, 64, 1, 1, 0),
                                             (66_000, 1100, 9, 10, 0)])
def test_flat_mfma_certified_matches_oracle(g, oracle_mod, monkeypatch, kind, N, D, B, k, metric):
    """K4 on i8 / bf16 MFMA (gvdb_flat.hip): candidates from the MFMA pass,
    exact rerank, certificate.  Ids equal and scores bit-identical to the
    oracle's storage.rs / index.rs flat search, with NO fallback taken (i8:
    neither the bf16 retry nor the exact rescan).  D=1100 covers the i8
    quantiser's second 1024-element pass and a ragged last chunk.  B = 256 at
    D in (640, 768] is the bench's exact-flat shape on k_flat_i8q: every one of
    its 8 query tiles holds real queries (waves 4-7 run the skewed epilogue),
    with planted and i.i.d. queries in every tile, duplicated rows (score ties)
    and duplicated queries."""
    monkeypatch.setenv("GVDB_FLAT", kind)
    x = rng_rows(N + D, N, D, dup=40)
    x[5] = 0.0  # zero-norm row scores 0 (cosine) / +inf (distance)
    Q = rng_rows(D + 11, B, D)
    r = np.random.default_rng(B)
    planted = r.integers(0, N, size=B)
    if B >= 128:  # planted and iid queries interleaved: every 32-query tile holds both
        sel = np.arange(B) % 2 == 0
        Q[sel] = x[planted[sel]] + 0.05 * Q[sel]
        for j in range(0, B, 37):  # a planted row duplicated 3x: a tie at the top of the list
            x[(planted[j] + 1) % N] = x[planted[j]]
            x[(planted[j] + 2) % N] = x[planted[j]]
        Q[B - 1] = Q[B - 2]  # duplicated queries in the last tile
    else:
        Q[: B // 2] = x[planted[: B // 2]] + 0.05 * Q[: B // 2]  # true near neighbours for half the batch
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    before = g.lib().gvdb_flat_fallback_count()
    before_i8 = g.lib().gvdb_flat_i8_fallback_count()
    ids, sc, n = ix.search_batch(Q, k, g.SearchParams(mode=1, metric=metric))
    assert g.lib().gvdb_flat_fallback_count() == before, "MFMA candidate pass was not certified"
    assert g.lib().gvdb_flat_i8_fallback_count() == before_i8, "i8 candidate pass was not certified"
    if B >= 128:  # the oracle's storage.rs / index.rs searches, one query per thread
        if metric == 0:
            ri_all, rs_all = oracle_mod.exact_topk_cosine_batch(Q, x, k, threads=16)
        else:
            ri_all, rs_all, _ = oracle_mod.flat_cosine_distance_batch(Q, x, k, threads=16)
        assert (n == k).all()
        assert (ids == ri_all).all()
        assert same_f32(sc, rs_all)
        return
    for b in range(B):
        if metric == 0:
            ri, rs = oracle_mod.storage_vector_search(Q[b], x, k)
        else:
            ri, rs = oracle_mod.flat_cosine_distance_search(Q[b], x, k)
        assert n[b] == len(ri)
        assert list(ids[b, : n[b]]) == list(ri), b
        assert same_f32(sc[b, : n[b]], rs)


def test_flat_i8_margin_too_wide_retries_on_bf16(g, oracle_mod, monkeypatch):
    """12000 rows at cosine 0.900..0.910 to the query e_0: with the i8 margin (the
    rows' ~1.6 % quantisation error) every one of them is a candidate, over the
    8192-candidate capacity; bf16's 2^-8 margin nominates ~40 % of them: the
    batch is retried on bf16, certified there, and the result is still exactly
    the oracle's."""
    N, D, k = 70_000, 64, 10
    r = np.random.default_rng(77)
    x = r.standard_normal((N, D)).astype(np.float32) * np.float32(0.05)
    x[:, 0] = 0.0
    special = r.choice(N, 12000, replace=False)
    c = np.linspace(0.90, 0.91, 12000, dtype=np.float64)
    u = r.standard_normal((12000, D))
    u[:, 0] = 0.0
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    x[special] = (c[:, None] * np.eye(D)[0] + np.sqrt(1 - c[:, None] ** 2) * u).astype(np.float32)
    Q = np.zeros((1, D), np.float32)
    Q[0, 0] = 1.0
    monkeypatch.setenv("GVDB_FLAT", "i8")
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    before = g.lib().gvdb_flat_fallback_count()
    before_i8 = g.lib().gvdb_flat_i8_fallback_count()
    ids, sc, n = ix.search_batch(Q, k, g.SearchParams(mode=1, metric=0))
    assert g.lib().gvdb_flat_i8_fallback_count() == before_i8 + 1
    assert g.lib().gvdb_flat_fallback_count() == before
    ri, rs = oracle_mod.storage_vector_search(Q[0], x, k)
    assert list(ids[0, : n[0]]) == list(ri) and same_f32(sc[0, : n[0]], rs)


def test_flat_nonfinite_row_takes_exact_scan(g, oracle_mod):
    """An +inf element makes a row's cosine NaN in the reference fold; the MFMA
    tiers refuse such a shard and the exact scan reproduces the reference."""
    N, D = 70_000, 64
    x = rng_rows(41, N, D)
    x[777, 3] = np.inf
    Q = rng_rows(42, 2, D)
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    before = g.lib().gvdb_flat_fallback_count()
    try:
        ids, sc, n = ix.search_batch(Q, 10, g.SearchParams(mode=1, metric=2))
    except g.QuantizationError:
        return  # the NaN score is reported as the reference's sort would panic
    assert g.lib().gvdb_flat_fallback_count() == before + 1
    for b in range(2):
        ri, rs = oracle_mod.flat_cosine_distance_search(Q[b], x, 10)
        assert list(ids[b, : n[b]]) == list(ri) and same_f32(sc[b, : n[b]], rs)


def test_flat_mfma_uncertifiable_falls_back_exactly(g, oracle_mod):
    """A zero query ties every row at 0.0: no certificate is possible, the exact
    full scan answers (storage.rs order: first k rows)."""
    N, D = 70_000, 64
    x = rng_rows(3, N, D)
    Q = np.zeros((2, D), np.float32)
    Q[1] = x[123]
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    before = g.lib().gvdb_flat_fallback_count()
    ids, sc, n = ix.search_batch(Q, 10, g.SearchParams(mode=1, metric=0))
    assert g.lib().gvdb_flat_fallback_count() == before + 1
    for b in range(2):
        ri, rs = oracle_mod.storage_vector_search(Q[b], x, 10)
        assert list(ids[b, : n[b]]) == list(ri) and same_f32(sc[b, : n[b]], rs)


def test_flat_device_api_without_out_n(g, oracle_mod):
    """gvdb_index_search_device with out_n = NULL (optional) on the MFMA flat path
    and, for a batch over 256 queries, across launch groups."""
    import torch

    N, D, B, k = 70_000, 64, 300, 5
    x = rng_rows(31, N, D)
    Q = rng_rows(32, B, D)
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    q = torch.from_numpy(Q).cuda()
    oi = torch.zeros((B, k), dtype=torch.int64, device="cuda")
    osc = torch.zeros((B, k), device="cuda")
    ix.search_device(q, k, oi, osc, None, g.SearchParams(mode=1, metric=0))
    torch.cuda.synchronize()
    ids, sc = oi.cpu().numpy(), osc.cpu().numpy()
    for b in (0, 255, 256, 299):
        ri, rs = oracle_mod.storage_vector_search(Q[b], x, k)
        assert list(ids[b]) == list(ri) and same_f32(sc[b], rs)


def test_flat_mfma_after_mutations(g, oracle_mod):
    """The bf16 mirror is rebuilt after add / remove (version counter)."""
    N, D = 80_000, 96
    x = rng_rows(21, N, D)
    Q = x[[10, 20_000, 79_999]] + 0.01
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    p = g.SearchParams(mode=1, metric=0)
    ids, _, _ = ix.search_batch(Q, 5, p)
    assert list(ids[:, 0]) == [10, 20_000, 79_999]
    extra = rng_rows(22, 1000, D)
    extra[7] = Q[1]  # exact match appended
    ix.add_batch(np.arange(N, N + 1000, dtype=np.uint64), extra)
    ids, _, _ = ix.search_batch(Q, 5, p)
    assert ids[1, 0] == N + 7
    assert ix.remove_vector_id(N + 7)
    ids, sc, n = ix.search_batch(Q, 5, p)
    allx = np.concatenate([x, np.delete(extra, 7, axis=0)])
    for b in range(3):
        ri, rs = oracle_mod.storage_vector_search(Q[b], allx, 5)
        live = np.concatenate([np.arange(N), np.delete(np.arange(N, N + 1000), 7)])
        assert list(ids[b, : n[b]]) == list(live[ri]) and same_f32(sc[b, : n[b]], rs)


@pytest.mark.parametrize("kind", ["i8", "bf16"])
@pytest.mark.parametrize("N,D,B", [(70_000, 64, 6), (200_000, 768, 256)])
def test_flat_prune_skips_orphans_and_keeps_ties(g, oracle_mod, monkeypatch, kind, N, D, B):
    """Candidate pruning (k_flat_prune) between the MFMA pass and the exact rerank:
    the k-th largest lower bound is taken over LIVE rows only.  Each query's 40
    nearest rows are re-added under their ids with far vectors, so the orphaned
    old rows still top the MFMA pass, and the live neighbours come in groups of 4
    exact duplicates (ties at the k-th score).  Certified on the MFMA tier (no
    fallback), ids and scores equal the oracle over the live rows.  The
    200K x 768 x 256 case is the bench's shape on k_flat_i8q (all 8 query
    tiles live, the late waves' skewed epilogue included)."""
    monkeypatch.setenv("GVDB_FLAT", kind)
    k = 10
    x = rng_rows(91, N, D)
    r = np.random.default_rng(92)
    centers = r.choice(N, B, replace=False)
    Q = x[centers] + np.float32(0.3) * rng_rows(93, B, D)
    xn = x / np.linalg.norm(x, axis=1, keepdims=True)
    sim = xn @ (Q / np.linalg.norm(Q, axis=1, keepdims=True)).T
    top = np.argpartition(-sim, 48, axis=0)[:48]  # the 48 nearest rows of each query (unordered)
    order = np.take_along_axis(top, np.argsort(-np.take_along_axis(sim, top, axis=0), axis=0, kind="stable"), axis=0)
    near = np.unique(order[:40].ravel())             # to be orphaned
    nxt = [c for c in order[40:48].T.ravel() if c not in set(near)]
    for j, c in enumerate(nxt[: len(nxt) // 4 * 4]):  # live neighbours in groups of 4 equal rows
        x[c] = x[nxt[j // 4 * 4]]
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    fresh = -x[near]  # cosine -c: far from every query
    ix.add_batch(near.astype(np.uint64), fresh)
    keep = np.setdiff1d(np.arange(N), near)
    live_x = np.concatenate([x[keep], fresh])
    live_id = np.concatenate([keep, near])
    before, before_i8 = g.lib().gvdb_flat_fallback_count(), g.lib().gvdb_flat_i8_fallback_count()
    ids, sc, n = ix.search_batch(Q, k, g.SearchParams(mode=1, metric=0))
    assert g.lib().gvdb_flat_fallback_count() == before, "MFMA candidate pass was not certified"
    assert g.lib().gvdb_flat_i8_fallback_count() == before_i8, "i8 candidate pass was not certified"
    ri_all, rs_all = oracle_mod.exact_topk_cosine_batch(Q, live_x, k, threads=16)
    for b in range(B):
        assert n[b] == k
        assert list(ids[b, : n[b]]) == list(live_id[ri_all[b]]), b
        assert same_f32(sc[b, : n[b]], rs_all[b])


@pytest.mark.parametrize("N,k", [(4000, 1), (4000, 10), (4000, 1000), (4000, 1024), (4000, 1500), (4000, 5000),
                                 (40000, 10), (40000, 1024)])
def test_flat_small_n_topk_matches_oracle_and_sort_path(g, oracle_mod, monkeypatch, N, k):
    """Small-N exact flat (the batched one-block-per-query top-k, limit <= 1024,
    keys staged in LDS up to 16K rows; larger limits take the per-query radix
    sort): heavy ties (3 distinct rows, zero-norm rows), both metrics, equal to
    the oracle and to the sort path."""
    D = 48
    base = rng_rows(21, 3, D)
    x = base[np.arange(N) % 3].copy()
    x[5] = 0.0
    x[123] = 0.0
    Q = rng_rows(22, 6, D)
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    for metric, ref in ((0, oracle_mod.storage_vector_search), (2, oracle_mod.flat_cosine_distance_search)):
        ids, sc, n = ix.search_batch(Q, k, g.SearchParams(mode=1, metric=metric))
        for b in range(len(Q)):
            ri, rs = ref(Q[b], x, k)
            assert list(ids[b, :n[b]]) == list(ri) and same_f32(sc[b, :n[b]], rs), (metric, b)
        monkeypatch.setenv("GVDB_FLAT_SORT", "1")
        ids2, sc2, n2 = ix.search_batch(Q, k, g.SearchParams(mode=1, metric=metric))
        monkeypatch.delenv("GVDB_FLAT_SORT")
        assert (n2 == n).all() and (ids2 == ids).all() and sc2.tobytes() == sc.tobytes()
    idx, sc, n = g.flat_search(Q, x, k, threshold=0.1)
    for b in range(len(Q)):
        ri, rs = oracle_mod.storage_vector_search(Q[b], x, k, threshold=0.1)
        assert list(idx[b, :n[b]]) == list(ri) and same_f32(sc[b, :n[b]], rs)


def test_flat_search_threshold(g, oracle_mod):
    N, D = 2000, 32
    x = rng_rows(11, N, D)
    Q = rng_rows(12, 3, D)
    idx, sc, n = g.flat_search(Q, x, 50, threshold=0.3)
    for b in range(3):
        ri, rs = oracle_mod.storage_vector_search(Q[b], x, 50, threshold=0.3)
        assert list(idx[b, :n[b]]) == list(ri) and same_f32(sc[b, :n[b]], rs)


# --------------------------------------------------------------------------- merges
def test_topk_merge_device_matches_host(g):
    import torch

    rng = np.random.default_rng(0)
    S, B, stride, limit = 4, 9, 50, 30
    ids = rng.integers(0, 10**9, (S, B, stride)).astype(np.uint64)
    sc = (rng.integers(0, 16, (S, B, stride)) / 16).astype(np.float32)
    cnt = rng.integers(0, stride + 1, (S, B)).astype(np.uint32)
    hi, hs, hn = g.topk_merge(ids, sc, cnt, limit)
    d = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32) if a.dtype == np.uint32 else a).cuda()
    oi = torch.zeros((B, limit), dtype=torch.int64, device="cuda")
    os_ = torch.zeros((B, limit), dtype=torch.float32, device="cuda")
    on = torch.zeros(B, dtype=torch.int32, device="cuda")
    t_ids, t_sc, t_cnt = d(ids), d(sc), d(cnt)  # keep the device copies alive across the call
    torch.cuda.synchronize()
    st = g.lib().gvdb_topk_merge_device(t_ids.data_ptr(), t_sc.data_ptr(), t_cnt.data_ptr(), S, B, stride, limit, 1,
                                        oi.data_ptr(), os_.data_ptr(), on.data_ptr(), None)
    assert st == 0
    torch.cuda.synchronize()
    n = on.cpu().numpy()
    assert (n == hn).all()
    for q in range(B):
        assert (oi.cpu().numpy()[q, :n[q]].view(np.uint64) == hi[q, :n[q]]).all()
        assert same_f32(os_.cpu().numpy()[q, :n[q]], hs[q, :n[q]])


def test_sharded_candidates_merge_equals_single_device(g, oracle_mod):
    """Exact sharded mode: per-shard candidates + one merge == one device."""
    import torch

    N, D, B, R, k, G = 40_000, 128, 8, 100, 10, 4
    x = rng_rows(21, N, D, dup=100)
    Q = rng_rows(22, B, D)
    bounds = [N * s // G for s in range(G + 1)]
    gids = np.zeros((G, B, R), np.uint64)
    dist = np.zeros((G, B, R), np.uint32)
    cosv = np.zeros((G, B, R), np.float32)
    counts = np.zeros((G, B), np.uint32)
    q = torch.from_numpy(Q).cuda()
    for s in range(G):
        lo, hi = bounds[s], bounds[s + 1]
        ix = g.GpuVectorIndex(dimension=D)
        ix.add_batch(np.arange(lo, hi, dtype=np.uint64), x[lo:hi])
        oi = torch.zeros((B, R), dtype=torch.int64, device="cuda")
        od = torch.zeros((B, R), dtype=torch.int32, device="cuda")
        oc = torch.zeros((B, R), dtype=torch.float32, device="cuda")
        st = g.lib().gvdb_index_bq_candidates_device(ix._h, q.data_ptr(), B, D, R, oi.data_ptr(), od.data_ptr(),
                                                      oc.data_ptr(), None)
        assert st == 0
        torch.cuda.synchronize()
        gids[s], dist[s], cosv[s] = oi.cpu().numpy().view(np.uint64), od.cpu().numpy().view(np.uint32), oc.cpu().numpy()
        counts[s] = R
    # device merge
    dg = torch.from_numpy(gids.view(np.int64)).cuda()
    dd = torch.from_numpy(dist.view(np.int32)).cuda()
    dc = torch.from_numpy(cosv).cuda()
    dn = torch.from_numpy(counts.view(np.int32)).cuda()
    mi = torch.zeros((B, k), dtype=torch.int64, device="cuda")
    ms = torch.zeros((B, k), dtype=torch.float32, device="cuda")
    mn = torch.zeros(B, dtype=torch.int32, device="cuda")
    st = g.lib().gvdb_bq_shard_merge_device(dg.data_ptr(), dd.data_ptr(), dc.data_ptr(), dn.data_ptr(), G, B, R, R, k,
                                            mi.data_ptr(), ms.data_ptr(), mn.data_ptr(), None)
    assert st == 0
    torch.cuda.synchronize()
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(x), Q, x, R, kind=0)
    assert (mi.cpu().numpy().view(np.uint64) == ri[:, :k]).all()
    assert same_f32(ms.cpu().numpy(), rs[:, :k])
    # the packed form: per rank [ids u64 B*R | dist u32 B*R | cos f32 B*R], as one all-gather delivers it
    packed = np.concatenate([gids.reshape(G, -1).view(np.uint32), dist.reshape(G, -1), cosv.reshape(G, -1).view(np.uint32)],
                            axis=1)
    dp = torch.from_numpy(np.ascontiguousarray(packed).view(np.int32)).cuda()
    pi = torch.zeros_like(mi)
    ps = torch.zeros_like(ms)
    pn = torch.zeros_like(mn)
    st = g.lib().gvdb_bq_shard_merge_packed_device(dp.data_ptr(), dn.data_ptr(), G, B, R, k, pi.data_ptr(),
                                                   ps.data_ptr(), pn.data_ptr(), None)
    assert st == 0
    torch.cuda.synchronize()
    assert (pi.cpu().numpy().view(np.uint64) == ri[:, :k]).all()
    assert same_f32(ps.cpu().numpy(), rs[:, :k])
    assert (pn.cpu().numpy() == k).all()


def test_reference_unit_tests_through_cpp_mirror(g):
    """The reference's own unit tests (quantization.rs:361-400, query.rs:428-483)
    re-run through the C++ host mirror grape-vector-db_amd/host/gvdb.hpp."""
    import os
    import subprocess

    exe = os.path.join(os.path.dirname(g.lib()._name), "build", "reference_tests")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


# --------------------------------------------------------------------------- filtered search
@pytest.mark.parametrize("metric", [0, 1, 2])
def test_search_filtered_matches_oracle_on_subset(g, oracle_mod, metric):
    """§8(f) rank 4: search restricted to an execute_filter id set = the
    exact scan (storage.rs:296-339 / index.rs:69-78 / index.rs:686-700) over
    those rows only."""
    N, D = 3000, 48
    x = rng_rows(31, N, D, dup=20)
    Q = rng_rows(32, 5, D)
    ix = g.GpuVectorIndex(dimension=D)
    ids = [f"doc{i}" for i in range(N)]
    ix.add_vectors(list(zip(ids, x)))
    ix.remove_vector("doc7")
    r = np.random.default_rng(33)
    sub = sorted(set(r.choice(N, 700, replace=False).tolist()) | {7})  # doc7 is gone: ignored
    allowed = [ids[i] for i in sub] + ["no-such-id"] + [ids[sub[0]]]  # unknown + repeated ids
    live = [i for i in sub if i != 7]
    p = g.SearchParams(mode=g._ffi.GVDB_SEARCH_FLAT, metric=metric)
    oi, osc, on = ix.search_batch_filtered(Q, 25, allowed, p)
    for b in range(len(Q)):
        got = [ix._str_of[int(u)] for u in oi[b, :on[b]]]
        if metric == 0:
            ri, rs = oracle_mod.storage_vector_search(Q[b], x[live], 25)
        elif metric == 2:
            ri, rs = oracle_mod.flat_cosine_distance_search(Q[b], x[live], 25)
        else:
            d = np.array([oracle_mod.l2_distance(Q[b], x[i]) for i in live], np.float32)
            ri = np.argsort(d, kind="stable")[:25]
            rs = d[ri]
        assert got == [ids[live[int(j)]] for j in ri]
        assert same_f32(osc[b, :on[b]], rs)
    # k larger than the subset; empty subset
    oi, osc, on = ix.search_batch_filtered(Q[:1], 10, [ids[3], ids[5]], p)
    assert on[0] == 2
    oi, osc, on = ix.search_batch_filtered(Q[:1], 10, ["nothing"], p)
    assert on[0] == 0


@pytest.mark.parametrize("N,D,B,keep,R,metric", [
    (3_000, 48, 5, 0.3, 40, 0),          # exact-threshold regime, cosine
    (3_000, 48, 5, 0.3, 0, 1),           # R from the subset (M as f32 * 0.1) as usize, L2
    (700_000, 768, 2, 0.6, 100, 0),      # sampled threshold over the 420K-row subset
    (400_000, 768, 128, 0.8, 100, 2),    # the FP4-MFMA scan over the subset, 1 - cosine
    (200_000, 256, 20, 0.5, 0, 0),       # default ratio over the ~100K-row subset: R ~ 10K, dense stage 1
])
def test_search_filtered_bq_matches_multi_stage_on_subset(g, oracle_mod, N, D, B, keep, R, metric):
    """BQ mode + filter = multi_stage_search (quantization.rs:151-193) over the
    allowed rows only: their codes compacted, stage 1 on them, rows mapped
    back for the rerank; ids and scores bit-identical to the oracle run on the
    subset (ties in subset order = index row order)."""
    x = rng_rows(N + D, N, D, dup=30)
    Q = rng_rows(D + 5, B, D)
    r = np.random.default_rng(N)
    sub = np.flatnonzero(r.random(N) < keep)
    Q[0] = x[sub[len(sub) // 2]]
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64) * 3 + 7, x)
    k = 10
    sp = g.SearchParams(metric=metric, rescore_count=R)
    allowed = (sub.astype(np.uint64) * 3 + 7)
    ids = np.zeros((B, k), np.uint64)
    sc = np.zeros((B, k), np.float32)
    n = np.zeros(B, np.uint32)
    import ctypes as C

    from gvdb._ffi import ptr

    c = sp.to_c()
    g.check(ix._lib.gvdb_index_search_filtered(ix._h, ptr(Q), B, D, k, C.byref(c), ptr(allowed), allowed.size,
                                               ptr(ids), ptr(sc), ptr(n)))
    M = len(sub)
    Reff = R if R else oracle_mod.rust_f32_as_usize(np.float32(M) * np.float32(0.1))
    Reff = min(max(Reff, k), M)
    xs = x[sub]
    ri, rs = oracle_mod.multi_stage_search_batch_r(oracle_mod.quantize(Q), oracle_mod.quantize(xs), Q, xs, Reff,
                                                   kind=metric)
    kk = min(k, Reff)
    assert (n == kk).all()
    assert (ids[:, :kk] == sub[ri[:, :kk].astype(np.int64)].astype(np.uint64) * 3 + 7).all()
    assert same_f32(sc[:, :kk], rs[:, :kk])


def test_sharded_packed_world1_equals_single_device(g):
    """ShardedBQSearch's packed path (candidates written into the all-gather
    send block, gvdb_bq_shard_merge_packed_device on it) with one rank returns
    exactly what the single-device search returns; more ranks are covered by
    the gloo test (host path) and the C-ABI merge test above."""
    import torch

    from gvdb.sharded import ShardedBQSearch, gpu_candidates_fn

    N, D, B, R, k = 300_000, 768, 128, 100, 10
    x = rng_rows(91, N, D, dup=50)
    Q = rng_rows(92, B, D)
    Q[5] = x[777]
    ix = g.GpuVectorIndex(dimension=D)
    ix.add_batch(np.arange(N, dtype=np.uint64), x)
    q = torch.from_numpy(Q).cuda()
    sh = ShardedBQSearch(gpu_candidates_fn(ix), [N], B, R, k, torch.device("cuda", 0))
    assert sh.packed
    pi, ps, pn = (t.clone() for t in sh.search(q))
    oi = torch.zeros((B, k), dtype=torch.int64, device="cuda")
    osc = torch.zeros((B, k), dtype=torch.float32, device="cuda")
    on = torch.zeros(B, dtype=torch.int32, device="cuda")
    ix.search_device(q, k, oi, osc, on, g.SearchParams(rescore_count=R))
    torch.cuda.synchronize()
    assert torch.equal(pi, oi) and torch.equal(pn, on)
    assert same_f32(ps.cpu().numpy(), osc.cpu().numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("N,D,B,R", [(1_200_000, 768, 256, 100), (600_000, 256, 128, 1000), (400_000, 384, 200, 100),
                                     (350_000, 512, 96, 4000), (1_250_000, 768, 300, 100), (200_000, 768, 256, 100),
                                     (70_000, 700, 128, 1000)])
def test_sample_histogram_mfma_thresholds_equal_valu(g, N, D, B, R):
    """The FP4-MFMA sample forms against the VALU histogram (GVDB_SAMPLE=valu):
    k_sample_mx (128 queries per block, bins d < 384, each block flushes only up
    to its own target-th distance; sampled shards N > 262144 only) gives exactly
    its thresholds; the default dense form (k_sample_dense + k_sample_select:
    per query the minimum of every 16 sample rows, windowed select of the
    target-th smallest minimum; also N <= 262144, where the "sample" is the
    whole shard) gives thresholds never below them.  The searches return the
    same ids and distances in every case (B = 300 spans two 256-query groups)."""
    import ctypes as C
    import os

    import torch

    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(N + D)
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N)
    for c0 in range(0, N, 1 << 19):
        n = min(1 << 19, N - c0)
        ix.add_device(torch.randn((n, D), generator=gen, device=dev), torch.arange(c0, c0 + n, device=dev))
    q = torch.randn((B, D), generator=gen, device=dev)
    L = g.lib()
    L.gvdb_debug_stage1_thresholds.argtypes = [C.POINTER(C.c_uint32), C.c_uint32]
    out = {}
    os.environ["GVDB_DEBUG_THR"] = "1"
    try:
        for mode in ("mfma", "dense", "valu"):
            os.environ["GVDB_SAMPLE"] = {"mfma": "mx", "dense": "dense", "valu": "valu"}[mode]
            rows = torch.zeros((B, R), dtype=torch.int64, device=dev)
            dist = torch.zeros((B, R), dtype=torch.int32, device=dev)
            ix.bq_topr_device(q, R, rows, dist)
            torch.cuda.synchronize()
            thr = (C.c_uint32 * B)()
            assert L.gvdb_debug_stage1_thresholds(thr, B) == 0
            out[mode] = (list(thr), rows.cpu().numpy(), dist.cpu().numpy())
    finally:
        os.environ.pop("GVDB_DEBUG_THR", None)
        os.environ.pop("GVDB_SAMPLE", None)
    # k_sample_mx: exactly the VALU thresholds; dense (16-row group minima): never
    # below them, equal unless two of the target smallest share a group
    assert out["mfma"][0] == out["valu"][0]
    assert all(a >= b for a, b in zip(out["dense"][0], out["valu"][0]))
    if N > 262_144:  # a sampled shard (small target): group collisions are rare
        assert np.mean([a == b for a, b in zip(out["dense"][0], out["valu"][0])]) > 0.5
    for mode in ("mfma", "dense"):
        assert max(out[mode][0]) < D  # a real estimate, not the no-pruning fallback
        assert (out[mode][1] == out["valu"][1]).all() and (out[mode][2] == out["valu"][2]).all(), mode


@pytest.mark.parametrize("N,D,B,R", [(1_250_000, 768, 256, 100), (400_000, 256, 300, 100), (200_000, 768, 100, 100),
                                     (70_003, 512, 256, 300), (300_001, 384, 160, 64)])
def test_fused_sample_prep_equals_separate_kernels(g, oracle_mod, N, D, B, R):
    """k_sample_prep (query packing + dense sample in one launch, round 5) against
    k_qprep + k_sample_dense (GVDB_PREP=0): the same group minima, so the same
    per-query thresholds, and the same search results; B = 300 spans two 256-query
    groups, N <= 262144 makes the "sample" the whole (ragged) shard.  A query
    equal to a row and two equal queries check the packing."""
    import ctypes as C
    import os

    import torch

    dev = torch.device("cuda", 0)
    gen = torch.Generator(device=dev).manual_seed(N + 3 * D)
    ix = g.GpuVectorIndex(dimension=D, capacity_hint=N)
    x0 = None
    for c0 in range(0, N, 1 << 19):
        n = min(1 << 19, N - c0)
        xc = torch.randn((n, D), generator=gen, device=dev)
        if c0 == 0:
            x0 = xc[:4].clone()
        ix.add_device(xc, torch.arange(c0, c0 + n, device=dev))
    q = torch.randn((B, D), generator=gen, device=dev)
    q[1] = x0[3]
    q[B - 1] = q[B - 2]
    L = g.lib()
    L.gvdb_debug_stage1_thresholds.argtypes = [C.POINTER(C.c_uint32), C.c_uint32]
    sp = g.SearchParams(rescore_count=R)
    out = {}
    os.environ["GVDB_DEBUG_THR"] = "1"
    try:
        for mode in ("fused", "separate"):
            if mode == "separate":
                os.environ["GVDB_PREP"] = "0"
            oi = torch.zeros((B, 10), dtype=torch.int64, device=dev)
            osc = torch.zeros((B, 10), dtype=torch.float32, device=dev)
            on = torch.zeros(B, dtype=torch.int32, device=dev)
            ix.search_device(q, 10, oi, osc, on, sp)
            torch.cuda.synchronize()
            thr = (C.c_uint32 * B)()
            assert L.gvdb_debug_stage1_thresholds(thr, B) == 0
            out[mode] = (list(thr), oi.cpu().numpy(), osc.cpu().numpy(), on.cpu().numpy())
    finally:
        os.environ.pop("GVDB_DEBUG_THR", None)
        os.environ.pop("GVDB_PREP", None)
    assert out["fused"][0] == out["separate"][0]
    assert max(out["fused"][0]) < D
    for i in (1, 2, 3):
        assert out["fused"][i].tobytes() == out["separate"][i].tobytes()
    assert out["fused"][1][1, 0] == 3
