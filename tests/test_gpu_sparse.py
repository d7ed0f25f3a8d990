"""GPU parity of the BM25 sparse path and RRF fusion (gvdb_sparse.hip)
against the oracle (oracle/bm25_oracle.cpp), through the C ABI.  Ids equal
and scores bit-identical (NaN compared as NaN); ties ordered by slot as the
oracle defines (the reference leaves them to HashMap order)."""
import numpy as np
import pytest

from test_bm25_oracle import zipf_docs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sp_mod(gvdb_mod):
    import torch

    assert torch.cuda.is_available()
    from gvdb import sparse

    return sparse


def build(sp_mod, oracle_mod, docs, id0=0):
    g, o = sp_mod.SparseIndex(), oracle_mod.Bm25()
    ptr = np.zeros(len(docs) + 1, np.uint64)
    for i, (t, _, _) in enumerate(docs):
        ptr[i + 1] = ptr[i] + t.size
    terms = np.concatenate([t for t, _, _ in docs])
    tfs = np.concatenate([v for _, v, _ in docs])
    dls = np.array([dl for _, _, dl in docs], np.float32)
    g.add_documents_u64(np.arange(id0, id0 + len(docs), dtype=np.uint64), ptr, terms, tfs, dls)
    for i, (t, v, dl) in enumerate(docs):
        o.add_document(id0 + i, t, v, dl)
    return g, o


def queries(seed, B, vocab, lo=1, hi=9):
    r = np.random.default_rng(seed)
    qs = []
    for _ in range(B):
        t = r.choice(vocab, size=int(r.integers(lo, hi)), replace=True).astype(np.uint32)
        qs.append((t, r.random(t.size).astype(np.float32)))
    return qs


def same(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return a.shape == b.shape and np.array_equal(np.isnan(a), np.isnan(b)) and \
        a[~np.isnan(a)].tobytes() == b[~np.isnan(b)].tobytes()


def check_batch(sp_mod, g, o, qs, limit):
    svs = [sp_mod.SparseVector(t.tolist(), v.tolist(), 1 << 32) for t, v in qs]
    ids, sc, n = g.search_bm25_batch(svs, limit)
    for b, (t, v) in enumerate(qs):
        ri, rs = o.search(t, v, limit)
        assert n[b] == len(ri), (b, n[b], len(ri))
        assert list(ids[b, : n[b]]) == list(ri), b
        assert same(sc[b, : n[b]], rs), b


@pytest.mark.parametrize("n_docs,limit", [(500, 10), (40_000, 1), (40_000, 20), (40_000, 200)])
def test_bm25_matches_oracle(sp_mod, oracle_mod, n_docs, limit):
    docs = zipf_docs(n_docs, n_docs, 2000, 40)
    g, o = build(sp_mod, oracle_mod, docs)
    st = g.get_stats()
    on, oavg, ov = o.stats()
    assert st.total_documents == on and np.float32(st.average_document_length) == oavg and st.vocabulary_size == ov
    check_batch(sp_mod, g, o, queries(n_docs + limit, 45, 2000), limit)


def test_bm25_ties_by_slot(sp_mod, oracle_mod):
    """20k documents scoring identically: the first `limit` slots win."""
    docs = [(np.array([3, 9], np.uint32), np.array([0.5, 0.5], np.float32), np.float32(1.0))] * 20_000
    g, o = build(sp_mod, oracle_mod, docs, id0=500)
    check_batch(sp_mod, g, o, [(np.array([3], np.uint32), np.array([1.0], np.float32))], 15)


def test_bm25_dense_fallback(sp_mod, oracle_mod):
    """limit 3000 with ~30k matching documents: the candidate buffer overflows
    and the dense key array + radix sort answers, still exactly."""
    docs = zipf_docs(77, 30_000, 50, 20)
    g, o = build(sp_mod, oracle_mod, docs)
    check_batch(sp_mod, g, o, queries(78, 3, 50, 2, 4), 3000)


def test_bm25_mutations(sp_mod, oracle_mod):
    docs = zipf_docs(5, 9000, 800, 30)
    g, o = build(sp_mod, oracle_mod, docs)
    for i in (3, 4000, 8999):  # re-adds (a second entry per term)
        t, v, dl = docs[(i * 13) % len(docs)]
        g.add_documents_u64(np.array([i], np.uint64), np.array([0, t.size], np.uint64), t, v, np.array([dl]))
        o.add_document(i, t, v, dl)
    for i in (4000, 10, 7777, 123456):
        r = bool(g._lib.gvdb_sparse_remove_document(g._h, i, None) == 0)
        assert r
        o.remove_document(i)
    st = g.get_stats()
    on, oavg, _ = o.stats()
    assert st.total_documents == on and np.float32(st.average_document_length) == oavg
    check_batch(sp_mod, g, o, queries(6, 40, 800), 25)


def test_bm25_nan_when_df_exceeds_n(sp_mod, oracle_mod):
    """remove_document keeps df while a posting list is non-empty
    (sparse.rs:128-133): df > total_documents makes idf NaN; NaN sorts last."""
    docs = [(np.array([7], np.uint32), np.array([1.0], np.float32), np.float32(1.0))] * 3 + \
           [(np.array([8], np.uint32), np.array([1.0], np.float32), np.float32(1.0))]
    g, o = build(sp_mod, oracle_mod, docs)
    for i in (0, 3):
        g.remove_document  # noqa: B018 (string-id API; u64 ids here)
        import ctypes as C

        r = C.c_int32(0)
        g._lib.gvdb_sparse_remove_document(g._h, i, C.byref(r))
        assert r.value == 1
        o.remove_document(i)
    check_batch(sp_mod, g, o, [(np.array([7, 8], np.uint32), np.array([1.0, 1.0], np.float32))], 5)


def test_bm25_empty_and_unknown_terms(sp_mod, oracle_mod):
    g = sp_mod.SparseIndex()
    assert g.search_bm25(sp_mod.SparseVector([1], [1.0], 10), 5) == []  # total_documents == 0
    docs = zipf_docs(4, 100, 30, 5)
    g, o = build(sp_mod, oracle_mod, docs)
    check_batch(sp_mod, g, o, [(np.array([999, 1000], np.uint32), np.array([1.0, 2.0], np.float32)),
                               (np.array([], np.uint32), np.array([], np.float32))], 5)


def test_string_api_roundtrip(sp_mod):
    tk = sp_mod.SimpleTokenizer()
    texts = {"d1": "gpu vector search on mi355x", "d2": "binary quantization search", "d3": "hybrid bm25 search"}
    vocab = tk.build_vocabulary(list(texts.values()))
    g = sp_mod.SparseIndex()
    for k, v in texts.items():
        g.add_document(tk.document_to_sparse_vector(k, v, vocab))
    q = tk.document_to_sparse_vector("q", "bm25 search", vocab).sparse_vector
    res = g.search_bm25(q, 3)
    assert res[0][0] == "d3" and len(res) == 3
    assert g.remove_document("d3") and not g.remove_document("nope")
    assert g.get_stats().total_documents == 2


def test_rrf_matches_oracle(sp_mod, oracle_mod):
    r = np.random.default_rng(11)
    B = 40
    D, S, T = [], [], []
    for _ in range(B):
        mk = lambda n: [(int(x), float(r.random())) for x in r.integers(0, 30, n)]  # noqa: E731
        D.append(mk(r.integers(0, 25)))
        S.append(mk(r.integers(0, 25)))
        T.append(mk(r.integers(0, 6)))
    got = sp_mod.rrf_fuse(D, S, T, 60.0, 20)
    for b in range(B):
        want = oracle_mod.rrf_fusion(D[b], S[b], T[b], 60.0)[:20]
        assert [x[0] for x in got[b]] == [w[0] for w in want], b
        assert np.array([x[1] for x in got[b]], np.float32).tobytes() == \
            np.array([w[1] for w in want], np.float32).tobytes()
        for x, w in zip(got[b], want):
            assert same([np.nan if v is None else v for v in x[2]], w[2:])


def test_hybrid_engine_rrf(gvdb_mod, sp_mod, oracle_mod):
    """HybridSearchEngine::search (hybrid.rs:286-356): dense top-2*limit (L2,
    HnswVectorIndex semantics) + BM25 top-2*limit + RRF, all on the GPU, equal
    to the oracle's fusion of the oracle's lists."""
    n, D, limit = 3000, 64, 7
    r = np.random.default_rng(21)
    x = r.standard_normal((n, D)).astype(np.float32)
    docs = zipf_docs(22, n, 300, 25)
    dense = gvdb_mod.GpuVectorIndex(dimension=D)
    dense.add_vectors([(f"doc{i}", x[i]) for i in range(n)])
    sparse = sp_mod.SparseIndex()
    for i, (t, v, dl) in enumerate(docs):
        sparse.add_document(sp_mod.DocumentSparseRepresentation(f"doc{i}", None, float(dl),
                                                                {int(a): float(b) for a, b in zip(t, v)}))
    eng = sp_mod.HybridSearchEngine(dense, sparse, rrf_k=60.0)
    reqs = []
    for qi in range(6):
        t = r.choice(300, 4).astype(np.uint32)
        reqs.append(sp_mod.HybridSearchRequest(dense_vector=x[qi * 11] + 0.1 * r.standard_normal(D).astype(np.float32),
                                               sparse_vector=sp_mod.SparseVector(t.tolist(), [1.0] * 4, 300),
                                               limit=limit))
    out = eng.search_batch(reqs)
    o = oracle_mod.Bm25()
    for i, (t, v, dl) in enumerate(docs):
        o.add_document(i, t, v, dl)
    for qi, req in enumerate(reqs):
        d_ids, d_sc, d_n = dense.search_batch(np.asarray(req.dense_vector)[None], 2 * limit, eng.dense_params)
        dl = [(int(d_ids[0, j]), float(d_sc[0, j])) for j in range(int(d_n[0]))]
        si, ss = o.search(np.array(req.sparse_vector.indices, np.uint32),
                          np.array(req.sparse_vector.values, np.float32), 2 * limit)
        want = oracle_mod.rrf_fusion(dl, list(zip(si.tolist(), ss.tolist())), [], 60.0)[:limit]
        assert [d for d, _, _ in out[qi]] == [f"doc{w[0]}" for w in want]
        assert np.array([s for _, s, _ in out[qi]], np.float32).tobytes() == \
            np.array([w[1] for w in want], np.float32).tobytes()


def test_bm25_unstaged_chunks(sp_mod, oracle_mod):
    """Documents with ~80 distinct terms of a 400-term vocabulary and 64
    queries of 8 terms: a 128-document chunk holds more postings of the
    group's terms than the 4096-entry LDS stage, so the rounds read the
    posting runs from HBM (k_bm25_taat's unstaged path)."""
    docs = zipf_docs(31, 6000, 400, 160, a=0.3)
    assert np.mean([t.size for t, _, _ in docs]) > 60
    g, o = build(sp_mod, oracle_mod, docs)
    check_batch(sp_mod, g, o, queries(32, 64, 400, 6, 10), 30)


def test_bm25_batch_groups_and_repeated_terms(sp_mod, oracle_mod):
    """150 queries (three launch groups of <= 64), every query repeating a
    term (each occurrence adds again, sparse.rs:167-190), re-added ids (a
    second posting of the same document in a run)."""
    docs = zipf_docs(33, 20_000, 3000, 30)
    g, o = build(sp_mod, oracle_mod, docs)
    for i in (5, 129, 130, 19_999):
        t, v, dl = docs[(i * 7) % len(docs)]
        g.add_documents_u64(np.array([i], np.uint64), np.array([0, t.size], np.uint64), t, v, np.array([dl]))
        o.add_document(i, t, v, dl)
    qs = []
    for t, v in queries(34, 150, 3000, 2, 7):
        qs.append((np.append(t, t[0]).astype(np.uint32), np.append(v, np.float32(0.25)).astype(np.float32)))
    check_batch(sp_mod, g, o, qs, 12)


def test_rrf_large_lists_match_oracle(sp_mod, oracle_mod):
    """limit 400 -> 800-entry dense / sparse lists (more than the old 1024-item
    cap in total) with overlapping and repeated ids."""
    r = np.random.default_rng(41)
    B = 6
    D, S, T = [], [], []
    for _ in range(B):
        mk = lambda n: [(int(x), float(r.random())) for x in r.integers(0, 1500, n)]  # noqa: E731
        D.append(mk(800))
        S.append(mk(800))
        T.append(mk(int(r.integers(0, 300))))
    got = sp_mod.rrf_fuse(D, S, T, 60.0, 400)
    for b in range(B):
        want = oracle_mod.rrf_fusion(D[b], S[b], T[b], 60.0)[:400]
        assert [x[0] for x in got[b]] == [w[0] for w in want], b
        assert np.array([x[1] for x in got[b]], np.float32).tobytes() == \
            np.array([w[1] for w in want], np.float32).tobytes()
        for x, w in zip(got[b], want):
            assert same([np.nan if v is None else v for v in x[2]], w[2:])


def test_rrf_over_capacity_is_an_error(sp_mod):
    big = [[(i, 1.0) for i in range(2100)]]
    with pytest.raises(Exception, match="4096"):
        sp_mod.rrf_fuse(big, big, [], 60.0, 10)


def test_bm25_long_queries(sp_mod, oracle_mod):
    """Queries of 17-60 live terms (past the 16 lane-resident rounds of the
    fast path), mixed with short ones in the same launch group."""
    docs = zipf_docs(35, 15_000, 1500, 40)
    g, o = build(sp_mod, oracle_mod, docs)
    qs = queries(36, 20, 1500, 17, 61) + queries(37, 20, 1500, 1, 5)
    check_batch(sp_mod, g, o, qs, 15)


def test_bm25_special_values(sp_mod, oracle_mod):
    """Zero, negative and infinite tf / q_tf and term ids up to 2^32 - 1: a
    posting whose tf_component is +0.0 still matches (score 0), a non-finite
    q_tf poisons only its own query (the per-term select path), and sparse
    32-bit term ids map through the index's dense vocabulary."""
    r = np.random.default_rng(31)
    vocab = np.array([0, 1, 2, 5, 77, 1 << 20, (1 << 31) + 3, 0xFFFFFFFE, 0xFFFFFFFF], np.uint32)
    docs = []
    for i in range(6000):
        t = np.unique(r.choice(vocab, size=int(r.integers(1, 6)), replace=False)).astype(np.uint32)
        v = r.choice(np.array([0.0, 1.0, 2.5, -1.0, 0.25], np.float32), size=t.size)
        docs.append((t, v.astype(np.float32), np.float32(r.integers(1, 20))))
    g, o = build(sp_mod, oracle_mod, docs)
    qs = [(np.array([0xFFFFFFFF, 1 << 20], np.uint32), np.array([1.0, 2.0], np.float32)),
          (np.array([5, 77], np.uint32), np.array([np.inf, 1.0], np.float32)),
          (np.array([2], np.uint32), np.array([0.0], np.float32)),
          (np.array([(1 << 31) + 3, 0, 1], np.uint32), np.array([1.0, -2.0, 0.5], np.float32)),
          (np.array([0xFFFFFFFE, 12345], np.uint32), np.array([np.nan, 1.0], np.float32))]
    for limit in (7, 300):
        check_batch(sp_mod, g, o, qs, limit)
