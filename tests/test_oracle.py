"""CPU: pin the oracle (oracle/gvdb_oracle.cpp) against the reference's own
known-answer tests (tests/golden/kat.json) and against an independent
pure-Python restatement that steps through the Rust f32 arithmetic one
operation at a time (np.float32 scalars: no FMA, no reassociation)."""
import json
import math
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "kat.json")))
f32 = np.float32


# ---------- independent pure-Python restatement (small cases only) ----------
def py_quantize(v, thr=0.0):
    D = len(v)
    out = [0] * ((D + 7) // 8)
    for i, x in enumerate(v):
        if f32(x) > f32(thr):  # NaN > t is False
            out[i >> 3] |= 0x80 >> (i & 7)
    return out


def py_hamming(a, b):
    return sum(bin(x ^ y).count("1") for x, y in zip(a, b))


def py_sum(vals):
    s = f32(-0.0)
    for v in vals:
        s = f32(s + f32(v))
    return s


def py_cos(a, b):
    dot = py_sum(f32(x) * f32(y) for x, y in zip(a, b))  # zip truncates
    na = f32(math.sqrt(py_sum(f32(x) * f32(x) for x in a)))
    nb = f32(math.sqrt(py_sum(f32(x) * f32(x) for x in b)))
    if na == 0 or nb == 0:
        return f32(0.0)
    return f32(dot / f32(na * nb))


def py_multi_stage(qv, cands, ratio, thr=0.0):
    qb = py_quantize(qv, thr)
    D = len(qv)
    s1 = []
    for i, c in enumerate(cands):
        d = py_hamming(qb, py_quantize(c, thr))
        s1.append((i, f32(f32(1.0) - f32(f32(d) / f32(D)))))
    s1.sort(key=lambda t: -t[1])  # Python sort is stable, like Rust's sort_by
    R = min(int(f32(len(cands)) * f32(ratio)) if f32(len(cands)) * f32(ratio) > 0 else 0, len(cands))
    s2 = [(i, py_cos(qv, cands[i])) for i, _ in s1[:R]]
    s2.sort(key=lambda t: -t[1])
    return s2


# ---------- KATs from the reference tests ----------
@pytest.mark.parametrize("case", KAT["quantize"])
def test_kat_quantize(oracle_mod, case):
    got = oracle_mod.quantize(case["vector"], case["threshold"])[0]
    assert list(got) == case["bytes"]
    assert py_quantize(case["vector"]) == case["bytes"]


@pytest.mark.parametrize("case", KAT["hamming"])
def test_kat_hamming(oracle_mod, case):
    a = oracle_mod.quantize(case["a"])[0]
    b = oracle_mod.quantize(case["b"])[0]
    d = oracle_mod.hamming(a, b)
    assert d == case["distance"] and d > 0
    assert oracle_mod.similarity(d, len(case["a"])) == case["similarity"]


@pytest.mark.parametrize("case", KAT["vector_search"])
def test_kat_vector_search(oracle_mod, case):
    ids = list(case["corpus"])
    rows = np.array([case["corpus"][i] for i in ids], np.float32)
    idx, sc = oracle_mod.storage_vector_search(case["query"], rows, case["limit"])
    assert ids[int(idx[0])] == case["top1"]


# ---------- oracle vs independent restatement ----------
def test_cosine_matches_stepwise(oracle_mod):
    rng = np.random.default_rng(1)
    for D in (1, 3, 7, 64, 100, 768):
        a = rng.standard_normal(D).astype(np.float32)
        b = rng.standard_normal(D).astype(np.float32)
        assert np.float32(oracle_mod.cosine_manual(a, b)).tobytes() == py_cos(a, b).tobytes()


def test_multi_stage_matches_stepwise(oracle_mod):
    rng = np.random.default_rng(2)
    for N, D, ratio in ((50, 16, 0.1), (200, 37, 0.25), (64, 128, 1.0), (30, 8, 0.5)):
        X = rng.standard_normal((N, D)).astype(np.float32)
        X[5] = X[3]  # duplicate row: equal Hamming AND equal cosine -> stable ties
        q = rng.standard_normal(D).astype(np.float32)
        cb = oracle_mod.quantize(X)
        qb = oracle_mod.quantize(q)[0]
        idx, cos = oracle_mod.multi_stage_search(qb, D, cb, D, q, X, ratio)
        ref = py_multi_stage(q, X, ratio)
        assert [int(i) for i in idx] == [i for i, _ in ref]
        assert np.array(cos, np.float32).tobytes() == np.array([c for _, c in ref], np.float32).tobytes()


def test_rescore_count_is_f32_truncation(oracle_mod):
    # (N as f32 * ratio) as usize — truncation of an f32 product
    assert oracle_mod.rust_f32_as_usize(f32(10_000_000) * f32(1e-5)) == int(f32(10_000_000) * f32(1e-5))
    assert oracle_mod.rust_f32_as_usize(f32(33) * f32(0.1)) == 3
    assert oracle_mod.rust_f32_as_usize(float("nan")) == 0
    assert oracle_mod.rust_f32_as_usize(-1.0) == 0


def test_dimension_mismatch_scores_zero(oracle_mod):
    # similarity().unwrap_or(0.0): every candidate ties at 0.0 -> index order
    rng = np.random.default_rng(3)
    X = rng.standard_normal((20, 16)).astype(np.float32)
    q = rng.standard_normal(8).astype(np.float32)
    idx, cos, s1i, s1s = oracle_mod.multi_stage_search(oracle_mod.quantize(q)[0], 8, oracle_mod.quantize(X), 16, q, X,
                                                       0.5, want_stage1=True)
    assert list(s1i) == list(range(20)) and all(s == 0.0 for s in s1s)
    # dot over the zip-truncated length, norms over each full vector (quantization.rs:207-209)
    for i, c in zip(idx, cos):
        assert np.float32(c).tobytes() == py_cos(q, X[int(i)]).tobytes()


def test_zero_dimension_panics_as_error(oracle_mod):
    X = np.zeros((3, 0), np.float32)
    with pytest.raises(RuntimeError):
        oracle_mod.multi_stage_search(np.zeros(0, np.uint8), 0, np.zeros((3, 0), np.uint8), 0, np.zeros(0), X, 1.0)


def test_storage_threshold_and_ties(oracle_mod):
    rows = np.array([[1, 0], [1, 0], [0, 1], [-1, 0], [0, 0]], np.float32)
    idx, sc = oracle_mod.storage_vector_search([1, 0], rows, 10, threshold=0.0)
    # zero vector scores 0.0 (>= 0.0 kept); ties keep record order
    assert list(idx) == [0, 1, 2, 4] and list(sc) == [1.0, 1.0, 0.0, 0.0]
    idx, sc = oracle_mod.storage_vector_search([1, 0], rows, 2)
    assert list(idx) == [0, 1]


def test_flat_cosine_distance(oracle_mod):
    rows = np.array([[0, 0], [1, 0], [0, 1], [1, 1]], np.float32)
    idx, sc = oracle_mod.flat_cosine_distance_search([1, 0], rows, 4)
    assert list(idx) == [1, 3, 2, 0]  # zero norm -> +inf distance, last
    assert math.isinf(sc[-1])


def test_l2_matches_stepwise(oracle_mod):
    rng = np.random.default_rng(4)
    a = rng.standard_normal(300).astype(np.float32)
    b = rng.standard_normal(300).astype(np.float32)
    ref = f32(math.sqrt(py_sum(f32(x - y) * f32(x - y) for x, y in zip(a, b))))
    assert np.float32(oracle_mod.l2_distance(a, b)) == ref


def test_shard_merge_stable(oracle_mod):
    ids = np.array([[1, 2, 3], [4, 5, 0]], np.uint64)
    sc = np.array([[0.9, 0.5, 0.1], [0.9, 0.7, 0.0]], np.float32)
    cnt = np.array([3, 2], np.uint64)
    oi, os_ = oracle_mod.shard_merge(ids, sc, cnt, 4)
    assert list(oi) == [1, 4, 5, 2]


def test_bq_topr_equals_stable_stage1(oracle_mod):
    rng = np.random.default_rng(5)
    X = rng.standard_normal((500, 64)).astype(np.float32)
    X[100:110] = X[7]  # heavy ties
    Q = rng.standard_normal((4, 64)).astype(np.float32)
    Q[1] = X[7]
    cb, qb = oracle_mod.quantize(X), oracle_mod.quantize(Q)
    ti, td = oracle_mod.bq_topr_batch(qb, cb, 64, 50)
    for b in range(4):
        _, _, s1i, _ = oracle_mod.multi_stage_search(qb[b], 64, cb, 64, Q[b], X, 0.1, want_stage1=True)
        assert list(ti[b]) == [int(i) for i in s1i[:50]]


def test_batched_flat_searches_equal_single(oracle_mod):
    """The threaded batch forms (the B >= 128 GPU flat checkers) are the
    per-query storage.rs / index.rs searches, bit for bit."""
    rng = np.random.default_rng(6)
    X = rng.standard_normal((700, 48)).astype(np.float32)
    X[10:20] = X[3]  # ties
    X[5] = 0.0
    Q = rng.standard_normal((9, 48)).astype(np.float32)
    Q[2] = X[3]
    ci, cs = oracle_mod.exact_topk_cosine_batch(Q, X, 15, threads=4)
    di, ds, dn = oracle_mod.flat_cosine_distance_batch(Q, X, 15, threads=4)
    for b in range(9):
        ri, rs = oracle_mod.storage_vector_search(Q[b], X, 15)
        assert list(ci[b]) == list(ri) and cs[b].tobytes() == rs.tobytes()
        ri, rs = oracle_mod.flat_cosine_distance_search(Q[b], X, 15)
        assert dn[b] == len(ri) and list(di[b]) == list(ri) and ds[b].tobytes() == rs.tobytes()
