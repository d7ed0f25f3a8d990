"""CPU: the C-ABI library (libgvdb.so) loads without a GPU and exports every
function include/gvdb.h declares; the host-only entry points (merges) agree
with the oracle.  No HIP compute is called here."""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gvdb.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gvdb_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_functions():
    fns = header_functions()
    assert "gvdb_index_search" in fns and "gvdb_bq_multi_stage_search" in fns
    assert len(fns) >= 25


def test_library_exports_every_declared_symbol(gvdb_lib_path):
    out = subprocess.run(["nm", "-D", "--defined-only", gvdb_lib_path], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (gvdb_\w+)", out))
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing


def test_python_binding_covers_header(gvdb_mod):
    from gvdb import _ffi

    assert sorted(_ffi.SIGNATURES) == header_functions()


def test_status_codes_consistent(gvdb_mod):
    from gvdb import _ffi

    txt = open(HEADER).read()
    codes = dict((k, int(v)) for k, v in re.findall(r"(GVDB_(?:OK|ERR_\w+))\s*=\s*(\d+)", txt))
    for k, v in codes.items():
        assert getattr(_ffi, k) == v, k
    L = gvdb_mod.lib()
    assert L.gvdb_abi_version() == 3
    assert L.gvdb_status_string(1) == b"IndexNotBuilt"
    assert L.gvdb_status_string(2) == b"DimensionMismatch"


def test_host_topk_merge_matches_oracle(gvdb_mod, oracle_mod):
    rng = np.random.default_rng(0)
    S, B, stride = 3, 5, 7
    ids = rng.integers(0, 1000, (S, B, stride)).astype(np.uint64)
    sc = rng.integers(0, 4, (S, B, stride)).astype(np.float32) / 4  # many ties
    cnt = rng.integers(0, stride + 1, (S, B)).astype(np.uint32)
    oi, os_, on = gvdb_mod.topk_merge(ids, sc, cnt, 10)
    for q in range(B):
        ri, rs = oracle_mod.shard_merge(ids[:, q, :], sc[:, q, :], cnt[:, q].astype(np.uint64), 10)
        assert on[q] == len(ri)
        assert list(oi[q, :on[q]]) == list(ri) and list(os_[q, :on[q]]) == list(rs)


def test_host_bq_shard_merge_matches_oracle(gvdb_mod, oracle_mod):
    import ctypes as C

    rng = np.random.default_rng(1)
    G, B, stride, R, k = 4, 6, 20, 30, 10
    gids = np.zeros((G, B, stride), np.uint64)
    for g in range(G):
        gids[g] = g * 1000 + rng.integers(0, 1000, (B, stride))
    dist = rng.integers(100, 110, (G, B, stride)).astype(np.uint32)
    cosv = (rng.integers(0, 8, (G, B, stride)) / 8).astype(np.float32)
    counts = rng.integers(10, stride + 1, (G, B)).astype(np.uint32)
    oi = np.zeros((B, k), np.uint64)
    os_ = np.zeros((B, k), np.float32)
    on = np.zeros(B, np.uint32)
    p = lambda a: a.ctypes.data
    st = gvdb_mod.lib().gvdb_bq_shard_merge(p(gids), p(dist), p(cosv), p(counts), G, B, stride, R, k, p(oi), p(os_),
                                            p(on))
    assert st == 0
    ri, rs, rn = oracle_mod.bq_shard_merge(gids, dist, cosv, counts.astype(np.uint64), R, k)
    assert (on == rn).all() and (oi == ri).all() and (os_ == rs).all()
