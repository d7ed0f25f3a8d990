"""CPU, world_size 2 and 3 (gloo): the sharded orchestrations (gvdb.sharded)
equal one multi_stage_search over the whole corpus.

* TwoExchangeSearch -- the production protocol: local stage-1
  keys -> all-gather -> global top-R by (Hamming, corpus row) + rerank of the
  rows this rank owns + local top-k -> all-gather -> merged top-k, through the
  host forms of libgvdb's merges (gvdb_shard_merge_host / _local_topk_host /
  _final_host; the device forms run the same blocks on the GPU).  Includes
  uneven shards and an EMPTY shard (it joins both exchanges with no entries).
* ShardedBQSearch -- the earlier one-exchange variant.
Per-shard stage 1 and cosines come from the oracle here (no GPU on this host)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

N, D, B, R, K = 3001, 64, 6, 40, 10


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    rng = np.random.default_rng(123)
    x = rng.standard_normal((N, D)).astype(np.float32)
    x[500:560] = x[10]  # ties across the shard boundary region
    x[1490:1530] = x[10]
    q = rng.standard_normal((B, D)).astype(np.float32)
    q[0] = x[10]
    return x, q


def _worker(rank, world, port, ret):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "grape-vector-db_amd")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import oracle
    from gvdb.sharded import ShardedBQSearch, shard_bounds

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x, q = _data()
    b = shard_bounds(N, world)
    lo, hi = b[rank], b[rank + 1]
    xs = x[lo:hi]

    def cand(qt, r):
        qn = qt.numpy()
        idx, dd = oracle.bq_topr_batch(oracle.quantize(qn), oracle.quantize(xs), D, r)
        cos = np.array([[oracle.cosine_manual(qn[i], xs[int(j)]) for j in idx[i]] for i in range(B)], np.float32)
        return (torch.from_numpy((idx.astype(np.int64) + lo)), torch.from_numpy(dd.astype(np.int32)),
                torch.from_numpy(cos))

    s = ShardedBQSearch(cand, [b[g + 1] - b[g] for g in range(world)], B, R, K, torch.device("cpu"))
    ids, sc, n = s.search(torch.from_numpy(q))
    ri, rs = oracle.multi_stage_search_batch_r(oracle.quantize(q), oracle.quantize(x), q, x, R)
    ok = bool((n.numpy() == K).all() and (ids.numpy().astype(np.uint64) == ri[:, :K]).all()
              and sc.numpy().tobytes() == rs[:, :K].tobytes())
    ret[rank] = int(ok)
    dist.destroy_process_group()


def _worker2(rank, world, port, ret, bounds, R):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "grape-vector-db_amd")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import oracle
    from gvdb.sharded import TwoExchangeSearch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x, q = _data()
    lo, hi = bounds[rank], bounds[rank + 1]
    xs = x[lo:hi]

    def stage1(qt, r):
        if hi == lo:
            return np.zeros((B, 0), np.uint64), np.zeros((B, 0), np.uint64)
        idx, dd = oracle.bq_topr_batch(oracle.quantize(qt.numpy()), oracle.quantize(xs), D, min(r, hi - lo))
        return idx, dd

    def cosine(i, local_rows):
        return np.array([oracle.cosine_manual(q[i], xs[int(j)]) for j in local_rows], np.float32)

    s = TwoExchangeSearch(B, R, K, torch.device("cpu"), stage1_fn=stage1, cosine_fn=cosine, id_offset=lo)
    ids, sc, n = s.search(torch.from_numpy(q))
    ri, rs = oracle.multi_stage_search_batch_r(oracle.quantize(q), oracle.quantize(x), q, x, R)
    ok = bool((n.numpy() == K).all() and (ids.numpy().astype(np.uint64) == ri[:, :K]).all()
              and sc.numpy().tobytes() == rs[:, :K].tobytes())
    ret[rank] = int(ok)
    dist.destroy_process_group()


def _worker_fail(rank, world, port, ret, bad_rank, phase, R=R):
    """One rank's stage 1 (phase 1) or cosine callable (phase 2) raises: every
    rank still completes both all-gathers (no hang), every query of the merge
    is poisoned on every rank, and only the failing rank raises."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "grape-vector-db_amd")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import oracle
    from gvdb.sharded import TwoExchangeSearch, shard_bounds

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x, q = _data()
    bnd = shard_bounds(N, world)
    lo, hi = bnd[rank], bnd[rank + 1]
    xs = x[lo:hi]

    def stage1(qt, r):
        if rank == bad_rank and phase == 1:
            raise ValueError("dimension mismatch on this shard")
        return oracle.bq_topr_batch(oracle.quantize(qt.numpy()), oracle.quantize(xs), D, min(r, hi - lo))

    def cosine(i, local_rows):
        if rank == bad_rank and phase == 2:
            raise ValueError("rerank failed on this shard")
        return np.array([oracle.cosine_manual(q[i], xs[int(j)]) for j in local_rows], np.float32)

    s = TwoExchangeSearch(B, R, K, torch.device("cpu"), stage1_fn=stage1, cosine_fn=cosine, id_offset=lo, dim=D)
    raised = False
    try:
        s.search(torch.from_numpy(q))
    except ValueError:
        raised = True
    # the merge ran on every rank: its outputs are the poisoned counts
    poisoned = bool((s.send2.numpy().view(np.uint32)[4 * B * K + 2 * B] == 1) == (rank == bad_rank))
    # a second search on the same ranks still works (nobody is stuck in a collective)
    s2 = TwoExchangeSearch(B, R, K, torch.device("cpu"), stage1_fn=lambda qt, r: oracle.bq_topr_batch(
        oracle.quantize(qt.numpy()), oracle.quantize(xs), D, min(r, hi - lo)), cosine_fn=lambda i, rows: np.array(
        [oracle.cosine_manual(q[i], xs[int(j)]) for j in rows], np.float32), id_offset=lo, dim=D)
    ids, sc, n = s2.search(torch.from_numpy(q))
    ok_after = bool((n.numpy() == K).all())
    ret[rank] = (raised == (rank == bad_rank), poisoned, ok_after)
    dist.destroy_process_group()


def _worker_fail_outputs(rank, world, port, ret):
    """The poisoned merge's outputs on a healthy rank: every out_n is POISONED."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "grape-vector-db_amd")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import oracle
    from gvdb._ffi import GVDB_N_POISONED
    from gvdb.sharded import TwoExchangeSearch, shard_bounds

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x, q = _data()
    bnd = shard_bounds(N, world)
    lo, hi = bnd[rank], bnd[rank + 1]
    xs = x[lo:hi]

    def stage1(qt, r):
        if rank == 1:
            raise ValueError("bad shard")
        return oracle.bq_topr_batch(oracle.quantize(qt.numpy()), oracle.quantize(xs), D, min(r, hi - lo))

    s = TwoExchangeSearch(B, R, K, torch.device("cpu"), stage1_fn=stage1,
                          cosine_fn=lambda i, rows: np.array([oracle.cosine_manual(q[i], xs[int(j)]) for j in rows],
                                                             np.float32), id_offset=lo)
    try:
        _, _, n = s.search(torch.from_numpy(q))
        ret[rank] = bool((n.numpy().view(np.uint32) == GVDB_N_POISONED).all())
    except ValueError:
        ret[rank] = rank == 1
    dist.destroy_process_group()


@pytest.mark.parametrize("phase,r", [(1, R), (2, R), (1, 9000), (2, 9000)])
def test_two_exchange_failing_rank_joins_both_exchanges(phase, r, oracle_mod, gvdb_lib_path):
    """Key form (R = 40) and deep form (R = 9000 > 8192: histogram exchange)."""
    world = 3
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    mp.spawn(_worker_fail, args=(world, _free_port(), ret, 1, phase, r), nprocs=world, join=True)
    assert dict(ret) == {r: (True, True, True) for r in range(world)}


def test_two_exchange_failing_rank_poisons_every_query(oracle_mod, gvdb_lib_path):
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    mp.spawn(_worker_fail_outputs, args=(2, _free_port(), ret), nprocs=2, join=True)
    assert dict(ret) == {0: True, 1: True}


@pytest.mark.parametrize("world,bounds,R", [(2, (0, 1500, N), 40), (3, (0, 900, 900, N), 40),
                                            (3, (0, 1000, 2000, N), 300)])
def test_two_exchange_equals_single_corpus(world, bounds, R, oracle_mod, gvdb_lib_path):
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    mp.spawn(_worker2, args=(world, _free_port(), ret, bounds, R), nprocs=world, join=True)
    assert dict(ret) == {r: 1 for r in range(world)}


@pytest.mark.parametrize("world", [2])
def test_sharded_equals_single_corpus(world, oracle_mod, gvdb_lib_path):
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), ret), nprocs=world, join=True)
    assert dict(ret) == {r: 1 for r in range(world)}


N3, D3, B3 = 26000, 64, 4


def _worker_deep(rank, world, port, ret, bounds, R):
    """The deep form (R > 8192): exchange 1 carries the Hamming histograms of
    the ranks' local top-R; the owned entries and the merge come from the host
    forms (gvdb_shard_deep_own_host / _local_topk_host / _final_host)."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "grape-vector-db_amd")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import oracle
    from gvdb.sharded import TwoExchangeSearch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(321)
    x = rng.standard_normal((N3, D3)).astype(np.float32)
    x[bounds[1]:bounds[1] + 30] = x[4]  # equal rows across a shard boundary
    x[7000:7030] = x[4]
    q = rng.standard_normal((B3, D3)).astype(np.float32)
    q[0] = x[4]
    lo, hi = bounds[rank], bounds[rank + 1]
    xs = x[lo:hi]

    def stage1(qt, r):
        if hi == lo:
            return np.zeros((B3, 0), np.uint64), np.zeros((B3, 0), np.uint64)
        idx, dd = oracle.bq_topr_batch(oracle.quantize(qt.numpy()), oracle.quantize(xs), D3, min(r, hi - lo))
        perm = np.random.default_rng(rank).permutation(idx.shape[1])  # membership, any order
        return idx[:, perm], dd[:, perm]

    def cosine(i, local_rows):
        return np.array([oracle.cosine_manual(q[i], xs[int(j)]) for j in local_rows], np.float32)

    s = TwoExchangeSearch(B3, R, K, torch.device("cpu"), stage1_fn=stage1, cosine_fn=cosine, id_offset=lo, dim=D3)
    ids, sc, n = s.search(torch.from_numpy(q))
    ri, rs = oracle.multi_stage_search_batch_r(oracle.quantize(q), oracle.quantize(x), q, x, R)
    ok = bool((n.numpy() == K).all() and (ids.numpy().astype(np.uint64) == ri[:, :K]).all()
              and sc.numpy().tobytes() == rs[:, :K].tobytes())
    ret[rank] = int(ok)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,bounds,R", [(2, (0, 13000, N3), 9000), (3, (0, 9000, 9000, N3), 12000),
                                            (3, (0, 2000, 20000, N3), 20000)])
def test_deep_two_exchange_equals_single_corpus(world, bounds, R, oracle_mod, gvdb_lib_path):
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    mp.spawn(_worker_deep, args=(world, _free_port(), ret, bounds, R), nprocs=world, join=True)
    assert dict(ret) == {r: 1 for r in range(world)}
