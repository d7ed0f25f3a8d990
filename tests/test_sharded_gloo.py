"""CPU, world_size 2 (gloo): the sharded orchestration (gvdb.sharded) —
contiguous row shards with global ids, one all-gather of (id, Hamming,
cosine) triplets, exact merge (the product's host merge in libgvdb) — equals
one multi_stage_search over the whole corpus.  Per-shard candidates come from
the oracle here (no GPU on this host); on the GPU box the same class runs
with gpu_candidates_fn and the device merge (bench.py)."""
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


@pytest.mark.parametrize("world", [2])
def test_sharded_equals_single_corpus(world, oracle_mod, gvdb_lib_path):
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), ret), nprocs=world, join=True)
    assert dict(ret) == {r: 1 for r in range(world)}
