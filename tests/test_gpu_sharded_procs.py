"""GPU, 2 and 3 processes: the two-exchange sharded search (SURVEY 8(e);
shard.rs:760-786) with its phases on the device in separate processes.

Each process owns one contiguous shard of the corpus as a GpuVectorIndex whose
ids are global row numbers, and runs gvdb.sharded.TwoExchangeSearch in device
mode (gvdb_shard_stage1_device -> all-gather -> gvdb_shard_rerank_device ->
all-gather -> gvdb_shard_final_device).  One GPU box cannot hold two RCCL ranks
on one device ("Duplicate GPU detected"), so the all-gathers go through gloo on
host copies of the same exchange blocks; everything else is the production
device path.  test_gpu_sharded.py emulates G = 8 shards in ONE process;
test_sharded_gloo.py runs the protocol across processes with host forms of the
phases; this runs the device forms across processes.  Every rank's merged
top-k must equal the oracle's multi_stage_search over the whole corpus (ids
and cosine bits), in the regular form (R <= 8192) and the deep form (R > 8192,
histogram exchange)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ret, N, D, B, R, k, bounds, seed):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "grape-vector-db_amd")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import gvdb
    import oracle
    from gvdb.sharded import TwoExchangeSearch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        rng = np.random.default_rng(seed)
        x = rng.standard_normal((N, D)).astype(np.float32)
        x[bounds[1] - 20:bounds[1] + 20] = x[3]  # equal rows across a shard boundary
        q = rng.standard_normal((B, D)).astype(np.float32)
        q[0] = x[3]
        q[1] = x[N - 5]
        lo, hi = bounds[rank], bounds[rank + 1]
        ix = gvdb.GpuVectorIndex(dimension=D, capacity_hint=max(hi - lo, 1))
        if hi > lo:
            ix.add_batch(np.arange(lo, hi, dtype=np.uint64), x[lo:hi])

        class GlooDeviceSearch(TwoExchangeSearch):
            def _gather(self, send, recv):  # the exchange blocks through gloo on host copies
                parts = [torch.empty_like(send, device="cpu") for _ in range(self.world)]
                dist.all_gather(parts, send.cpu())
                recv.copy_(torch.stack(parts).to(recv.device))

        s = GlooDeviceSearch(B, R, k, dev, index=ix, dim=D)
        ids, sc, n = s.search(torch.from_numpy(q).to(dev))
        torch.cuda.synchronize()
        ri, rs = oracle.multi_stage_search_batch_r(oracle.quantize(q), oracle.quantize(x), q, x, R, threads=8)
        ok = bool((n.cpu().numpy() == k).all() and (ids.cpu().numpy().astype(np.uint64) == ri[:, :k]).all()
                  and sc.cpu().numpy().tobytes() == np.ascontiguousarray(rs[:, :k]).tobytes()
                  and int(ids[0, 0]) == 3)
        ret[rank] = int(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N,D,B,R,bounds", [
    (2, 60_000, 256, 8, 100, (0, 30_000, 60_000)),
    (3, 60_000, 768, 6, 300, (0, 10_000, 45_000, 60_000)),
    (2, 40_000, 128, 4, 12_000, (0, 16_000, 40_000)),  # deep form: histogram exchange
])
def test_two_exchange_device_phases_across_processes(world, N, D, B, R, bounds, gvdb_lib_path):
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), ret, N, D, B, R, 10, bounds, N + D + R), nprocs=world, join=True)
    assert dict(ret) == {r: 1 for r in range(world)}
