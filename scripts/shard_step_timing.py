"""Per-rank cost of one sharded step at the 8-GPU shard size (1.25M x 768,
batch 256) on ONE GPU: the single-device search vs the sharded orchestration
(local candidates + pack + world-1 'gather' copy + unpack + merge) without the
collective.  Timing only (no parity claim); run under rocprofv3 for the
per-kernel breakdown."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "grape-vector-db_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import gvdb  # noqa: E402
from gvdb.sharded import ShardedBQSearch, gpu_candidates_fn  # noqa: E402

n = int(os.environ.get("SHARD_N", 1_250_000))
D, B, R, k = 768, 256, 100, 10
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
q = bench.gen_queries(B, D, dev)
ix = gvdb.GpuVectorIndex(dimension=D, device=0, capacity_hint=n)
for c in range((n + bench.CHUNK - 1) // bench.CHUNK):
    lo, hi = c * bench.CHUNK, min(n, (c + 1) * bench.CHUNK)
    ix.add_device(bench.gen_chunk(c, hi - lo, D, dev), torch.arange(lo, hi, device=dev))
sp = gvdb.SearchParams(rescore_count=R)
oi = torch.zeros((B, k), dtype=torch.int64, device=dev)
osc = torch.zeros((B, k), dtype=torch.float32, device=dev)
on = torch.zeros(B, dtype=torch.int32, device=dev)
sh = ShardedBQSearch(gpu_candidates_fn(ix), [n], B, R, k, dev)


def timeit(name, fn, steps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3 / steps
    print(f"{name}: {ms:.4f} ms/step  ({B / ms * 1e3:,.0f} QPS per rank)", flush=True)


timeit("single-device search_device", lambda: ix.search_device(q, k, oi, osc, on, sp))
timeit("sharded step (world 1, no collective)", lambda: sh.search(q))
a = sh.search(q)[0].clone()
ix.search_device(q, k, oi, osc, on, sp)
print("same ids:", bool((a == oi).all()))
