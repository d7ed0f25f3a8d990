#!/usr/bin/env python3
"""Batch-256 BQ search timing on one GPU (timing only): step time and the
stage-1 scan's HIP-event average, for N = $SHARD_N rows (default 10M x 768);
GVDB_LIB_PATH selects a timing variant of libgvdb.so.  With RCCL=1 also the
in-library sharded step over a 1-rank communicator."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "grape-vector-db_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import gvdb  # noqa: E402

n = int(os.environ.get("SHARD_N", 10_000_000))
D, B, R, k = int(os.environ.get("DIM", 768)), 256, 100, 10
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
L = gvdb.lib()
tag = os.environ.get("TAG", os.path.basename(os.environ.get("GVDB_LIB_PATH", "base")))


def timeit(name, fn, steps=40):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    L.gvdb_timing_reset()
    L.gvdb_timing_enable(1)
    t = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3 / steps
    L.gvdb_timing_enable(0)
    tm, tn = C.c_double(), C.c_uint64()
    L.gvdb_timing_read(1, C.byref(tm), C.byref(tn))
    scan = tm.value / max(tn.value, 1)
    print(f"[{tag}] N={n} {name}: {ms:.4f} ms/step ({B / ms * 1e3:,.0f} QPS), scan {scan:.4f} ms", flush=True)


timeit("search_device", lambda: ix.search_device(q, k, oi, osc, on, sp))
if os.environ.get("RCCL"):
    from gvdb.sharded import RcclShardedSearch

    sh = RcclShardedSearch(ix, R, k)
    timeit("sharded (RCCL comm, world 1)", lambda: sh.search_into(q, oi, osc, on))
    sh.close()
