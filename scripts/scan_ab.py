#!/usr/bin/env python3
"""Same-box A/B of stage-1 scan variants (timing only): one index of N rows
(env SHARD_N, default 10M x 768; the bench's synthetic corpus), batch-256 BQ
search steps, alternating GVDB_SCAN values (env SCANS, comma list; "" = the
default) REPS times; prints step ms and the scan's HIP-event average."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "grape-vector-db_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import gvdb  # noqa: E402

D, B, R, k = 768, 256, 100, 10
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
q = bench.gen_queries(B, D, dev)
L = gvdb.lib()
scans = os.environ.get("SCANS", "mx5,").split(",")
reps = int(os.environ.get("REPS", 3))
for n in [int(x) for x in os.environ.get("SHARD_N", "10000000").split(",")]:
    ix = gvdb.GpuVectorIndex(dimension=D, device=0, capacity_hint=n)
    for c in range((n + bench.CHUNK - 1) // bench.CHUNK):
        lo, hi = c * bench.CHUNK, min(n, (c + 1) * bench.CHUNK)
        ix.add_device(bench.gen_chunk(c, hi - lo, D, dev), torch.arange(lo, hi, device=dev))
    sp = gvdb.SearchParams(rescore_count=R)
    oi = torch.zeros((B, k), dtype=torch.int64, device=dev)
    osc = torch.zeros((B, k), dtype=torch.float32, device=dev)
    on = torch.zeros(B, dtype=torch.int32, device=dev)
    ref = None
    for rep in range(reps):
        for sc in scans:
            if sc:
                os.environ["GVDB_SCAN"] = sc
            else:
                os.environ.pop("GVDB_SCAN", None)
            for _ in range(5):
                ix.search_device(q, k, oi, osc, on, sp)
            torch.cuda.synchronize()
            res = (oi.cpu().clone(), osc.cpu().clone())
            if ref is None:
                ref = res
            same = bool((res[0] == ref[0]).all() and (res[1] == ref[1]).all())
            L.gvdb_timing_reset()
            L.gvdb_timing_enable(1)
            steps = 40
            t = time.perf_counter()
            for _ in range(steps):
                ix.search_device(q, k, oi, osc, on, sp)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) * 1e3 / steps
            L.gvdb_timing_enable(0)
            tm, tn = C.c_double(), C.c_uint64()
            L.gvdb_timing_read(1, C.byref(tm), C.byref(tn))
            print(f"[scan_ab] N={n} scan={sc or 'default'} rep={rep}: {ms:.4f} ms/step ({B / ms * 1e3:,.0f} QPS), "
                  f"scan {tm.value / max(tn.value, 1):.4f} ms, same_results={same}", flush=True)
    del ix
    torch.cuda.empty_cache()
