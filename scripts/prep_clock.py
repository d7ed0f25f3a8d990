#!/usr/bin/env python3
"""Timing study of k_sample_prep per wave (variant build -DGVDB_PREP_CLK): at the
1.25M-row shard, batch 256: us from the earliest wave start to the end of the
packing, the fragment build and the sample loop."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "grape-vector-db_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import gvdb  # noqa: E402

D, B, R, k, n = 768, 256, 100, 10, int(os.environ.get("SHARD_N", 1_250_000))
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
L = gvdb.lib()
q = bench.gen_queries(B, D, dev)
ix = gvdb.GpuVectorIndex(dimension=D, device=0, capacity_hint=n)
for c in range((n + bench.CHUNK - 1) // bench.CHUNK):
    lo, hi = c * bench.CHUNK, min(n, (c + 1) * bench.CHUNK)
    ix.add_device(bench.gen_chunk(c, hi - lo, D, dev), torch.arange(lo, hi, device=dev))
sp = gvdb.SearchParams(rescore_count=R)
oi = torch.zeros((B, k), dtype=torch.int64, device=dev)
osc = torch.zeros((B, k), dtype=torch.float32, device=dev)
on = torch.zeros(B, dtype=torch.int32, device=dev)
for _ in range(30):
    ix.search_device(q, k, oi, osc, on, sp)
torch.cuda.synchronize()
buf = (C.c_ulonglong * (2048 * 5))()
assert L.gvdb_debug_prep_clock(buf) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(2048, 5).astype(np.float64)
t0 = a[:, 0].min()
us = (a[:, :4] - t0) / 100.0
for i, nm in enumerate(["start", "packed", "fragments", "sampled"]):
    print(f"[prepclk] {nm:10s} min {us[:, i].min():7.2f} med {np.median(us[:, i]):7.2f} max {us[:, i].max():7.2f} us",
          flush=True)
