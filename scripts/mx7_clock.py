#!/usr/bin/env python3
"""Timing study of k_scan_mx7 (the stage-1 FP4 scan) per wave: where a launch's
time goes at the 8-GPU shard (1.25M x 768) and at 10M rows, batch 256, R = 100.
Needs the variant build with -DGVDB_MX7_CLK (scripts/build_variant.sh mx7clk
"-DGVDB_MX7_CLK"; run with GVDB_LIB_PATH pointing at it).  Prints, over the
waves of the last launch (s_memrealtime, 100 MHz -> us from the earliest wave
start): start skew, prologue, full rounds, tail units, flush, end; and the tile
tests that took the hit path per wave."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "grape-vector-db_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import gvdb  # noqa: E402

D, B, R, k = 768, 256, 100, 10
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
L = gvdb.lib()
fn = L.gvdb_debug_mx7_clock
fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_uint32]
q = bench.gen_queries(B, D, dev)
for n in [int(x) for x in os.environ.get("SHARD_N", "1250000,10000000").split(",")]:
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
    waves = 256 * 8
    buf = (C.c_ulonglong * (waves * 6))()
    assert fn(buf, waves) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(waves, 6).astype(np.float64)
    os.makedirs("gpurun_out", exist_ok=True)
    np.save(f"gpurun_out/mx7clk_{n}.npy", a)  # raw per-wave clocks (wave gw = 8 * block + wave)
    t0 = a[:, 0].min()
    us = (a[:, :5] - t0) / 100.0  # 100 MHz ticks -> us
    ph = np.diff(us, axis=1)
    names = ["prologue", "full rounds", "tail units", "flush"]
    print(f"[mx7clk] N={n}: start skew max {us[:, 0].max():.2f} us, end min/med/max "
          f"{us[:, 4].min():.2f}/{np.median(us[:, 4]):.2f}/{us[:, 4].max():.2f} us", flush=True)
    for i, nm in enumerate(names):
        print(f"[mx7clk] N={n}:   {nm:12s} mean {ph[:, i].mean():7.2f}  max {ph[:, i].max():7.2f} us", flush=True)
    print(f"[mx7clk] N={n}:   hit-path tile tests per wave: mean {a[:, 5].mean():.1f}, max {a[:, 5].max():.0f} "
          f"(of ~{8 * ((n + 31) // 32) / waves:.0f} tile tests)", flush=True)
    del ix
    torch.cuda.empty_cache()
