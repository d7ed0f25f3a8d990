"""Timing study of the stage-1 scan variants (GPU box).  Builds a 10M x 768
index once, then times batch-256 stage-1 scans under GVDB_SCAN /
GVDB_SCAN_DBG settings (ablations give invalid results; timing only)."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "grape-vector-db_amd")]
import torch  # noqa: E402

import gvdb  # noqa: E402

N, D, B = int(os.environ.get("N", 10_000_000)), 768, 256
dev = torch.device("cuda", 0)
ix = gvdb.GpuVectorIndex(dimension=D, capacity_hint=N)
g = torch.Generator(device=dev).manual_seed(1)
for c0 in range(0, N, 1 << 20):
    n = min(1 << 20, N - c0)
    x = torch.randn((n, D), generator=g, device=dev)
    ix.add_device(x, torch.arange(c0, c0 + n, dtype=torch.int64, device=dev))
q = torch.randn((B, D), generator=g, device=dev)
rows = torch.zeros((B, 100), dtype=torch.int64, device=dev)
dist = torch.zeros((B, 100), dtype=torch.int32, device=dev)
L = gvdb.lib()
configs = sys.argv[1:] or ["fp4:0", "fp4:1", "fp4:2", "fp4:3", "fp4u:0", "i8:0", "valu:0"]
for cfg in configs:
    scan, dbg = cfg.split(":")
    os.environ["GVDB_SCAN"] = scan
    os.environ["GVDB_SCAN_DBG"] = dbg
    for _ in range(2):
        ix.bq_topr_device(q, 100, rows, dist)
    L.gvdb_timing_reset()
    L.gvdb_timing_enable(1)
    for _ in range(5):
        ix.search_device(q, 10, torch.zeros((B, 10), dtype=torch.int64, device=dev),
                         torch.zeros((B, 10), device=dev), None, gvdb.SearchParams(rescore_count=100))
    L.gvdb_timing_enable(0)
    ms, n = C.c_double(), C.c_uint64()
    L.gvdb_timing_read(1, C.byref(ms), C.byref(n))
    print(f"{cfg:10s} scan {ms.value / max(n.value, 1):.3f} ms", flush=True)
    if int(dbg) & 16:  # per-phase shader-clock deltas of block 0, waves 0 (early half) and 4 (late)
        import numpy as np
        st = np.zeros((2, 64, 8), dtype=np.uint64)
        L.gvdb_debug_stamps(C.c_void_p(st.ctypes.data))
        d = np.diff(st[:, 4:60, :5].astype(np.int64), axis=2)
        mf = (st[:, 4:60, 5].astype(np.int64) - st[:, 4:60, 0].astype(np.int64))
        e6 = (st[:, 4:60, 6].astype(np.int64) - st[:, 4:60, 0].astype(np.int64))
        e7 = (st[:, 4:60, 7].astype(np.int64) - st[:, 4:60, 0].astype(np.int64))
        per = np.diff(st[:, 4:60, 0].astype(np.int64), axis=1)
        for h, name in enumerate(("early", "late")):
            print(f"  {name}: phase cycles (mean) {d[h].mean(0).round(0).tolist()} tile {per[h].mean():.0f}"
                  f"  consume-MFMA end at {mf[h].mean():.0f} cmp0 {e6[h].mean():.0f} emit0 {e7[h].mean():.0f}  samples {d[h][:6].tolist()}", flush=True)
