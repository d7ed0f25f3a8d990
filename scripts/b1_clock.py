#!/usr/bin/env python3
"""Timing study of the batch-1 tail kernel (GVDB_B1_CLK=1): phase wall clocks
(100 MHz) of block 0 and of the last block of k_b1_tail, median over queries."""
import ctypes as C
import os
import sys

import numpy as np

os.environ["GVDB_B1_CLK"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "grape-vector-db_amd")]
import torch  # noqa: E402

import gvdb  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    D, k = 768, 10
    dev = torch.device("cuda", 0)
    ix = gvdb.GpuVectorIndex(dimension=D, capacity_hint=N)
    g = torch.Generator(device=dev).manual_seed(5)
    for c0 in range(0, N, 1 << 20):
        n = min(1 << 20, N - c0)
        x = torch.randn((n, D), generator=g, device=dev)
        ix.add_device(x, torch.arange(c0, c0 + n, dtype=torch.int64, device=dev))
    q = torch.randn((64, D), generator=g, device=dev)
    oi = torch.zeros((1, k), dtype=torch.int64, device=dev)
    osc = torch.zeros((1, k), dtype=torch.float32, device=dev)
    L = gvdb.lib()
    L.gvdb_debug_b1_clock.restype = C.c_int
    rows = []
    for i in range(64):
        ix.search_device(q[i:i + 1].contiguous(), k, oi, osc, None, gvdb.SearchParams(rescore_count=100))
        torch.cuda.synchronize()
        buf = (C.c_ulonglong * 16)()
        L.gvdb_debug_b1_clock(buf)
        c = np.array(buf[:], dtype=np.int64)
        b0, b1, bl = c[:4], c[4:8], c[8:14]
        t0 = min(b0[0], b1[0], bl[0])
        rows.append([b0[1] - b0[0], b0[3] - t0, b1[1] - b1[0], b1[2] - b1[1], b1[3] - t0, bl[3] - t0,
                     bl[4] - bl[3], bl[5] - bl[4], bl[5] - t0, c[14]])
    r = np.median(np.array(rows[4:]), axis=0)
    names = ["select (block 0)", "block 0 arrives", "b1 rerank loads", "b1 rerank fold", "block 1 arrives",
             "last block arrives", "last final sort", "last emit+clean", "tail total", "candidates"]
    for n_, v in zip(names, r):
        print(f"{n_:22s} {v * 0.01 if n_ != 'candidates' else v:8.2f}{' us' if n_ != 'candidates' else ''}")


if __name__ == "__main__":
    main()
