#!/usr/bin/env python3
"""The reference's DEFAULT rescore depth at scale (src/quantization.rs:27,178:
R = (N as f32 * 0.1) as usize): batched BQ search with rescore_ratio 0.1 on
the bench corpus at N = 1M (R = 100K) and 10M (R = 1M), batch 8 / 64 / 256,
k = 10, through gvdb_index_search_device: by default the certified search
(exact cosine top-64 of the shard filtered by the stage-1 membership rule;
"certified" counts the batches it answered), with GVDB_DEEP_CERT=0 the exact
top-R stage 1, rerank of all R rows and k_topk_big (gvdb_bigr.hip).  With --check the first queries of the
1M run are compared with the oracle's multi_stage_search (ids + cosine bits).
Prints one JSON line per point."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "grape-vector-db_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import gvdb  # noqa: E402


def deep_counts():
    import ctypes as C

    L = gvdb.lib()
    L.gvdb_debug_deep_cert.argtypes = [C.POINTER(C.c_uint64)]
    out = (C.c_uint64 * 2)()
    L.gvdb_debug_deep_cert(out)
    return int(out[0]), int(out[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="1000000,10000000")
    ap.add_argument("--batches", default="8,64,256")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--check", type=int, default=2, help="oracle-checked queries at the first N (0: none)")
    a = ap.parse_args()
    D, k = 768, 10
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    for ni, n in enumerate(int(x) for x in a.n.split(",")):
        ix = gvdb.GpuVectorIndex(dimension=D, device=0, capacity_hint=n)
        host = np.empty((n, D), np.float32) if (a.check and ni == 0) else None
        for c in range((n + bench.CHUNK - 1) // bench.CHUNK):
            lo, hi = c * bench.CHUNK, min(n, (c + 1) * bench.CHUNK)
            x = bench.gen_chunk(c, hi - lo, D, dev)
            ix.add_device(x, torch.arange(lo, hi, device=dev))
            if host is not None:
                host[lo:hi] = x.cpu().numpy()
        sp = gvdb.SearchParams(rescore_ratio=0.1)
        R = int(np.float32(n) * np.float32(0.1))
        for B in (int(x) for x in a.batches.split(",")):
            q = bench.gen_queries(B, D, dev)
            oi = torch.zeros((B, k), dtype=torch.int64, device=dev)
            osc = torch.zeros((B, k), dtype=torch.float32, device=dev)
            on = torch.zeros(B, dtype=torch.int32, device=dev)
            ix.search_device(q, k, oi, osc, on, sp)
            torch.cuda.synchronize()
            c0 = deep_counts()
            ts = []
            for _ in range(a.steps):
                t = time.perf_counter()
                ix.search_device(q, k, oi, osc, on, sp)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t)
            ms = 1e3 * float(np.median(ts))
            line = {"rows": n, "dim": D, "R": R, "batch": B, "k": k, "ms_per_batch": ms, "qps": B / ms * 1e3,
                    "rerank_bytes_per_batch": B * R * (4 * D + 12), "all_k": bool((on.cpu() == k).all())}
            c1 = deep_counts()
            line["certified_batches"], line["rerank_batches"] = c1[0] - c0[0], c1[1] - c0[1]
            if host is not None and B == 8:
                import oracle  # checker only

                nq = min(a.check, B)
                qn = q[:nq].cpu().numpy()
                t = time.perf_counter()
                ri, rs = oracle.multi_stage_search_batch_r(oracle.quantize(qn), oracle.quantize(host), qn, host, R,
                                                           threads=16)
                line["oracle"] = {"queries": nq, "seconds": time.perf_counter() - t,
                                  "ids_equal": bool((ri[:, :k] == oi[:nq].cpu().numpy().astype(np.uint64)).all()),
                                  "cosine_bit_exact": rs[:, :k].tobytes() == osc[:nq].cpu().numpy().tobytes()}
            print(json.dumps(line), flush=True)
        del ix
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
