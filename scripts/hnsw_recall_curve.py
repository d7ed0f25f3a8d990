#!/usr/bin/env python3
"""Recall@10 vs ef_search of the CPU-HNSW restatement (oracle/hnsw_oracle.cpp,
instant-distance 0.6.1 as HnswVectorIndex uses it: M = 32, ef_construction =
100, index.rs:150) at D = 768, against exact ground truth; QPS on this host.

  python scripts/hnsw_recall_curve.py --n 50000 --out profiles/r06/hnsw_recall_curve_50Kx768.json

Two corpora: i.i.d. N(0,1) rows L2-normalised (the bench's data: cosine = L2
order) and the same rows un-normalised (L2 ground truth), with random queries
and planted queries (x_j + 0.1 n, |n| = 1, normalised; recall@1 = x_j found)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402  (CPU restatement; test/measurement infrastructure)


def unit(a):
    return (a / np.linalg.norm(a.astype(np.float64), axis=1, keepdims=True)).astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--queries", type=int, default=100)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--ef", type=int, nargs="+", default=[10, 50, 100, 200, 400, 1000, 2000, 5000])
    ap.add_argument("--out", default="")
    ap.add_argument("--unit-only", action="store_true", help="only the unit-row corpus (the bench's data)")
    a = ap.parse_args()
    rng = np.random.default_rng(a.n)
    raw = rng.standard_normal((a.n, a.dim)).astype(np.float32)
    qr = rng.standard_normal((a.queries, a.dim)).astype(np.float32)
    j = rng.integers(0, a.n, a.queries)
    noise = unit(rng.standard_normal((a.queries, a.dim)).astype(np.float32))
    res = {"n": a.n, "dim": a.dim, "queries": a.queries, "threads": a.threads, "M": 32, "ef_construction": 100,
           "corpora": []}
    names = ["unit rows (cosine = L2 order)"] + ([] if a.unit_only else ["un-normalised rows (L2 order)"])
    for name in names:
        unit_rows = name.startswith("unit")
        x = unit(raw) if unit_rows else raw
        q = unit(qr) if unit_rows else qr
        qp = unit(x[j] + 0.1 * noise * (1.0 if unit_rows else np.sqrt(a.dim)))
        x64 = x.astype(np.float64)

        def truth(qq):
            d2 = (x64 ** 2).sum(1)[None, :] - 2.0 * qq.astype(np.float64) @ x64.T
            return np.argsort(d2, axis=1, kind="stable")[:, :10]

        g_iid, g_pl = truth(q), truth(qp)
        t0 = time.time()
        h = oracle.Hnsw(x, threads=a.threads)
        build = time.time() - t0
        pts = []
        for ef in a.ef:
            p = {"ef_search": ef}
            for tag, qq, gg in (("iid", q, g_iid), ("planted", qp, g_pl)):
                t0 = time.time()
                ids, _, _ = h.search(qq, k=10, ef_search=ef, threads=a.threads)
                dt = time.time() - t0
                ids = ids.astype(np.int64)
                p[f"{tag}_recall_at_10"] = float(np.mean([len(set(u.tolist()) & set(v.tolist())) / 10
                                                          for u, v in zip(ids, gg)]))
                p[f"{tag}_recall_at_1"] = float(np.mean(ids[:, 0] == gg[:, 0]))
                p[f"{tag}_qps"] = qq.shape[0] / dt
            pts.append(p)
            print(json.dumps(p), flush=True)
        res["corpora"].append({"corpus": name, "build_s": build, "points": pts})
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
