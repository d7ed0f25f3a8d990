#!/usr/bin/env python3
"""BASELINE.json configs[0]: MockEmbeddingProvider (embeddings.rs:222-266),
10k x 128 f32, HNSW m=16 / ef_search=64.

  * corpus: 10000 seeded synthetic sentences, 256 query sentences, embedded
    by gvdb.embeddings.MockEmbeddingProvider(128) (bit-identical to the
    reference's f32 formula);
  * CPU leg (oracle/hnsw_oracle.cpp, instant-distance restated): the requested
    m=16 / ef_construction=200 / ef_search=64 -- NOT expressible in the
    reference, whose HnswVectorIndex builds with Builder::default()
    (index.rs:140-154) -- and that default, M=32 / ef=100;
  * GPU leg: the same corpus in a GpuVectorIndex: BQ + exact rerank (R=100)
    at batch 256 and batch 1, and the exact flat search; stage-1/2 results
    checked against the oracle's multi_stage_search (ids + cosine bits).
Writes profiles/r02/config1.json (or --out) and prints it.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "grape-vector-db_amd")]


SYL = ["gra", "pe", "vec", "tor", "da", "ta", "ba", "se", "in", "dex", "qu", "ery", "se", "arch", "ham", "ming",
       "co", "sine", "rank", "fu", "sion", "shard", "mer", "ge", "lo", "ad", "sa", "ve", "bit", "code"]


def texts(n, seed):
    """n synthetic sentences (3-12 words of 1-4 syllables each), seeded: the
    mock embedder only sees bytes, so any text works; short repetitive texts
    ("document i") collapse into a few tight clusters by length."""
    r = np.random.default_rng([0x6772617065, seed])
    out = []
    for _ in range(n):
        words = ["".join(SYL[j] for j in r.integers(0, len(SYL), r.integers(1, 5))) for _ in range(r.integers(3, 13))]
        out.append(" ".join(words))
    return out


def recall(found, truth):
    k = truth.shape[1]
    return float(np.mean([len(set(map(int, f[:k])) & set(map(int, t))) / k for f, t in zip(found, truth)]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--queries", type=int, default=256)
    ap.add_argument("--no-gpu", action="store_true")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02", "config1.json"))
    a = ap.parse_args()
    import oracle  # CPU baseline + checker
    from gvdb.embeddings import MockEmbeddingProvider

    t0 = time.time()
    prov = MockEmbeddingProvider(a.dim)
    docs, queries = texts(a.n, 1), texts(a.queries, 2)
    x = prov.generate_embeddings(docs)
    q = prov.generate_embeddings(queries)
    k = 10
    # exact ground truth by L2 (index.rs:64-79), ties by row
    d2 = ((q[:, None, :].astype(np.float64) - x[None, :, :].astype(np.float64)) ** 2).sum(-1)
    truth = np.argsort(d2, axis=1, kind="stable")[:, :k]
    res = {"config": "BASELINE configs[0]: Mock provider, 10k x 128 f32",
           "corpus": f"MockEmbeddingProvider({a.dim}) of {a.n} seeded synthetic sentences; {a.queries} query sentences",
           "embed_s": time.time() - t0}
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    cpu = []
    for M, efc, efs, label in [(16, 200, 64, "m=16 ef_search=64 (requested; not expressible in the reference: "
                                              "HnswVectorIndex uses Builder::default())"),
                               (32, 100, 100, "M=32 ef=100 (instant-distance Builder::default, the reference)")]:
        tb = time.perf_counter()
        h = oracle.Hnsw(x, M=M, ef_construction=efc, threads=threads)
        tb = time.perf_counter() - tb
        h.search(q[:threads], k=k, ef_search=efs, threads=threads)
        t = time.perf_counter()
        ids, _, _ = h.search(q, k=k, ef_search=efs, threads=threads)
        t = time.perf_counter() - t
        cpu.append({"hnsw": label, "M": M, "ef_construction": efc, "ef_search": efs, "build_s": tb,
                    "qps": a.queries / t, "cores": threads, "recall_at_10": recall(ids.astype(np.int64), truth)})
        del h
    res["cpu_hnsw"] = cpu
    if not a.no_gpu:
        import torch

        import gvdb

        dev = torch.device("cuda", 0)
        ix = gvdb.GpuVectorIndex(dimension=a.dim)
        ix.add_batch(np.arange(a.n, dtype=np.uint64), x)
        qd = torch.from_numpy(q).to(dev)
        gpu = []
        for name, sp in [("bq R=100", gvdb.SearchParams(rescore_count=100)),
                         ("exact flat", gvdb.SearchParams(mode=1))]:
            oi = torch.zeros((a.queries, k), dtype=torch.int64, device=dev)
            osc = torch.zeros((a.queries, k), dtype=torch.float32, device=dev)
            ix.search_device(qd, k, oi, osc, None, sp)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(20):
                ix.search_device(qd, k, oi, osc, None, sp)
            torch.cuda.synchronize()
            t = (time.perf_counter() - t) / 20
            found = oi.cpu().numpy()
            o1i = torch.zeros((1, k), dtype=torch.int64, device=dev)
            o1s = torch.zeros((1, k), dtype=torch.float32, device=dev)
            t1 = time.perf_counter()
            for i in range(a.queries):
                ix.search_device(qd[i:i + 1], k, o1i, o1s, None, sp)
            torch.cuda.synchronize()
            t1 = (time.perf_counter() - t1) / a.queries
            gpu.append({"search": name, "qps_batch256": a.queries / t, "qps_batch1": 1.0 / t1,
                        "recall_at_10": recall(found, truth)})
        res["gpu"] = gpu
        ri, rs = oracle.multi_stage_search_batch_r(oracle.quantize(q), oracle.quantize(x), q, x, 100, kind=0)
        gi, gs, gn = ix.search_batch(q, k, gvdb.SearchParams(rescore_count=100))
        res["bq_parity_vs_oracle"] = {"queries": a.queries, "ids_equal": bool((gi == ri[:, :k]).all()),
                                      "cosine_bit_exact": gs.tobytes() == rs[:, :k].tobytes()}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
