#!/usr/bin/env python3
"""Equal-recall comparison at matched N: CPU HNSW (instant-distance restated,
oracle/hnsw_oracle.cpp; the path HnswVectorIndex takes, index.rs:140-154,
212-231) vs the GPU search paths on the SAME corpus and queries.

The corpus is generated with numpy from a fixed seed (i.i.d. N(0,1) f32 rows,
L2-normalised through float64 norms so the bits do not depend on the host's
SIMD path), so the CPU leg and the GPU leg can run on different machines and
still see identical data; ground truth = exact top-10 by cosine (= by L2 for
unit rows), computed in float64 on the host.

  --leg cpu : build the HNSW graph (M, ef_construction), sweep ef_search, write
              <out>/hnsw_cpu_<N>.json (QPS on this host's cores, recall@10).
  --leg gpu : build the GPU index, sweep BQ rescore depth R and the exact flat
              search, read the CPU json and write <out>/equal_recall_<N>.json:
              for every HNSW point the fastest GPU point with recall >= it.
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "grape-vector-db_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

SEED = 0x6772617065
CH = 1 << 18


def gen_rows(n, d, seed):
    out = np.empty((n, d), np.float32)
    for c0 in range(0, n, CH):
        c1 = min(n, c0 + CH)
        x = np.random.default_rng([seed, c0 // CH]).standard_normal((c1 - c0, d), dtype=np.float32)
        nrm = np.sqrt(np.square(x.astype(np.float64)).sum(1, keepdims=True)).astype(np.float32)
        out[c0:c1] = x / nrm
    return out


def exact_truth(x, q, k, pad=20):
    """Exact top-k by cosine: f32 BLAS shortlists the top-(k+pad) per query,
    float64 re-scores the shortlist (ties by row)."""
    kk = k + pad
    best_v = np.full((q.shape[0], kk), -np.inf, np.float32)
    best_i = np.zeros((q.shape[0], kk), np.int64)
    for c0 in range(0, x.shape[0], CH):
        s = q @ x[c0:c0 + CH].T
        part = np.argpartition(-s, kk - 1, axis=1)[:, :kk]
        v = np.concatenate([best_v, np.take_along_axis(s, part, 1)], 1)
        i = np.concatenate([best_i, part + c0], 1)
        o = np.argpartition(-v, kk - 1, axis=1)[:, :kk]
        best_v = np.take_along_axis(v, o, 1)
        best_i = np.take_along_axis(i, o, 1)
        print(f"[data] truth rows {c0 + s.shape[1]}", flush=True)
    exact = np.einsum("bd,bkd->bk", q.astype(np.float64), x[best_i].astype(np.float64))
    o = np.lexsort((best_i, -exact), axis=1)[:, :k]
    return np.take_along_axis(best_i, o, 1)


def recall(found, truth):
    k = truth.shape[1]
    return float(np.mean([len(set(map(int, f[:k])) & set(map(int, t))) / k for f, t in zip(found, truth)]))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def leg_cpu(a, x, q, truth):
    import oracle  # CPU baseline (test / bench infrastructure)

    threads = a.threads or len(os.sched_getaffinity(0))
    t0 = time.perf_counter()
    h = oracle.Hnsw(x, M=a.M, ef_construction=a.ef_c, threads=threads)
    build = time.perf_counter() - t0
    print(f"[cpu] build {x.shape[0]}x{x.shape[1]} M={a.M} ef_c={a.ef_c}: {build:.1f}s on {threads} threads",
          flush=True)
    points = []
    for ef in a.ef:
        h.search(q[:threads], k=a.k, ef_search=ef, threads=threads)
        t = time.perf_counter()
        ids, _, _ = h.search(q, k=a.k, ef_search=ef, threads=threads)
        t = time.perf_counter() - t
        t1 = time.perf_counter()
        h.search(q[:8], k=a.k, ef_search=ef, threads=1)
        t1 = (time.perf_counter() - t1) / 8
        p = {"ef_search": ef, "qps": q.shape[0] / t, "recall_at_10": recall(ids.astype(np.int64), truth),
             "single_thread_ms_per_query": 1e3 * t1}
        points.append(p)
        print(f"[cpu] ef={ef}: {p}", flush=True)
    return {"n": x.shape[0], "dim": x.shape[1], "queries": q.shape[0], "M": a.M, "ef_construction": a.ef_c,
            "build_s": build, "threads": threads, "cpu": cpu_model(), "points": points,
            "kind": "port (instant-distance 0.6.1 restated, oracle/hnsw_oracle.cpp; one query per thread)"}


def leg_gpu(a, x, q, truth):
    import torch

    import gvdb

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n, d = x.shape
    ix = gvdb.GpuVectorIndex(dimension=d, capacity_hint=n)
    for c0 in range(0, n, CH):
        xs = torch.from_numpy(x[c0:c0 + CH]).to(dev)
        ix.add_device(xs, torch.arange(c0, c0 + xs.shape[0], dtype=torch.int64, device=dev))
    torch.cuda.synchronize()
    B = a.batch
    points = []
    for name, sp in [(f"bq R={r}", gvdb.SearchParams(rescore_count=r)) for r in a.R] + \
                    [("exact flat", gvdb.SearchParams(mode=1))]:
        found = np.zeros((q.shape[0], a.k), np.int64)
        oi = torch.zeros((B, a.k), dtype=torch.int64, device=dev)
        osc = torch.zeros((B, a.k), dtype=torch.float32, device=dev)
        qd = torch.from_numpy(q).to(dev)
        batches = [qd[b0:b0 + B].contiguous() for b0 in range(0, q.shape[0], B)]
        for i, qb in enumerate(batches):  # results (untimed; also the warm-up)
            ix.search_device(qb, a.k, oi[:qb.shape[0]], osc[:qb.shape[0]], None, sp)
            found[i * B:i * B + qb.shape[0]] = oi[:qb.shape[0]].cpu().numpy()
        torch.cuda.synchronize()
        reps, t = 0, time.perf_counter()
        while reps < 2 or time.perf_counter() - t < 1.0:
            for qb in batches:
                ix.search_device(qb, a.k, oi[:qb.shape[0]], osc[:qb.shape[0]], None, sp)
            torch.cuda.synchronize()
            reps += 1
        qps = q.shape[0] * reps / (time.perf_counter() - t)
        p = {"search": name, "qps": qps, "recall_at_10": recall(found, truth), "batch": B}
        points.append(p)
        print(f"[gpu] {p}", flush=True)
    return points


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--leg", choices=["cpu", "gpu"], required=True)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--queries", type=int, default=1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--M", type=int, default=32)
    ap.add_argument("--ef-c", dest="ef_c", type=int, default=100)
    ap.add_argument("--ef", type=int, nargs="+", default=[64, 100, 200, 400])
    ap.add_argument("--R", type=int, nargs="+", default=[100, 1000, 4000, 16000])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02"))
    a = ap.parse_args()
    t0 = time.time()
    x = gen_rows(a.n, a.dim, SEED)
    q = gen_rows(a.queries, a.dim, SEED + 1)
    truth = exact_truth(x, q, a.k)
    print(f"[data] {a.n}x{a.dim} + {a.queries} queries + exact truth: {time.time() - t0:.1f}s", flush=True)
    os.makedirs(a.out, exist_ok=True)
    cpu_path = os.path.join(a.out, f"hnsw_cpu_{a.n}x{a.dim}.json")
    if a.leg == "cpu":
        res = leg_cpu(a, x, q, truth)
        with open(cpu_path, "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res))
        return
    gpu = leg_gpu(a, x, q, truth)
    res = {"n": a.n, "dim": a.dim, "queries": a.queries, "gpu_points": gpu}
    if os.path.exists(cpu_path):
        with open(cpu_path) as f:
            cpu = json.load(f)
        res["cpu_hnsw"] = cpu
        cmp = []
        for hp in cpu["points"]:
            best = max((g for g in gpu if g["recall_at_10"] >= hp["recall_at_10"] - 1e-9), key=lambda g: g["qps"],
                       default=None)
            if best:
                cmp.append({"hnsw_ef_search": hp["ef_search"], "hnsw_qps": hp["qps"],
                            "hnsw_recall_at_10": hp["recall_at_10"], "gpu_search": best["search"],
                            "gpu_qps": best["qps"], "gpu_recall_at_10": best["recall_at_10"],
                            "speedup": best["qps"] / hp["qps"]})
        res["equal_recall"] = cmp
    with open(os.path.join(a.out, f"equal_recall_{a.n}x{a.dim}.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
