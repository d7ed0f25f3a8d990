#!/usr/bin/env python3
"""GPU side of the 10M x 768 equal-recall experiment: the SAME corpus and
queries as scripts/hnsw10m_cpu.py (scripts/hnsw10m_data.py regenerates them
bit for bit), scored against the ground truth that script committed
(profiles/r03/hnsw10M_gt.npz).  Runs on one MI355X: the BQ rescore sweep
(R = 10 .. 8000) and the exact flat search (recall 1.0) at batch 256, plus
batch-1 BQ, on the iid and the planted query sets; prints one JSON line and
writes gpurun_out/hnsw10m_gpu.json.  The pairing with the CPU-HNSW points is
done by scripts/hnsw10m_pair.py."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "grape-vector-db_amd"), os.path.join(ROOT, "scripts")]

import torch  # noqa: E402

import gvdb  # noqa: E402
import hnsw10m_data as data  # noqa: E402


def log(*a):
    print(time.strftime("%H:%M:%S"), *a, file=sys.stderr, flush=True)


def recall(found, truth):
    k = truth.shape[1]
    return float(np.mean([len(set(f[:k].tolist()) & set(t.tolist())) / k for f, t in zip(found, truth)]))


def main():
    N, D, B, k = 10_000_000, 768, 256, 10
    # HNSW10M_GT: the ground truth the CPU side wrote (default: round 3's)
    gt = np.load(os.environ.get("HNSW10M_GT", os.path.join(ROOT, "profiles", "r03", "hnsw10M_gt.npz")))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    ix = gvdb.GpuVectorIndex(dimension=D, capacity_hint=N)
    t0 = time.time()
    host = {}
    workers = min(16, len(os.sched_getaffinity(0)))
    for lo, rows in data.chunks(N, D, workers=workers):
        t = torch.from_numpy(rows).to(dev)
        ix.add_device(t, torch.arange(lo, lo + rows.shape[0], dtype=torch.int64, device=dev))
        host[lo] = rows  # kept for the planted queries (x_j rows)
        if (lo // data.CHUNK) % 8 == 0:
            log(f"rows {lo + rows.shape[0]} / {N} ({time.time() - t0:.0f}s)")
    torch.cuda.synchronize()

    def rows_at(j):
        return np.stack([host[(int(v) // data.CHUNK) * data.CHUNK][int(v) % data.CHUNK] for v in j])

    q_iid, q_pl, pj = data.queries(rows_at, N, D, gt["iid"].shape[0], gt["planted"].shape[0])
    assert (pj == gt["planted_rows"]).all(), "planted rows differ from the CPU side's"
    del host
    sets = {"iid": (q_iid, gt["iid"]), "planted": (q_pl, gt["planted"])}
    pts = []
    for name, (Q, truth) in sets.items():
        nq = (Q.shape[0] // B) * B
        qd = torch.from_numpy(Q[:nq]).to(dev)
        oi = torch.zeros((B, k), dtype=torch.int64, device=dev)
        osc = torch.zeros((B, k), dtype=torch.float32, device=dev)
        for label, prm in [(f"bq R={r}", gvdb.SearchParams(rescore_count=r))
                           for r in (10, 30, 100, 300, 1000, 3000, 8000)] + \
                          [("bq R=0.1 N (reference default, certified)", gvdb.SearchParams(rescore_ratio=0.1)),
                           ("exact flat", gvdb.SearchParams(mode=1))]:
            found = np.zeros((nq, k), np.int64)
            ix.search_device(qd[:B], k, oi, osc, None, prm)  # warm
            torch.cuda.synchronize()
            t = time.perf_counter()
            for b0 in range(0, nq, B):
                ix.search_device(qd[b0:b0 + B], k, oi, osc, None, prm)
                found[b0:b0 + B] = oi.cpu().numpy()
            torch.cuda.synchronize()
            t = time.perf_counter() - t
            pts.append({"search": label, "queries": name, "batch": B, "qps": nq / t,
                        "recall_at_10": recall(found, truth[:nq]),
                        "recall_at_1": float(np.mean(found[:, 0] == truth[:nq, 0]))})
            log(pts[-1])
        # batch 1 (latency), BQ R=100 and R=1000
        o1i = torch.zeros((1, k), dtype=torch.int64, device=dev)
        o1s = torch.zeros((1, k), dtype=torch.float32, device=dev)
        for r in (100, 1000):
            prm = gvdb.SearchParams(rescore_count=r)
            n1 = 200
            found = np.zeros((n1, k), np.int64)
            ix.search_device(qd[:1], k, o1i, o1s, None, prm)
            torch.cuda.synchronize()
            t = time.perf_counter()
            res = []
            for i in range(n1):
                ix.search_device(qd[i:i + 1], k, o1i, o1s, None, prm)
                res.append(o1i.clone())
            torch.cuda.synchronize()
            t = time.perf_counter() - t
            found = torch.cat(res).cpu().numpy()
            pts.append({"search": f"bq R={r}", "queries": name, "batch": 1, "qps": n1 / t,
                        "recall_at_10": recall(found, truth[:n1]),
                        "recall_at_1": float(np.mean(found[:, 0] == truth[:n1, 0]))})
            log(pts[-1])
        # 64 concurrent single-query callers through the C ABI (bench.py's driver, library-coalesced)
        from bench import concurrent_b1_points
        for p in concurrent_b1_points(ix, D, k, Q[:nq], truth[:nq], None, None,
                                      [("bq R=100", gvdb.SearchParams(rescore_count=100)),
                                       ("exact flat", gvdb.SearchParams(mode=1))], threads=64):
            p["queries"] = name
            p["batch"] = "concurrent64"
            pts.append(p)
            log(pts[-1])
    out = {"rows": N, "dim": D, "points": pts,
           "note": "same rows / queries / ground truth as profiles/r03/hnsw10M_cpu.json (scripts/hnsw10m_data.py); "
                   "qps = queries / wall time of the search loop (result copies included)"}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "hnsw10m_gpu.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
