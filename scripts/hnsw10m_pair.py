#!/usr/bin/env python3
"""Pairs the two sides of the 10M x 768 equal-recall experiment (BASELINE
north_star: ">= 10x the CPU-HNSW QPS at equal recall@10 on 10M x 768"):

  CPU  profiles/r03/hnsw10M_cpu.json  scripts/hnsw10m_cpu.py: the instant-distance
                                       0.6.1 restatement (HnswVectorIndex's
                                       Builder::default(), index.rs:150) on the host
  GPU  profiles/r03/hnsw10M_gpu.json  scripts/hnsw10m_gpu.py: BQ R sweep + exact flat
                                       on one MI355X

Same rows, same queries, same ground truth (scripts/hnsw10m_data.py).  Every
CPU point (ef_search, query set, distance form) is paired with the fastest GPU
point on the same query set whose recall@10 is >= the CPU point's (strict), and
separately >= the CPU point's - 0.02 (the bench's matched-recall rule), at batch
256 and at batch 1.  Writes profiles/r03/equal_recall_10000000x768.json."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def best(gpu_pts, qset, batch, need, key="recall_at_10"):
    ok = [p for p in gpu_pts if p["queries"] == qset and p["batch"] == batch and p[key] >= need]
    return max(ok, key=lambda p: p["qps"]) if ok else None


def main():
    d = os.environ.get("HNSW10M_DIR", os.path.join(ROOT, "profiles", "r03"))
    cpu = json.load(open(sys.argv[1] if len(sys.argv) > 1 else os.path.join(d, "hnsw10M_cpu.json")))
    gpu = json.load(open(sys.argv[2] if len(sys.argv) > 2 else os.path.join(d, "hnsw10M_gpu.json")))
    pairs = []
    for c in cpu["points"]:
        row = {"cpu": c}
        for batch in (256, 1, "concurrent64"):
            for tag, need in (("strict", c["recall_at_10"]), ("minus_0.02", c["recall_at_10"] - 0.02)):
                g = best(gpu["points"], c["queries"], batch, need)
                row[f"gpu_b{batch}_{tag}"] = None if g is None else {
                    "search": g["search"], "qps": g["qps"], "recall_at_10": g["recall_at_10"],
                    "speedup": g["qps"] / c["qps"]}
            # recall@1 (the planted set's top-1 is its planted row: a non-degenerate target)
            g = best(gpu["points"], c["queries"], batch, c["recall_at_1"], "recall_at_1")
            row[f"gpu_b{batch}_recall1"] = None if g is None else {
                "search": g["search"], "qps": g["qps"], "recall_at_1": g["recall_at_1"],
                "speedup": g["qps"] / c["qps"]}
        pairs.append(row)
    strict256 = [r["gpu_b256_strict"]["speedup"] for r in pairs if r["gpu_b256_strict"]]
    hi = [r for r in pairs if r["cpu"]["recall_at_10"] >= 0.9 or r["cpu"]["recall_at_1"] >= 0.9]
    out = {"rows": cpu["rows"], "dim": cpu["dim"],
           "cpu_host": cpu.get("host"), "cpu_model": cpu.get("cpu_model"),
           "cpu_build_threads": cpu.get("build_threads"), "cpu_search_threads": cpu.get("search_threads"),
           "cpu_build_s": cpu.get("build_s"),
           "min_speedup_b256_strict": min(strict256) if strict256 else None,
           "cpu_points_at_recall_0.9": [{"ef_search": r["cpu"]["ef_search"], "queries": r["cpu"]["queries"],
                                          "distance": r["cpu"]["distance"], "cpu_qps": r["cpu"]["qps"],
                                          "recall_at_10": r["cpu"]["recall_at_10"],
                                          "recall_at_1": r["cpu"]["recall_at_1"],
                                          "gpu_recall10_pairs": {b: r[f"gpu_b{b}_strict"] for b in (256, 1, "concurrent64")},
                                          "gpu_recall1_pairs": {b: r[f"gpu_b{b}_recall1"] for b in (256, 1, "concurrent64")}}
                                         for r in hi],
           "pairs": pairs,
           "rule": "fastest GPU point with recall@10 >= the CPU point's (strict) / >= it - 0.02, same query set; "
                   "recall1 pairs: the same with recall@1"}
    path = os.path.join(d, "equal_recall_10000000x768.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    for r in pairs:
        c, g = r["cpu"], r["gpu_b256_strict"]
        print(f"ef {c['ef_search']:4d} {c['queries']:8s} {c['distance'][:6]:6s}: CPU {c['qps']:9.1f} QPS @ "
              f"{c['recall_at_10']:.3f}  | GPU b256 {g['search'] if g else '-':12s} "
              f"{(g or {}).get('qps', 0):10.0f} QPS @ {(g or {}).get('recall_at_10', 0):.3f}  "
              f"x{(g or {}).get('speedup', 0):.0f}  | recall@1 {c['recall_at_1']:.3f}: "
              f"x{(r['gpu_b256_recall1'] or {}).get('speedup', 0):.0f} (b256), "
              f"x{(r['gpu_bconcurrent64_recall1'] or {}).get('speedup', 0):.0f} (64 callers)")
    print("min speedup (batch 256, strict):", out["min_speedup_b256_strict"], "->", path)


if __name__ == "__main__":
    main()
