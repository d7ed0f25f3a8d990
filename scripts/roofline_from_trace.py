#!/usr/bin/env python3
"""Recompute bench.py's roofline fractions from a rocprofv3 kernel trace of the
same command (profiles/rNN/): the average duration of exactly the launches
bench.py times with HIP events --

* batch 256: k_scan_mx7 launches (warmup + 1) .. (warmup + steps) in order
  (the search loop is the first user of the scan; warmup steps come first);
* batch 1: the first `b1` k_b1_scan launches (the pass whose HIP events give
  batch1.roofline.avg_launch_ms);
* exact flat: the full-corpus k_flat_i8q launches (operating_points[].emit_roofline; the
  CPU-HNSW leg's 100K-row launches are the short ones and are left out);

and the fractions from the same algorithmic work bench.py uses.  Usage:
roofline_from_trace.py TRACE.csv BENCH.json [--warmup 3 --steps 20 --b1 200]"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--b1", type=int, default=200)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    bench = json.loads(open(a.bench).read().strip().splitlines()[-1])

    def durs(prefix):
        return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows
                if r["Kernel_Name"].startswith(prefix)]

    out = {}
    scan = durs("void gvdb::k_scan_mx7<")[a.warmup:a.warmup + a.steps]
    if scan:
        roof = bench["roofline"]
        avg = sum(scan) / len(scan)
        ach = roof["algorithmic_ops_per_launch"] / (avg * 1e-3) / 1e12
        out["batch256"] = {"kernel": "k_scan_mx7", "launches": len(scan), "avg_launch_ms_rocprof": avg,
                           "avg_launch_ms_hip_events": roof["avg_launch_ms"], "achieved_rocprof": ach,
                           "frac_rocprof": ach / roof["peak"], "frac_hip_events": roof["frac"],
                           "agreement": avg / roof["avg_launch_ms"]}
    b1 = durs("void gvdb::k_b1_scan<")[:a.b1]
    if b1 and bench.get("batch1"):
        roof = bench["batch1"]["roofline"]
        avg = sum(b1) / len(b1)
        ach = roof["algorithmic_bytes_per_launch"] / (avg * 1e-3) / 1e9
        out["batch1"] = {"kernel": "k_b1_scan", "launches": len(b1), "avg_launch_ms_rocprof": avg,
                         "avg_launch_ms_hip_events": roof["avg_launch_ms"], "achieved_rocprof_GBs": ach,
                         "frac_rocprof": ach / roof["peak"], "frac_hip_events": roof["frac"],
                         "agreement": avg / roof["avg_launch_ms"]}
    fl = durs("void gvdb::k_flat_i8q<")
    # the 10M-row launches (the CPU-HNSW leg also runs the flat search on its 100K-row prefix)
    fl = [d for d in fl if fl and d >= 0.5 * max(fl)]
    fr = next((p.get("emit_roofline") for p in bench.get("operating_points") or [] if p.get("emit_roofline")), None)
    if fl and fr:
        avg = sum(fl) / len(fl)
        ach = fr["algorithmic_bytes_per_launch"] / (avg * 1e-3) / 1e9
        out["flat_emit"] = {"kernel": "k_flat_i8q", "launches": len(fl), "avg_launch_ms_rocprof": avg,
                            "avg_launch_ms_hip_events": fr["avg_launch_ms"], "achieved_rocprof_GBs": ach,
                            "frac_rocprof": ach / fr["peak"], "frac_hip_events": fr["frac"],
                            "agreement": avg / fr["avg_launch_ms"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
