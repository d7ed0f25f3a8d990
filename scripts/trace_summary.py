#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (CSV): per-kernel average duration and,
for a repeated step, the per-step timeline (kernel start offsets and the idle
gaps between consecutive kernels).  Usage: trace_summary.py run_kernel_trace.csv [first_kernel_substring]"""
import csv
import os
import re
import sys
from collections import defaultdict

def _quiet_pipe(exc_type, exc, tb):  # `| head` in a pipefail script: a closed pipe is not a failure
    if exc_type is BrokenPipeError:
        os._exit(0)
    sys.__excepthook__(exc_type, exc, tb)


sys.excepthook = _quiet_pipe
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[2] if len(sys.argv) > 2 else None
dur = defaultdict(list)
for r in rows:
    m = re.search(r"(k_\w+)", r["Kernel_Name"])  # anonymous-namespace kernels by their own name
    dur[m.group(1) if m else r["Kernel_Name"].split("(")[0][:70]].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"{'kernel':70s} {'calls':>6s} {'avg us':>9s}")
for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:70s} {len(v):6d} {sum(v) / len(v):9.1f}")
if anchor:
    starts = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    if len(starts) >= 3:
        i0, i1 = starts[-3], starts[-2]
        print(f"\none step (kernels {i0}..{i1 - 1}), times in us from the step's first kernel:")
        t0 = int(rows[i0]["Start_Timestamp"])
        prev_end = t0
        busy = 0
        for r in rows[i0:i1]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            busy += e - s
            print(f"  start {(s - t0) / 1e3:8.1f}  dur {(e - s) / 1e3:7.1f}  gap {(s - prev_end) / 1e3:6.1f}  "
                  f"{r['Kernel_Name'].split('(')[0][:60]}")
            prev_end = e
        span = int(rows[i1]["Start_Timestamp"]) - t0
        print(f"  step span {span / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us")
try:
    sys.stdout.flush()
except BrokenPipeError:
    os._exit(0)
