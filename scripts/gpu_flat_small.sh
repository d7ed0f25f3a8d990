#!/bin/bash
# Small-N exact flat (config 1 shape): timing and a per-dispatch kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02/flat_small_${TAG:-a}
mkdir -p $OUT
N=${N:-10000} D=${D:-128} BS=${BS:-256,1} timeout -k 10 300 python3 -u scripts/flat_timing.py > $OUT/timing.log 2>&1 || { tail -5 $OUT/timing.log; exit 1; }
grep -v amdgpu.ids $OUT/timing.log | tail -6
N=${N:-10000} D=${D:-128} BS=256 FLAT_REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 scripts/flat_timing.py > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 1; }
f=$(find $OUT/kt -name "*kernel_trace.csv" | head -1)
python3 - "$f" > $OUT/dispatch.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    k = r["Kernel_Name"][:70]
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
    print(f"{k:70s} {n:5d} {t / n:10.1f} us avg {t:10.1f} us total")
PY
rm -rf $OUT/kt
cat $OUT/dispatch.txt
