#!/bin/bash
# BM25 leg probe: timing, per-dispatch kernel trace, one SQ counter pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02/bm25_${TAG:-p}
mkdir -p $OUT
timeout -k 10 300 python3 -u scripts/bm25_timing.py ${BARGS} > $OUT/timing.log 2>&1 || { tail -5 $OUT/timing.log; exit 1; }
tail -1 $OUT/timing.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 scripts/bm25_timing.py --steps 2 ${BARGS} > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 1; }
f=$(find $OUT/kt -name "*kernel_trace.csv" | head -1)
python3 - "$f" > $OUT/dispatch.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    k = r["Kernel_Name"]
    if any(s in k for s in ("bm25", "ta_dir", "inv_", "rrf")):
        print(f'{k[:60]:60s} {(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3:10.1f} us grid={r.get("Grid_Size_X", r.get("Grid_Size", ""))}')
PY
rm -rf $OUT/kt
tail -24 $OUT/dispatch.txt
if [ -n "$PMC" ]; then
    timeout -s KILL 200 rocprofv3 --pmc $PMC --output-format csv -d $OUT/pmc -o run -- python3 scripts/bm25_timing.py --steps 1 ${BARGS} > $OUT/pmc.log 2>&1 || { tail -5 $OUT/pmc.log; exit 1; }
    f=$(find $OUT/pmc -name "*counter_collection.csv" | head -1)
    head -1 "$f" > $OUT/counters_p1.csv; grep -E "bm25_taat|ta_dir" "$f" >> $OUT/counters_p1.csv; rm -rf $OUT/pmc
    python3 scripts/pmc_summary.py $OUT | tee $OUT/pmc_summary.txt
fi
