#!/bin/bash
# HBM traffic passes only (FETCH_SIZE, WRITE_SIZE; one rocprofv3 --pmc run each)
# over the scan-dominated bench run; rows of the stage-1 kernels kept.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG:-traffic}
mkdir -p $OUT
ARGS="--no-cpu-baseline --no-points --steps 10 --warmup 2 --b1-queries 50 --hnsw-rows 0"
i=0
for set in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
    rc=$?
    echo "pass $i ($set) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
    f=$(find $OUT/p$i -name "*counter_collection.csv" | head -1)
    if [ -n "$f" ]; then head -1 "$f" > $OUT/counters_p$i.csv; grep -E "k_scan|k_rerank|k_sample_hist|k_select" "$f" >> $OUT/counters_p$i.csv; fi
    rm -rf $OUT/p$i
done
python3 scripts/pmc_summary.py $OUT
