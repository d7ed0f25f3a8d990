#!/bin/bash
# PMC passes (separate runs) over the hybrid bench at 1M docs; k_bm25 rows only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/pmc_bm25_$TAG
mkdir -p $OUT
i=0
SETS=${SETS:-"SQ_WAVES|SQ_BUSY_CYCLES|GRBM_GUI_ACTIVE|SQ_INSTS_VALU|SQ_INSTS_LDS|SQ_INSTS_SALU|SQ_WAVE_CYCLES|SQ_INSTS_VMEM;SQ_WAIT_ANY|SQ_WAIT_INST_ANY|SQ_ACTIVE_INST_ANY|SQ_ACTIVE_INST_LDS|SQ_WAIT_INST_LDS|SQ_LDS_BANK_CONFLICT|SQ_ACTIVE_INST_VALU|SQ_INSTS_BRANCH"}
IFS=';' read -ra ALL <<< "$SETS"
for set in "${ALL[@]}"; do
    set=${set//|/ }
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 scripts/bench_hybrid.py --n ${N:-1000000} --no-cpu-baseline --steps 3 --warmup 1 > $OUT/p$i.log 2>&1
    rc=$?
    echo "pass $i ($set) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
    f=$(find $OUT/p$i -name "*counter_collection.csv" | head -1)
    if [ -n "$f" ]; then head -1 "$f" > $OUT/counters_p$i.csv; grep -E "k_bm25" "$f" >> $OUT/counters_p$i.csv; fi
    rm -rf $OUT/p$i
done
