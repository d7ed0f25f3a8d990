#!/bin/bash
# PMC counter passes (separate runs) over the flat-search timing script
# (default B=256).  Keeps only the rows of the flat kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/pmc_flat_$TAG
mkdir -p $OUT
export BS=${BS:-256} FLAT_REPS=${FLAT_REPS:-3}
i=0
SETS=${SETS:-"SQ_WAVES|SQ_BUSY_CYCLES|GRBM_GUI_ACTIVE|SQ_INSTS_VALU|SQ_INSTS_MFMA|SQ_INSTS_LDS|SQ_INSTS_SALU|SQ_WAVE_CYCLES;SQ_VALU_MFMA_BUSY_CYCLES|SQ_WAIT_INST_LDS|SQ_LDS_BANK_CONFLICT|SQ_WAIT_ANY|SQ_ACTIVE_INST_VALU|SQ_WAIT_INST_ANY;FETCH_SIZE"}
IFS=';' read -ra ALL <<< "$SETS"
for set in "${ALL[@]}"; do
    set=${set//|/ }
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 scripts/flat_timing.py > $OUT/p$i.log 2>&1
    rc=$?
    echo "pass $i ($set) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
    f=$(find $OUT/p$i -name "*counter_collection.csv" | head -1)
    if [ -n "$f" ]; then head -1 "$f" > $OUT/counters_p$i.csv; grep -E "k_flat|k_rerank" "$f" >> $OUT/counters_p$i.csv; fi
    rm -rf $OUT/p$i
done
ls -la $OUT
