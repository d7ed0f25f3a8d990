#!/bin/bash
# PMC passes (one counter set per run) over the batch-256 timing script at 10M x 768;
# keeps the k_scan_mx5 / k_scan_mx3 rows.  LIB=<name> picks abl/libgvdb_<name>.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG:-mx5}
mkdir -p $OUT
[ -n "$LIB" ] && export GVDB_LIB_PATH=$PWD/abl/libgvdb_$LIB.so
i=0
for set in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 scripts/b256_timing.py > $OUT/p$i.log 2>&1
    rc=$?
    echo "pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
    f=$(find $OUT/p$i -name "*counter_collection.csv" | head -1)
    if [ -n "$f" ]; then head -1 "$f" > $OUT/counters_p$i.csv; grep -E "k_scan_mx" "$f" >> $OUT/counters_p$i.csv; fi
    rm -rf $OUT/p$i
done
python3 scripts/pmc_summary.py $OUT --json $OUT/pmc.json || true
