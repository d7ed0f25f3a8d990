#!/bin/bash
# BM25 phase ablation (timing only; results are wrong with ablation bits set).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02/bm25_abl_${TAG:-a}
mkdir -p $OUT
for A in ${ABLS:-0 1 2 4 3 7}; do
    GVDB_BM25_ABL=$A timeout -k 10 300 python3 -u scripts/bm25_timing.py --steps 5 ${BARGS} > $OUT/abl$A.log 2>&1 || { tail -5 $OUT/abl$A.log; exit 1; }
    echo "abl=$A $(tail -1 $OUT/abl$A.log)"
done
