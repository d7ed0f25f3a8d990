#!/bin/bash
# BM25 launch-group size sweep (GVDB_BM25_GROUP_TERMS) on the 5M timing workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02/bm25_grp
mkdir -p $OUT
for G in ${GROUPS_:-511 255 128}; do
    GVDB_BM25_GROUP_TERMS=$G timeout -k 10 300 python3 -u scripts/bm25_timing.py --steps 5 --check > $OUT/g$G.log 2>&1 || { tail -5 $OUT/g$G.log; exit 1; }
    echo "group_terms=$G $(tail -1 $OUT/g$G.log)"
done
