#!/bin/bash
# batch-1 timing sweep over knobs (each setting in its own process: knobs are read once)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02
out=gpurun_out/r02/b1_sweep.log
: > $out
for div in ${DIVS:-32 64 128}; do
    GVDB_B1_SAMPLE_DIV=$div TAG=" div=$div" NQ=400 STREAMS=${STREAMS:-0} timeout -k 10 200 python scripts/b1_timing.py 2>&1 | grep batch-1 >> $out || exit 1
done
cat $out
