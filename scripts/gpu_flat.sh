#!/bin/bash
# Flat (K4) parity tests + i8/bf16 timing + a kernel-trace profile of the i8 path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 6 "gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
    return 0
}
step pytest_flat 600 python -u -m pytest tests/test_gpu_parity.py -k "flat" -x -v -rf --timeout 300 --timeout-method thread
GVDB_FLAT=i8 step flat_i8 300 python scripts/flat_timing.py
step flat_bf16 300 python scripts/flat_timing.py
BS=256 step prof_flat 300 rocprofv3 --kernel-trace --stats --output-format csv -T -d gpurun_out/prof_flat_$TAG -o run -- python3 scripts/flat_timing.py
find gpurun_out/prof_flat_$TAG -type f ! -name "*_stats.csv" -delete
head -12 gpurun_out/prof_flat_$TAG/run_kernel_stats.csv | cut -c1-150
