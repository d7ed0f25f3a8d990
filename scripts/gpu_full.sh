#!/bin/bash
# Full-size bench + kernel-trace profile.  Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 4 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return 0
}
if [ -z "$SKIP_TESTS" ]; then step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread; fi
step bench_full 900 python bench.py
step prof_full 900 rocprofv3 --kernel-trace --stats --output-format csv -T -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2
# keep only the summaries (the per-dispatch trace is large)
find gpurun_out/prof_$TAG -type f ! -name "*_stats.csv" -delete
ls -la gpurun_out/prof_$TAG
