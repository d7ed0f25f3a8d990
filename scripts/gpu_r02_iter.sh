#!/bin/bash
# Round 2 iteration: selected GPU tests ($TESTS), optionally the full suite
# ($FULL=1), the bench without CPU legs, and a kernel-trace profile ($PROF=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/r02/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 3 "gpurun_out/r02/$name.log" | cut -c1-3000
    if [ $rc -ne 0 ]; then exit $rc; fi
    return 0
}
if [ -n "$TESTS" ]; then
    step pytest_sel 600 python -u -m pytest $TESTS -x -v -rf --timeout 240 --timeout-method thread
fi
if [ -n "$FULL" ]; then
    step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread
fi
if [ -z "$NO_BENCH" ]; then
    step bench 600 python bench.py --no-cpu-baseline --hnsw-rows 0 ${BENCH_ARGS}
fi
if [ -n "$PROF" ]; then
    step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -T -d gpurun_out/r02/prof_$PROF -o run -- python3 bench.py --no-cpu-baseline --no-points --hnsw-rows 0 --steps 10 --warmup 2
    find gpurun_out/r02/prof_$PROF -type f ! -name "*_stats.csv" -delete
fi
