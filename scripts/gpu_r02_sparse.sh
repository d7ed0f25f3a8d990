#!/bin/bash
# Round 2: BM25 term-at-a-time + RRF: GPU parity tests, the 5M hybrid bench
# (with its oracle parity leg) and a kernel-trace profile of it ($PROF=tag).
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
step pytest_sparse 600 python -u -m pytest ${TESTS:-tests/test_gpu_sparse.py} -x -v -rf --timeout 240 --timeout-method thread
if [ -z "$NO_BENCH" ]; then
    step bench_hybrid 600 python -u scripts/bench_hybrid.py --cpu-seconds 10 ${HARGS}
fi
if [ -n "$PROF" ]; then
    step prof_hybrid 600 rocprofv3 --kernel-trace --stats --output-format csv -T -d gpurun_out/r02/prof_$PROF -o run -- python3 -u scripts/bench_hybrid.py --no-cpu-baseline --steps 5 --warmup 1
    find gpurun_out/r02/prof_$PROF -type f ! -name "*_stats.csv" -delete
fi
