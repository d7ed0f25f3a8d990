#!/bin/bash
# All GPU parity tests, flat timing, a quick 10M bench and a flat kernel-trace profile.
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
    if [ $rc -ne 0 ]; then exit $rc; fi
    return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread
step flat_bf16 300 python scripts/flat_timing.py
step bench_quick 600 python bench.py --no-cpu-baseline --hnsw-rows 0 --steps 10
BS=256 step prof_flat 300 rocprofv3 --kernel-trace --stats --output-format csv -T -d gpurun_out/prof_flat_$TAG -o run -- python3 scripts/flat_timing.py
find gpurun_out/prof_flat_$TAG -type f ! -name "*_stats.csv" -delete
head -12 gpurun_out/prof_flat_$TAG/run_kernel_stats.csv | cut -c1-150
