#!/bin/bash
# Round-end validation: GPU tests, smoke(), default bench, kernel-trace profile.
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
step pytest_gpu_final 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread
step smoke_final 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_final 900 python bench.py
step prof_final 900 rocprofv3 --kernel-trace --stats --output-format csv -T -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-cpu-baseline --no-points --steps 10 --warmup 2
find gpurun_out/prof_$TAG -type f ! -name "*_stats.csv" -delete
