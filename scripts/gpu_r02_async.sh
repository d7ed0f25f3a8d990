#!/bin/bash
# Round 2: the host-sync-free search path (async tests, full GPU suite, bench).
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
step pytest_async 300 python -u -m pytest tests/test_gpu_async.py -x -v -rf --timeout 200 --timeout-method thread
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread
step bench 600 python bench.py --no-cpu-baseline --hnsw-rows 0
