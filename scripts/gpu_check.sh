#!/bin/bash
# GPU-box check: parity tests, smoke, a reduced bench.  Stops at the first
# crash/timeout (exit codes other than 0/1) and never retries a GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_1m 600 python bench.py --n 1000000 --steps 5 --warmup 2 --no-cpu-baseline --b1-queries 50
