#!/bin/bash
# Config 4 (10M x 3072) measurements on one GPU: the per-GPU shard of the
# 8-way C4 split (1.25M x 3072) and the whole 10M x 3072 corpus.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-c4}
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 2 "gpurun_out/$name.log" | cut -c1-1500
    if [ $rc -ne 0 ]; then exit $rc; fi
    return 0
}
if [ -n "$C4_TESTS" ]; then
    step pytest_c4 600 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread -k "$C4_TESTS"
fi
step bench_c4_shard_$TAG 600 python bench.py --n 1250000 --dim 3072 --hnsw-rows 0 --steps 10
step bench_c4_full_$TAG 900 python bench.py --n 10000000 --dim 3072 --hnsw-rows 0 --no-cpu-baseline --no-points --steps 10 --b1-queries 50
