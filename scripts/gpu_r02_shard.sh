#!/bin/bash
# Round 2: sharded-path GPU tests (RCCL comm in libgvdb, G=8 merge at D=3072)
# and the full-size config-4 emulation on one GPU (8 x 1.25M x 3072 shards).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02
step() {
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/r02/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 3 "gpurun_out/r02/$name.log" | cut -c1-2000
    if [ $rc -ne 0 ]; then exit $rc; fi
    return 0
}
step pytest_sharded 300 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_parity.py -m gpu -x -v -rf --timeout 200 --timeout-method thread -k "shard or rccl"
if [ -z "$NO_C4" ]; then
step c4_emulate 900 python -u scripts/c4_emulate.py
fi
