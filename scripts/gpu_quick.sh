#!/bin/bash
# quick check: GPU parity suite of the BQ path, then batch-256 timing (10M x 768) twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  TAG=quick timeout -k 10 300 python -u scripts/b256_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
done
