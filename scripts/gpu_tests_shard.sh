#!/bin/bash
# Full GPU test suite, then the per-rank sharded-step timing + profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -n 4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_shard_timing.sh
