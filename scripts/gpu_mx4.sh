#!/bin/bash
# k_scan_mx4 (wide codes) parity tests, then the C4 measurements.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -rf --timeout 300 --timeout-method thread -k "mfma_batches" > gpurun_out/pytest_mx4.log 2>&1
rc=$?; echo "pytest_mx4 rc=$rc"; tail -n 14 gpurun_out/pytest_mx4.log
[ $rc -eq 0 ] || exit $rc
TAG=${TAG:-mx4} bash scripts/gpu_c4.sh
