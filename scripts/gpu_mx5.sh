#!/bin/bash
# stage-1 FP4 scan check: MFMA-scan parity tests (default vs GVDB_SCAN variants vs oracle),
# then batch-256 timing of the default scan and the GVDB_SCAN variants in $SCANS at 10M x 768.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "mfma_batches or stage1_topr or index_search_matches" --timeout 120 --timeout-method thread > gpurun_out/mx5_tests.log 2>&1
rc=$?; tail -4 gpurun_out/mx5_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/mx5_timing.log
for v in default ${SCANS:-mx3 mx6} default ${SCANS:-mx3 mx6}; do
  if [ $v = default ]; then unset GVDB_SCAN; else export GVDB_SCAN=$v; fi
  TAG=$v timeout -k 10 300 python -u scripts/b256_timing.py >> gpurun_out/mx5_timing.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/mx5_timing.log
for v in ${LIBS}; do
  unset GVDB_SCAN
  GVDB_LIB_PATH=$PWD/abl/libgvdb_$v.so TAG=lib_$v timeout -k 10 300 python -u scripts/b256_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
done
