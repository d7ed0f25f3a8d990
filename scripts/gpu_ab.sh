#!/bin/bash
# same-box A/B of the batch-256 step: the in-tree libgvdb.so vs abl/libgvdb_$PREV.so, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; [ -n "$SKIP_TESTS" ] || { tail -2 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2 3; do
  TAG=new timeout -k 10 300 python -u scripts/b256_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
  GVDB_LIB_PATH=$PWD/abl/libgvdb_${PREV:-prev}.so TAG=${PREV:-prev} timeout -k 10 300 python -u scripts/b256_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
done
