#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1
rc=$?; grep -E "passed|failed|Error" gpurun_out/pytest_parity.log | tail -3; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_b1.sh || exit 1
for v in 0 4096; do
  echo "== GVDB_RERANK_SMALL=$v"; SHARD_N=10000000 GVDB_RERANK_SMALL=$v timeout -k 10 200 python scripts/shard_step_timing.py 2>&1 | grep -E "single|same" || exit 1
done
