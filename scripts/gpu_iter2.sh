#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_tests_shard.sh > gpurun_out/step1.log 2>&1; rc=$?; grep -E "passed|failed|Error" gpurun_out/pytest_gpu.log | tail -3; grep -E "single|sharded|same" gpurun_out/shard_timing.log; [ $rc -eq 0 ] || exit $rc
for f in 65536 32768 16384; do
  echo "== floor $f"; GVDB_SAMPLE_FLOOR=$f timeout -k 10 200 python scripts/shard_step_timing.py 2>&1 | grep -E "single|sharded|same" || exit 1
done
