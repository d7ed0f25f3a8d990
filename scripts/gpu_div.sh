#!/bin/bash
# Sample-size sweep (GVDB_SAMPLE_DIV) at the 10M single-GPU shard: step time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for dv in 64 128 32 96 48; do
  echo "== div $dv"; SHARD_N=10000000 GVDB_SAMPLE_DIV=$dv timeout -k 10 200 python scripts/shard_step_timing.py 2>&1 | grep -E "single|same" || exit 1
done
