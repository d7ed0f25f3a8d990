#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/shard_step_timing.py > gpurun_out/shard_timing.log 2>&1 || { tail gpurun_out/shard_timing.log; exit 1; }
cat gpurun_out/shard_timing.log | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -T -d gpurun_out/prof_shard -o run -- python3 scripts/shard_step_timing.py > gpurun_out/prof_shard.log 2>&1 || exit 1
find gpurun_out/prof_shard -type f ! -name "*_stats.csv" -delete
cut -d, -f1-8 gpurun_out/prof_shard/run_kernel_stats.csv | head -25 | cut -c1-200
