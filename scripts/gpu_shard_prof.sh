#!/bin/bash
# Kernel-trace breakdown of the batch-256 step at the 8-GPU shard size (1.25M x 768), with the
# in-library sharded step over a 1-rank RCCL communicator.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SHARD_N=1250000 RCCL=1 timeout -k 10 300 python -u scripts/b256_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
SHARD_N=1250000 RCCL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_shard -o run -- python3 scripts/b256_timing.py > gpurun_out/prof_shard.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_shard/run_kernel_stats.csv')):
    n = r['Name'].split('(')[0]
    print(n[:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
" | head -30
find gpurun_out/prof_shard -type f ! -name "*_kernel_stats.csv" -delete
