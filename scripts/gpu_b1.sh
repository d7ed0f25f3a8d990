#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/b1_timing.py > gpurun_out/b1.log 2>&1 || { tail gpurun_out/b1.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b1.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -T -d gpurun_out/prof_b1 -o run -- python3 scripts/b1_timing.py > gpurun_out/prof_b1.log 2>&1 || exit 1
find gpurun_out/prof_b1 -type f ! -name "*_stats.csv" -delete
cut -d, -f1-4 gpurun_out/prof_b1/run_kernel_stats.csv | head -14
