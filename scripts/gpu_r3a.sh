#!/bin/bash
# round 3: dense FP4 sample + precomputed query fragments -- parity of the
# thresholds / stage-1 lists, then timing + kernel trace at the 8-GPU shard and 10M
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "thresholds_equal_valu or stage1_mfma or stage1_topr or index_search_matches" > gpurun_out/r3a_tests.log 2>&1 || { tail -30 gpurun_out/r3a_tests.log; exit 1; }
tail -3 gpurun_out/r3a_tests.log
SHARD_N=1250000 RCCL=1 timeout -k 10 300 python3 -u scripts/b256_timing.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python3 -u scripts/b256_timing.py 2>&1 | grep -v amdgpu.ids
SHARD_N=1250000 RCCL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3a -o run -- python3 scripts/b256_timing.py > gpurun_out/r3a.log 2>&1
