#!/bin/bash
# round 3: two-exchange sharded search -- GPU tests, config-3 8-shard emulation, per-rank trace
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sharded.py > gpurun_out/r3b_tests.log 2>&1 || { tail -40 gpurun_out/r3b_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r3b_tests.log | tail -3
timeout -k 10 600 python -u scripts/c3_emulate.py > gpurun_out/r3b_c3.json 2> gpurun_out/r3b_c3.log || { tail -20 gpurun_out/r3b_c3.log; exit 1; }
tail -5 gpurun_out/r3b_c3.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3b -o run -- python3 scripts/c3_emulate.py --no-single --oracle-queries 0 --steps 10 > gpurun_out/r3b_prof.log 2>&1
