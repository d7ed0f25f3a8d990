#!/bin/bash
# FP4-MFMA sample histogram: threshold-equality + MFMA-scan parity tests, then batch-256
# timing with the MFMA and the VALU sample histogram (GVDB_SAMPLE=valu) at 10M x 768.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "sample_histogram or mfma_batches or stage1_topr" --timeout 200 --timeout-method thread > gpurun_out/smx_tests.log 2>&1
rc=$?; [ -n "$SKIP_TESTS" ] || { tail -4 gpurun_out/smx_tests.log; [ $rc -eq 0 ] || exit $rc; }
: > gpurun_out/smx_timing.log
for v in mx valu mx valu; do
  export GVDB_SAMPLE=$v
  TAG=sample_$v timeout -k 10 300 python -u scripts/b256_timing.py >> gpurun_out/smx_timing.log 2>&1 || exit 1
done
export GVDB_SAMPLE=mx
TAG=shard_mx SHARD_N=1250000 timeout -k 10 300 python -u scripts/b256_timing.py >> gpurun_out/smx_timing.log 2>&1 || exit 1
GVDB_SAMPLE=valu TAG=shard_valu SHARD_N=1250000 timeout -k 10 300 python -u scripts/b256_timing.py >> gpurun_out/smx_timing.log 2>&1 || exit 1
TAG=shard_mx SHARD_N=1250000 timeout -k 10 300 python -u scripts/b256_timing.py >> gpurun_out/smx_timing.log 2>&1 || exit 1
GVDB_SAMPLE=valu TAG=shard_valu SHARD_N=1250000 timeout -k 10 300 python -u scripts/b256_timing.py >> gpurun_out/smx_timing.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/smx_timing.log
unset GVDB_SAMPLE
GVDB_SAMPLE=mx SHARD_N=${PROF_N:-1250000} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_smx -o run -- python3 scripts/b256_timing.py > gpurun_out/prof_smx.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_smx/run_kernel_stats.csv')):
    n = r['Name'].split('(')[0]
    if 'gvdb::' in n: print(n[:44], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
"
find gpurun_out/prof_smx -type f ! -name "*_kernel_stats.csv" -delete
