#!/bin/bash
# k_scan_mx5 timing ablations (results invalid in the variants): batch-256 step and scan at 10M x 768.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/mx5_abl.log; : > $out
for v in base ${VARIANTS:-1 2 4 6 7}; do
    if [ $v = base ]; then unset GVDB_LIB_PATH; else export GVDB_LIB_PATH=$PWD/abl/libgvdb_$v.so; fi
    TAG=abl$v timeout -k 10 300 python -u scripts/b256_timing.py >> $out 2>&1 || { tail $out; exit 1; }
done
grep -v amdgpu.ids $out
