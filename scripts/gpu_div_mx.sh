#!/bin/bash
# sample-size sweep with the FP4 sample histogram forced (GVDB_SAMPLE=mx): batch-256 step at 10M x 768
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp GVDB_SAMPLE=mx
for div in 64 32 48 96 64; do
  GVDB_SAMPLE_DIV=$div TAG="div=$div" timeout -k 10 300 python -u scripts/b256_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
done
