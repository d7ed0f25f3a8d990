#!/bin/bash
# Emit-pass timing of the production k_flat_mx and of the FX_ABL ablation
# builds (abl/, scripts/build_flat_abl.sh); ablation results are invalid, so
# those runs suppress emission (GVDB_FLAT_DBG_NOEMIT) and time one batch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export BS=${BS:-256,1}
echo "production"
timeout -k 10 200 python scripts/flat_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "production, no emission"
GVDB_FLAT_DBG_NOEMIT=1 FLAT_REPS=1 timeout -k 10 200 python scripts/flat_timing.py 2>&1 | grep "k_flat_mx" || exit 1
for v in ${ABL:-1 2 3 4 8 12 14}; do
    echo "FX_ABL=$v"
    GVDB_LIB_PATH=$PWD/abl/libgvdb_abl$v.so GVDB_FLAT_DBG_NOEMIT=1 FLAT_REPS=1 timeout -k 10 200 python scripts/flat_timing.py 2>&1 | grep "k_flat_mx" || exit 1
done
