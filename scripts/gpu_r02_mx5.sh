#!/bin/bash
# k_scan_mx5 round: PMC passes (counters + HBM traffic), then the round-end validation
# (all GPU tests, smoke, default bench, kernel-trace profile).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_pmc_mx5.sh || exit 1
TAG=${TAG:-r02c} bash scripts/gpu_final.sh
