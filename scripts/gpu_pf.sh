#!/bin/bash
# k_scan_mx3 A-fragment ring depth (MX3_PF builds in abl/) vs the default (4), 10M shard.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in base pf2 pf3 base pf2 pf3; do
  if [ $v = base ]; then unset GVDB_LIB_PATH; else export GVDB_LIB_PATH=$PWD/abl/libgvdb_$v.so; fi
  echo "== $v"; SHARD_N=10000000 timeout -k 10 200 python scripts/shard_step_timing.py 2>&1 | grep -E "single|same" || exit 1
done
