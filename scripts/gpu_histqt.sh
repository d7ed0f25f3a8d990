#!/bin/bash
# VALU sample-histogram queries per block (GVDB_HIST_LDS_WORDS / (D+1)) at the 10M shard.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for w in 12288 6144 24576 3072 12288 6144 24576 3072; do
  echo "== words $w"; SHARD_N=10000000 GVDB_HIST_LDS_WORDS=$w timeout -k 10 200 python scripts/shard_step_timing.py 2>&1 | grep -E "single|same" || exit 1
done
