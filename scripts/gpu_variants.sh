#!/bin/bash
# Time libgvdb.so variants (abl/libgvdb_<name>.so) against the default build on
# the batch-256 path: VARIANTS="p1 p2", SIZES="10000000 1250000", REPS=2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02
out=gpurun_out/r02/variants.log
: > $out
for rep in $(seq ${REPS:-2}); do
  for n in ${SIZES:-10000000}; do
    for v in base $VARIANTS; do
      if [ $v = base ]; then unset GVDB_LIB_PATH; else export GVDB_LIB_PATH=$PWD/abl/libgvdb_$v.so; fi
      SHARD_N=$n TAG=$v timeout -k 10 200 python scripts/b256_timing.py 2>&1 | grep "\[" >> $out || exit 1
    done
  done
done
cat $out
