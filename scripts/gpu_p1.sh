#!/bin/bash
# k_scan_mx3 single-pass (MX3_PASSES=1, abl/libgvdb_p1.so) vs the default two-pass build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 10000000 1250000; do
  for v in base p1 base p1; do
    if [ $v = base ]; then unset GVDB_LIB_PATH; else export GVDB_LIB_PATH=$PWD/abl/libgvdb_$v.so; fi
    echo "== n=$n $v"; SHARD_N=$n timeout -k 10 200 python scripts/shard_step_timing.py 2>&1 | grep -E "single|same" || exit 1
  done
done
unset GVDB_LIB_PATH
d=gpurun_out/p1prof
GVDB_LIB_PATH=$PWD/abl/libgvdb_p1.so SHARD_N=10000000 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -T -d $d -o run -- python3 scripts/shard_step_timing.py > $d.log 2>&1 || exit 1
grep -E '"k_scan_mx3"' $d/run_kernel_stats.csv | cut -d, -f1,2,4
