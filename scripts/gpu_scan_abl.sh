#!/bin/bash
# k_scan_mx3 emit/flush ablation (timing only): kernel times at the 8-GPU
# shard size (1.25M) and the 10M single-GPU shard.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 1250000 10000000; do
  for v in ${VARIANTS:-base 1 2}; do
    if [ $v = base ]; then unset GVDB_LIB_PATH; else export GVDB_LIB_PATH=$PWD/abl/libgvdb_mx3abl$v.so; fi
    d=gpurun_out/abl_${v}_$n
    SHARD_N=$n timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -T -d $d -o run -- python3 scripts/shard_step_timing.py > $d.log 2>&1 || { echo "fail $v $n"; tail $d.log; exit 1; }
    find $d -type f ! -name "*_kernel_stats.csv" -delete
    echo "== n=$n variant=$v: $(grep 'single-device' $d.log)"
    grep -E '"(k_scan_mx3|k_sample_hist|k_select|k_rerank)"' $d/run_kernel_stats.csv | cut -d, -f1,2,4
  done
done
