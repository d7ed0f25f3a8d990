bash scripts/gpu_tests_shard.sh > gpurun_out/step1.log 2>&1; rc=$?; tail -8 gpurun_out/step1.log; [ $rc -eq 0 ] || exit $rc
VARIANTS=base bash scripts/gpu_scan_abl.sh || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline --hnsw-rows 0 --no-points > gpurun_out/bench_quick.log 2>&1 || exit 1
tail -1 gpurun_out/bench_quick.log | cut -c1-300
