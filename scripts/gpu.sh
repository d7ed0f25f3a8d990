#!/bin/bash
# One entry point for the GPU-box runs (gpurun -- 'bash scripts/gpu.sh TASK[+TASK...] [ARGS]').
# Every step runs under its own time limit; the first failing step ends the run.
#
#   tests        pytest -m gpu (all GPU tests, one process)            -> gpurun_out/pytest_gpu.log
#   tests:EXPR   pytest -m gpu -k EXPR
#   smoke        __graft_entry__.smoke()                                -> gpurun_out/smoke.log
#   bench        python bench.py (the driver's default command)         -> gpurun_out/bench.json / .log
#   benchprof    the same command under rocprofv3 --kernel-trace --stats -> gpurun_out/prof_bench/
#   b256         scripts/b256_timing.py at 10M (SHARD_N / RCCL env pass through)
#   coalesce     build/coalesce_bench: concurrent batch-1 callers, B=1 searches vs the coalescer -> gpurun_out/coalesce.json
#   bigr         scripts/bigr_timing.py: R = 0.1 N at 1M / 10M rows -> gpurun_out/bigr.json
#   scanab       scripts/scan_ab.py: stage-1 scan timing at 10M and 1.25M rows (SCANS: GVDB_SCAN values) -> gpurun_out/scanab.log
#   c3           scripts/c3_emulate.py (config 3, 8 shards on one GPU)  -> gpurun_out/c3.json / .log
#   c3prof       c3_emulate (no single index, no oracle) under rocprofv3 -> gpurun_out/prof_c3/
#   c4           scripts/c4_emulate.py (config 4, 8 shards of 1.25M x 3072; one-exchange merge)
#   c4x2         scripts/c3_emulate.py --dim 3072: config 4 on the two-exchange protocol
#   hybrid       scripts/bench_hybrid.py (config 5)                     -> gpurun_out/hybrid.json / .log
#   hnsw10m      scripts/hnsw10m_gpu.py (GPU side of the 10M equal-recall experiment)
#   pmc:NAME:REGEX:CMD[:FIRST]   rocprofv3 --pmc passes (one counter set per run) over python3 CMD (spaces as ','),
#                        rows whose kernel name matches REGEX -> gpurun_out/pmc_NAME/pmc.json; FIRST = the
#                        pmc_summary.py --first filter (kernel=N/...: only each kernel's first N dispatches)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out

run() {  # run LIMIT_S LOG cmd...
    local lim=$1 log=$2
    shift 2
    echo "[gpu.sh] $(date +%T) $*" >&2
    timeout -k 10 "$lim" "$@" > "$log" 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then
        echo "[gpu.sh] FAILED rc=$rc: $*" >&2
        tail -30 "$log" >&2
        exit $rc
    fi
}

PMC_SETS=("GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
          "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT"
          "FETCH_SIZE" "WRITE_SIZE")

IFS='+' read -ra TASKS <<< "$1"
for t in "${TASKS[@]}"; do
    case "$t" in
        tests)
            run 1500 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
            grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2 ;;
        tests:*)
            run 1500 gpurun_out/pytest_gpu_k.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${t#tests:}"
            grep -E "passed|failed" gpurun_out/pytest_gpu_k.log | tail -2 ;;
        smoke)
            run 300 gpurun_out/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
            tail -3 gpurun_out/smoke.log ;;
        bench)
            run 900 gpurun_out/bench.log python -u bench.py
            grep '^{' gpurun_out/bench.log > gpurun_out/bench.json; tail -c 600 gpurun_out/bench.json; echo ;;
        benchprof)
            run 900 gpurun_out/benchprof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py
            grep '^{' gpurun_out/benchprof.log > gpurun_out/benchprof.json || true ;;
        warm)  # bench.py's scan time vs its warmup count (clock ramp?), then scan_ab, one box
            run 600 gpurun_out/warm_w3.log python3 -u bench.py --no-cpu-baseline --no-points --b1-queries 0
            run 600 gpurun_out/warm_w200.log python3 -u bench.py --no-cpu-baseline --no-points --b1-queries 0 --warmup 200
            SHARD_N=10000000 SCANS="," REPS=1 run 600 gpurun_out/warm_scanab.log python3 -u scripts/scan_ab.py
            for f in warm_w3 warm_w200; do grep -o '"ms_per_step": [0-9.]*\|"scan": [0-9.]*' gpurun_out/$f.log | tr '\n' ' '; echo; done
            grep '^\[scan_ab\]' gpurun_out/warm_scanab.log ;;
        c2)  # BASELINE configs[1]: 1M x 768, batch 256, bench.py's own pipeline at N = 1M
            run 900 gpurun_out/c2.log python3 -u bench.py --n 1000000
            grep '^{' gpurun_out/c2.log > gpurun_out/c2.json; tail -c 300 gpurun_out/c2.json; echo ;;
        c1)  # BASELINE configs[0]: MockEmbeddingProvider 10k x 128
            run 600 gpurun_out/c1.log python3 -u scripts/config1_mock.py
            grep '^{' gpurun_out/c1.log > gpurun_out/c1.json; tail -c 300 gpurun_out/c1.json; echo ;;
        c3ab)  # config-3 emulation A/B: VARIANTS (abl/libgvdb_NAME.so, "base" = product) alternating, one box
            for v in ${VARIANTS:-base}; do
                lib=""; [ "$v" != base ] && lib=grape-vector-db_amd/abl/libgvdb_$v.so
                GVDB_LIB_PATH=$lib run 300 gpurun_out/c3ab_$v.log python3 -u scripts/c3_emulate.py --no-single --oracle-queries 0 --steps 20
                echo "$v $(grep 'per-rank step' gpurun_out/c3ab_$v.log) p2 $(grep -o '"merge_rerank_topk_ms": [0-9.]*' gpurun_out/c3ab_$v.log | head -8 | awk '{s+=$2} END {print s/NR}') $(grep -o '"host_enqueue_us_per_call": {[^}]*}' gpurun_out/c3ab_$v.log || true)"
            done ;;
        envab)  # bench.py's batch-256 step under env variants (ENVS: ';'-separated "NAME=V,NAME=V" sets, "-" = none), one box
            IFS=';' read -ra SETS <<< "${ENVS:--}"
            for e in "${SETS[@]}" "${SETS[@]}"; do
                envs=(); [ "$e" != "-" ] && IFS=',' read -ra envs <<< "$e"
                env "${envs[@]}" timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-points --b1-queries 0 > gpurun_out/envab.log 2>&1 || { tail -20 gpurun_out/envab.log; exit 1; }
                echo "[$e] $(grep -o '"ms_per_step": [0-9.]*\|"stage_ms_per_step": {[^}]*}' gpurun_out/envab.log | tr '\n' ' ')"
            done ;;
        ablscan)  # k_scan timing variants (abl/libgvdb_NAME.so, scripts/build_variant.sh) against the product
                  # build, one box; VARIANTS: space-separated names ("base" = the product build)
            for v in ${VARIANTS:-base}; do
                lib=""; [ "$v" != base ] && lib=grape-vector-db_amd/abl/libgvdb_$v.so
                GVDB_LIB_PATH=$lib SHARD_N=10000000 SCANS="" REPS=2 run 300 gpurun_out/ablscan_$v.log python3 -u scripts/scan_ab.py
                echo "$v $(grep '^\[scan_ab\]' gpurun_out/ablscan_$v.log | tail -1)"
            done ;;
        scanvar)  # k_scan timing of build variants at 10M and the 1.25M shard (VARIANTS, "base" = product), one box
            for v in ${VARIANTS:-base}; do
                lib=""; [ "$v" != base ] && lib=grape-vector-db_amd/abl/libgvdb_$v.so
                GVDB_LIB_PATH=$lib SHARD_N=10000000,1250000 SCANS="" REPS=2 run 400 gpurun_out/scanvar_$v.log python3 -u scripts/scan_ab.py
                grep '^\[scan_ab\]' gpurun_out/scanvar_$v.log | sed "s/^/$v /"
            done ;;
        scanab)  # stage-1 scan timing at 10M and the 1.25M shard (same box, alternating SCANS)
            SHARD_N=10000000,1250000 SCANS="${SCANS:-,}" REPS=3 run 900 gpurun_out/scanab.log python3 -u scripts/scan_ab.py
            grep '^\[scan_ab\]' gpurun_out/scanab.log ;;
        coalesce)  # concurrent batch-1 callers at 10M x 768: B=1 searches vs the request coalescer
            run 900 gpurun_out/coalesce.log grape-vector-db_amd/build/coalesce_bench 10000000 768 100 10 4 1 8 64
            grep '^{' gpurun_out/coalesce.log > gpurun_out/coalesce.json; cat gpurun_out/coalesce.json ;;
        bigr)  # the reference's default depth R = 0.1 N at 1M and 10M rows, batch 8 / 64 / 256
            run 1100 gpurun_out/bigr.log python3 -u scripts/bigr_timing.py
            grep '^{' gpurun_out/bigr.log > gpurun_out/bigr.json; cat gpurun_out/bigr.json ;;
        b256)
            run 600 gpurun_out/b256.log python3 -u scripts/b256_timing.py
            grep -v amdgpu.ids gpurun_out/b256.log | tail -4 ;;
        c3)
            run 900 gpurun_out/c3.log python -u scripts/c3_emulate.py
            grep '^{' gpurun_out/c3.log > gpurun_out/c3.json; grep '^\[c3\]' gpurun_out/c3.log | tail -4 ;;
        c4prof)  # kernel trace of config 4's per-rank step (8 shards of 1.25M x 3072, batch 256)
            run 900 gpurun_out/c4prof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o run -- python3 scripts/c3_emulate.py --dim 3072 --no-single --oracle-queries 0 --steps 5
            python3 scripts/trace_summary.py gpurun_out/prof_c4/run_kernel_trace.csv > gpurun_out/c4_kernels.txt; head -20 gpurun_out/c4_kernels.txt ;;
        c3prof)
            run 600 gpurun_out/c3prof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 scripts/c3_emulate.py --no-single --oracle-queries 0 --steps 10
            python3 scripts/trace_summary.py gpurun_out/prof_c3/run_kernel_trace.csv | head -16 ;;
        deepprof)  # kernel trace of the deep form (1M, R = 100K, batch 256; 10M, R = 1M, batch 64)
            run 600 gpurun_out/deepprof_1M.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_deep1M -o run -- python3 scripts/c3_emulate.py --n 1000000 --R 100000 --no-single --oracle-queries 0 --steps 2
            python3 scripts/trace_summary.py gpurun_out/prof_deep1M/run_kernel_trace.csv > gpurun_out/deep1M_kernels.txt
            run 900 gpurun_out/deepprof_10M.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_deep10M -o run -- python3 scripts/c3_emulate.py --n 10000000 --R 1000000 --batch 64 --no-single --oracle-queries 0 --steps 2
            python3 scripts/trace_summary.py gpurun_out/prof_deep10M/run_kernel_trace.csv > gpurun_out/deep10M_kernels.txt ;;
        c3floor)  # c3 per-rank step with the default sample floor vs 131072 / 262144 sample rows (same box)
            for f in ${FLOORS:-0 131072 262144}; do
                GVDB_SAMPLE_FLOOR=$f run 600 gpurun_out/c3floor_$f.log python3 scripts/c3_emulate.py --oracle-queries 0 --steps 20
                echo "== floor $f"; grep '^\[c3\]' gpurun_out/c3floor_$f.log | tail -2
            done ;;
        mx7clk)  # k_scan_mx7 per-wave phase clocks (variant build abl/libgvdb_mx7clk.so) at 1.25M and 10M rows
            GVDB_LIB_PATH=$PWD/grape-vector-db_amd/abl/libgvdb_mx7clk.so run 600 gpurun_out/mx7clk.log python3 -u scripts/mx7_clock.py
            grep '^\[mx7clk\]' gpurun_out/mx7clk.log ;;
        prepclk)  # k_sample_prep per-wave phase clocks (variant build abl/libgvdb_prepclk.so)
            GVDB_LIB_PATH=$PWD/grape-vector-db_amd/abl/libgvdb_prepclk.so run 300 gpurun_out/prepclk.log python3 -u scripts/prep_clock.py
            grep '^\[prepclk\]' gpurun_out/prepclk.log ;;
        c3clk)
            run 600 gpurun_out/c3clk.log python3 scripts/c3_emulate.py --no-single --oracle-queries 0 --steps 10 --p2clk
            grep '^\[c3\]' gpurun_out/c3clk.log ;;
        flatab)  # exact flat at 10M x 768, one box: candidate pruning (default) | every candidate reranked
            for v in prune noprune; do
                case $v in
                    prune) BS=256 FLAT_REPS=10 run 600 gpurun_out/flatab_$v.log python3 scripts/flat_timing.py ;;
                    noprune) GVDB_FLAT_PRUNE=0 BS=256 FLAT_REPS=10 run 600 gpurun_out/flatab_$v.log python3 scripts/flat_timing.py ;;
                esac
                echo "== $v"; grep -E "B=|emit" gpurun_out/flatab_$v.log | tail -2
            done ;;
        flatevery)  # exact flat sample-pass stride A/B (GVDB_FLAT_EVERY; default 64 tiles)
            for v in 64 128; do
                GVDB_FLAT_EVERY=$v BS=256 FLAT_REPS=10 run 600 gpurun_out/flatevery_$v.log python3 scripts/flat_timing.py
                echo "== every $v"; grep -E "B=|emit" gpurun_out/flatevery_$v.log | tail -2
            done ;;
        probeprof:*)  # k_flat_probes (and every flat kernel) per build variant: kernel stats of flat_timing
            IFS=',' read -ra VARS <<< "${t#probeprof:}"
            for v in "${VARS[@]}"; do
                lib=""; [ "$v" != base ] && lib=$PWD/grape-vector-db_amd/abl/libgvdb_$v.so
                GVDB_LIB_PATH=$lib BS=256 FLAT_REPS=5 run 600 gpurun_out/probeprof_$v.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_probe_$v -o run -- python3 scripts/flat_timing.py
                echo "== $v"; grep -E "k_flat_probes|k_flat_i8q|k_rerank2" gpurun_out/prof_probe_$v/run_kernel_stats.csv | cut -d, -f1-4
            done ;;
        flatvar:*)  # k_flat_i8q build variants A/B: flatvar:a,b,... runs abl/libgvdb_<a>.so ... ("base" = libgvdb.so)
            IFS=',' read -ra VARS <<< "${t#flatvar:}"
            for v in "${VARS[@]}"; do
                lib=""; [ "$v" != base ] && lib=$PWD/grape-vector-db_amd/abl/libgvdb_$v.so
                GVDB_FLAT=i8 GVDB_LIB_PATH=$lib BS=${FBS:-256} FLAT_REPS=10 run 600 gpurun_out/flatvar_$v.log python3 scripts/flat_timing.py
                echo "== $v"; grep -E "B=|emit" gpurun_out/flatvar_$v.log | tail -2
            done ;;
        flatshard)  # the flat pass at the 8-GPU shard (1.25M x 768), batch 64, k = 10 and 32, kernel trace
            for kk in 10 32; do
                N=1250000 K=$kk GVDB_FLAT=i8 BS=64 FLAT_REPS=10 run 600 gpurun_out/flatshard_$kk.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_flatshard_$kk -o run -- python3 scripts/flat_timing.py
                echo "== k $kk"; grep -E "B=|emit" gpurun_out/flatshard_$kk.log | tail -2
                python3 scripts/trace_summary.py gpurun_out/prof_flatshard_$kk/run_kernel_trace.csv | head -14
            done ;;
        flatshardab)  # the flat pass at the 8-GPU shard, batch 64, k = 32: sample stride and prune variants
            for v in e64 e16 e4 noprune; do
                case $v in
                    e64) ENVV="GVDB_FLAT_EVERY=64" ;;
                    e16) ENVV="GVDB_FLAT_EVERY=16" ;;
                    e4) ENVV="GVDB_FLAT_EVERY=4" ;;
                    noprune) ENVV="GVDB_FLAT_PRUNE=0" ;;
                esac
                env $ENVV N=1250000 K=32 GVDB_FLAT=i8 BS=64 FLAT_REPS=10 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fsab_$v -o run -- python3 scripts/flat_timing.py > gpurun_out/fsab_$v.log 2>&1 || { echo "FAILED $v"; exit 1; }
                echo "== $v"; grep -E "B=|emit" gpurun_out/fsab_$v.log | tail -2
                python3 scripts/trace_summary.py gpurun_out/prof_fsab_$v/run_kernel_trace.csv | head -12
            done ;;
        flatstats)  # candidate counts of the flat pass (variant build abl/libgvdb_fstats.so), 1.25M and 10M rows
            for nn in 1250000 10000000; do
                GVDB_LIB_PATH=$PWD/grape-vector-db_amd/abl/libgvdb_fstats.so N=$nn K=32 GVDB_FLAT=i8 BS=64 FLAT_REPS=2 run 600 gpurun_out/fstats_$nn.log python3 scripts/flat_timing.py
                grep flatstats gpurun_out/fstats_$nn.log | tail -2
            done ;;
        flatrr)  # flat pass rerank variants (GVDB_RERANK = default | items) at the shard (k 32, B 64) and 10M (k 10, B 256)
            for v in ${RRV:-def items}; do
                ENVV="GVDB_RERANK=$v"
                [ "$v" = dma ] && ENVV="GVDB_RERANK_DMA=1"
                env $ENVV N=1250000 K=32 GVDB_FLAT=i8 BS=64 FLAT_REPS=10 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_frr_$v -o run -- python3 scripts/flat_timing.py > gpurun_out/frr_$v.log 2>&1 || { echo "FAILED $v"; exit 1; }
                echo "== shard $v"; grep -E "B=|emit" gpurun_out/frr_$v.log | tail -2
                python3 scripts/trace_summary.py gpurun_out/prof_frr_$v/run_kernel_trace.csv | grep -E "rerank|i8q"
                env $ENVV N=10000000 K=10 GVDB_FLAT=i8 BS=256 FLAT_REPS=10 timeout -k 10 600 python3 scripts/flat_timing.py > gpurun_out/frr10_$v.log 2>&1 || { echo "FAILED 10M $v"; exit 1; }
                echo "== 10M $v"; grep -E "B=|emit" gpurun_out/frr10_$v.log | tail -2
            done ;;
        flatevery2)  # flat sample stride A/B at the shard (k 32, B 64) and 10M (k 10, B 256)
            for v in 64 32 16; do
                GVDB_FLAT_EVERY=$v N=1250000 K=32 GVDB_FLAT=i8 BS=64 FLAT_REPS=10 run 600 gpurun_out/fe2s_$v.log python3 scripts/flat_timing.py
                echo "== shard every $v"; grep -E "B=|emit" gpurun_out/fe2s_$v.log | tail -2
                GVDB_FLAT_EVERY=$v N=10000000 K=10 GVDB_FLAT=i8 BS=256 FLAT_REPS=10 run 600 gpurun_out/fe2l_$v.log python3 scripts/flat_timing.py
                echo "== 10M every $v"; grep -E "B=|emit" gpurun_out/fe2l_$v.log | tail -2
            done ;;
        probeab)  # flat pass probe selection blocks per query (GVDB_PROBE_PARTS 1 / 4 / default) at 10M B 256 k 10 and the shard
            for v in 1 4 0; do
                GVDB_PROBE_PARTS=$v N=10000000 K=10 GVDB_FLAT=i8 BS=256 FLAT_REPS=10 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pab_$v -o run -- python3 scripts/flat_timing.py > gpurun_out/pab_$v.log 2>&1 || { echo "FAILED $v"; exit 1; }
                echo "== 10M parts $v"; grep -E "B=|emit" gpurun_out/pab_$v.log | tail -2
                python3 scripts/trace_summary.py gpurun_out/prof_pab_$v/run_kernel_trace.csv | grep -E "i8q|rerank|k_flat" | head -10
                GVDB_PROBE_PARTS=$v N=1250000 K=32 GVDB_FLAT=i8 BS=64 FLAT_REPS=10 run 600 gpurun_out/pabs_$v.log python3 scripts/flat_timing.py
                echo "== shard parts $v"; grep -E "B=|emit" gpurun_out/pabs_$v.log | tail -2
            done ;;
        flatwide)  # flat pass at D = 3072 (k_flat_mx path) on the config-4 shard, variants: flatwide:base,prevflush
            IFS=',' read -ra VARS <<< "${FWV:-base,prevflush}"
            for v in "${VARS[@]}"; do
                lib=""; [ "$v" != base ] && lib=$PWD/grape-vector-db_amd/abl/libgvdb_$v.so
                GVDB_LIB_PATH=$lib N=1250000 D=3072 K=10 BS=256,64 FLAT_REPS=10 run 600 gpurun_out/flatwide_$v.log python3 scripts/flat_timing.py
                echo "== $v"; grep -E "B=|emit" gpurun_out/flatwide_$v.log | tail -4
            done ;;
        flatwidestats)  # candidate counts of the flat tiers at 1.25M x 3072 (variant abl/libgvdb_fstats.so)
            for tier in i8 bf16; do
                for b in 64 256; do
                    GVDB_FLAT=$tier GVDB_LIB_PATH=$PWD/grape-vector-db_amd/abl/libgvdb_fstats.so N=1250000 D=3072 K=10 BS=$b FLAT_REPS=1 run 600 gpurun_out/fws_${tier}_$b.log python3 scripts/flat_timing.py
                    echo "== $tier B=$b"; grep -E "flatstats|B=" gpurun_out/fws_${tier}_$b.log | sort | uniq -c | sort -rn | head -6
                done
            done ;;
        flatprof)  # exact flat search at 10M x 768, batch 256, per-dispatch kernel trace
            BS=256 FLAT_REPS=5 run 600 gpurun_out/flatprof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_flat -o run -- python3 scripts/flat_timing.py
            grep -E "B=|emit" gpurun_out/flatprof.log | tail -3 ;;
        deep)  # the deep two-exchange form at the reference's default ratio: 8 shards of 1M (R = 100K) and 10M (R = 1M)
            run 900 gpurun_out/deep_1M.log python3 -u scripts/c3_emulate.py --n 1000000 --R 100000 --batch 256 --steps 3 --oracle-queries 8
            grep '^{' gpurun_out/deep_1M.log > gpurun_out/deep_1M.json
            run 1100 gpurun_out/deep_10M.log python3 -u scripts/c3_emulate.py --n 10000000 --R 1000000 --batch 64 --steps 2 --oracle-queries 2
            grep '^{' gpurun_out/deep_10M.log > gpurun_out/deep_10M.json
            grep '\[c3\]' gpurun_out/deep_1M.log gpurun_out/deep_10M.log ;;
        deepearly)  # deep 10M with / without the early flat list (GVDB_DEEP_EARLY=0), same box
            for v in 1 0; do
                GVDB_DEEP_EARLY=$v run 900 gpurun_out/deepearly_$v.log python3 -u scripts/c3_emulate.py --n 10000000 --R 1000000 --batch 64 --steps 3 --oracle-queries 0 --no-single
                echo "== early $v"; grep '\[c3\]' gpurun_out/deepearly_$v.log | tail -2
            done ;;
        deepab)  # deep 10M (R = 1M, batch 64) per-rank step, VARIANTS (abl/libgvdb_NAME.so, "base" = product), one box
            for v in ${VARIANTS:-base}; do
                lib=""; [ "$v" != base ] && lib=$PWD/grape-vector-db_amd/abl/libgvdb_$v.so
                GVDB_LIB_PATH=$lib run 900 gpurun_out/deepab_$v.log python3 -u scripts/c3_emulate.py --n 10000000 --R 1000000 --batch 64 --steps 3 --oracle-queries 0 --no-single
                echo "== $v $(grep 'per-rank step' gpurun_out/deepab_$v.log)"
            done ;;
        mx4var:*)  # k_scan_mx4 build variants at 10M x 3072 (b256_timing, one box): mx4var:base,ch8,...
            IFS=',' read -ra VARS <<< "${t#mx4var:}"
            for v in "${VARS[@]}"; do
                lib=""; [ "$v" != base ] && lib=$PWD/grape-vector-db_amd/abl/libgvdb_$v.so
                DIM=3072 GVDB_LIB_PATH=$lib TAG=$v run 600 gpurun_out/mx4var_$v.log python3 -u scripts/b256_timing.py
                grep "scan" gpurun_out/mx4var_$v.log | tail -1
            done ;;
        flatvar)  # exact flat timing at 10M x 768 (BS, default 256,64), VARIANTS (abl/libgvdb_NAME.so, "base" = product) alternating
            for v in ${VARIANTS:-base}; do
                lib=""; [ "$v" != base ] && lib=$PWD/grape-vector-db_amd/abl/libgvdb_$v.so
                GVDB_LIB_PATH=$lib BS=${BS:-256,64} FLAT_REPS=10 run 600 gpurun_out/flatvar_$v.log python3 -u scripts/flat_timing.py
                echo "== $v"; grep -E "B=|emit" gpurun_out/flatvar_$v.log | tail -4
            done ;;
        bm25ab)  # BM25 leg at 5M docs, one box: VARIANTS (abl/libgvdb_NAME.so, "base" = product) alternating twice
            for v in ${VARIANTS:-base} ${VARIANTS:-base}; do
                lib=""; [ "$v" != base ] && lib=grape-vector-db_amd/abl/libgvdb_$v.so
                GVDB_LIB_PATH=$lib run 300 gpurun_out/bm25ab_$v.log python3 -u scripts/bm25_timing.py --check --steps 20
                echo "$v $(tail -1 gpurun_out/bm25ab_$v.log)"
            done ;;
        bm25prof)  # BM25 leg at 5M docs under rocprofv3 (kernel trace) and the phase clocks, per VARIANT
            for v in ${VARIANTS:-base}; do
                lib=""; [ "$v" != base ] && lib=$PWD/grape-vector-db_amd/abl/libgvdb_$v.so
                GVDB_LIB_PATH=$lib run 300 gpurun_out/bm25prof_$v.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bm25_$v -o run -- python3 scripts/bm25_timing.py --steps 10
                python3 scripts/trace_summary.py gpurun_out/prof_bm25_$v/run_kernel_trace.csv > gpurun_out/bm25_kernels_$v.txt; echo "== $v"; head -8 gpurun_out/bm25_kernels_$v.txt
                GVDB_LIB_PATH=$lib GVDB_BM25_ABL=8 run 300 gpurun_out/bm25clk_$v.log python3 -u scripts/bm25_timing.py --steps 2
                grep "bm25 prof" gpurun_out/bm25clk_$v.log | tail -1
            done ;;
        bm25clk)  # BM25 leg at 5M docs: timing, then the per-phase shader clocks (GVDB_BM25_ABL=8)
            run 600 gpurun_out/bm25t.log python3 -u scripts/bm25_timing.py --check
            tail -3 gpurun_out/bm25t.log
            GVDB_BM25_ABL=8 run 600 gpurun_out/bm25clk.log python3 -u scripts/bm25_timing.py --steps 2
            grep "bm25 prof" gpurun_out/bm25clk.log | tail -2
            GVDB_BM25_ABL=1 run 600 gpurun_out/bm25norounds.log python3 -u scripts/bm25_timing.py
            echo "== no rounds (results invalid)"; tail -1 gpurun_out/bm25norounds.log ;;
        c4x2)  # config 4 (10M x 3072, 8 shards) on the TWO-exchange protocol, vs one 10M x 3072 index
            run 1100 gpurun_out/c4x2.log python -u scripts/c3_emulate.py --dim 3072 --oracle-queries 0 --steps 10
            grep '^{' gpurun_out/c4x2.log > gpurun_out/c4x2.json; grep '^\[c3\]' gpurun_out/c4x2.log | tail -4 ;;
        c4)
            run 1100 gpurun_out/c4.log python -u scripts/c4_emulate.py
            grep '^{' gpurun_out/c4.log > gpurun_out/c4.json; tail -3 gpurun_out/c4.log ;;
        hybrid)
            run 900 gpurun_out/hybrid.log python -u scripts/bench_hybrid.py
            grep '^{' gpurun_out/hybrid.log > gpurun_out/hybrid.json; tail -3 gpurun_out/hybrid.log ;;
        hnsw10m)
            run 1100 gpurun_out/hnsw10m_gpu.log python -u scripts/hnsw10m_gpu.py
            tail -5 gpurun_out/hnsw10m_gpu.log ;;
        pmc:*)
            IFS=':' read -r _ name regex cmd first <<< "$t"
            cmd=${cmd//,/ }
            out=gpurun_out/pmc_$name
            mkdir -p "$out"
            i=0
            for set in "${PMC_SETS[@]}"; do
                i=$((i + 1))
                # shellcheck disable=SC2086
                run 300 "$out/p$i.log" rocprofv3 --pmc $set --output-format csv -d "$out/p$i" -o run -- python3 $cmd
                f=$(find "$out/p$i" -name "*counter_collection.csv" | head -1)
                if [ -n "$f" ]; then head -1 "$f" > "$out/counters_p$i.csv"; grep -E "$regex" "$f" >> "$out/counters_p$i.csv" || true; fi
                rm -rf "${out:?}/p$i"
            done
            if [ -n "$first" ]; then
                python3 scripts/pmc_summary.py "$out" --first "${first//\//,}" --json "$out/pmc.json" | tail -40
            else
                python3 scripts/pmc_summary.py "$out" --json "$out/pmc.json" | tail -40
            fi ;;
        *)
            echo "[gpu.sh] unknown task $t" >&2
            exit 2 ;;
    esac
done
