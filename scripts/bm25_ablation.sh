cd $GRAFT_REPO_ROOT
for v in base bm1 bm2 bm3; do
  if [ $v = base ]; then unset GVDB_LIB_PATH; else export GVDB_LIB_PATH=$PWD/abl/libgvdb_$v.so; fi
  echo "== $v"; timeout -k 10 300 python scripts/bench_hybrid.py --n 2000000 --no-cpu-baseline 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['stage_ms_per_step'])" || exit 1
done
