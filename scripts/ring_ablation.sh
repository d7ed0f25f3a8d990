cd $GRAFT_REPO_ROOT
for v in base ring3; do
  if [ $v = base ]; then unset GVDB_LIB_PATH; else export GVDB_LIB_PATH=$PWD/abl/libgvdb_$v.so; fi
  echo "== $v"; timeout -k 10 200 python scripts/scan_ablation.py fp4:0 fp4:0 fp4:0 2>&1 | grep scan || exit 1
done
