cd $GRAFT_REPO_ROOT
export BS=256
export FLAT_REPS=3
for d in 0 1 2 4 3 6; do
  echo "dbg=$d"; GVDB_FLAT_DBG_NOEMIT=1 GVDB_FLAT_DBG=$d timeout -k 10 200 python scripts/flat_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
done
