set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for n in 1250000 2500000 5000000 10000000; do SHARD_N=$n timeout -k 10 300 python3 -u scripts/b256_timing.py 2>&1 | grep -v amdgpu.ids | grep ms/step; done
SHARD_N=1250000 TAG=noflush GVDB_LIB_PATH=$PWD/grape-vector-db_amd/abl/libgvdb_noflush.so timeout -k 10 300 python3 -u scripts/b256_timing.py 2>&1 | grep ms/step
for f in 16384 32768 131072; do SHARD_N=1250000 TAG=floor$f GVDB_SAMPLE_FLOOR=$f timeout -k 10 300 python3 -u scripts/b256_timing.py 2>&1 | grep ms/step; done
bash scripts/gpu.sh c3+c3prof
bash scripts/gpu.sh hnsw10m
