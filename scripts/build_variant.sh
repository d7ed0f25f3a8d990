#!/bin/bash
# Build a timing variant of libgvdb.so with extra compile flags:
#   scripts/build_variant.sh NAME "-DFLAG=V ..."  ->  grape-vector-db_amd/abl/libgvdb_NAME.so
# (A/B runs load it with GVDB_LIB_PATH; abl/ is git-ignored, gpurun ships it.)
set -e
cd "$(dirname "$0")/../grape-vector-db_amd"
name=$1
flags=$2
b=abl/build_$name
mkdir -p "$b"
objs=()
for f in csrc/*.hip; do
    o=$b/$(basename "${f%.hip}").o
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wall -Wno-unused-result $flags -c "$f" -o "$o" &
    objs+=("$o")
done
g++ -O2 -std=c++17 -fPIC -Wall -c csrc/gvdb_persist.cpp -o "$b/gvdb_persist.o"
g++ -O2 -std=c++17 -fPIC -Wall -c csrc/gvdb_coalesce.cpp -o "$b/gvdb_coalesce.o"
wait
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -shared -o "abl/libgvdb_$name.so" "${objs[@]}" "$b/gvdb_persist.o" "$b/gvdb_coalesce.o" -lz -ldl -lpthread
rm -rf "$b"
echo "abl/libgvdb_$name.so"
