#!/bin/bash
# Timing variants of libgvdb.so: each argument NAME=FLAGS builds abl/libgvdb_NAME.so
# with gvdb_kernels.hip compiled with FLAGS (e.g. mx3p1=-DMX3_PRIO=1).  CPU host only.
set -e
cd "$(dirname "$0")/../grape-vector-db_amd"
make -s libgvdb.so
F="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wno-unused-result"
mkdir -p ../abl
for kv in "$@"; do
    name=${kv%%=*}; flags=${kv#*=}
    /opt/rocm/bin/hipcc $F $flags -c csrc/gvdb_kernels.hip -o ../abl/kern_$name.o &
done
wait
for kv in "$@"; do
    name=${kv%%=*}
    /opt/rocm/bin/hipcc $F -shared -o ../abl/libgvdb_$name.so ../abl/kern_$name.o build/gvdb_flat.o build/gvdb_sparse.o build/gvdb_capi.o build/gvdb_comm.o build/gvdb_persist.o -lz -ldl
    rm ../abl/kern_$name.o
done
ls -la ../abl
