#!/bin/bash
# Timing-ablation builds of libgvdb.so with k_scan_mx3 parts disabled via
# MX3_ABL=<v> (results invalid) into abl/libgvdb_mx3abl<v>.so.  CPU host only.
set -e
cd "$(dirname "$0")/../grape-vector-db_amd"
F="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wno-unused-result"
mkdir -p ../abl
for v in "$@"; do
    /opt/rocm/bin/hipcc $F -DMX3_ABL=$v -c csrc/gvdb_kernels.hip -o ../abl/kern_$v.o &
done
wait
for v in "$@"; do
    /opt/rocm/bin/hipcc $F -shared -o ../abl/libgvdb_mx3abl$v.so ../abl/kern_$v.o build/gvdb_flat.o build/gvdb_sparse.o build/gvdb_capi.o build/gvdb_persist.o -lz
    rm ../abl/kern_$v.o
done
ls -la ../abl
