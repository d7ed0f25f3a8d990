#!/bin/bash
# Timing-ablation builds of libgvdb.so (k_flat_mx with parts disabled via
# FX_ABL; results invalid) into abl/libgvdb_abl<N>.so.  Run on the CPU host.
set -e
cd "$(dirname "$0")/../grape-vector-db_amd"
F="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wno-unused-result"
mkdir -p ../abl
for v in "$@"; do
    /opt/rocm/bin/hipcc $F -DFX_ABL=$v -c csrc/gvdb_flat.hip -o ../abl/flat_$v.o &
done
wait
for v in "$@"; do
    /opt/rocm/bin/hipcc $F -shared -o ../abl/libgvdb_abl$v.so build/gvdb_kernels.o ../abl/flat_$v.o build/gvdb_sparse.o build/gvdb_capi.o
    rm ../abl/flat_$v.o
done
ls -la ../abl
