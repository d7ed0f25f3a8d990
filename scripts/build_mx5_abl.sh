#!/bin/bash
# Timing builds of libgvdb.so with k_scan_mx5 knobs, one per argument
# "<name>=<-D flags>" (e.g. abl7="-DMX5_ABL=7", prio1="-DMX5_PRIO=1") into
# abl/libgvdb_<name>.so.  MX5_ABL variants give invalid results.  CPU host only.
set -e
cd "$(dirname "$0")/../grape-vector-db_amd"
F="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wno-unused-result"
mkdir -p ../abl
for a in "$@"; do
    name=${a%%=*}; flags=${a#*=}
    /opt/rocm/bin/hipcc $F $flags -c csrc/gvdb_kernels.hip -o ../abl/kern_$name.o &
done
wait
for a in "$@"; do
    name=${a%%=*}
    /opt/rocm/bin/hipcc $F -shared -o ../abl/libgvdb_$name.so ../abl/kern_$name.o build/gvdb_flat.o build/gvdb_sparse.o build/gvdb_capi.o build/gvdb_comm.o build/gvdb_persist.o -lz -ldl
    rm ../abl/kern_$name.o
done
ls -la ../abl
