#!/bin/bash
# build_variant.sh NAME "-DFLAGS..." [SOURCE=nns_frs.hip] : libo3dml_amd.so with SOURCE built with extra flags
# -> open3d-ml_amd/lib_NAME/  (the other objects come from the current in-tree build)
set -e
SRC=${3:-nns_frs.hip}
cd "$(dirname "$0")/../open3d-ml_amd/csrc"
mkdir -p ../lib_$1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fvisibility=hidden -munsafe-fp-atomics $2 -c $SRC -o /tmp/${SRC%.hip}_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib_$1/libo3dml_amd.so /tmp/${SRC%.hip}_$1.o $(ls ../build/*.o | grep -v ${SRC})
