#!/bin/bash
# build_variant.sh NAME "-DFLAGS..." : libo3dml_amd.so with nns_frs.hip built with extra flags -> open3d-ml_amd/lib_NAME/
set -e
cd "$(dirname "$0")/../open3d-ml_amd/csrc"
mkdir -p ../lib_$1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fvisibility=hidden -munsafe-fp-atomics $2 -c nns_frs.hip -o /tmp/nns_frs_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib_$1/libo3dml_amd.so /tmp/nns_frs_$1.o $(ls ../build/*.o | grep -v nns_frs)
