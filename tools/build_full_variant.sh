#!/bin/bash
# build_full_variant.sh NAME "-DFLAGS..." : every csrc source rebuilt with the
# extra flags (for header-level knobs) -> open3d-ml_amd/lib_NAME/libo3dml_amd.so
set -e
cd "$(dirname "$0")/../open3d-ml_amd/csrc"
O=/tmp/var_$1; mkdir -p $O ../lib_$1
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fvisibility=hidden -munsafe-fp-atomics $2"
ls *.hip *.cpp | xargs -P 8 -I{} sh -c "/opt/rocm/bin/hipcc $F -c {} -o $O/{}.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib_$1/libo3dml_amd.so $O/*.o -L/opt/rocm/lib -lrocblas -Wl,-rpath,/opt/rocm/lib
