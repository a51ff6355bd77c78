#!/bin/bash
# sparse-conv GEMM probe per library build, interleaved (one box session):
# ab_libs_gemm.sh <lib dir>...  (relative to open3d-ml_amd/); SHAPES as gemm_probe.py
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib"
    O3DML_AMD_LIB=$PWD/open3d-ml_amd/$lib/libo3dml_amd.so timeout -k 10 200 python3 tools/gemm_probe.py 2>/dev/null | grep cin || exit 1
  done
done
