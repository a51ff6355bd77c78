#!/bin/bash
# Round-4 session 22: sparse-conv GEMM workgroup size A/B (O3DML_GEMM_THREADS
# 256 / 128 / 64 builds): GEMM probe, SCN frames, sparse tests on the winner.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s22
O=gpurun_out/r4s22
export SHAPES=32x32,64x32,64x64,128x128
timeout -k 10 600 bash tools/ab_libs_gemm.sh lib lib_t128 lib_t64 > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
cat $O/ab.log
for lib in lib lib_t64 lib_t128 lib lib_t64 lib_t128; do
  O3DML_AMD_LIB=$PWD/open3d-ml_amd/$lib/libo3dml_amd.so timeout -k 10 120 python tools/scn_frames.py 20 > $O/scn.log 2>&1 || { tail -5 $O/scn.log; exit 1; }
  echo "$lib $(grep 'SCN frame' $O/scn.log)"
done
O3DML_AMD_LIB=$PWD/open3d-ml_amd/lib_t64/libo3dml_amd.so timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -k "sparse or scn or unet or c4" \
    > $O/tests64.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" $O/tests64.log | head -30; exit 1; }
tail -1 $O/tests64.log
echo done
