#!/bin/bash
# Round-4 session 20: sparse-conv GEMM split-K target A/B at the C4 widths.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s20
export SHAPES=32x32,64x64,128x128
timeout -k 10 500 bash tools/ab_env_gemm.sh O3DML_GEMM_TARGET_WAVES=4096 O3DML_GEMM_TARGET_WAVES=8192 O3DML_GEMM_TARGET_WAVES=16384 O3DML_GEMM_TARGET_WAVES=2048 > gpurun_out/r4s20/ab.log 2>&1 || { tail -5 gpurun_out/r4s20/ab.log; exit 1; }
cat gpurun_out/r4s20/ab.log
