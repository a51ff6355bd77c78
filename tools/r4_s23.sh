#!/bin/bash
# Round-4 session 23: two stages in flight (O3DML_GEMM_DEPTH=2) after the
# map-tile preamble fix, with and without split-K (target waves 2,048 = none at 32->32).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s23
export SHAPES=32x32,64x32
timeout -k 10 600 bash tools/ab_env_gemm.sh "O3DML_GEMM_DEPTH=1" "O3DML_GEMM_DEPTH=2" "O3DML_GEMM_DEPTH=1 O3DML_GEMM_TARGET_WAVES=2048" "O3DML_GEMM_DEPTH=2 O3DML_GEMM_TARGET_WAVES=2048" > gpurun_out/r4s23/ab.log 2>&1 || { tail -5 gpurun_out/r4s23/ab.log; exit 1; }
cat gpurun_out/r4s23/ab.log
