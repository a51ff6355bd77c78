#!/bin/bash
# Sparse-conv GEMM check on the GPU box: sparse-conv / SCN GPU tests, then the
# GEMM probe under rocprofv3 kernel-trace -> gpurun_out/$TAG/
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-sc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_conv.py tests/test_gpu_scn.py -x -q --timeout 120 \
    --timeout-method thread > "$OUT/t.log" 2>&1 || { tail -30 "$OUT/t.log"; exit 1; }
tail -1 "$OUT/t.log"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/s" -o run --output-format csv \
    -- python3 "$R/tools/gemm_probe.py" > "$OUT/probe.log" 2>&1 || { tail -20 "$OUT/probe.log"; exit 1; }
grep cin "$OUT/probe.log"
python3 "$R/tools/gemm_shapes.py" "$OUT/s/run_kernel_trace.csv"
