#!/bin/bash
# Sparse-conv GEMM A/B of the product precisions: bf16x6 (default), exact f32
# MFMA (O3DML_SPARSE_CONV_EXACT=1), bf16x3 (=2): sparse-conv tests, then the GEMM probe under
# rocprofv3 kernel-trace for each -> gpurun_out/$TAG/{x6,f32,x3}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-scab}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_conv.py -x -q --timeout 120 \
    --timeout-method thread > "$OUT/t.log" 2>&1 || { tail -30 "$OUT/t.log"; exit 1; }
tail -1 "$OUT/t.log"
for v in ${MODES:-x6 f32 x3}; do
  ex=0; [ $v = f32 ] && ex=1; [ $v = x3 ] && ex=2
  (cd /tmp && O3DML_SPARSE_CONV_EXACT=$ex timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o run \
      --output-format csv -- python3 "$R/tools/gemm_probe.py" > "$OUT/probe_$v.log" 2>&1) \
      || { tail -20 "$OUT/probe_$v.log"; exit 1; }
  echo "== $v"; grep cin "$OUT/probe_$v.log"
  python3 "$R/tools/gemm_shapes.py" "$OUT/$v/run_kernel_trace.csv"
done
