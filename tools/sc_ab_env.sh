#!/bin/bash
# Sparse-conv GEMM A/B over environment switches: sparse-conv + SCN GPU tests,
# then tools/gemm_probe.py under rocprofv3 kernel-trace once per variant.
# VARIANTS="name:VAR=val[,VAR=val] ..." -> gpurun_out/$TAG/<name>/
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-scenv}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_conv.py tests/test_gpu_scn.py -x -q --timeout 120 \
    --timeout-method thread > "$OUT/t.log" 2>&1 || { tail -30 "$OUT/t.log"; exit 1; }
tail -1 "$OUT/t.log"
for v in $VARIANTS; do
  name=${v%%:*}; envs=${v#*:}
  (cd /tmp && env ${envs//,/ } timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run \
      --output-format csv -- python3 "$R/tools/gemm_probe.py" > "$OUT/probe_$name.log" 2>&1) \
      || { tail -20 "$OUT/probe_$name.log"; exit 1; }
  echo "== $name ($envs)"; grep cin "$OUT/probe_$name.log"
  python3 "$R/tools/gemm_shapes.py" "$OUT/$name/run_kernel_trace.csv" | grep -v radix
done
