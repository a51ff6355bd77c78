#!/bin/bash
# Round-end GPU session: full GPU test suite, smoke, default bench line, the
# sparse-conv GEMM probe under rocprofv3 kernel-trace --stats, and the
# SparseConvUnet eval / training step times (exact f32 vs default products).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out/${TAG:-final}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { echo "pytest rc=$?"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke rc=$?"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/full_bench.log" 2>&1 || { echo "bench rc=$?"; tail -5 "$OUT/full_bench.log"; exit 1; }
tail -1 "$OUT/full_bench.log" | cut -c1-200
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/gemm" -o run --output-format csv \
    -- python3 "$R/tools/gemm_probe.py" > "$OUT/gemm_probe.log" 2>&1) || { echo "probe rc=$?"; exit 1; }
grep cin "$OUT/gemm_probe.log"
for ex in 0 1; do
  for tr in 0 1; do
    O3DML_SPARSE_CONV_EXACT=$ex TRAIN=$tr timeout -k 10 200 python tools/scn_probe.py > "$OUT/scn_${ex}_${tr}.log" 2>&1 \
        || { echo "scn rc=$?"; exit 1; }
    echo "exact=$ex $(grep ms/frame "$OUT/scn_${ex}_${tr}.log")"
  done
done
