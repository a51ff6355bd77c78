#!/bin/bash
# Sparse-conv GEMM probe with the presplit operands on / off (A/B) ->
# gpurun_out/$TAG/gemm_{on,off}.log, then rocprofv3 kernel stats of the
# presplit run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
D=$R/gpurun_out/${TAG:-gemm}
mkdir -p "$D"
export TMPDIR=/tmp
for on in 1 0; do
  O3DML_GEMM_PRESPLIT=$on timeout -k 10 180 python3 -u tools/gemm_probe.py > "$D/gemm_$on.log" 2>&1 || { echo "probe $on rc=$?"; tail -5 "$D/gemm_$on.log"; exit 1; }
  echo "presplit=$on"; cat "$D/gemm_$on.log"
done
cd /tmp && REPS=5 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$D/prof" -o run --output-format csv \
    -- python3 "$R/tools/gemm_probe.py" > "$D/prof.log" 2>&1
echo "prof rc=$?"
