#!/bin/bash
# Kernel timeline of the C4 32->32 SparseConv layer call (bench sparse_conv
# section, rulebook rebuilt per call) -> gpurun_out/$TAG/
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out/${TAG:-sclayer}; mkdir -p "$OUT"; export TMPDIR=/tmp
(cd /tmp && REPS=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/t" -o run --output-format csv \
    -- python3 "$R/tools/sc_probe.py" > "$OUT/probe.log" 2>&1) || { tail -20 "$OUT/probe.log"; exit 1; }
tail -1 "$OUT/probe.log" | cut -c1-300
