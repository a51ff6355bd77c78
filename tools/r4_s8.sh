#!/bin/bash
# Round-4 session 8: SparseConvUnet eval frame time and kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/r4s8
timeout -k 10 200 python tools/scn_frames.py 20 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r4s8/scn" -o run --output-format csv \
    -- python3 "$R/tools/scn_frames.py" 10 > "$R/gpurun_out/r4s8/scn.log" 2>&1) || exit 1
f=$(find gpurun_out/r4s8/scn -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py "$f" 40 > gpurun_out/r4s8/scn_top.txt
cat gpurun_out/r4s8/scn_top.txt
