#!/bin/bash
# SparseConvUnet eval forward on the C4 room: wall ms/frame, torch profiler
# table, and rocprofv3 kernel stats + trace (REPS frames after a warm-up)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
D=$R/gpurun_out/${TAG:-scn}
mkdir -p "$D"
export TMPDIR=/tmp
TORCHPROF=1 REPS=5 timeout -k 10 200 python3 -u tools/scn_probe.py > "$D/probe.log" 2>&1 || { echo "probe rc=$?"; tail -5 "$D/probe.log"; exit 1; }
grep "ms/frame" "$D/probe.log"
cd /tmp && REPS=5 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$D/prof" -o run --output-format csv \
    -- python3 "$R/tools/scn_probe.py" > "$D/prof.log" 2>&1
echo "prof rc=$?"
