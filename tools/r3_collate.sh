#!/bin/bash
# KPFCNN collate: wall time + cProfile, then a kernel trace of REPS calls
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); D=$R/gpurun_out/${TAG:-collate}; mkdir -p "$D"; export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/collate_probe.py > "$D/probe.log" 2>&1 || { echo "probe rc=$?"; tail -5 "$D/probe.log"; exit 1; }
grep "ms per" "$D/probe.log"
cd /tmp && PROFILE=0 REPS=4 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$D/prof" -o run --output-format csv \
    -- python3 "$R/tools/collate_probe.py" > "$D/prof.log" 2>&1
echo "prof rc=$?"
