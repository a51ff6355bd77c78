#!/bin/bash
# Small-call overhead of one C1 scene (2^16 points): wall time + cProfile
# split, then a kernel trace of 20 calls and the per-call timeline.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
D=$R/gpurun_out/${TAG:-c1small}
mkdir -p "$D"
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/frs_host_overhead.py 65536 > "$D/host.log" 2>&1 || { echo "host rc=$?"; tail -5 "$D/host.log"; exit 1; }
head -3 "$D/host.log"
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d "$D/trace" -o run --output-format csv \
    -- python3 "$R/tools/frs_single.py" 16 20 > "$D/trace.log" 2>&1 || { echo "trace rc=$?"; exit 1; }
f=$(ls "$D"/trace/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find "$D/trace" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/step_timeline.py" "$f" "frs_group_kernel<1, false, false, 0" 15 | tee "$D/timeline.txt"
