#!/bin/bash
# Round-end evidence: FRS profile + PMC passes (round_profile.sh), the full bench line,
# and the sparse-conv GEMM probe under rocprofv3 kernel-trace -> gpurun_out/r02s4/
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r02s4 bash tools/round_profile.sh || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r02s4/full_bench.log 2>&1 || { echo "bench rc=$?"; exit 1; }
tail -1 gpurun_out/r02s4/full_bench.log | cut -c1-300
R=$(pwd); export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r02s4/sc" -o run --output-format csv \
    -- python3 "$R/tools/gemm_probe.py" > "$R/gpurun_out/r02s4/gemm_probe.log" 2>&1) || { echo "probe rc=$?"; exit 1; }
grep cin gpurun_out/r02s4/gemm_probe.log
