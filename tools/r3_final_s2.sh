#!/bin/bash
# Round-3 end evidence (second session): the -m gpu suite, smoke, the default
# bench line, a kernel trace + stats of the FRS-only bench (step timeline),
# and the collate probe.  Stops at the first step that crashes or times out.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r3fin}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_gpu.log"; [ $rc -le 1 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke rc=$?"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/full_bench.log" 2>&1 || { echo "bench rc=$?"; tail -5 "$OUT/full_bench.log"; exit 1; }
tail -1 "$OUT/full_bench.log" | cut -c1-160
BARGS="--steps 10 --warmup 3 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv \
    -- python3 "$R/bench.py" $BARGS > "$OUT/stats.log" 2>&1) || { echo "stats rc=$?"; exit 1; }
f=$(find "$OUT/stats" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/step_timeline.py" "$f" "frs_group_kernel<1, false, false, 0" 6 > "$OUT/frs_step_timeline.txt"
tail -1 "$OUT/frs_step_timeline.txt"
PROFILE=0 timeout -k 10 200 python -u tools/collate_probe.py 2>/dev/null | grep "ms per" > "$OUT/collate.txt"; cat "$OUT/collate.txt"
