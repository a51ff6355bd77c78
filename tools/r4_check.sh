#!/bin/bash
# Final-tree check: full GPU suite and smoke.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4check
O=gpurun_out/r4check
( while true; do sleep 45; echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest_gpu.log | tail -20; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py > $O/full_bench.log 2>&1 || { tail -5 $O/full_bench.log; exit 1; }
tail -1 $O/full_bench.log | cut -c1-200
