#!/bin/bash
# Round-4 session 24: SparseConvUnet level grids on a side stream
# (size reads wait only for the grid kernels): SCN tests, frames, kernel trace (stats only kept).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s24
O=gpurun_out/r4s24
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -k "scn or sparse or unet or c4" \
    > $O/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 120 python tools/scn_frames.py 20 > $O/scn.log 2>&1 || { tail -5 $O/scn.log; exit 1; }
  grep 'SCN frame' $O/scn.log
done
timeout -k 10 120 python tools/scn_frames.py 20 prof > $O/scn_cprof.log 2>&1 || { tail -5 $O/scn_cprof.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/scn -o run --output-format csv -- python3 tools/scn_frames.py 10 > $O/scn_prof.log 2>&1 || { tail -5 $O/scn_prof.log; exit 1; }
grep 'SCN frame' $O/scn_prof.log
echo done
