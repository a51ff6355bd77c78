#!/bin/bash
# Round-4 session 25: SparseConvUnet level grids, front vs side stream (same box, interleaved).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s25
O=gpurun_out/r4s25
for m in front side front side front side; do
  O3DML_SCN_GRIDS=$m timeout -k 10 120 python tools/scn_frames.py 30 > $O/scn.log 2>&1 || { tail -5 $O/scn.log; exit 1; }
  echo "$m $(grep 'SCN frame' $O/scn.log)"
done
O3DML_SCN_GRIDS=side timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -k "scn or unet or c4" \
    > $O/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -k "scn or unet or c4" \
    > $O/tests2.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" $O/tests2.log | head -30; exit 1; }
tail -1 $O/tests2.log
