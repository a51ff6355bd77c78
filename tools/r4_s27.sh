#!/bin/bash
# Round-4 session 27: padded exchange buffers in the one-workgroup radix sort:
# sort + SCN tests, SCN frames, sort kernel times under the kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s27
O=gpurun_out/r4s27; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_sort.py tests -m gpu -q --timeout 150 --timeout-method thread -k "sort or scn or unet or c4 or grid or voxel" \
    > $O/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 120 python tools/scn_frames.py 30 > $O/scn.log 2>&1 || { tail -5 $O/scn.log; exit 1; }
  grep 'SCN frame' $O/scn.log
done
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/scn" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/tools/scn_frames.py" 10 > "$GRAFT_REPO_ROOT/$O/scn_prof.log" 2>&1) || { echo "prof failed"; exit 1; }
rm -f $O/scn/run_kernel_trace.csv
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/r4s27/scn/run_kernel_stats.csv')):
    if 'block_radix' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:8.1f} us x {r['Calls']}  {r['Name'][:70]}")
PY
echo done
