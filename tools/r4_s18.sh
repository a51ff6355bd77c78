#!/bin/bash
# Round-4 session 18: one-workgroup LSD radix sort (o3dml_sort_pairs tests, the
# GPU suite) and SparseConvUnet frames, radix vs bitonic small sorts.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s18
O=gpurun_out/r4s18
timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py -x -q --timeout 120 --timeout-method thread \
    > $O/sort.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" $O/sort.log | head -30; exit 1; }
tail -1 $O/sort.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
    > $O/pytest.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
for k in 1 0 1 0; do
  O3DML_BS_KIND=$k timeout -k 10 120 python tools/scn_frames.py 20 > $O/scn_$k.log 2>&1 || { tail -5 $O/scn_$k.log; exit 1; }
  echo "kind $k $(grep 'SCN frame' $O/scn_$k.log)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/scn -o run -- python3 tools/scn_frames.py 10 > $O/scn_prof.log 2>&1 || { tail -5 $O/scn_prof.log; exit 1; }
echo done
