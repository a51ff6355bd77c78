#!/bin/bash
# Round-4 session 2: FRS parity, A/B of the query-bin / gather changes, the
# 2^24 single scene, a full default bench line.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/r4s2
timeout -k 10 400 python -u -m pytest tests/test_gpu_frs.py tests/test_gpu_many.py -q -x --timeout 150 --timeout-method thread \
    > gpurun_out/r4s2/frs_tests.log 2>&1 || { tail -30 gpurun_out/r4s2/frs_tests.log; exit 1; }
tail -1 gpurun_out/r4s2/frs_tests.log
bash tools/ab_libs_frs.sh lib lib_oldbins || exit 1
for e in "O3DML_FRS_QGATHER=0" "O3DML_FRS_QGATHER=1" "O3DML_FRS_QGATHER=0" "O3DML_FRS_QGATHER=1"; do
  echo "$e $(env $e timeout -k 10 120 python tools/frs_big_time.py 24 7)" || exit 1
done
echo "22: $(timeout -k 10 120 python tools/frs_big_time.py 22 9)" || exit 1
timeout -k 10 500 python bench.py > gpurun_out/r4s2/bench.log 2>&1 || { tail -5 gpurun_out/r4s2/bench.log; exit 1; }
tail -1 gpurun_out/r4s2/bench.log | cut -c1-400
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r4s2/bench.log").read().strip().splitlines()[-1])
print("randla", d.get("randlanet", {}).get("frames_per_s"), "kpconv", d.get("kpconv", {}).get("ms_per_step"),
      "pp", d.get("pointpillars", {}).get("ms_per_step"), "scn", d.get("sparse_conv", {}).get("unet"),
      "sweep", {k: v["Mpoints_s"] for k, v in d.get("c1_sweep", {}).items()}, "cpu", d.get("cpu_baseline"))
PY
exit 0
