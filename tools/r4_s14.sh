#!/bin/bash
# Round-4 session 14: the default bench.py line (all sections) twice.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s14
( while true; do sleep 45; echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
for i in 1 2; do
  timeout -k 10 500 python bench.py > gpurun_out/r4s14/bench$i.log 2>&1 || { tail -5 gpurun_out/r4s14/bench$i.log; exit 1; }
  python3 - $i <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r4s14/bench{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(d["value"], d["roofline"]["frac"], "randla", d["randlanet"]["frames_per_s"], "kpconv", d["kpconv"]["ms_per_step"],
      "pp", d["pointpillars"]["ms_per_step"], "scn", d["sparse_conv"]["unet"]["ms_per_frame"],
      "sweep24", d["c1_sweep"]["16777216"]["Mpoints_s"], "cpu", d["cpu_baseline"]["value"])
PY
done
