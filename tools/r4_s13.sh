#!/bin/bash
# Round-4 session 13: C5 PointPillars step, NCHW vs channels-last backbone.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s13
( while true; do sleep 45; echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
A="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 --sweep-reps 0 --pointpillars-steps 10"
for e in 0 1 0 1; do
  O3DML_PP_NHWC=$e timeout -k 10 300 python bench.py $A > gpurun_out/r4s13/pp.log 2>&1 || { tail -5 gpurun_out/r4s13/pp.log; exit 1; }
  echo "NHWC=$e pp $(python3 -c "import json;d=json.loads(open('gpurun_out/r4s13/pp.log').read().strip().splitlines()[-1]);print(d['pointpillars']['ms_per_step'])")"
done
