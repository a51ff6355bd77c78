#!/bin/bash
# Round-4 session 12: C5 PointPillars step with MIOpen solver search
# (torch.backends.cudnn.benchmark) and find modes; C3 step after the BN tree
# finalize default.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s12
( while true; do sleep 45; echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
A="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 --sweep-reps 0 --pointpillars-steps 10"
for e in "X=1" "O3DML_CUDNN_BENCHMARK=1" "MIOPEN_FIND_MODE=1" "X=1" "O3DML_CUDNN_BENCHMARK=1" "MIOPEN_FIND_MODE=1"; do
  env $e timeout -k 10 300 python bench.py $A > gpurun_out/r4s12/pp.log 2>&1 || { tail -5 gpurun_out/r4s12/pp.log; exit 1; }
  echo "$e pp $(python3 -c "import json;d=json.loads(open('gpurun_out/r4s12/pp.log').read().strip().splitlines()[-1]);print(d['pointpillars']['ms_per_step'])")"
done
A="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --pointpillars-steps 0 --sweep-reps 0"
for i in 1 2 3; do
  timeout -k 10 200 python bench.py $A > gpurun_out/r4s12/kp.log 2>&1 || { tail -5 gpurun_out/r4s12/kp.log; exit 1; }
  echo "c3 $(python3 -c "import json;d=json.loads(open('gpurun_out/r4s12/kp.log').read().strip().splitlines()[-1]);k=d['kpconv'];print(k['ms_per_step'], k['ms_collate'])")"
done
