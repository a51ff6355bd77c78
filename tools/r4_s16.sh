#!/bin/bash
# Round-4 session 16: RandLA frames/s vs the dense split-K plan.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s16
A="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0"
for rep in 1 2; do
  for e in "X=1" "O3DML_DENSE_TARGET=256" "O3DML_DENSE_TARGET=512" "O3DML_DENSE_MIN_CHUNKS=4" "O3DML_DENSE_MIN_CHUNKS=8"; do
    env $e timeout -k 10 200 python bench.py $A > gpurun_out/r4s16/rl.log 2>&1 || { tail -5 gpurun_out/r4s16/rl.log; exit 1; }
    echo "$e $(python3 -c "import json;d=json.loads(open('gpurun_out/r4s16/rl.log').read().strip().splitlines()[-1]);print(d['randlanet']['frames_per_s'])")"
  done
done
