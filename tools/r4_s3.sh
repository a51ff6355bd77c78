#!/bin/bash
# Round-4 session 3: RandLA frames/s spread and its kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/r4s3
A="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0"
for i in 1 2; do
  timeout -k 10 200 python bench.py $A --randla-frames 6 > gpurun_out/r4s3/rl$i.log 2>&1 || { tail -5 gpurun_out/r4s3/rl$i.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r4s3/rl$i.log').read().strip().splitlines()[-1]);print(d['randlanet'])"
done
SECTION=randla TAG=r4s3 bash tools/prof_section.sh || exit 1
f=$(find gpurun_out/r4s3/randla -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py "$f" 40 > gpurun_out/r4s3/randla_top.txt
cat gpurun_out/r4s3/randla_top.txt
