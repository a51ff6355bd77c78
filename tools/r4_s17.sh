#!/bin/bash
# Round-4 session 17: selection chunking (count / write at 1,024 keys per
# workgroup): radix tests, RandLA tests, frames/s.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s17
timeout -k 10 400 python -u -m pytest tests/test_gpu_many.py tests/test_gpu_randla.py tests/test_gpu_pipeline.py -q --timeout 150 --timeout-method thread \
    > gpurun_out/r4s17/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" gpurun_out/r4s17/tests.log | head -30; exit 1; }
tail -1 gpurun_out/r4s17/tests.log
A="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0"
for i in 1 2 3; do
  timeout -k 10 200 python bench.py $A > gpurun_out/r4s17/rl.log 2>&1 || { tail -5 gpurun_out/r4s17/rl.log; exit 1; }
  echo "randla $(python3 -c "import json;d=json.loads(open('gpurun_out/r4s17/rl.log').read().strip().splitlines()[-1]);print(d['randlanet']['frames_per_s'])")"
done
