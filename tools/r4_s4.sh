#!/bin/bash
# Round-4 session 4: multi-workgroup radix selection (crop / k > 2048) parity,
# RandLA frames/s, then the RandLA section under rocprofv3 (kernel stats).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/r4s4
timeout -k 10 400 python -u -m pytest tests/test_gpu_many.py tests/test_gpu_randla.py tests/test_gpu_pipeline.py -q --timeout 150 --timeout-method thread \
    > gpurun_out/r4s4/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" gpurun_out/r4s4/tests.log | head -30; exit 1; }
tail -1 gpurun_out/r4s4/tests.log
A="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0"
timeout -k 10 200 python bench.py $A --randla-frames 6 > gpurun_out/r4s4/rl.log 2>&1 || { tail -5 gpurun_out/r4s4/rl.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r4s4/rl.log').read().strip().splitlines()[-1]);print(d['randlanet'])"
SECTION=randla TAG=r4s4 bash tools/prof_section.sh || { grep -v "^frame\|^W20\|^E20" gpurun_out/r4s4/randla.log | head -20; exit 1; }
f=$(find gpurun_out/r4s4/randla -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py "$f" 40 > gpurun_out/r4s4/randla_top.txt
cat gpurun_out/r4s4/randla_top.txt
