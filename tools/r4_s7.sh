#!/bin/bash
# Round-4 session 7: rocBLAS GEMM entry point + one-node KPFCNN ops: parity,
# C3 step (default backend and both torch backends), host split, kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s7
timeout -k 10 600 python -u -m pytest tests/test_gpu_batchnorm.py tests/test_gpu_kpconv.py tests/test_gpu_kpfcnn.py tests/test_gpu_full.py tests/test_gpu_determinism.py -q --timeout 200 --timeout-method thread \
    > gpurun_out/r4s7/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" gpurun_out/r4s7/tests.log | head -40; exit 1; }
tail -1 gpurun_out/r4s7/tests.log
A="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --pointpillars-steps 0 --sweep-reps 0 --kpconv-steps 10"
for e in "X=1" "X=2" "X=3"; do
  env $e timeout -k 10 200 python bench.py $A > gpurun_out/r4s7/kp.log 2>&1 || { tail -5 gpurun_out/r4s7/kp.log; exit 1; }
  echo "$e $(python3 -c "import json;d=json.loads(open('gpurun_out/r4s7/kp.log').read().strip().splitlines()[-1]);k=d['kpconv'];print(k['ms_per_step'], k['ms_collate'])")"
done
timeout -k 10 300 python tools/kp_host.py > gpurun_out/r4s7/kp_host.log 2>&1 && head -3 gpurun_out/r4s7/kp_host.log
SECTION=kpconv TAG=r4s7 bash tools/prof_section.sh || exit 1
f=$(find gpurun_out/r4s7/kpconv -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py "$f" 30 > gpurun_out/r4s7/kpconv_top.txt
head -30 gpurun_out/r4s7/kpconv_top.txt
