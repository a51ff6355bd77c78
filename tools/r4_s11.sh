#!/bin/bash
# Round-4 session 11: one-call KPFCNN layer ops (csrc/kpfcnn_ops.cpp): parity,
# C3 step, host split.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s11
timeout -k 10 600 python -u -m pytest tests/test_gpu_batchnorm.py tests/test_gpu_kpconv.py tests/test_gpu_kpfcnn.py tests/test_gpu_full.py tests/test_gpu_determinism.py -q --timeout 200 --timeout-method thread \
    > gpurun_out/r4s11/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" gpurun_out/r4s11/tests.log | head -40; exit 1; }
tail -1 gpurun_out/r4s11/tests.log
A="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --pointpillars-steps 0 --sweep-reps 0"
for i in 1 2 3; do
  timeout -k 10 200 python bench.py $A > gpurun_out/r4s11/kp.log 2>&1 || { tail -5 gpurun_out/r4s11/kp.log; exit 1; }
  echo "c3 $(python3 -c "import json;d=json.loads(open('gpurun_out/r4s11/kp.log').read().strip().splitlines()[-1]);k=d['kpconv'];print(k['ms_per_step'], k['ms_collate'])")"
done
timeout -k 10 300 python tools/kp_host.py > gpurun_out/r4s11/kp_host.log 2>&1 && head -3 gpurun_out/r4s11/kp_host.log
