#!/bin/bash
# Round-4 session 5: fused BN + LeakyReLU and MFMA KPConv aggregation —
# parity (BN vs torch, MFMA vs wave kernels, KPFCNN / C3 vs reference), the
# C3 step time, its kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/r4s5
timeout -k 10 600 python -u -m pytest tests/test_gpu_batchnorm.py tests/test_gpu_kpconv.py tests/test_gpu_kpfcnn.py tests/test_gpu_full.py tests/test_gpu_determinism.py -q --timeout 200 --timeout-method thread \
    > gpurun_out/r4s5/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" gpurun_out/r4s5/tests.log | head -40; exit 1; }
tail -1 gpurun_out/r4s5/tests.log
A="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --pointpillars-steps 0 --sweep-reps 0"
for i in 1 2; do
  timeout -k 10 200 python bench.py $A --kpconv-steps 10 > gpurun_out/r4s5/kp$i.log 2>&1 || { tail -5 gpurun_out/r4s5/kp$i.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r4s5/kp$i.log').read().strip().splitlines()[-1]);print(d['kpconv'])"
done
SECTION=kpconv TAG=r4s5 bash tools/prof_section.sh || { grep -v "^frame\|^W20\|^E20" gpurun_out/r4s5/kpconv.log | head -20; exit 1; }
f=$(find gpurun_out/r4s5/kpconv -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py "$f" 40 > gpurun_out/r4s5/kpconv_top.txt
cat gpurun_out/r4s5/kpconv_top.txt
