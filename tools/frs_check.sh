#!/bin/bash
# FRS parity tests + two FRS-only bench lines (value, ms/step, kernel ms).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -m pytest tests/test_gpu_frs.py tests/test_gpu_golden.py tests/test_gpu_sparse_conv.py -q -x --timeout 120 --timeout-method thread 2>&1 | tail -2
[ ${PIPESTATUS[0]} -le 1 ] || exit 1
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 \
      --pointpillars-steps 0 --sweep-reps 0 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_all'])" || exit 1
done
