#!/bin/bash
# FRS-only bench.py line per environment setting, interleaved 3x in one box session:
# ab_env_frs.sh "VAR=a" "VAR=b" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2 3; do
  for e in "$@"; do
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --randla-frames 0 --sparse-conv-reps 0 \
      --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0 2>/dev/null | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$e', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_all'])" || exit 1
  done
done
