#!/bin/bash
# C1 FRS bench line (bench.py, FRS only) under environment settings,
# interleaved twice:  bash tools/frs_ab.sh ENV1=a,ENV2=b ENV1=c ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0"
for rep in 1 2; do
  for cfg in "$@"; do
    echo -n "$cfg (rep $rep): "
    env ${cfg//,/ } timeout -k 10 300 python bench.py $ARGS 2>/dev/null | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
r = d['roofline']
print('Mpts/s', d['value'], 'ms/step', d['ms_per_step'], 'kernels', r.get('kernel_ms_all'))" || exit 1
  done
done
