#!/bin/bash
# Whole bench.py (no CPU legs, no sweep) under environment settings, interleaved
# twice, one summary line per run:  bash tools/bench_ab.sh ENV1=a,ENV2=b ENV1=c ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGS="--no-cpu-baseline --sweep-reps 0 ${BENCH_ARGS:-}"
for rep in 1 2; do
  for cfg in "$@"; do
    echo -n "$cfg (rep $rep): "
    env ${cfg//,/ } timeout -k 10 400 python bench.py $ARGS 2>/dev/null | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
g = lambda *k: (lambda v: [v := v.get(x, {}) if isinstance(v, dict) else None for x in k][-1])(d)
print('C1', d['value'], 'RandLA fps', g('randlanet', 'frames_per_s'), 'SCN ms', g('sparse_conv', 'unet', 'ms_per_frame'),
      'C3 ms', g('kpconv', 'ms_per_step'), 'C5 ms', g('pointpillars', 'ms_per_step'))" || exit 1
  done
done
