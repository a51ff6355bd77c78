#!/bin/bash
# A/B the RandLA-Net bench section across environment settings in ONE box
# session: ab_env_randla.sh "VAR=a" "VAR=b" ...  (each twice, interleaved)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
B="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --randla-frames 4 --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0"
for rep in 1 2; do
  for e in "$@"; do
    env $e timeout -k 10 300 python bench.py $B 2>/dev/null | \
      python3 -c "import json,sys; d=json.load(sys.stdin)['randlanet']; print('$e', d['ms_per_frame'])" || exit 1
  done
done
