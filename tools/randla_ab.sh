#!/bin/bash
# RandLA-Net section of bench.py (frames/s on the C2 scans) under environment
# settings, interleaved twice:  bash tools/randla_ab.sh ENV1=a,ENV2=b ENV1=c ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --randla-frames ${FRAMES:-4} --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0"
for rep in 1 2; do
  for cfg in "$@"; do
    echo -n "$cfg (rep $rep): "
    env ${cfg//,/ } timeout -k 10 300 python bench.py $ARGS 2>/dev/null | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())['randlanet']
print('frames/s', d['frames_per_s'], 'ms/frame', d['ms_per_frame'], 'cold', d['cold_frames_per_s'])" || exit 1
  done
done
