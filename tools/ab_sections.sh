#!/bin/bash
# ab_sections.sh DIR1 DIR2 ... : bench.py model sections (no FRS timing, no CPU baseline) from each repo
# checkout (a git worktree inside the tree, e.g. ab_r1, or "." for this one), alternating, twice.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOTD=$(pwd)
mkdir -p gpurun_out/absec
for rep in 1 2; do
  for d in "$@"; do
    (cd "$ROOTD/$d" && timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --scenes 4 \
        > "$ROOTD/gpurun_out/absec/$(basename $d)_$rep.log" 2>&1) || exit $?
    python3 -c "
import json;d=json.loads(open('$ROOTD/gpurun_out/absec/$(basename $d)_$rep.log').read().strip().splitlines()[-1])
print('$d', 'randla fps', d['randlanet']['frames_per_s'], 'kpconv ms', d['kpconv']['ms_per_step'], 'pp ms', d['pointpillars']['ms_per_step'], 'unet ms', d['sparse_conv']['unet']['ms_per_frame'])"
  done
done
