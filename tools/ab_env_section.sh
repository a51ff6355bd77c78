#!/bin/bash
# A/B one bench.py section across environment settings in ONE box session:
# ab_env_section.sh <randla|kpconv|pp|sc> "VAR=a" "VAR=b" ...  (each twice, interleaved)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
sec=$1; shift
case "$sec" in
  randla) A="--randla-frames 4"; K=randlanet; F=ms_per_frame;;
  kpconv) A="--kpconv-steps 10"; K=kpconv; F=ms_per_step;;
  pp) A="--pointpillars-steps 10"; K=pointpillars; F=ms_per_step;;
  sc) A="--sparse-conv-reps 20"; K=sparse_conv; F=ms_layer;;
esac
B="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0"
for rep in 1 2; do
  for e in "$@"; do
    env $e timeout -k 10 300 python bench.py $B $A 2>/dev/null | \
      python3 -c "import json,sys; d=json.load(sys.stdin)['$K']; print('$sec $e', d['$F'])" || exit 1
  done
done
