#!/bin/bash
# rocprofv3 kernel stats of one bench.py section (the FRS part shrunk to one
# scene / one step): SECTION=randla|kpconv|pp|sc  TAG=name -> gpurun_out/$TAG/
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-sec}
mkdir -p "$OUT"
export TMPDIR=/tmp
A="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0"
case "$SECTION" in
  randla) A="$A --randla-frames 3";;
  kpconv) A="$A --kpconv-steps 5";;
  pp) A="$A --pointpillars-steps 5";;
  sc) A="$A --sparse-conv-reps 10";;
esac
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$SECTION" -o run --output-format csv \
    -- python3 "$R/bench.py" $A > "$OUT/$SECTION.log" 2>&1
echo "$SECTION rc=$?"
