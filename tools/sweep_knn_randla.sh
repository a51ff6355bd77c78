#!/bin/bash
# kNN grid density (O3DML_KNN_TARGET) sweep: kNN probe per size, then the
# RandLA-Net bench section per setting (interleaved, one box session).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/swr
for t in ${TARGETS:-0.125 0.25 0.5}; do
  O3DML_KNN_TARGET=$t timeout -k 10 120 python tools/knn_probe.py > gpurun_out/swr/knn_$t.log 2>&1 || exit 1
  echo "target $t: $(tail -1 gpurun_out/swr/knn_$t.log)"
done
B="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --randla-frames 4 --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0"
for rep in 1 2; do
  for t in ${TARGETS:-0.125 0.25 0.5}; do
    O3DML_KNN_TARGET=$t timeout -k 10 300 python bench.py $B 2>/dev/null | \
      python3 -c "import json,sys; d=json.load(sys.stdin)['randlanet']; print('target $t', d['ms_per_frame'])" || exit 1
  done
done
