#!/bin/bash
# FRS-only bench.py line per library build, interleaved, in ONE box session:
# ab_libs_frs.sh <lib dir>... (relative to open3d-ml_amd/)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2 3; do
  for lib in "$@"; do
    O3DML_AMD_LIB=$PWD/open3d-ml_amd/$lib/libo3dml_amd.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 \
      --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0 2>/dev/null | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$lib', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_all'])" || exit 1
  done
done
