#!/bin/bash
# run_variants.sh v1 v2 ... : FRS-only bench.py line with each open3d-ml_amd/lib_<v>/ build
# ("main" = the in-tree open3d-ml_amd/lib build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/variants
for v in "$@"; do
  if [ "$v" = main ]; then LIBV=$PWD/open3d-ml_amd/lib/libo3dml_amd.so; else LIBV=$PWD/open3d-ml_amd/lib_$v/libo3dml_amd.so; fi
  O3DML_AMD_LIB=$LIBV timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0 > gpurun_out/variants/$v.log 2>&1 || exit $?
  python -c "import json,sys;d=json.loads(open('gpurun_out/variants/$v.log').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d['roofline']['kernel_ms_all'])"
done
