#!/bin/bash
# rocprofv3 kernel stats of the FRS-only bench for each library build (A/B in one session):
# stats_ab.sh lib lib_old ...  -> gpurun_out/sab/<lib>/
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); export TMPDIR=/tmp
mkdir -p $R/gpurun_out/sab
for l in "$@"; do
  (cd /tmp && O3DML_AMD_LIB=$R/open3d-ml_amd/$l/libo3dml_amd.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
     -d $R/gpurun_out/sab/$l -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline \
     --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0 > $R/gpurun_out/sab/$l.log 2>&1) || exit 1
  echo "$l ok"
done
