#!/bin/bash
# Round-4 session 1b: FRS parity of every variant build, the FRS cost split and
# A/B (DIAG and micro-opt variants), C3 / C5 kernel stats, the 2^24-point
# single-scene stats.  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); export TMPDIR=/tmp
VARS="${VARS:-main nodpp oob dma dma3}"
for v in $VARS; do
  if [ "$v" = main ]; then L=$R/open3d-ml_amd/lib/libo3dml_amd.so; else L=$R/open3d-ml_amd/lib_$v/libo3dml_amd.so; fi
  O3DML_AMD_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_frs.py -q -x --timeout 120 --timeout-method thread \
      -k "self_search or c1_config or bench_batch or voxel_classes or group_sizes or overflow or one_call" > gpurun_out/r4s1b_frs_$v.log 2>&1 \
      || { echo "parity FAILED for $v"; tail -20 gpurun_out/r4s1b_frs_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r4s1b_frs_$v.log)"
done
bash tools/r4_diag.sh $VARS diag1 diag2 || exit $?
[ -n "$NOPROF" ] && exit 0
for s in kpconv pp; do SECTION=$s TAG=r4s1 bash tools/prof_section.sh || exit $?; done
for s in kpconv pp; do
  f=$(find gpurun_out/r4s1/$s -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && python3 tools/kstats.py "$f" 30 > gpurun_out/r4s1/${s}_top.txt
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r4s1/single24" -o run --output-format csv \
    -- python3 "$R/tools/frs_single.py" 24 5 > "$R/gpurun_out/r4s1/single24.log" 2>&1) || exit 1
f=$(find gpurun_out/r4s1/single24 -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py "$f" 25 > gpurun_out/r4s1/single24_top.txt
cat gpurun_out/r4s1/single24_top.txt
bash tools/ab_env_scn.sh "O3DML_BS_MAX=8192" "O3DML_BS_MAX=1024" "O3DML_BS_MAX=0" || exit 1
exit 0
