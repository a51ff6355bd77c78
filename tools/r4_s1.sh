#!/bin/bash
# Round-4 session 1: parity tests of this round's changes, the FRS cost split
# (DIAG variants), C3 / C5 kernel stats.  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PYTEST_FILES="tests/test_gpu_many.py tests/test_gpu_pipeline.py tests/test_gpu_full.py tests/test_gpu_randla.py tests/test_capi.py tests/test_gpu_pointpillars.py tests/test_torch_ops.py tests/test_gpu_sparse_conv.py tests/test_gpu_frs.py" \
  TAG=r4s1 bash tools/r3_tests.sh || exit $?
bash tools/r4_diag.sh main diag1 diag2 || exit $?
for s in kpconv pp; do SECTION=$s TAG=r4s1 bash tools/prof_section.sh || exit $?; done
for s in kpconv pp; do
  f=$(find gpurun_out/r4s1/$s -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && python3 tools/kstats.py "$f" 30 > gpurun_out/r4s1/${s}_top.txt
done
exit 0
