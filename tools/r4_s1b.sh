#!/bin/bash
# Round-4 session 1b: the FRS cost split (DIAG variants) and C3 / C5 kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/r4_diag.sh main diag1 diag2 || exit $?
for s in kpconv pp; do SECTION=$s TAG=r4s1 bash tools/prof_section.sh || exit $?; done
for s in kpconv pp; do
  f=$(find gpurun_out/r4s1/$s -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && python3 tools/kstats.py "$f" 30 > gpurun_out/r4s1/${s}_top.txt
done
exit 0
