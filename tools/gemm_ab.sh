#!/bin/bash
# Sparse-conv GEMM probe A/B over environment settings, interleaved twice:
#   bash tools/gemm_ab.sh ENV1=a,ENV2=b ENV1=c ...   (a comma joins the settings of one
#   configuration; SHAPES / REPS from the caller)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for cfg in "$@"; do
    echo "== $cfg (rep $rep)"
    env ${cfg//,/ } timeout -k 10 120 python tools/gemm_probe.py 2>/dev/null | grep -v "^$" || exit 1
  done
done
