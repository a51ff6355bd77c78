#!/bin/bash
# sparse-conv GEMM probe per environment setting, interleaved (one box session):
# ab_env_gemm.sh "VAR=a" "VAR=b" ...  (SHAPES as gemm_probe.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for e in "$@"; do
    echo "== $e"
    env $e timeout -k 10 200 python3 tools/gemm_probe.py 2>/dev/null | grep cin || exit 1
  done
done
