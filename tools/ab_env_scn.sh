#!/bin/bash
# SparseConvUnet eval ms/frame per environment setting, interleaved twice in
# one box session: ab_env_scn.sh "VAR=a" "VAR=b" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for e in "$@"; do
    echo "== $e $(env $e REPS=10 timeout -k 10 200 python3 tools/scn_probe.py 2>/dev/null | grep ms/frame)" || exit 1
  done
done
