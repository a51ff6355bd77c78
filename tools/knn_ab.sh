#!/bin/bash
# Batched kNN probe A/B over environment settings, interleaved twice:
#   bash tools/knn_ab.sh ENV1=a,ENV2=b ENV1=c ...   (a comma joins the settings of one configuration)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for cfg in "$@"; do
    echo "== $cfg (rep $rep)"
    env ${cfg//,/ } timeout -k 10 120 python tools/knn_probe.py 2>&1 | grep -v "^$" | tail -3 || exit 1
  done
done
