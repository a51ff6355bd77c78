#!/bin/bash
# SparseConvUnet eval frames (tools/scn_frames.py) under environment settings,
# interleaved twice:  bash tools/scn_ab.sh "ENV1=a ENV2=b" "ENV1=c" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for cfg in "$@"; do
    echo -n "$cfg (rep $rep): "
    env $cfg timeout -k 10 120 python tools/scn_frames.py 20 2>/dev/null | grep "SCN frame" || exit 1
  done
done
