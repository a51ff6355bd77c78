#!/bin/bash
# SparseConvUnet eval frames with each product precision of the sparse-conv
# GEMMs (O3DML_SPARSE_CONV_EXACT: 0 bf16x6, 1 exact f32), interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for mode in 0 1; do
    echo -n "mode=$mode rep=$rep "
    O3DML_SPARSE_CONV_EXACT=$mode timeout -k 10 120 python tools/scn_frames.py 20 2>/dev/null | grep "SCN frame" || exit 1
  done
done
