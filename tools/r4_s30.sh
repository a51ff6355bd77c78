#!/bin/bash
# Round-4 session 30: SparseConvUnet frames vs the split-K wave target (fewer
# split-K reduce launches on the host-bound frame), interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s30
O=gpurun_out/r4s30
for rep in 1 2; do
  for t in 4096 2048 1024 512; do
    O3DML_GEMM_TARGET_WAVES=$t timeout -k 10 120 python tools/scn_frames.py 30 > $O/scn.log 2>&1 || { tail -5 $O/scn.log; exit 1; }
    echo "target $t $(grep 'SCN frame' $O/scn.log)"
  done
done
