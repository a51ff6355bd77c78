#!/bin/bash
# presplit GEMM row-block A/B: O3DML_GEMM_SPLIT_RB = 1, 2, 4 and presplit off
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/${TAG:-gemmrb}
mkdir -p "$D"
for v in 1 2 4; do
  O3DML_GEMM_SPLIT_RB=$v timeout -k 10 180 python3 -u tools/gemm_probe.py > "$D/rb$v.log" 2>&1 || { echo "rb $v rc=$?"; tail -5 "$D/rb$v.log"; exit 1; }
  echo "rb=$v"; grep cin "$D/rb$v.log"
done
O3DML_GEMM_PRESPLIT=0 timeout -k 10 180 python3 -u tools/gemm_probe.py > "$D/off.log" 2>&1 || exit 1
echo "presplit off"; grep cin "$D/off.log"
