#!/bin/bash
# PMC passes over tools/knn_probe.py (k=16 self kNN on RandLA patch sizes) ->
# gpurun_out/$TAG/p*/ ; summary: tools/pmc_summary.py gpurun_out/$TAG knn_group
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out/${TAG:-pmck}; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run --output-format csv \
      -- python3 "$R/tools/knn_probe.py" > "$OUT/p$i.log" 2>&1) || { echo "pass $i rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
python3 "$R/tools/pmc_summary.py" "$OUT" "knn_group_kernel<16"
