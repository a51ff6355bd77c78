#!/bin/bash
# Round profile: bench line + rocprofv3 kernel stats of the same command + PMC
# HBM passes (FETCH_SIZE and WRITE_SIZE in separate passes, kernel-trace only)
# -> gpurun_out/$TAG/.  Copy the summaries into profiles/<round>/ afterwards
# (tools/pmc_traffic.py writes the traffic JSON bench.py reads).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOTDIR=$(pwd)
OUT=$ROOTDIR/gpurun_out/${TAG:-prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
BARGS_X="--no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0"
BARGS="--steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0"
timeout -k 10 300 python bench.py $BARGS > "$OUT/bench.log" 2>&1 || { echo "bench rc=$?"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-200
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv \
    -- python3 "$ROOTDIR/bench.py" $BARGS > "$OUT/stats.log" 2>&1) || { echo "stats rc=$?"; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run --output-format csv \
      -- python3 "$ROOTDIR/bench.py" --steps 2 --warmup 1 $BARGS_X > "$OUT/p$i.log" 2>&1) \
      || { echo "pmc pass $i rc=$?"; exit 1; }
  echo "pmc pass $i ok"
done
