#!/bin/bash
# PMC passes over the sparse-conv GEMM probe (SHAPES, default 128x128) ->
# gpurun_out/$TAG/p*/ ; summarise with tools/pmc_summary.py gpurun_out/$TAG implicit_gemm
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-pmcg}
mkdir -p "$OUT"
export TMPDIR=/tmp SHAPES=${SHAPES:-128x128} REPS=3
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o run --output-format csv \
      -- python3 "$R/tools/gemm_probe.py" > "$OUT/p$i.log" 2>&1) || { echo "pass $i rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok: $grp"
done < "$R/tools/pmc_groups_gemm.txt"
python3 "$R/tools/pmc_summary.py" "$OUT" implicit_gemm
