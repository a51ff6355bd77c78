#!/bin/bash
# Round-4 session 10: radix tile A/B (lib vs lib_rs16) on the FRS bench line,
# SCN frames and the C3 step, interleaved; the RandLA section and the 2^24
# single scene (u32 temp rows) under rocprofv3 (stats + HBM PMC passes).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); export TMPDIR=/tmp; OUT=$R/gpurun_out/r4s10; mkdir -p $OUT
( while true; do sleep 45; echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
A="--steps 1 --warmup 1 --scenes 1 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --pointpillars-steps 0 --sweep-reps 0 --kpconv-steps 10"
for rep in 1 2 3; do
  for lib in lib lib_rs16; do
    L=$R/open3d-ml_amd/$lib/libo3dml_amd.so
    f=$(O3DML_AMD_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_ms_all'])") || exit 1
    s=$(O3DML_AMD_LIB=$L timeout -k 10 120 python tools/scn_frames.py 20) || exit 1
    k=$(O3DML_AMD_LIB=$L timeout -k 10 200 python bench.py $A 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['kpconv']['ms_per_step'])") || exit 1
    echo "$lib | frs $f | $s | c3 $k"
  done
done
for m in 0 2; do
  (cd /tmp && O3DML_BN_FINALIZE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/bn$m" -o run --output-format csv \
      -- python3 "$R/bench.py" $A > "$OUT/bn$m.log" 2>&1) || { echo "bn$m prof rc=$?"; exit 1; }
  f=$(find $OUT/bn$m -name '*kernel_trace.csv' | head -1)
  echo "BN_FINALIZE=$m: $(python3 tools/trace_window_stats.py $f nll_loss_forward 5 60 | grep -E 'window|bn_' | tr -s ' ' | tr '\n' ';')"
done
SECTION=randla TAG=r4s10 bash tools/prof_section.sh || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/single24" -o run --output-format csv \
    -- python3 "$R/tools/frs_single.py" 24 5 > "$OUT/single24.log" 2>&1) || { echo "single24 rc=$?"; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/single24_p$i" -o run --output-format csv \
      -- python3 "$R/tools/frs_single.py" 24 2 > "$OUT/single24_p$i.log" 2>&1) || { echo "single24 pmc $i rc=$?"; exit 1; }
  echo "single24 pmc pass $i ok"
done
echo "all done"
