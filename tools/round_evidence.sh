#!/bin/bash
# Round evidence session (TAG=name): full GPU suite, smoke, default bench line, FRS
# kernel stats + PMC (tools/round_profile.sh), the C3 / C5 / RandLA sections
# and SparseConvUnet frames under rocprofv3 --kernel-trace --stats, the 2^24-point single scene stats
# and its HBM PMC passes (u32 temp rows).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); T=${TAG:-rfin}; OUT=$R/gpurun_out/$T; mkdir -p "$OUT"; export TMPDIR=/tmp
( while true; do sleep 45; echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { echo "pytest rc=$?"; grep -E "^(FAILED|ERROR)|passed|failed" "$OUT/pytest_gpu.log" | tail -20; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke rc=$?"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 500 python bench.py > "$OUT/full_bench.log" 2>&1 || { echo "bench rc=$?"; tail -5 "$OUT/full_bench.log"; exit 1; }
tail -1 "$OUT/full_bench.log" | cut -c1-300
TAG=$T/frs bash tools/round_profile.sh || exit 1
for s in kpconv pp randla; do SECTION=$s TAG=$T bash tools/prof_section.sh || exit 1; done
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/scn" -o run --output-format csv \
    -- python3 "$R/tools/scn_frames.py" 10 > "$OUT/scn.log" 2>&1) || { echo "scn rc=$?"; exit 1; }
grep "SCN frame" "$OUT/scn.log"
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
