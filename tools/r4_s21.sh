#!/bin/bash
# Round-4 session 21: sparse-conv GEMM map tiles loaded with every load in
# flight: sparse-conv / SCN tests, GEMM probe, SCN frames, bench sparse_conv leg.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s21
O=gpurun_out/r4s21
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -k "sparse or scn or unet or c4 or gemm" \
    > $O/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
SHAPES=32x32,64x64,128x128,64x32 timeout -k 10 200 python3 tools/gemm_probe.py > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
grep cin $O/probe.log
for i in 1 2 3; do
  timeout -k 10 120 python tools/scn_frames.py 20 > $O/scn.log 2>&1 || { tail -5 $O/scn.log; exit 1; }
  grep 'SCN frame' $O/scn.log
done
A="--steps 2 --warmup 1 --scenes 4 --no-cpu-baseline --randla-frames 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0"
timeout -k 10 300 python bench.py $A > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);s=d['sparse_conv'];print(s['ms_gemm'], s['unet'], json.dumps(s['mfma_roofline'])[:700])"
echo done
