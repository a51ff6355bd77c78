#!/bin/bash
# Round-4 session 28: filters split once per call for the narrow GEMM (BS):
# bitwise test, sparse/SCN tests, GEMM probe on vs off, bench sparse_conv leg.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s28
O=gpurun_out/r4s28
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -k "sparse or scn or unet or c4 or gemm" \
    > $O/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
export SHAPES=32x32,64x32,32x16
timeout -k 10 500 bash tools/ab_env_gemm.sh O3DML_GEMM_BSPLIT=1 O3DML_GEMM_BSPLIT=0 > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
cat $O/ab.log
A="--steps 2 --warmup 1 --scenes 4 --no-cpu-baseline --randla-frames 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0"
for b in 1 0; do
  O3DML_GEMM_BSPLIT=$b timeout -k 10 300 python bench.py $A > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);s=d['sparse_conv'];print('bsplit $b', s['ms_gemm'], s['unet']['ms_per_frame'], [(m['channels'],m['products'],m['kernel_us'],m['frac']) for m in s['mfma_roofline']])"
done
echo done
