#!/bin/bash
# Round-4 session 29: filter split restricted to cin 32: full GPU suite, smoke, default bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s29
O=gpurun_out/r4s29
( while true; do sleep 45; echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { grep -E "^(FAILED|ERROR)|passed|failed" $O/pytest_gpu.log | tail -20; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py > $O/full_bench.log 2>&1 || { tail -5 $O/full_bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/full_bench.log').read().strip().splitlines()[-1]);s=d['sparse_conv'];print(d['value'], d['roofline']['frac'], s['unet']['ms_per_frame'], [(m['channels'],m['products'],m['kernel_us'],m['frac']) for m in s['mfma_roofline']], d['kpconv']['ms_per_step'], d['pointpillars']['ms_per_step'], d['randlanet']['frames_per_s'])"
