#!/bin/bash
# Round-4 session 26: host trims (to_dev fast path for resident tensors, cached
# sparse-conv workspace sizes): GPU suite, SCN frames, C1 sweep.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r4s26
O=gpurun_out/r4s26
( while true; do sleep 45; echo "[hb] $(date +%T)"; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread \
    > $O/pytest.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|Error|assert" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  timeout -k 10 120 python tools/scn_frames.py 30 > $O/scn.log 2>&1 || { tail -5 $O/scn.log; exit 1; }
  grep 'SCN frame' $O/scn.log
done
A="--steps 5 --warmup 2 --no-cpu-baseline --randla-frames 0 --kpconv-steps 3 --pointpillars-steps 0 --sparse-conv-reps 5"
timeout -k 10 400 python bench.py $A > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);print(d['value'], d['sparse_conv']['unet'], d['kpconv']['ms_per_step'], {k:v['ms'] for k,v in d['c1_sweep'].items()})"
echo done
