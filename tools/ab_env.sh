#!/bin/bash
# ab_env.sh "ENV=val ..." "ENV=val ..." ... : FRS-only bench.py line per environment setting (in-tree lib)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/abenv
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0 > gpurun_out/abenv/$i.log 2>&1 || exit $?
  python -c "import json,sys;d=json.loads(open('gpurun_out/abenv/$i.log').read().strip().splitlines()[-1]);print('$e',d['value'],d['ms_per_step'],d['roofline']['kernel_ms_all'])"
done
