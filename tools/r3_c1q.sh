#!/bin/bash
# C1 small-call A/B over the queries per wave of the FRS search (O3DML_FRS_QLOG)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/${TAG:-c1q}
mkdir -p "$D"
for q in 6 5 4; do
  O3DML_FRS_QLOG=$q timeout -k 10 120 python3 -u tools/frs_host_overhead.py 65536 > "$D/q$q.log" 2>&1 || { echo "q $q rc=$?"; exit 1; }
  echo "qlog=$q $(grep 'ms per call' $D/q$q.log)"
done
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 20 > "$D/bench.log" 2>&1 || exit 1
python3 - "$D/bench.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("value", d["value"], "ms_per_step", d["ms_per_step"])
for k, v in d.get("c1_sweep", {}).items():
    print(k, v)
PY
