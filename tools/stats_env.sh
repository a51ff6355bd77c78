#!/bin/bash
# stats_env.sh TAG "ENV=.. ENV2=.." cmd... : rocprofv3 kernel stats of one command under extra env
# -> gpurun_out/senv/TAG/ and a top-8 kernel summary on stdout
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift; ENVS=$1; shift
export TMPDIR=/tmp
mkdir -p $R/gpurun_out/senv
for kv in $ENVS; do export "$kv"; done
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/senv/$TAG -o run --output-format csv -- "$@" > $R/gpurun_out/senv/$TAG.log 2>&1) || exit 1
f=$(find $R/gpurun_out/senv/$TAG -name "*kernel_stats.csv" | head -1)
python3 - "$f" "$TAG" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(sys.argv[2], "total_ms", round(tot / 1e6, 3))
for r in rows[:8]:
    print("  ", r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), r["Name"][:70])
PY
