#!/bin/bash
# Copy a tools/round_evidence.sh session (gpurun_out/$1) into profiles/$2:
# bench line, pytest log, kernel stats of every section, FRS search PMC
# (pmc_frs_group_search.json, read by bench.py), 2^24 scene PMC.
set -e
S=gpurun_out/$1; D=profiles/$2; mkdir -p "$D"
cp "$S/full_bench.log" "$D/full_bench.log"; cp "$S/pytest_gpu.log" "$D/pytest_gpu.log"; cp "$S/smoke.log" "$D/smoke.log"
python3 tools/pmc_traffic.py "$S/frs" "$D" "frs_group_kernel<1, false, false, 0" frs_group_search > /dev/null
for s in kpconv:c3_kpfcnn pp:c5_pointpillars randla:randla_section scn:scn_eval single24:frs_single24; do
  src=${s%%:*}; dst=${s##*:}
  f=$(find "$S/$src" -name run_kernel_stats.csv | head -1); [ -n "$f" ] && cp "$f" "$D/${dst}_kernel_stats.csv"
done
T=$(mktemp -d); ln -s "$(pwd)/$S/single24_p1" "$T/p1"; ln -s "$(pwd)/$S/single24_p2" "$T/p2"
python3 - "$T" "$D" <<'PY'
import json, sys
sys.path.insert(0, "tools")
from pmc_summary import load
res = load(sys.argv[1], "frs_")
out = {}
for k, c in res.items():
    out[k] = {"hbm_read_bytes_2x_fetch": int(2 * c.get("FETCH_SIZE", 0) * 1024),
              "hbm_write_bytes": int(c.get("WRITE_SIZE", 0) * 1024), "dur_us_mean": c.get("dur_us_mean")}
json.dump(out, open(sys.argv[2] + "/pmc_frs_single24.json", "w"), indent=1, sort_keys=True)
PY
rm -rf "$T"
ls "$D" | wc -l
