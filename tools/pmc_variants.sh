#!/bin/bash
# pmc_variants.sh v1 v2 ... : one SQ instruction-count PMC pass of the FRS bench per library build
# (open3d-ml_amd/lib_<v>/, "main" = open3d-ml_amd/lib) -> per-launch means of the MODE-0 search kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); export TMPDIR=/tmp; mkdir -p $R/gpurun_out/pv
for v in "$@"; do
  if [ "$v" = main ]; then L=$R/open3d-ml_amd/lib/libo3dml_amd.so; else L=$R/open3d-ml_amd/lib_$v/libo3dml_amd.so; fi
  (cd /tmp && O3DML_AMD_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/pv/$v -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --randla-frames 0 --sparse-conv-reps 0 --kpconv-steps 0 --pointpillars-steps 0 --sweep-reps 0 > $R/gpurun_out/pv/$v.log 2>&1) || exit 1
  python3 - "$R/gpurun_out/pv/$v" "$v" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "frs_group_kernel<1, false, false, 0" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: round(sum(v) / len(v) / 1e6, 2) for k, v in sorted(acc.items())}, "(M per launch)")
PY
done
