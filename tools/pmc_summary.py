"""Summarise rocprofv3 --pmc passes (counter_collection.csv) per kernel:
mean counter value per dispatch, for kernels matching a substring."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(dirpath, match):
    acc = defaultdict(list)
    durs = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(dirpath, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if match not in name:
                continue
            acc[(name[:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for f in sorted(glob.glob(os.path.join(dirpath, "p*", "run_kernel_trace.csv"))):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if match in name:
                durs[name[:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {}
    for (k, c), v in acc.items():
        out.setdefault(k, {})[c] = sum(v) / len(v)
    for k, v in durs.items():
        out.setdefault(k, {})["dur_us_mean"] = sum(v) / len(v)
    return out


if __name__ == "__main__":
    res = load(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
    print(json.dumps(res, indent=1, sort_keys=True))
