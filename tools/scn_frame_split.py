"""Split one SparseConvUnet eval frame of a rocprofv3 kernel trace (mode 3:
o3dml_scn_plan + the replayed body) into plan / body kernels: counts, busy
time, span, and the body's kernels grouped by name.
  python tools/scn_frame_split.py <run_kernel_trace.csv> [top]"""
import csv
import sys
from collections import defaultdict

f = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = sorted(csv.DictReader(open(f)), key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "scn_splits_kernel" in r["Kernel_Name"]]
seg = rows[idx[-3]:idx[-2]]
i = [j for j, r in enumerate(seg) if "lattice_stats" in r["Kernel_Name"]][0]


def dur(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3


def span(rs):
    return (int(rs[-1]["End_Timestamp"]) - int(rs[0]["Start_Timestamp"])) / 1e3


for name, part in (("plan", seg[:i]), ("body", seg[i:])):
    print(f"{name}: {len(part)} kernels, busy {sum(map(dur, part)):.1f} us, span {span(part):.1f} us")
print(f"frame span {span(seg):.1f} us")
agg = defaultdict(lambda: [0, 0.0])
for r in seg[i:]:
    k = r["Kernel_Name"].split("(")[0][:100]
    agg[k][0] += 1
    agg[k][1] += dur(r)
for k, v in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print("%4d %8.1f %s" % (v[0], v[1], k))
