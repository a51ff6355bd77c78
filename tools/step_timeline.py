"""Per-step kernel timeline from a rocprofv3 kernel trace: the kernels between
two consecutive launches of an anchor kernel, with gaps and durations.
usage: step_timeline.py run_kernel_trace.csv [anchor substring] [step index]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
anchor = sys.argv[2] if len(sys.argv) > 2 else "frs_group_kernel<1, false, false, 0"
k = int(sys.argv[3]) if len(sys.argv) > 3 else 6
idx = [i for i, x in enumerate(rows) if anchor in x["Kernel_Name"]]
a, b = idx[k], idx[k + 1]
t0 = int(rows[a]["Start_Timestamp"])
prev = None
busy = 0
for x in rows[a:b]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    busy += e - s
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{(s - t0) / 1e3:8.1f} gap {gap:6.1f} dur {(e - s) / 1e3:7.1f} {x['Kernel_Name'][:90]}")
    prev = e
print(f"step span {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us, {b - a} kernels")
