"""Print the top kernels of a rocprofv3 *_kernel_stats.csv (ms total, calls, us avg)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us  "
          f"{r['Name'][:100]}")
print(f"total {tot/1e6:.3f} ms")
