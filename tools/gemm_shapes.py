"""Median duration per (kernel, grid) of the sparse-conv GEMM kernels in a
rocprofv3 kernel_trace.csv: python tools/gemm_shapes.py <trace.csv>"""
import collections
import csv
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if any(s in n for s in ("implicit_gemm", "dweight", "split_reduce", "reduce_slabs", "mask_keys", "radix")):
        key = (n.split("(")[0][-40:], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
        d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    v.sort()
    print(f"{k[0]:40s} grid {k[1]:>7s} x {k[2]:>3s} x {k[3]:>3s}  n {len(v):4d}  median {v[len(v) // 2]:8.1f} us")
