"""Steady-state kernel stats from a rocprofv3 kernel trace: the window of the
last N steps, a step ending at each launch of a once-per-step marker kernel
(e.g. the optimizer's multi_tensor_apply_kernel) — so warm-up launches
(MIOpen find, first-call tuning) stay out.  Prints per kernel: total ms per
step, launches per step, average us; and busy / span per step.
usage: python tools/trace_window_stats.py run_kernel_trace.csv MARKER N [top]"""
import collections
import csv
import sys


def main(path, marker, n, top=30):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(ends) < n + 1:
        raise SystemExit(f"only {len(ends)} marker launches")
    a, b = ends[-n - 1] + 1, ends[-1] + 1
    seg = rows[a:b]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    d = collections.defaultdict(lambda: [0, 0])
    for r in seg:
        k = r["Kernel_Name"]
        d[k][0] += 1
        d[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print(f"window: last {n} steps (marker '{marker}'), {len(seg) / n:.0f} launches/step, "
          f"busy {busy / n / 1e6:.3f} ms/step, span {(t1 - t0) / n / 1e6:.3f} ms/step")
    print(f"{'ms/step':>9} {'calls/step':>10} {'avg us':>9}  kernel")
    for k, (c, t) in sorted(d.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{t / n / 1e6:9.3f} {c / n:10.1f} {t / c / 1e3:9.1f}  {k[:110]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else 30)
