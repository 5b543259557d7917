"""Per-(kernel, grid) time summary from a rocprofv3 kernel_trace.csv, normalised per step.

usage: python tools/kernel_by_shape.py <run_kernel_trace.csv> <steps> [top] [t_from_frac t_to_frac]
The optional fractions select a window of the trace by dispatch order (e.g. 0 0.5 for the first half)."""
import csv
import sys
from collections import defaultdict


def main(path, steps, top=45, lo=0.0, hi=1.0):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    n = len(rows)
    rows = rows[int(lo * n):int(hi * n)]
    agg = defaultdict(lambda: [0, 0])
    for r in rows:
        k = (r["Kernel_Name"], r["Grid_Size_X"], r["Grid_Size_Y"], r["VGPR_Count"], r["Accum_VGPR_Count"])
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[k][0] += 1
        agg[k][1] += d
    tot = sum(v[1] for v in agg.values())
    print(f"{'us/step':>9s} {'n/step':>7s} {'avg_us':>8s}  kernel  grid_x grid_y vgpr agpr")
    for k, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{d / 1e3 / steps:9.1f} {c / steps:7.1f} {d / 1e3 / c:8.1f}  {k[0][:110]}  {k[1]} {k[2]} {k[3]} {k[4]}")
    print(f"total {tot / 1e3 / steps:.1f} us/step over {n} dispatches")


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], float(a[1]), int(a[2]) if len(a) > 2 else 45, float(a[3]) if len(a) > 3 else 0.0,
         float(a[4]) if len(a) > 4 else 1.0)
