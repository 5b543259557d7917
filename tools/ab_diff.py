"""Per-kernel total-time difference of the two kernel traces tools/ab_tree.sh leaves (A = ab_base, B = this tree)."""
import csv
import sys


def load(p):
    d = {}
    for r in csv.DictReader(open(p)):
        k = r["Name"][:80]
        c, t = d.get(k, (0, 0.0))
        d[k] = (c + int(r["Calls"]), t + float(r["TotalDurationNs"]) / 1e3)
    return d


base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab_tree"
A, B = load(f"{base}/tA/run_kernel_stats.csv"), load(f"{base}/tB/run_kernel_stats.csv")
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
for k in sorted(set(A) | set(B), key=lambda k: -abs(B.get(k, (0, 0))[1] - A.get(k, (0, 0))[1])):
    a, b = A.get(k, (0, 0.0)), B.get(k, (0, 0.0))
    if abs(b[1] - a[1]) > thr:
        print(f"{a[0]:4d} {a[1]:9.1f} | {b[0]:4d} {b[1]:9.1f} | {b[1] - a[1]:+8.1f}  {k}")
print(f"total {sum(v[1] for v in A.values()):.1f} | {sum(v[1] for v in B.values()):.1f}")
