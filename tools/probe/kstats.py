"""Per-kernel average durations from a rocprofv3 --kernel-trace --stats output directory (the *_kernel_stats.csv
or the rocpd .db).  usage: python tools/probe/kstats.py <dir> [name-substring ...]"""
import csv
import glob
import os
import sqlite3
import sys


def rows(d):
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                yield r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3
        return
    for f in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(f)
        for n, calls, tot, avg in c.execute("select name,total_calls,total_duration,average from top_kernels"):
            yield n, int(calls), float(tot) / 1e3 if tot > 1e6 else float(tot), float(avg)
        return


if __name__ == "__main__":
    keys = sys.argv[2:]
    for n, calls, tot, avg in rows(sys.argv[1]):
        if not keys or any(k in n for k in keys):
            print(f"{avg:9.1f} us avg  {calls:6d} calls  {n[:110]}")
