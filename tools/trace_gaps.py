"""Busy vs idle time of the GPU over a window of a rocprofv3 kernel trace: how much of the step wall time is
kernel execution and how much is gaps between dispatches (graph launch latency, host waits).

usage: python tools/trace_gaps.py <run_kernel_trace.csv> <steps> [from_frac] [to_frac]"""
import csv
import sys


def main(path, steps, lo=0.5, hi=1.0):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    n = len(rows)
    rows = rows[int(lo * n):int(hi * n)]
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e in iv:
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = iv[-1][1] - iv[0][0]
    gaps.sort()
    print(f"dispatches {len(rows)}  span {span / 1e3:.1f} us  busy {busy / 1e3:.1f} us ({100 * busy / span:.1f} %)  "
          f"idle {(span - busy) / 1e3:.1f} us in {len(gaps)} gaps (median {gaps[len(gaps) // 2] / 1e3:.2f} us, "
          f"max {gaps[-1] / 1e3:.1f} us)")
    print(f"per step (/{steps}): span {span / 1e3 / steps:.1f} us, idle {(span - busy) / 1e3 / steps:.1f} us")


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], float(a[1]), *(float(x) for x in a[2:4]))
