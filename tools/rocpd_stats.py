"""Per-kernel duration summary from a rocprofv3 rocpd SQLite database (when the run was not written as CSV)."""
import sqlite3
import sys


def main(path, top=40):
    c = sqlite3.connect(path)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    disp = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    sym = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    cols = [r[1] for r in c.execute(f"pragma table_info({sym})")]
    name_col = "display_name" if "display_name" in cols else ("kernel_name" if "kernel_name" in cols else "name")
    q = (f"select s.{name_col}, count(*), sum(d.end - d.start), avg(d.end - d.start) from {disp} d "
         f"join {sym} s on d.kernel_id = s.id group by s.{name_col} order by sum(d.end - d.start) desc")
    rows = list(c.execute(q))
    tot = sum(r[2] for r in rows)
    print(f"{'kernel':80s} {'calls':>6s} {'total_ms':>9s} {'avg_us':>9s} {'pct':>6s}")
    for n, cnt, s, a in rows[:top]:
        print(f"{n[:80]:80s} {cnt:6d} {s / 1e6:9.3f} {a / 1e3:9.2f} {100 * s / tot:6.2f}")
    print(f"total kernel time {tot / 1e6:.3f} ms over {sum(r[1] for r in rows)} dispatches")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
