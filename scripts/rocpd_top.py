"""Per-kernel totals from a rocprofv3 rocpd SQLite database (the default output of `rocprofv3 --kernel-trace`):
us per update, calls per update, mean us -- the busiest kernels first. Usage: rocpd_top.py DB [UPDATES] [N] [MARKER]
(MARKER: a once-per-update kernel; only the last UPDATES updates are counted)."""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    upd = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    marker = sys.argv[4] if len(sys.argv) > 4 else None
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    where = ""
    if marker:   # only the last UPDATES updates: dispatches from the UPDATES-th last start of the marker kernel on
        starts = [r[0] for r in c.execute(f"select start from kernels where {name} like ? order by start",
                                          (f"%{marker}%",))]
        t0 = starts[-int(upd)]
        where = f"where start >= {t0}"
    rows = c.execute(f"select {name}, count(*), sum(end - start) from kernels {where} group by {name} "
                     "order by sum(end - start) desc").fetchall()
    if marker:
        span = c.execute(f"select min(start), max(end) from kernels {where}").fetchone()
        print("wall per update (first..last dispatch): %.1f us" % ((span[1] - span[0]) / 1e3 / upd))
    tot = sum(r[2] for r in rows)
    print("%10s %8s %9s  %s" % ("us/upd", "n/upd", "avg_us", "kernel"))
    for nm, cnt, t in rows[:n]:
        print("%10.2f %8.1f %9.2f  %s" % (t / 1e3 / upd, cnt / upd, t / 1e3 / cnt, nm[:110]))
    print("total kernel us per update: %.1f; dispatches per update: %.1f" % (tot / 1e3 / upd,
                                                                           sum(r[1] for r in rows) / upd))


if __name__ == "__main__":
    main()
