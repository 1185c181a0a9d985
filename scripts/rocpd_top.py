"""Per-kernel totals from a rocprofv3 rocpd SQLite database (the default output of `rocprofv3 --kernel-trace`):
us per update, calls per update, mean us -- the busiest kernels first. Usage: rocpd_top.py DB [UPDATES] [N]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    upd = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name}, count(*), sum(end - start) from kernels group by {name} "
                     "order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    print("%10s %8s %9s  %s" % ("us/upd", "n/upd", "avg_us", "kernel"))
    for nm, cnt, t in rows[:n]:
        print("%10.2f %8.1f %9.2f  %s" % (t / 1e3 / upd, cnt / upd, t / 1e3 / cnt, nm[:110]))
    print("total kernel us per update: %.1f; dispatches per update: %.1f" % (tot / 1e3 / upd,
                                                                           sum(r[1] for r in rows) / upd))


if __name__ == "__main__":
    main()
