"""Per-update kernel time from a rocprofv3 kernel trace: only the last `--updates` updates (graph replays after
warm-up/tuning), identified by the env-step kernel that runs `--per-update` times per update."""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--updates", type=int, default=40)
ap.add_argument("--marker", default="pong_step_kernel")
ap.add_argument("--per-update", type=int, default=5)
a = ap.parse_args()
if a.trace.endswith(".db"):   # rocprofv3 >= 7 default output (rocpd SQLite): same fields as the CSV kernel trace
    import sqlite3
    con = sqlite3.connect(a.trace)
    rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
            for n, s, e in con.execute("select name, start, end from kernels")]
else:
    rows = list(csv.DictReader(open(a.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
need = a.updates * a.per_update
start = marks[-need]
# include the kernels of the first update that precede its first env step: back up to the previous update's end
prev_end = marks[-need - 1] if len(marks) > need else 0
seg = rows[start:]
first_t = int(rows[start]["Start_Timestamp"])
last_t = int(rows[-1]["End_Timestamp"])
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    k = r["Kernel_Name"][:90]
    agg[k][0] += 1
    agg[k][1] += d
tot = sum(v[1] for v in agg.values())
print("%9s %7s %8s  %s" % ("us/upd", "n/upd", "avg_us", "kernel"))
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%9.2f %7.1f %8.2f  %s" % (t / a.updates, n / a.updates, t / n, k))
print("sum of kernel time per update: %.1f us; dispatches per update: %.1f; wall per update (first..last): %.1f us"
      % (tot / a.updates, len(seg) / a.updates, (last_t - first_t) / 1e3 / a.updates))
