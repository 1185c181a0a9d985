"""Profiling tools: scripts/rocpd_top.py summarises a rocprofv3 rocpd database (synthetic database of the same
schema subset: the `kernels` view with name / start / end)."""
import os
import sqlite3
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _db(path):
    c = sqlite3.connect(path)
    c.execute("create table kernels (name text, start integer, end integer)")
    t = 0
    rows = []
    for upd in range(3):                       # 3 updates: marker + 2 x k1 (5 us) + k2 (20 us)
        for nm, d in (("aca::marker_kernel(args)", 1000), ("aca::k1(args)", 5000), ("aca::k1(args)", 5000),
                      ("aca::k2(args)", 20000 if upd else 90000)):   # the first update is a warm-up outlier
            rows.append((nm, t, t + d))
            t += d + 100
    c.executemany("insert into kernels values (?, ?, ?)", rows)
    c.commit()
    c.close()


def test_rocpd_top_last_updates(tmp_path):
    db = str(tmp_path / "run_results.db")
    _db(db)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rocpd_top.py"), db, "2", "10", "marker"],
                         capture_output=True, text=True, check=True).stdout
    lines = {l.split()[-1]: l.split() for l in out.splitlines() if l.strip().startswith(tuple("0123456789"))}
    # only the last two updates: k2 20 us per update (the 90 us warm-up excluded), k1 2 x 5 us
    assert abs(float(lines["aca::k2(args)"][0]) - 20.0) < 1e-6, out
    assert abs(float(lines["aca::k1(args)"][0]) - 10.0) < 1e-6 and float(lines["aca::k1(args)"][1]) == 2.0, out
    assert "dispatches per update: 4.0" in out, out
