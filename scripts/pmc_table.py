#!/usr/bin/env python3
"""Per-kernel roofline table from rocprofv3 ``--pmc`` passes (CSV output), one pass per counter group.

    python scripts/pmc_table.py --tail 540 pass1_counter_collection.csv pass2_... [--last 20]

Steady state only: ``--tail D`` keeps the last D dispatches of each pass (the timed graph replays, after every
autotuning candidate has run), and within that each kernel's last ``--last`` dispatches. For every kernel it
joins the counters of all passes and derives, per dispatch:
  * time (kernel-trace start/end of the PMC runs; profiled runs clock ~2-5 % lower than unprofiled ones),
  * MFMA busy share of the whole chip = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x clock cycles), where clock cycles =
    GRBM_GUI_ACTIVE / 8 (rocprofv3 sums GRBM over the 8 XCDs; MI355X_MICROARCH.md 'DVFS give-back'),
  * bf16 matrix FLOP = SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 and F32-MFMA FLOP = MOPS_F32 x 512 (one MOP = 512 FLOP),
    achieved TF/s and the share of the 2.5 PF dense bf16 (157 TF f32-MFMA) peak,
  * HBM-side bytes: FETCH_SIZE (KiB; x2 for wide streaming reads on gfx950, see the microarch guide -- reported raw
    here and doubled in the TB/s column) and WRITE_SIZE, achieved TB/s against 8 TB/s,
  * LDS bank-conflict share = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, L2 hit rate = TCC_HIT / (TCC_HIT + TCC_MISS).
"""
from __future__ import annotations

import argparse
import collections
import csv

PEAK_BF16 = 2.5e15
PEAK_F32 = 157.3e12
PEAK_HBM = 8.0e12


def load(files, last, tail=0):
    per = collections.defaultdict(lambda: collections.defaultdict(list))   # kernel -> counter -> values
    for fn in files:
        disp = collections.defaultdict(dict)
        meta = {}
        with open(fn) as f:
            for r in csv.DictReader(f):
                d = int(r["Dispatch_Id"])
                disp[d][r["Counter_Name"]] = disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                meta[d] = (r["Kernel_Name"], int(r.get("Grid_Size", 0) or 0), int(r.get("VGPR_Count", 0) or 0),
                           int(r.get("LDS_Block_Size", 0) or 0),
                           int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) if "End_Timestamp" in r else 0)
        bykern = collections.defaultdict(list)
        ids = sorted(disp)
        if tail:
            ids = ids[-tail:]
        for d in ids:
            bykern[meta[d][0]].append(d)
        for k, ds in bykern.items():
            for d in ds[-last:]:
                for c, v in disp[d].items():
                    per[k][c].append(v)
                per[k]["_dur_ns"].append(meta[d][4])
                per[k]["_n"].append(len(ds))
                per[k]["_grid"].append(meta[d][1])
                per[k]["_vgpr"].append(meta[d][2])
                per[k]["_lds"].append(meta[d][3])
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}


def short(name, n=64):
    name = name.replace("aca::", "").replace("void ", "")
    return name if len(name) <= n else name[:n - 1] + "~"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--tail", type=int, default=0, help="keep only the last D dispatches of each pass")
    a = ap.parse_args()
    rows = load(a.files, a.last, a.tail)
    out = sorted(rows.items(), key=lambda kv: -kv[1].get("_dur_ns", 0) * kv[1].get("_n", 1))[:a.top]
    hdr = ("%-64s %5s %8s %7s %5s %6s %9s %7s %6s %8s %8s %7s %6s %6s" %
           ("kernel", "n", "us", "grid", "vgpr", "mfma%", "GFLOP", "TF/s", "%pk", "fetchKB", "writeKB", "TB/s",
            "ldsC%", "L2hit"))
    print(hdr)
    for k, v in out:
        dur = v.get("_dur_ns", 0) * 1e-9
        clk = v.get("GRBM_GUI_ACTIVE", 0) / 8.0
        busy = v.get("SQ_VALU_MFMA_BUSY_CYCLES")
        mfma = 100.0 * busy / (1024.0 * clk) if busy is not None and clk > 0 else float("nan")
        fb = v.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512
        ff = v.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0) * 512
        flop = fb + ff
        tfs = flop / dur / 1e12 if dur > 0 else 0.0
        pk = 100.0 * (fb / PEAK_BF16 + ff / PEAK_F32) / dur if dur > 0 else 0.0
        fetch = v.get("FETCH_SIZE", float("nan"))
        write = v.get("WRITE_SIZE", float("nan"))
        byts = (2 * (fetch if fetch == fetch else 0) + (write if write == write else 0)) * 1024
        tbs = byts / dur / 1e12 if dur > 0 else 0.0
        lc = v.get("SQ_LDS_BANK_CONFLICT")
        la = v.get("SQ_LDS_IDX_ACTIVE")
        ldsc = 100.0 * lc / la if lc is not None and la else float("nan")
        h, m = v.get("TCC_HIT_sum", v.get("TCC_HIT")), v.get("TCC_MISS_sum", v.get("TCC_MISS"))
        l2 = 100.0 * h / (h + m) if h is not None and m is not None and h + m > 0 else float("nan")
        print("%-64s %5d %8.2f %7d %5d %6.1f %9.3f %7.1f %6.2f %8.1f %8.1f %7.3f %6.1f %6.1f" %
              (short(k), v.get("_n", 0), dur * 1e6, v.get("_grid", 0), v.get("_vgpr", 0), mfma, flop / 1e9, tfs, pk, fetch, write,
               tbs, ldsc, l2))


if __name__ == "__main__":
    main()
