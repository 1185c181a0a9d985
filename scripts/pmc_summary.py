"""Per-kernel PMC summary from rocprofv3 --pmc CSV(s): the last N dispatches of each kernel (steady state),
averaged; derived per-wave metrics. Usage: python scripts/pmc_summary.py run_counter_collection.csv [...]"""
import collections
import csv
import sys

files = [a for a in sys.argv[1:] if not a.startswith("--")]
last = 20
vals = collections.defaultdict(lambda: collections.defaultdict(list))   # kernel -> counter -> [per dispatch]
for fn in files:
    rows = list(csv.DictReader(open(fn)))
    by_disp = collections.defaultdict(dict)
    names = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        by_disp[d][r["Counter_Name"]] = float(r["Counter_Value"])
        names[d] = (r["Kernel_Name"][:70], int(r["Grid_Size"]), int(r["VGPR_Count"]), int(r["LDS_Block_Size"]),
                    int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for d in sorted(by_disp):
        k = names[d][0]
        for c, v in by_disp[d].items():
            vals[k][c].append(v)
        vals[k]["_dur_ns"].append(names[d][4])
        vals[k]["_grid"].append(names[d][1])
out = []
for k, cs in vals.items():
    avg = {c: sum(v[-last:]) / len(v[-last:]) for c, v in cs.items()}
    out.append((avg.get("_dur_ns", 0), k, avg))
out.sort(reverse=True)
for dur, k, a in out[:24]:
    waves = max(a.get("SQ_WAVES", 1), 1)
    line = f"{dur / 1e3:8.2f}us grid={int(a['_grid']):7d} {k}\n   "
    for c in ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_INSTS_VALU", "SQ_INSTS_SALU",
              "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_VMEM_RD", "SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES",
              "SQ_ACTIVE_INST_VALU", "SQ_INST_LEVEL_VMEM", "SQ_IFETCH", "GRBM_GUI_ACTIVE"):
        if c in a:
            v = a[c]
            per = v / waves if c.startswith("SQ_INSTS") or c in ("SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                                                                  "SQ_ACTIVE_INST_VALU", "SQ_IFETCH") else v
            line += f" {c[3:] if c.startswith('SQ_') else c}={per:.0f}"
    print(line)
