"""Per-kernel instruction mix and stall breakdown from rocprofv3 counter_collection CSVs (scripts/exp/r4m.sh):
instructions per wave by class, and WAVE_CYCLES split into active-issue / parked (s_waitcnt, barrier) / issue-stall
(SQ_ACTIVE_INST_* , SQ_WAIT_* count quad-cycles, MFMA busy counts cycles; MI355X_MICROARCH.md PMC table)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from pmc_table import load, short  # noqa: E402


def main():
    per = load(sys.argv[1:], last=8)
    for k, c in per.items():
        if "cnn_trunk" not in k and "pong_fused" not in k:
            continue
        w = c.get("SQ_WAVES", 0) or 1
        print(f"== {short(k, 100)}  (dur {c['_dur_ns'] / 1e3:.1f} us, grid {int(c['_grid'])}, waves {int(w)})")
        print("  insts/wave: " + "  ".join(f"{n[9:]} {c[n] / w:.0f}" for n in
              ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU")
              if n in c))
        wc = c.get("SQ_WAVE_CYCLES", 0)
        if wc:
            parts = [(n, c[n]) for n in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                         "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_INST_LDS") if n in c]
            print("  of WAVE_CYCLES: " + "  ".join(f"{n[3:]} {v / wc * 100:.1f}%" for n, v in parts))
        if "SQ_BUSY_CYCLES" in c and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            print(f"  MFMA busy / (BUSY_CYCLES x 4 SIMD x 256 CU)... raw: MFMA_BUSY {c['SQ_VALU_MFMA_BUSY_CYCLES']:.3g} "
                  f"COEXEC {c.get('SQ_VALU_MFMA_COEXEC_CYCLES', 0):.3g} BUSY {c['SQ_BUSY_CYCLES']:.3g}")
        rest = {n: v for n, v in c.items() if n.startswith("SQ_") and n in (
            "SQ_INST_CYCLES_VMEM_WR", "SQ_INST_CYCLES_VMEM_RD", "SQ_VMEM_TA_ADDR_FIFO_FULL", "SQ_VMEM_WR_TA_DATA_FIFO_FULL",
            "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE")}
        if rest:
            print("  " + "  ".join(f"{n[3:]} {v:.3g}" for n, v in rest.items()))


if __name__ == "__main__":
    main()
