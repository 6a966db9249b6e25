"""MFMA-busy per kernel from one rocprofv3 PMC pass:
    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE ...

Per dispatch (rocprofv3 serialises dispatches while it collects counters, so each kernel runs alone):
  * mfma_busy_chip = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)  -- rocprofv3's derived
    `MfmaUtil` (counter_defs.yaml): the fraction of the whole chip's MFMA-pipe cycles busy over the dispatch.
    GRBM_GUI_ACTIVE comes back summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS paragraph).
  * mfma_busy_per_busy_cu = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CU_CYCLES * 4 SIMDs): the same busy cycles
    over the cycles the CUs that held waves were busy -- separates "few workgroups" from "slow workgroups".
    SQ_BUSY_CU_CYCLES reads as CU-cycles summed over the CUs on gfx950 (counter_defs.yaml says quad-cycles):
    for conv1_res_kernel on 128 workgroups it gives ~104 busy CUs on average, and the quad-cycle reading would
    give ~415 of the chip's 256.
  * mfma_flop = SQ_INSTS_VALU_MFMA_MOPS_F16 * 512 (counter_defs.yaml `MfmaFlopsF16`), a check of the
    algorithmic FLOP count the bench prices `achieved` on.
  * clock_ghz = GRBM_GUI_ACTIVE / 8 / dispatch time (reads high below ~0.3 ms dispatches).
Usage: python tools/pmc_mfma.py COUNTERS.csv [kernel-substring ...] > profiles/rNN_pmc_mfma_fp16.json
"""
import csv
import json
import sys
from collections import defaultdict

SIMDS = 1024  # 256 CUs x 4 SIMDs
XCDS = 8


def main():
    rows = defaultdict(dict)  # (kernel, dispatch) -> counter -> value
    span = {}
    for r in csv.DictReader(open(sys.argv[1])):
        key = (r["Kernel_Name"], r["Dispatch_Id"])
        rows[key][r["Counter_Name"]] = rows[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        span[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    pats = sys.argv[2:] or [""]
    per = defaultdict(list)
    for (name, _), c in rows.items():
        if any(p in name for p in pats) and "GRBM_GUI_ACTIVE" in c and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            per[name].append((c, span[(name, _)]))
    out = {}
    for name, lst in sorted(per.items()):
        n = len(lst)
        busy = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"] for c, _ in lst) / n
        gui = sum(c["GRBM_GUI_ACTIVE"] for c, _ in lst) / n
        cu = sum(c.get("SQ_BUSY_CU_CYCLES", 0.0) for c, _ in lst) / n
        mops = sum(c.get("SQ_INSTS_VALU_MFMA_MOPS_F16", 0.0) for c, _ in lst) / n
        t = sum(s for _, s in lst) / n
        out[name] = {
            "dispatches": n,
            "dispatch_us": round(t * 1e6, 2),
            "SQ_VALU_MFMA_BUSY_CYCLES": busy, "GRBM_GUI_ACTIVE": gui, "SQ_BUSY_CU_CYCLES": cu,
            "SQ_INSTS_VALU_MFMA_MOPS_F16": mops,
            "mfma_busy_chip": busy / (gui / XCDS * SIMDS) if gui else None,
            "mfma_busy_per_busy_cu": busy / (cu * 4) if cu else None,
            "busy_cus_mean": round(cu / (gui / XCDS), 1) if gui else None,
            "mfma_flop_f16": mops * 512,
            "clock_ghz": round(gui / XCDS / t * 1e-9, 3) if t > 0 else None,
        }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
