"""VALU-side counters per kernel from one rocprofv3 --pmc pass (a hardware figure for
the VALU-bound north_star kernels, chamfer_cull / chamfer_screen / knn3 / fps_reg), launch-averaged:

  valu_busy      = SQ_ACTIVE_INST_VALU x 4 / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8): the fraction of the
                   chip's SIMD-cycles spent issuing VALU over the kernel's lifetime (the derived
                   counter VALUBusy; SQ_ACTIVE_INST_* count quad-cycles, GRBM_GUI_ACTIVE is summed over
                   the 8 XCDs -- MI355X_MICROARCH.md 'DVFS give-back')
  valu_per_wave  = SQ_INSTS_VALU / SQ_WAVES
  wait_frac      = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barriers)
  active_cus     = SQ_BUSY_CYCLES share of the chip (how much of it the launch occupies)
  clock_ghz      = GRBM_GUI_ACTIVE / 8 / duration

    python tools/pmc_valu.py <counter_collection.csv> out.json
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    per = defaultdict(lambda: defaultdict(float))
    dur = {}
    for r in csv.DictReader(open(sys.argv[1])):
        k = r["Kernel_Name"]
        per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[(k, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg = defaultdict(lambda: defaultdict(float))
    n = defaultdict(int)
    for (k, d), c in per.items():
        n[k] += 1
        agg[k]["_s"] += dur[(k, d)]
        for name, v in c.items():
            agg[k][name] += v
    out = {}
    for k, c in agg.items():
        L = n[k]
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0 / L
        row = {"launches": L, "avg_us": c["_s"] / L * 1e6}
        if cyc > 0:
            row["valu_busy"] = c["SQ_ACTIVE_INST_VALU"] / L * 4.0 / 1024.0 / cyc
            row["clock_ghz"] = cyc / (c["_s"] / L) / 1e9 if c["_s"] else None
        if c["SQ_WAVES"]:
            row["valu_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
            row["salu_per_wave"] = c["SQ_INSTS_SALU"] / c["SQ_WAVES"]
            row["lds_per_wave"] = c["SQ_INSTS_LDS"] / c["SQ_WAVES"]
        if c["SQ_WAVE_CYCLES"]:
            row["wait_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
        out[k] = row
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["launches"]):
        print(f"{v['avg_us']:9.1f} us x{v['launches']:3d}  valu_busy {v.get('valu_busy', 0):.3f}  "
              f"wait {v.get('wait_frac', 0):.2f}  {k[:110]}")


if __name__ == "__main__":
    main()
