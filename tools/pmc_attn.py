"""Summarise one rocprofv3 --pmc pass over the attention kernels into
counter-based utilisation per kernel (launch-averaged):

  mfma_util   = SQ_VALU_MFMA_BUSY_CYCLES / (busy cycles x 1024 SIMDs)
                (the matrix pipe's busy fraction over the kernel's lifetime;
                SQ_VALU_MFMA_BUSY_CYCLES counts 32 cycles per 32x32x16 bf16 MFMA,
                MI355X_MICROARCH.md 's_memtime tick vs SQ PMC units')
  valu_per_mfma = SQ_INSTS_VALU / SQ_INSTS_MFMA (VALU instructions issued per MFMA)
  valu_active_frac = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (both quad-cycles): fraction of
                wave-cycles spent issuing VALU
  busy cycles = the kernel's duration in shader cycles: (End-Start) ns x clock

    python tools/pmc_attn.py <counter_collection.csv> [clock_GHz] > summary.json
"""
import csv
import json
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    clock = float(sys.argv[2]) if len(sys.argv) > 2 else 2.4
    per = defaultdict(lambda: defaultdict(float))
    dur = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if k.startswith("_Z"):  # mangled: keep the readable stem
            import re
            m = re.search(r"(attn_\w+?_kernel)ILi(\d+)ELi(\d+)", k)
            k = f"{m.group(1)}<{m.group(2)}, {m.group(3)}...>" if m else k
        d = r["Dispatch_Id"]
        per[(k, d)][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[k][d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg = defaultdict(lambda: defaultdict(float))
    n = defaultdict(int)
    for (k, d), c in per.items():
        n[k] += 1
        for name, v in c.items():
            agg[k][name] += v
        agg[k]["seconds"] += dur[k][d]
    out = {}
    for k, c in agg.items():
        L = n[k]
        cyc = c["seconds"] / L * clock * 1e9
        mfma_busy = c["SQ_VALU_MFMA_BUSY_CYCLES"] / L
        out[k] = {
            "launches": L,
            "avg_us": c["seconds"] / L * 1e6,
            "mfma_insts": c["SQ_INSTS_MFMA"] / L,
            "valu_insts": c["SQ_INSTS_VALU"] / L,
            "lds_insts": c["SQ_INSTS_LDS"] / L,
            "mfma_util": mfma_busy / (cyc * 1024),
            "mfma_util_grbm": mfma_busy / (c["GRBM_GUI_ACTIVE"] / L * 1024) if c["GRBM_GUI_ACTIVE"] else None,
            "valu_per_mfma": c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"] if c["SQ_INSTS_MFMA"] else None,
            "valu_active_frac": c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"] if c["SQ_WAVE_CYCLES"] else None,
            "sq_busy_frac": c["SQ_BUSY_CYCLES"] / L / cyc if cyc else None,
        }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
