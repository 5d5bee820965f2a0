"""Launch-averaged counter summary of one rocprofv3 --pmc csv, per kernel:
every counter's mean per launch, the mean duration, and the effective clock
GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md 'DVFS give-back').

    python tools/pmc_summary.py <counter_collection.csv> [kernel-regex]
"""
import csv
import re
import sys
from collections import defaultdict


def main():
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    per = defaultdict(lambda: defaultdict(float))
    dur = {}
    for r in csv.DictReader(open(sys.argv[1])):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if pat and not pat.search(k):
            continue
        per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[(k, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg = defaultdict(lambda: defaultdict(float))
    n = defaultdict(int)
    for (k, d), c in per.items():
        n[k] += 1
        agg[k]["_s"] += dur[(k, d)]
        for name, v in c.items():
            agg[k][name] += v
    for k, c in agg.items():
        L = n[k]
        s = c["_s"] / L
        print(f"{k}  launches={L}  avg_ms={s * 1e3:.3f}")
        for name in sorted(x for x in c if not x.startswith("_")):
            print(f"    {name:28s} {c[name] / L:16.1f}")
        if "GRBM_GUI_ACTIVE" in c:
            print(f"    effective clock (GHz)        {c['GRBM_GUI_ACTIVE'] / L / 8 / s / 1e9:16.3f}")


if __name__ == "__main__":
    main()
