"""Per-kernel totals of one graph replay in a rocprofv3 kernel trace (csv / csv.gz),
grouped by kernel name (templates kept) and grid size, filtered by a regex.
    python tools/trace_kernels.py run_kernel_trace.csv.gz [regex] [step_ms] [--seq]"""
import csv
import gzip
import re
import sys
from collections import defaultdict

path = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
step_ms = float(sys.argv[3]) if len(sys.argv) > 3 else 58.0
seq = "--seq" in sys.argv
rows = list(csv.DictReader((gzip.open if path.endswith(".gz") else open)(path, "rt")))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Grid_Size_X"]) for r in rows)
W = int(step_ms * 1e6)
best, j = None, 0
for i in range(len(ev)):  # the step_ms window with the most dispatches = one graph replay
    while j < len(ev) and ev[j][0] < ev[i][0] + W:
        j += 1
    if best is None or j - i > best[0]:
        best = (j - i, i, j)
_, i, j = best


def short(n):
    m = re.search(r"([A-Za-z_]\w*)<([^()]*)>\(", n)
    if m and "at::native" not in n:
        return f"{m.group(1)}<{m.group(2)}>"
    return re.sub(r"\(.*", "", n)[:100]


tot, cnt = defaultdict(float), defaultdict(int)
for s, e, n, g in ev[i:j]:
    if not pat.search(n):
        continue
    if seq:
        print(f"{(e - s) / 1e3:8.1f} us  grid {g:>8}  {short(n)}")
    k = (short(n), g)
    tot[k] += (e - s) / 1e6
    cnt[k] += 1
allt = 0.0
for k, v in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"{v:7.3f} ms {cnt[k]:4d} x {v / cnt[k] * 1e3:7.1f} us  grid {k[1]:>8}  {k[0]}")
    allt += v
print(f"total {allt:.3f} ms")
