"""Per-kernel statistics of exactly the timed steps of a bench.py run traced with
rocprofv3 --kernel-trace under PCOPS_TRACE_MARKS=1 (a spin kernel on each side
of the timed region): no warm-up, no MIOpen search, no kernel-timing steps.
    python tools/trace_window.py <kernel_trace.csv[.gz]> <steps> <out.csv>"""
import csv
import gzip
import re
import sys
from collections import defaultdict

path, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rows = list(csv.DictReader((gzip.open if path.endswith(".gz") else open)(path, "rt")))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
marks = [i for i, e in enumerate(ev) if "spin_kernel" in e[2]]
if len(marks) < 2:
    sys.exit(f"expected two spin_kernel markers, found {len(marks)}")
a, b = marks[0], marks[1]
t0, t1 = ev[a][1], ev[b][0]
win = [e for e in ev[a + 1:b] if e[0] >= t0 and e[1] <= t1]


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    m = re.search(r"([A-Za-z_]\w*)<([^()]*)>\(", n)
    if m and "at::native" not in n:
        return f"{m.group(1)}<{m.group(2)}>"
    return re.sub(r"\(.*", "", n)[:120]


tot, cnt = defaultdict(int), defaultdict(int)
for s, e, n in win:
    tot[short(n)] += e - s
    cnt[short(n)] += 1
busy = sum(tot.values())
with open(out, "w", newline="") as f:
    wr = csv.writer(f)
    wr.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "CallsPerStep", "MsPerStep"])
    for n in sorted(tot, key=lambda k: -tot[k]):
        wr.writerow([n, cnt[n], tot[n], tot[n] // cnt[n], round(100.0 * tot[n] / busy, 3), cnt[n] / steps,
                     round(tot[n] / steps / 1e6, 4)])
print(f"window {(t1 - t0) / 1e6:.2f} ms over {steps} steps = {(t1 - t0) / 1e6 / steps:.2f} ms/step; "
      f"{len(win)} kernels, kernel time {busy / 1e6 / steps:.2f} ms/step (streams overlap)")
