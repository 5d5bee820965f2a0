"""Per-queue busy time and idle gaps of one graph replay in a rocprofv3
kernel trace (csv or csv.gz): which queue is the critical path of the step.
    python tools/trace_streams.py run_kernel_trace.csv.gz [step_ms]"""
import csv
import gzip
import sys
from collections import defaultdict

path = sys.argv[1]
step_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 60.0
rows = list(csv.DictReader((gzip.open if path.endswith(".gz") else open)(path, "rt")))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in rows)
# the timed replays: the densest run of dispatches -- take the 10 windows of step_ms ending before the last
# long gap (eager timing steps follow the replays); pick the window with the most dispatches
t0, t1 = ev[0][0], ev[-1][1]
W = int(step_ms * 1e6)
best = None
j = 0
for i in range(len(ev)):
    while j < len(ev) and ev[j][0] < ev[i][0] + W:
        j += 1
    busy = sum(min(e[1], ev[i][0] + W) - e[0] for e in ev[i:j])
    if best is None or busy > best[0]:
        best = (busy, i, j)
_, i, j = best
win = ev[i:j]
ws, we = win[0][0], win[0][0] + W
per_q = defaultdict(float)
names = defaultdict(lambda: defaultdict(float))
for s, e, q, n in win:
    per_q[q] += (min(e, we) - s) / 1e6
    names[q][n[:60]] += (min(e, we) - s) / 1e6
# union coverage
cov, cur_s, cur_e = 0.0, None, None
for s, e, q, n in win:
    e = min(e, we)
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            cov += (cur_e - cur_s) / 1e6
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
cov += (cur_e - cur_s) / 1e6
print(f"window {step_ms} ms: {len(win)} dispatches, union busy {cov:.2f} ms ({100 * cov / step_ms:.0f} %)")
for q, t in sorted(per_q.items(), key=lambda kv: -kv[1]):
    print(f"  queue {q}: busy {t:.2f} ms")
    for n, tt in sorted(names[q].items(), key=lambda kv: -kv[1])[:6]:
        print(f"      {tt:7.3f} ms  {n}")
