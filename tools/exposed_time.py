"""Exposed time of a kernel group in the timed steps of a PCOPS_TRACE_MARKS=1 kernel trace: the
part of the group's busy time during which NO other kernel runs anywhere on the GPU (what the step
would lose if the group took zero time and everything else stayed put), next to its total kernel
time and the part that runs with the main stream idle.
    python tools/exposed_time.py <kernel_trace.csv[.gz]> <steps> [regex=fps_(reg|wave|stream|mw)_kernel]"""
import csv
import gzip
import re
import sys

path, steps = sys.argv[1], int(sys.argv[2])
pat = re.compile(sys.argv[3] if len(sys.argv) > 3 else r"fps_(reg|wave|stream|mw)_kernel")
rows = list(csv.DictReader((gzip.open if path.endswith(".gz") else open)(path, "rt")))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
marks = [i for i, e in enumerate(ev) if "spin_kernel" in e[2]]
if len(marks) < 2:
    sys.exit(f"expected two spin_kernel markers, found {len(marks)}")
t0, t1 = ev[marks[0]][1], ev[marks[1]][0]
win = [e for e in ev if e[0] >= t0 and e[1] <= t1 and "spin_kernel" not in e[2]]


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def length(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    out, i, j = [], 0, 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def subtract(a, b):   # a minus b, both unions
    out = []
    for s, e in a:
        cur = s
        for bs, be in b:
            if be <= cur or bs >= e:
                continue
            if bs > cur:
                out.append([cur, bs])
            cur = max(cur, be)
        if cur < e:
            out.append([cur, e])
    return out


grp = union([(s, e) for s, e, n in win if pat.search(n)])
other = union([(s, e) for s, e, n in win if not pat.search(n)])
total = sum(e - s for s, e, n in win if pat.search(n))
alone = length(subtract(grp, other))
print(f"{pat.pattern}: {total / 1e6 / steps:.3f} ms/step kernel time, busy {length(grp) / 1e6 / steps:.3f} ms/step, "
      f"exposed (no other kernel running) {alone / 1e6 / steps:.3f} ms/step over {(t1 - t0) / 1e6 / steps:.2f} ms steps")
