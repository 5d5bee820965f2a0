"""Per-launch-shape exposure of selected kernels in a rocprofv3 kernel trace cut to the timed replays
(the two torch spin kernels PCOPS_TRACE_MARKS=1 puts around them): for each (kernel, grid) group,
launches per step, kernel time per step and the time during which NO other kernel ran (on the step's
critical path whatever the stream).

    python tools/exposed_launches.py run_kernel_trace.csv[.gz] steps [regex]
"""
import bisect
import collections
import csv
import gzip
import re
import sys


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    pat = re.compile(sys.argv[3] if len(sys.argv) > 3 else r"fps|chamfer|knn|emd")
    op = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
    rows = list(csv.DictReader(op))
    spin = [r for r in rows if "spin_kernel" in r["Kernel_Name"]]
    a, b = int(spin[0]["End_Timestamp"]), int(spin[-1]["Start_Timestamp"])
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Grid_Size_X"], r.get("Grid_Size_Y"))
          for r in rows if int(r["Start_Timestamp"]) >= a and int(r["End_Timestamp"]) <= b]
    ev = sorted([(s, 1) for s, *_ in ks] + [(e, -1) for _, e, *_ in ks])
    single, cnt, last = [], 0, None
    for t, d in ev:
        if cnt == 1 and last is not None and t > last:
            single.append((last, t))
        cnt += d
        last = t

    def exposed(s, e):
        tot, i = 0, bisect.bisect_left(single, (s, 0))
        for j in range(max(0, i - 1), len(single)):
            x, y = single[j]
            if x >= e:
                break
            tot += max(0, min(e, y) - max(s, x))
        return tot

    def short(n):
        m = re.search(r"(\w+_kernel)(<[^>(]*>)?", n.replace("(anonymous namespace)::", ""))
        return (m.group(1) + (m.group(2) or "")) if m else n[:60]

    agg = collections.defaultdict(lambda: [0, 0, 0])
    for s, e, n, gx, gy in ks:
        if pat.search(n):
            g = agg[(short(n), gx, gy)]
            g[0] += 1
            g[1] += e - s
            g[2] += exposed(s, e)
    print(f"window {(b - a) / 1e6 / steps:.3f} ms per step over {steps} steps")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][2]):
        print(f"{v[0] / steps:5.1f}/step  kernel {v[1] / steps / 1e6:7.3f} ms  exposed {v[2] / steps / 1e6:7.3f} ms  "
              f"{k[0]} grid {k[1]}x{k[2]}")


if __name__ == "__main__":
    main()
