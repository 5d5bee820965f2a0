"""Torch glue in a replay-only kernel-stats CSV (tools/trace_window.py output): time and launches per
step of ATen's own kernels (elementwise, copies / casts, cat, reductions, fills), the fused optimizer
listed apart, and the step's total launch count.
    python tools/glue_from_trace.py profiles/r4_kernel_stats_replay.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
glue = defaultdict(lambda: [0.0, 0.0])
opt = [0.0, 0.0]
launches = 0.0
for r in rows:
    n, ms, calls = r["Name"], float(r["MsPerStep"]), float(r["CallsPerStep"])
    launches += calls
    if "FusedAdam" in n or "FusedOptimizer" in n:
        opt[0] += ms
        opt[1] += calls
    elif "at::native" in n:
        kind = ("cat" if "CatArrayBatched" in n else "reduce" if "reduce_kernel" in n else
                "copy/cast" if ("copy" in n or "direct_copy" in n) else "fill" if "Fill" in n else "elementwise")
        glue[kind][0] += ms
        glue[kind][1] += calls
tot = sum(v[0] for v in glue.values())
print(f"torch glue: {tot:.3f} ms/step in {sum(v[1] for v in glue.values()):.0f} launches; "
      f"fused optimizer {opt[0]:.3f} ms ({opt[1]:.0f}); all kernels {launches:.0f} launches/step")
for k, (ms, c) in sorted(glue.items(), key=lambda kv: -kv[1][0]):
    print(f"  {k:12s} {ms:7.3f} ms  {c:5.0f} launches")
