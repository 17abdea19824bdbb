"""Per-kernel time of the dispatches after the last idle gap (> 0.3 s) of a rocprofv3 kernel trace:
the steady-state forwards of scripts/prof_abstract.py.  usage: trace_after_gap.py run_kernel_trace.csv [n_iters]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
n_it = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
cut = 0
for i in range(1, len(ev)):
    if ev[i][0] - ev[i - 1][1] > 300_000_000:
        cut = i
tail = ev[cut:]
tot = defaultdict(float)
for s, e, n in tail:
    tot[n] += (e - s) / 1e6
wall = (tail[-1][1] - tail[0][0]) / 1e6
print(f"steady-state dispatches {len(tail)}, wall {wall / n_it:.2f} ms per forward, busy {sum(tot.values()) / n_it:.2f} ms")
for n, t in sorted(tot.items(), key=lambda kv: -kv[1])[:25]:
    print(f"{t / n_it:9.3f} ms  {n[:110]}")
