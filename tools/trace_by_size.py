"""Per-(kernel, grid) breakdown of a rocprofv3 kernel trace (tooling, not product): which launch sizes
of a kernel take the time.  usage: trace_by_size.py kernel_trace.csv steps [name-substring ...]"""
import collections
import csv
import sys

path, steps = sys.argv[1], float(sys.argv[2])
pats = sys.argv[3:]
rows = list(csv.DictReader(open(path)))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    k = r["Kernel_Name"]
    if pats and not any(p in k for p in pats):
        continue
    g = tuple(int(r.get(f"Grid_Size_{a}", r.get(f"Grid_Size{a}", 0)) or 0) for a in "XYZ")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a = agg[(k[:70], g)]
    a[0] += 1
    a[1] += d
tot = sum(v[1] for v in agg.values())
for (k, g), (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:60]:
    print(f"{us / steps / 1e3:8.2f} ms/step {n / steps:6.1f}/step avg {us / n:8.1f} us grid {g} {k}")
print(f"total {tot / steps / 1e3:.1f} ms/step")
