"""Summarize a rocprofv3 kernel trace: per-step kernel time table and small-kernel census."""
import collections
import csv
import sys

path, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
rows = list(csv.DictReader(open(path)))
dur = collections.Counter()
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:100]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    dur[k] += d
    cnt[k] += 1
tot = sum(dur.values())
print(f"launches/step {len(rows)/steps:.0f}  kernel ms/step {tot/steps/1e3:.1f}")
for k, v in dur.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
    print(f"{v/steps/1e3:8.2f} ms {100*v/tot:5.1f}% n={cnt[k]/steps:6.0f} avg={v/cnt[k]:8.1f}us {k}")
