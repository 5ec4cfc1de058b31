"""Launches and kernel time per headline step from a rocprofv3 kernel trace of a bench.py run (tools/gpu_r06_prof.sh):
the trace is split at each step's log-mel tile launch, and segments FIRST .. FIRST + COUNT - 1 are averaged --
bench.py runs W warm-up steps, K timed steps, two steps from an idle GPU and one probed step, so with the default
--warmup 2 --steps 5 the timed steps are segments 2..6 (eager launches since round 5).
usage: replay_step.py run_kernel_trace.csv [tag] [first=2] [count=5]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
tag = sys.argv[2] if len(sys.argv) > 2 else ""
first = int(sys.argv[3]) if len(sys.argv) > 3 else 2
count = int(sys.argv[4]) if len(sys.argv) > 4 else 5
segs, cur = [], None
for r in rows:
    if "logmel_tiles" in r["Kernel_Name"]:
        cur = []
        segs.append(cur)
    if cur is not None:
        cur.append(r)
print(f"rocprofv3 kernel trace {tag}: per-step numbers below are the mean of segments {first}..{first + count - 1}"
      " (the timed steps; segments start at each step's logmel_tiles launch)")
for s in segs:
    print("segment launches", len(s))
rep = segs[first:first + count]
dur = collections.defaultdict(float)
cnt = collections.Counter()
for s in rep:
    for r in s:
        dur[r["Kernel_Name"]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / len(rep)
        cnt[r["Kernel_Name"]] += 1
wall = sum((int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) for s in rep) / len(rep)
print(f"launches/step {sum(len(s) for s in rep) / len(rep):.0f}  kernel ms/step {sum(dur.values()) / 1e6:.1f} "
      f"(kernels of the side streams overlap the main stream: step wall ~{wall / 1e6:.0f} ms)")
for k, v in sorted(dur.items(), key=lambda kv: -kv[1])[:40]:
    n = cnt[k] / len(rep)
    print(f"{v / 1e6:8.2f} ms n={n:5.0f} avg={v / n / 1e3:9.1f}us {k[:140]}")
