"""Launches and kernel time per headline step from a rocprofv3 kernel trace of tools/gpu_prof.sh: the
trace is split at each step's log-mel tile launch; the last three segments are the timed steps (eager launches
since round 5; graph replays before, and with bench.py --graph).
usage: replay_step.py run_kernel_trace.csv [tag]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
tag = sys.argv[2] if len(sys.argv) > 2 else ""
segs, cur = [], None
for r in rows:
    if "logmel_tiles" in r["Kernel_Name"]:
        cur = []
        segs.append(cur)
    if cur is not None:
        cur.append(r)
print(f"rocprofv3 kernel trace of tools/gpu_prof.sh {tag} (2 warm-ups + 3 timed steps of the headline step);")
print("per-step numbers below are the mean of the 3 timed steps (segments start at each step's logmel_tiles launch)")
for s in segs:
    print("segment launches", len(s))
rep = segs[-3:]
dur = collections.defaultdict(float)
cnt = collections.Counter()
for s in rep:
    for r in s:
        dur[r["Kernel_Name"]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 3
        cnt[r["Kernel_Name"]] += 1
wall = sum((int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) for s in rep) / 3
print(f"launches/step {sum(len(s) for s in rep) / 3:.0f}  kernel ms/step {sum(dur.values()) / 1e6:.1f} "
      f"(kernels of the side streams overlap the main stream: step wall ~{wall / 1e6:.0f} ms)")
for k, v in sorted(dur.items(), key=lambda kv: -kv[1])[:40]:
    n = cnt[k] / 3
    print(f"{v / 1e6:8.2f} ms n={n:5.0f} avg={v / n / 1e3:9.1f}us {k[:140]}")
