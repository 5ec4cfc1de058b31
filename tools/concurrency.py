"""Per-queue busy time and kernel concurrency of one step from a rocprofv3 kernel trace (segments split at each
step's logmel_tiles launch; the last segment is analysed).  usage: concurrency.py run_kernel_trace.csv"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
segs, cur = [], None
for r in rows:
    if "logmel_tiles" in r["Kernel_Name"]:
        cur = []
        segs.append(cur)
    if cur is not None:
        cur.append(r)
s = segs[-1]
t0 = int(s[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in s)
print(f"last step: span {(t1 - t0) / 1e6:.1f} ms, {len(s)} launches")
byq = collections.defaultdict(list)
for r in s:
    byq[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for q, v in sorted(byq.items()):
    print(f"queue {q}: {len(v)} kernels, busy {sum(e - b for b, e in v) / 1e6:.1f} ms, "
          f"from {(v[0][0] - t0) / 1e6:.1f} to {(max(e for _, e in v) - t0) / 1e6:.1f} ms")
ev = sorted([(b, 1) for v in byq.values() for b, _ in v] + [(e, -1) for v in byq.values() for _, e in v])
c, last, conc = 0, t0, collections.Counter()
for t, d in ev:
    conc[c] += t - last
    last, c = t, c + d
print("ms with k kernels running:", {k: round(v / 1e6, 1) for k, v in sorted(conc.items())})
