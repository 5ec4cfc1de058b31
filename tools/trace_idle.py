"""Where the GPU idles inside one step of a rocprofv3 kernel trace (the last step: segments split at each step's
logmel_tiles launch): the union of kernel intervals over every queue, the idle time in tenths of the step's span,
and the longest gaps with the kernels either side.  Idle time is time the host's issue is behind the GPU.
usage: trace_idle.py run_kernel_trace.csv [top]"""
import csv
import sys

top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
segs, cur = [], None
for r in rows:
    if "logmel_tiles" in r["Kernel_Name"]:
        cur = []
        segs.append(cur)
    if cur is not None:
        cur.append(r)
s = segs[-1]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in s)
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
span = t1 - t0
gaps, end, prev = [], iv[0][1], iv[0][2]
for b, e, k in iv[1:]:
    if b > end:
        gaps.append((b - end, end, prev, k))
    if e > end:
        end, prev = e, k
idle = sum(g[0] for g in gaps)
print(f"last step: span {span / 1e6:.2f} ms, {len(s)} launches, GPU idle {idle / 1e6:.2f} ms "
      f"({100.0 * idle / span:.1f} %) in {len(gaps)} gaps, {sum(1 for g in gaps if g[0] > 5000)} longer than 5 us")
tenth = [0.0] * 10
for g, at, _, _ in gaps:
    tenth[min(9, int(10 * (at - t0) / span))] += g
print("idle ms per tenth of the step:", [round(v / 1e6, 2) for v in tenth])
for g, at, a, b in sorted(gaps, reverse=True)[:top]:
    print(f"  {g / 1e3:8.1f} us at {(at - t0) / 1e6:7.2f} ms  after {a}  before {b}")
