"""Per-(kernel, grid) durations from a rocprofv3 kernel trace (graph replay: real kernel times, no
host gaps).  usage: trace_shapes.py <run_kernel_trace.csv> [steps] [top]"""
import collections
import csv
import sys

steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
top = int(sys.argv[3]) if len(sys.argv) > 3 else 45
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    k = (r["Kernel_Name"][:80], f'{r["Grid_Size_X"]}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]}', r["VGPR_Count"],
         r["Scratch_Size"])
    d[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in d.values())
rows = sorted(((sum(v) / steps / 1e3, len(v) / steps, sum(v) / len(v) / 1e3, k) for k, v in d.items()), reverse=True)
print(f"kernel time per step {tot / steps / 1e6:.1f} ms")
for x in rows[:top]:
    print(f"{x[0]:8.1f} us/step {x[1]:6.1f}/step {x[2]:8.1f} us  grid {x[3][1]:>14} vgpr {x[3][2]:>3} scr {x[3][3]:>3} {x[3][0]}")
