"""Per-kernel HBM traffic per launch from the FETCH_SIZE / WRITE_SIZE rocprofv3 passes of
tools/prof3.sh (MI355X_MICROARCH.md HBM: FETCH_SIZE is KB and reports half of a wide streaming
read on gfx950, so it is doubled; WRITE_SIZE is KB, exact for 16-B stores).
usage: pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> [name filter]"""
import collections
import csv
import sys


def load(path, ctr):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == ctr:
            per[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return per


fetch = load(sys.argv[1], "FETCH_SIZE")
write = load(sys.argv[2], "WRITE_SIZE")
pat = sys.argv[3] if len(sys.argv) > 3 else ""
print("kernel,launches,avg_fetch_bytes_x2,avg_write_bytes,avg_hbm_bytes")
rows = []
for k in fetch:
    if pat not in k:
        continue
    f = 2.0 * sum(fetch[k]) / len(fetch[k])
    w = sum(write.get(k, [0.0])) / max(len(write.get(k, [])), 1)
    rows.append((f + w, k, len(fetch[k]), f, w))
for tot, k, n, f, w in sorted(rows, reverse=True):
    print(f'"{k[:90]}",{n},{f:.0f},{w:.0f},{tot:.0f}')
