"""MFMA utilisation per kernel from one rocprofv3 --pmc pass (SQ_VALU_MFMA_BUSY_CYCLES,
SQ_INSTS_MFMA, GRBM_GUI_ACTIVE) plus its kernel trace (tools/gpu_mfma_pmc.sh).
util = MFMA busy cycles / (kernel cycles x 1024 SIMDs), kernel cycles = GRBM_GUI_ACTIVE / 8 (the
counter is summed over the 8 XCDs, MI355X_MICROARCH.md 'DVFS give-back'); busy cycles are per SIMD
(32 per 32x32x16 and 16 per 16x16x32 bf16 MFMA, same section), which the cycles-per-MFMA column
checks.  usage: pmc_mfma.py <counter_collection.csv> [min launches]"""
import collections
import csv
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    d = r.get("Dispatch_Id") or r.get("Correlation_Id")
    vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(d)
rows = []
for k, c in vals.items():
    n = max(len(disp[k]), 1)
    busy, insts, gui = c["SQ_VALU_MFMA_BUSY_CYCLES"], c["SQ_INSTS_MFMA"], c["GRBM_GUI_ACTIVE"]
    if busy == 0:
        continue
    util = busy / (gui / 8.0 * 1024.0) if gui > 0 else 0.0
    rows.append((busy, k, n, util, busy / insts if insts else float('nan'), gui / 8.0 / n))
print("kernel,launches,mfma_util,busy_cycles_per_mfma,avg_kernel_cycles,share_of_mfma_busy")
tot = sum(r[0] for r in rows)
for busy, k, n, util, cpm, cyc in sorted(rows, reverse=True):
    print(f'"{k[:90]}",{n},{util:.4f},{cpm:.1f},{cyc:.0f},{busy / tot:.3f}')
