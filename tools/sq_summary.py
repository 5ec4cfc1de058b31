"""Summarise a rocprofv3 --pmc counter_collection.csv of the SQ issue / wait counters (tools/gpu_sq_pmc.sh):
per kernel (name prefix) and grid size, the mean per dispatch of each counter and the wave-cycle split
(SQ_WAIT_ANY = parked on s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue stall, SQ_ACTIVE_INST_ANY = issuing;
MI355X_MICROARCH.md rocprofv3 section).  usage: sq_summary.py run_counter_collection.csv [name-regex]"""
import collections
import csv
import re
import sys

pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else "asrx")
acc = collections.defaultdict(lambda: collections.defaultdict(list))
meta = {}
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"]
    if not pat.search(name):
        continue
    key = (name[:70], int(r["Grid_Size"]))
    acc[key][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    meta[key] = (r["VGPR_Count"], r["LDS_Block_Size"])
for key, d in acc.items():
    per = collections.defaultdict(list)
    for (disp, cn), vals in d.items():
        per[cn].append(sum(vals))
    m = {cn: sum(v) / len(v) for cn, v in per.items()}
    n = len(next(iter(per.values())))
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{key[0]}  grid {key[1]}  vgpr {meta[key][0]}  lds {meta[key][1]}  dispatches {n}")
    print("   wave-cycles split: wait %.2f  issue-stall %.2f  active %.2f   (wait_inst_lds %.2f)" % (
        m.get("SQ_WAIT_ANY", 0) / wc, m.get("SQ_WAIT_INST_ANY", 0) / wc, m.get("SQ_ACTIVE_INST_ANY", 0) / wc,
        m.get("SQ_WAIT_INST_LDS", 0) / wc))
    print("   " + "  ".join(f"{cn}={v:.3g}" for cn, v in sorted(m.items())))
