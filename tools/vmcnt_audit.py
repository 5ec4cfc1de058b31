"""Loop-level s_waitcnt audit of a gfx950 assembly listing (hipcc --offload-device-only -S): per kernel matching
the regex, every loop with its number of vmcnt(0) waits and the counted waits, to find prefetch pipelines the
compiler drains every iteration.  usage: vmcnt_audit.py file.s regex"""
import collections
import re
import sys

L = open(sys.argv[1]).read().splitlines()
pat = re.compile(sys.argv[2])
name = None
loops = collections.OrderedDict()
cur = None


def flush():
    if name and pat.search(name):
        print(name[:90])
        for lab, w in loops.items():
            print(f"  loop {lab}: {len(w)} vmcnt waits, {w.count(0)} x vmcnt(0), counted {sorted(set(w))[:14]}")


for t in L:
    m = re.match(r"^(_Z\w+):", t)
    if m:
        flush()
        name, loops, cur = m.group(1), collections.OrderedDict(), None
        continue
    lab = re.match(r"^\.(LBB\w+):(.*)", t)
    if lab:
        h = re.search(r"Loop Header: Depth=\d+", lab.group(2))
        g = re.search(r"in Loop: Header=(\w+)", lab.group(2))
        cur = lab.group(1).replace("LBB", "BB") if h else (g.group(1) if g else None)
        if cur:
            loops.setdefault(cur, [])
        continue
    if cur:
        w = re.search(r"s_waitcnt.*vmcnt\((\d+)\)", t)
        if w:
            loops[cur].append(int(w.group(1)))
flush()
