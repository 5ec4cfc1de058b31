"""Static instruction mix of device functions in a gfx950 assembly listing (hipcc --cuda-device-only -S):
per matching kernel, total / VALU / transcendental / LDS / global / scratch instruction counts and the most
frequent opcodes.  usage: isa_count.py file.s regex"""
import collections
import re
import sys

L = open(sys.argv[1]).read().splitlines()
pat = re.compile(sys.argv[2])
for i, l in enumerate(L):
    m = re.match(r"^(_Z\w+):", l)
    if not m or not pat.search(m.group(1)):
        continue
    ins = []
    for t in L[i + 1:]:
        t = t.strip()
        if t.startswith("s_endpgm") or t.startswith(".Lfunc_end"):
            break
        if t and not t.startswith((".", ";")) and not t.endswith(":"):
            ins.append(t.split()[0])
    c = collections.Counter(ins)
    pick = lambda *p: sum(n for k, n in c.items() if k.startswith(p))  # noqa: E731
    print(m.group(1)[:70])
    print(f"  total {len(ins)}  valu {pick('v_')}  salu {pick('s_')}  trans "
          f"{pick('v_exp_', 'v_log_', 'v_rcp_', 'v_sqrt_', 'v_rsq_')}  div_fixup {c['v_div_fixup_f32']}  "
          f"lds {pick('ds_')}  global {pick('global_')}  scratch {pick('scratch_', 'buffer_')}  "
          f"dpp {sum(1 for k in ins if '_dpp' in k)}")
    print("  top", c.most_common(16))
