"""MSheath control step alone (asrx_msheath_ctrl_fwd3) and asrx_row_tiles, back-to-back launches on synthetic state;
ASRX_LIB selects the library build to time (A/B of kernel variants).  usage: python tools/ctrl_micro.py [B L D]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import lib  # noqa: E402

B, L, D = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (8, 6002, 768)
dev = torch.device("cuda:0")
P = lib.ptr
nl, i = 12, 3
nchunk = int(lib.load().asrx_mem_chunks(L))
rows = B * L
E = lambda *s: torch.rand(*s, device=dev)  # noqa: E731
policy, gp, ion = E(B, 3), E(B, 3), E(B, L)
mgw, mgb, memv, memw = E(D), E(1), E(B), E(D)
part, mem, js = E(B, nchunk, D), E(B, D), E(3)
next_i = torch.randint(0, 6, (B,), device=dev).float()
alpha, beta, gam, mwo, active, nxt = E(B), E(B), E(B, D), E(B, D), E(B), E(B)
rec = torch.empty(B * int(lib.load().asrx_msheath_rec_bytes()), dtype=torch.uint8, device=dev)
ntl = int(lib.load().asrx_row_tiles_max(rows))
tl, cnt = torch.empty(ntl, dtype=torch.int32, device=dev), torch.empty(1, dtype=torch.int32, device=dev)
st = lib.stream()
args = (P(policy), P(gp), 3, P(ion), P(mgw), P(mgb), P(memv), P(memw), 0, P(part), P(mem), P(js), P(next_i), i, nl, B,
        L, D, P(alpha), P(beta), P(gam), P(mwo), P(active), P(nxt), P(rec))


def f3():
    lib.call("asrx_msheath_ctrl_fwd3", *args, st)


def rt():
    lib.call("asrx_row_tiles", P(nxt), i + 1, L, rows, P(tl), P(cnt), st)


def t(fn, n=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


f3()
torch.cuda.synchronize()
m0 = mem.clone()
print(f"{os.path.basename(lib.LIB_PATH)} B={B} L={L} D={D} nchunk={nchunk}: ctrl_fwd3 {t(f3):.2f} us, row_tiles "
      f"{t(rt):.2f} us, mem checksum {float(m0.double().sum()):.9e}")
