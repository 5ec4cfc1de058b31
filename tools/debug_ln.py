import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch
from asrx import lib, gemm as G, prec
dev = torch.device("cuda")
g = torch.Generator().manual_seed(0)
rows, D = 2002, 384
x = (torch.randn(rows, D, generator=g) * 3).to(dev)
w = torch.randn(D, generator=g).to(dev); b = torch.randn(D, generator=g).to(dev)
gw = torch.randn(D, generator=g).to(dev); gb = torch.randn(1, generator=g).to(dev)
outs = []
for yb in (0, 1):
    y = torch.empty(rows, D, device=dev, dtype=torch.bfloat16 if yb else torch.float32)
    m, r, gt = (torch.empty(rows, device=dev) for _ in range(3))
    lib.call("asrx_layernorm_fwd3", lib.ptr(x), lib.ptr(w), lib.ptr(b), lib.ptr(y), yb, lib.ptr(m), lib.ptr(r), None,
             lib.ptr(gw), lib.ptr(gb), lib.ptr(gt), 1, rows, D, 1e-5, lib.stream())
    outs.append(y)
torch.cuda.synchronize()
print("LN bf16 == round(LN fp32):", torch.equal(outs[1], outs[0].to(torch.bfloat16)),
      int((outs[1] != outs[0].to(torch.bfloat16)).sum()))
W = (torch.randn(1536, D, generator=g) / D ** 0.5).to(dev); bias = torch.randn(1536, generator=g).to(dev)
with prec.precision("bf16"):
    y32 = G.linear_fwd(outs[0], W, bias, act="silu")
    y16 = G.linear_fwd(outs[1], W, bias, act="silu")
    yr = G.linear_fwd(outs[0].to(torch.bfloat16).float(), W, bias, act="silu")
torch.cuda.synchronize()
print("GEMM fp32-A vs bf16-A equal:", torch.equal(y32, y16), "vs rounded-fp32:", torch.equal(yr, y16),
      float((y32 - y16).abs().max()))
