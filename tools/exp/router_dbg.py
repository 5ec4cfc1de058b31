import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch
from asrx import gemm as G
dev = torch.device("cuda:0")
for M in (3001, 12000, 3000, 128, 1024, 2048, 4096, 8192):
    N = 384
    g = torch.Generator().manual_seed(M)
    x = torch.randn(M, N, generator=g).to(dev)
    W1 = (torch.randn(N, N, generator=g) / N ** 0.5).to(dev)
    b1 = torch.randn(N, generator=g).to(dev)
    W2 = (torch.randn(3, N, generator=g) / N ** 0.5).to(dev)
    ref_h = x.to(torch.bfloat16).double() @ W1.to(torch.bfloat16).double().t() + b1.double()
    ref_l = torch.nn.functional.silu(ref_h) @ W2.double().t()
    for keep in (True, False):
        h, l = G.router_fwd(x, W1, b1, W2, keep)
        err = (l.double() - ref_l).abs().max(dim=1).values
        bad = (err > 1e-3).nonzero().flatten()
        print(M, keep, "bad rows", bad.numel(), bad[:10].tolist(), flush=True)
