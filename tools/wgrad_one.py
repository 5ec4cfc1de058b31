"""One weight-gradient GEMM shape, a few launches (for rocprofv3 --pmc passes); not product code."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import gemm as G  # noqa: E402

R, N, K = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (192064, 384, 384)))
dev = torch.device("cuda:0")
dy = torch.randn(R, N, device=dev)
x = torch.randn(R, K, device=dev)
out = torch.zeros(N, K, device=dev)
for _ in range(3):
    G.linear_wgrad(dy, x, out=out, accumulate=True)
torch.cuda.synchronize()
print("ok")
