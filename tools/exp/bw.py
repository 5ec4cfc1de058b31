import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..")]
import torch
from microbench import timeit
dev = torch.device("cuda:0")
for n in (192064 * 384, 96032 * 1536):
    x = torch.empty(n, device=dev)
    y = torch.empty(n, device=dev)
    t = timeit(lambda: x.fill_(1.0))
    print(f"fill {n*4/1e6:.0f} MB: {t*1e6:.1f} us {n*4/t/1e9:.0f} GB/s")
    t = timeit(lambda: y.copy_(x))
    print(f"copy {n*4/1e6:.0f} MB: {t*1e6:.1f} us {2*n*4/t/1e9:.0f} GB/s (r+w)")
    t = timeit(lambda: x.sum())
    print(f"sum {n*4/1e6:.0f} MB: {t*1e6:.1f} us {n*4/t/1e9:.0f} GB/s")
