"""Do kernels on two HIP streams overlap, and does a rocprofv3 kernel trace show it?  Two 1-workgroup spin kernels
(torch.cuda._sleep) on two streams: the wall time says whether they ran together; under rocprofv3 --kernel-trace the
trace's timestamps say whether the profiler saw (or forced) the same.  usage: python tools/conc_check.py"""
import time

import torch

torch.cuda.init()
a, b = torch.cuda.Stream(), torch.cuda.Stream()
cyc = 20_000_000
torch.cuda._sleep(1000)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    with torch.cuda.stream(a):
        torch.cuda._sleep(cyc)
    with torch.cuda.stream(b):
        torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    t2 = time.perf_counter() - t0
    t0 = time.perf_counter()
    with torch.cuda.stream(a):
        torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    t1 = time.perf_counter() - t0
    print(f"one spin {t1 * 1e3:.2f} ms, two spins on two streams {t2 * 1e3:.2f} ms", flush=True)
