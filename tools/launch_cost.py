"""Host cost of issuing work on the GPU box (calibration, not product): N small asrx launches (asrx_zero of 4 KB)
issued eagerly, and the same N captured in one HIP graph and replayed, each while the stream is held busy by a
long spin kernel (so the issue time is not hidden behind execution; N is kept below the queue depth); and
torch.empty on the device.  usage: launch_cost.py [N]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import lib  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 500
dev = torch.device("cuda:0")
buf = torch.empty(1024, device=dev)


def issue():
    for _ in range(N):
        lib.call("asrx_zero", lib.ptr(buf), 4096, lib.stream())


issue()
torch.cuda.synchronize()
for rep in range(3):
    torch.cuda._sleep(200_000_000)
    t0 = time.perf_counter()
    issue()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"eager: {N} launches issued in {(t1 - t0) * 1e3:.2f} ms = {(t1 - t0) / N * 1e6:.2f} us/launch", flush=True)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    issue()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    issue()
torch.cuda.synchronize()
for rep in range(3):
    torch.cuda._sleep(200_000_000)
    t0 = time.perf_counter()
    g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"graph: replay of {N} nodes issued in {(t1 - t0) * 1e3:.2f} ms = {(t1 - t0) / N * 1e6:.2f} us/node", flush=True)
t0 = time.perf_counter()
for _ in range(N):
    torch.empty(384 * 1000, device=dev)
t1 = time.perf_counter()
print(f"torch.empty (cached): {(t1 - t0) / N * 1e6:.2f} us")
t0 = time.perf_counter()
for _ in range(N):
    torch.cuda.current_stream().cuda_stream
t1 = time.perf_counter()
print(f"torch.cuda.current_stream().cuda_stream: {(t1 - t0) / N * 1e6:.2f} us; lib.stream(): ", end="")
t0 = time.perf_counter()
for _ in range(N):
    lib.stream()
print(f"{(time.perf_counter() - t0) / N * 1e6:.2f} us")
