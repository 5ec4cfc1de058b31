"""GPU debug aid: fp32 parity attention on the model's regime -- scores of 1e3-1e4 (rotary scales q / k by
the source row norm), near one-hot softmax rows -- against float64, next to torch's own fp32 (CPU) on
the same inputs.  Prints max relative output / gradient errors of both."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from asrx import ops, prec  # noqa: E402


def ref(q, k, v, causal):
    s = (q.transpose(1, 2) @ k.transpose(1, 2).transpose(-1, -2)) / q.shape[-1] ** 0.5
    if causal:
        s = s.masked_fill(torch.ones(s.shape[-2], s.shape[-1], dtype=torch.bool).triu(1), float("-inf"))
    return (torch.softmax(s, -1) @ v.transpose(1, 2)).transpose(1, 2)


def rel(a, b):
    return float((a - b).abs().max() / b.abs().max())


for (B, Lq, Lk, H, hd, mag, causal) in [(2, 64, 1001, 6, 64, 30.0, False), (2, 64, 64, 6, 64, 30.0, True),
                                         (1, 256, 3001, 6, 64, 30.0, False), (2, 64, 1001, 6, 64, 3.0, False)]:
    g = torch.Generator().manual_seed(B + Lq + Lk)
    q = torch.randn(B, Lq, H, hd, generator=g, dtype=torch.float64) * mag
    k = torch.randn(B, Lk, H, hd, generator=g, dtype=torch.float64) * mag
    v = torch.randn(B, Lk, H, hd, generator=g, dtype=torch.float64)
    go = torch.randn(B, Lq, H, hd, generator=g, dtype=torch.float64)
    q32, k32, v32 = (t.float() for t in (q, k, v))
    # float64 reference on the fp32-rounded inputs
    qd, kd, vd = (t.double().requires_grad_(True) for t in (q32, k32, v32))
    od = ref(qd, kd, vd, causal)
    od.backward(go)
    # torch fp32 CPU
    qc, kc, vc = (t.clone().requires_grad_(True) for t in (q32, k32, v32))
    oc = ref(qc, kc, vc, causal)
    oc.backward(go.float())
    # HIP fp32 parity kernels
    qg, kg, vg = (t.cuda().requires_grad_(True) for t in (q32, k32, v32))
    with prec.precision("fp32"):
        og = ops.attention(qg, kg, vg, causal)
        og.backward(go.float().cuda())
    torch.cuda.synchronize()
    s = (q32.double().transpose(1, 2) @ k32.double().transpose(1, 2).transpose(-1, -2)) / hd ** 0.5
    print(f"B{B} Lq{Lq} Lk{Lk} mag{mag} causal{causal}: |s|max {float(s.abs().max()):.0f}")
    print(f"   out   cpu32 {rel(oc.double(), od):.2e}   hip32 {rel(og.double().cpu(), od):.2e}")
    for nm, a, c, d in (("dq", qc.grad, qg.grad, qd.grad), ("dk", kc.grad, kg.grad, kd.grad),
                        ("dv", vc.grad, vg.grad, vd.grad)):
        print(f"   {nm}    cpu32 {rel(a.double(), d):.2e}   hip32 {rel(c.double().cpu(), d):.2e}")
