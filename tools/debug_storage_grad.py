"""Debug aid (GPU box): bf16 storage on vs off -- per-parameter gradient differences (relative to the
model's largest gradient), with variants that switch storage sites off, to locate a backward that
differs by more than the attention-Delta rounding."""
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import msheath, ops, prec  # noqa: E402
from asrx import model as M  # noqa: E402
from asrx.config import Dimensions  # noqa: E402
from asrx.model import Model  # noqa: E402

torch.manual_seed(0)
cfg = Dimensions(tokens=1000, mels=128, dims=384, head=6, layer=2, act="gelu", n_type="AbbyNormal")
model = Model(cfg).cuda().train()
model.fused_ce = False  # both runs through the same (unfused) logits + CE
g = torch.Generator().manual_seed(4)
B, T, S = 2, 16, 1001
spec = torch.randn(B, 128, S, generator=g).cuda()
pitch = (torch.rand(B, 1, S, generator=g) * 200).cuda()
wav = (torch.randn(B, 1, S - 1, generator=g) * 0.1).cuda()
ids = torch.randint(3, 1000, (B, T), generator=g)
ids[:, 0] = 1
labels = torch.cat([ids[:, 1:], torch.full((B, 1), 2)], 1).cuda()
ids = ids.cuda()


def run(on, patch=None, prec_mode="bf16"):
    saved = {}
    if patch:
        for mod, attr, val in patch:
            saved[(mod, attr)] = getattr(mod, attr)
            setattr(mod, attr, val)
    try:
        model.zero_grad(set_to_none=True)
        model.set_noise(3, 1)
        with prec.precision(prec_mode), prec.storage(on):
            out = model(labels=labels, text_ids=ids, spectrogram=spec, pitch=pitch, waveform=wav)
            out["loss"].backward()
        torch.cuda.synchronize()
        return float(out["loss"]), {n: p.grad.detach().double().cpu().clone() for n, p in model.named_parameters()
                                    if p.grad is not None}
    finally:
        for (mod, attr), v in saved.items():
            setattr(mod, attr, v)


l0, off = run(False)
l0b, off2 = run(False)
gmax = max(float(v.abs().max()) for v in off.values())
print("loss", l0, "repeat identical:", all(torch.equal(off[n], off2[n]) for n in off))
fake_prec = types.SimpleNamespace(**{k: getattr(prec, k) for k in dir(prec) if not k.startswith("__")})
fake_prec.bf16_storage = lambda: False
fake_prec.attn_bf16_io = lambda: False

def _force_off(fn, pos=None):
    def w(*a, **k):
        if "out_bf16" in k:
            k["out_bf16"] = False
        if pos is not None and len(a) > pos:
            a = a[:pos] + (False,) + a[pos + 1:]
        return fn(*a, **k)
    return w


fake_io = types.SimpleNamespace(**{k: getattr(prec, k) for k in dir(prec) if not k.startswith("__")})
fake_io.attn_bf16_io = lambda: False
variants = {
    "all_on": None,
    "ops_off": [(ops, "prec", fake_prec)],
    "linear_off": [(ops, "linear", _force_off(ops.linear))],
    "abby_off": [(ops, "abby_normal", _force_off(ops.abby_normal, 7))],
    "attn_off": [(ops, "attention", _force_off(ops.attention))],
    "tgate_off": [(ops, "tgate", _force_off(ops.tgate))],
    "attn_io_off": [(M, "prec", fake_io), (ops, "prec", fake_io)],
}
for name, patch in variants.items():
    l1, on = run(True, patch)
    rows = sorted(((float((on[n] - off[n]).abs().max()) / gmax, float(off[n].abs().max()) / gmax,
                    float(on[n].abs().max()) / gmax, n) for n in off), reverse=True)
    print(f"== {name}: loss {l1} (off {l0})")
    for r in rows[:8]:
        print(f"   diff {r[0]:.3e}  |off| {r[1]:.3e}  |on| {r[2]:.3e}  {r[3]}")
