"""Debug aid (GPU box): bisect which bf16-storage site changes the forward (variants switch sites off)."""
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
g = torch.Generator().manual_seed(4)
B, T, S = 2, 16, 1001
spec = torch.randn(B, 128, S, generator=g).cuda()
pitch = (torch.rand(B, 1, S, generator=g) * 200).cuda()
wav = (torch.randn(B, 1, S - 1, generator=g) * 0.1).cuda()
ids = torch.randint(3, 1000, (B, T), generator=g)
ids[:, 0] = 1
ids = ids.cuda()


def run(on, patch=None):
    saved = {}
    if patch:
        for mod, attr, val in patch:
            saved[(mod, attr)] = getattr(mod, attr)
            setattr(mod, attr, val)
    try:
        model.set_noise(3, 1)
        with prec.precision("bf16"), prec.storage(on), torch.no_grad():
            return model(text_ids=ids, spectrogram=spec, pitch=pitch, waveform=wav)["logits"].float().cpu()
    finally:
        for (mod, attr), v in saved.items():
            setattr(mod, attr, v)


off = run(False)
fake_prec = types.SimpleNamespace(**{k: getattr(prec, k) for k in dir(prec) if not k.startswith("__")})
fake_prec.bf16_storage = lambda: False
fake_prec.attn_bf16_io = lambda: False
variants = {
    "all_on": None,
    "msheath_off": [(msheath, "prec", fake_prec)],
    "ops_off": [(ops, "prec", fake_prec)],
    "model_off": [(M, "prec", fake_prec)],
    "ops_model_off": [(ops, "prec", fake_prec), (M, "prec", fake_prec)],
}
for name, patch in variants.items():
    y = run(True, patch)
    print(f"{name:16s} equal to off: {torch.equal(y, off)}  max diff {float((y - off).abs().max()):.4g}")
