"""Debug aid (GPU box): run one forward with bf16 activation storage off and on, record the hard
decisions of both, and print the first sites (in execution order) where they differ."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import decisions, prec  # noqa: E402
from asrx.config import Dimensions  # noqa: E402
from asrx.model import Model  # noqa: E402
from asrx.noise import site_key  # noqa: E402

torch.manual_seed(0)
layer = int(sys.argv[1]) if len(sys.argv) > 1 else 2
cfg = Dimensions(tokens=1000, mels=128, dims=384, head=6, layer=layer, act="gelu", n_type="AbbyNormal")
model = Model(cfg).cuda().train()
g = torch.Generator().manual_seed(4)
B, T, S = 2, 16, 1001
spec = torch.randn(B, 128, S, generator=g).cuda()
pitch = (torch.rand(B, 1, S, generator=g) * 200).cuda()
wav = (torch.randn(B, 1, S - 1, generator=g) * 0.1).cuda()
ids = torch.randint(3, 1000, (B, T), generator=g)
ids[:, 0] = 1
labels = torch.cat([ids[:, 1:], torch.full((B, 1), 2)], 1).cuda()
ids = ids.cuda()
names = {}
for i in range(layer):
    for base in ("ta", "tb", "tc", "td", "tg", "audio", "xa", "tg.xa"):
        for suf in ("", ".ln0", ".ln1", ".ln2", ".mlp.ln0", ".mlp.ln1", ".ln", ".sa.q", ".sa.kv", ".sa.qh", ".sa.kh",
                    ".ca.q", ".ca.kv", ".ca.qh", ".ca.kh", ".jump"):
            names[site_key(3, 1, f"b{i}.{base}{suf}")] = f"b{i}.{base}{suf}"
names[site_key(3, 1, "final.ln")] = "final.ln"
conc = len(sys.argv) <= 2 or sys.argv[2] != "serial"
model.processor.concurrent_dead_text = conc
print("concurrent dead text:", conc)
modes = [False, True, True, False]
recs = []
for on in modes:
    model.set_noise(3, 1)
    decisions.enable()
    with prec.precision("bf16"), prec.storage(on), torch.no_grad():
        out = model(labels=labels, text_ids=ids, spectrogram=spec, pitch=pitch, waveform=wav)
    torch.cuda.synchronize()
    recs.append((decisions.disable(), out["logits"].float().cpu()))
for i, j in ((0, 3), (1, 2), (0, 1)):
    print(f"run {i} ({modes[i]}) vs run {j} ({modes[j]}): logits equal", torch.equal(recs[i][1], recs[j][1]))
a, b = recs[0][0], recs[1][0]
n = 0
for k in a:
    if k not in b:
        print("missing", k)
        continue
    va, vb = a[k], b[k]
    same = (va == vb) if not torch.is_tensor(va) else torch.equal(va, vb)
    if not same:
        print("DIFF", k[0], names.get(k[1], k[1]), k[2:], "" if not torch.is_tensor(va) else int((va != vb).sum()))
        n += 1
        if n > 12:
            break
print("decisions:", len(a), "first diffs shown:", n)
