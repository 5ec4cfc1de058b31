"""Launch census of one training step without a GPU: asrx.lib.call is replaced by a recorder and
the model runs on CPU tensors (kernels are not executed, values are garbage).  Lists every C-ABI
call with its problem sizes, so launch counts and GEMM shapes can be read off per step."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
import torch  # noqa: E402

from asrx import lib  # noqa: E402

calls = []
sites = []


def _record(name, *a):
    calls.append((name, a))
    f, chain = sys._getframe(1), []
    while f is not None and len(chain) < 3:
        fn = os.path.basename(f.f_code.co_filename)
        if fn not in ("gemm.py", "lib.py") and "torch" not in f.f_code.co_filename:
            chain.append(f"{fn}:{f.f_lineno}")
        f = f.f_back
    sites.append(" <- ".join(chain))


lib.call = _record
lib.require_gpu = lambda *t: None
class _FakeLib:
    """Size queries the host code makes (what the real library answers); everything else returns 64."""
    asrx_msheath_rec_bytes = staticmethod(lambda: 36)
    asrx_mem_chunks = staticmethod(lambda L: (L + 63) // 64)
    asrx_row_tiles_max = staticmethod(lambda M: (M + 127) // 128 + 64)
    asrx_jump_bwd_part_floats = staticmethod(lambda B, L, d: B * ((L + 127) // 128) * (2 * ((d // 4 + 31) // 32) + d))
    asrx_wconv_entry_bytes = staticmethod(lambda: 40)

    def __getattr__(self, name):
        return lambda *a: 64


lib.load = lambda: _FakeLib()

from asrx import prec, synth  # noqa: E402
from asrx.config import CONFIGS  # noqa: E402
from asrx.model import Model  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
prec.set_precision("bf16")
torch.cuda.current_stream = lambda *a: type("S", (), {"cuda_stream": 0})()
cfg = CONFIGS["tiny"]
model = Model(cfg).train()
model.set_noise(seed=0, step=0)
wav = synth.waveform(B, 30.0)
pitch = synth.pitch(B)
ids, labels = synth.text(B, 256, cfg.tokens)
spec = torch.zeros(B, 128, 3001)
wf = torch.zeros(B, 1, 3000)
from torch.profiler import ProfilerActivity, profile  # noqa: E402

# torch-side device work of the step (copies, fills, cats, elementwise ops outside the library): on the
# GPU every one of these aten ops is a kernel (or a copy / fill) launch of its own
with profile(activities=[ProfilerActivity.CPU]) as prof:
    out = model(labels=labels, text_ids=ids, spectrogram=spec, pitch=pitch, waveform=wf)
    nf = len(calls)
    out["loss"].backward()
LAUNCHING = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::cat", "aten::add_", "aten::mul", "aten::add",
             "aten::sub", "aten::div", "aten::where", "aten::index", "aten::gather", "aten::scatter", "aten::sum",
             "aten::mean", "aten::clamp", "aten::neg", "aten::exp", "aten::log", "aten::masked_fill_",
             "aten::_to_copy", "aten::stack", "aten::index_put_", "aten::cumsum", "aten::ones_like",
             "aten::zeros_like", "aten::mul_", "aten::div_", "aten::max", "aten::argmax", "aten::eq", "aten::ne",
             "aten::lt", "aten::gt", "aten::ge", "aten::le", "aten::any", "aten::all", "aten::pow", "aten::sqrt")
tops = collections.Counter()
for ev in prof.key_averages():
    if ev.key in LAUNCHING:
        tops[ev.key] += ev.count
print("torch ops that launch on a GPU (top-level counts include nested):", sum(tops.values()))
for k, v in tops.most_common(20):
    print(f"{v:6d} {k}")
c = collections.Counter(n for n, _ in calls)
print(f"calls fwd {nf} bwd {len(calls)-nf}")
for n, v in c.most_common():
    print(f"{v:6d} {n}")
g = collections.Counter()
for n, a in calls:
    if n == "asrx_gemm_wn":
        g[("wn", a[11], a[12], a[13], a[17], a[2])] += 1  # M N K nj conv
    elif n == "asrx_gemm":
        g[("gemm", a[16], a[17], a[18], a[19], a[4], a[9])] += 1  # M N K batch a_kc b_kc
for k, v in sorted(g.items(), key=lambda kv: -kv[1] * kv[0][1] * kv[0][2] * kv[0][3]):
    print(v, k)
ge = collections.Counter()
for n, a in calls:
    if n == "asrx_gemm_wn_ex" and a[18] != 0:
        ge[("wn_ex act", a[13], a[14], a[15], a[18], "Z" if a[12] else "-", "ab" if a[1] else "a32")] += 1
    elif n == "asrx_act_bwd_bias":
        ge[("act_bwd_bias", a[4], a[5], a[6])] += 1
    elif n == "asrx_gemm_wn_gact":
        ge[("gact", a[11], a[12], a[13], a[14])] += 1
for k, v in sorted(ge.items(), key=lambda kv: -kv[1]):
    print(v, k)
gf = collections.Counter()
for (n, a), site in zip(calls, sites):
    if n == "asrx_gemm_wn_ex" and not a[1] and (a[13] >= 32768 or os.environ.get("CENSUS_ALL")):
        gf[("fp32-A", a[13], a[14], a[15], "nj", a[19], "conv" if a[3] else "", "act", a[18], "Z" if a[12] else "",
            "beta" if a[17] else "", "cb" if a[9] else "", site)] += 1
    elif n in ("asrx_gemm_wn_res", "asrx_gemm_wn_router") and a[-5 if n == "asrx_gemm_wn_res" else -4] >= 32768:
        gf[(n,) + tuple(a[-5:-1])] += 1
for k, v in sorted(gf.items(), key=lambda kv: -kv[1]):
    print(v, k)
