"""Model.generate (model.py:674-701): the hoisted audio side + last-block decode
must reproduce the naive reference loop (full processor forward with seq=True over the prefix at
every step, all blocks) token for token, with the same keyed noise."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("layer", [2, 4])
def test_generate_matches_naive_loop(cuda, layer):
    from asrx import prec
    from asrx.config import Dimensions
    from asrx.model import Model
    from asrx.noise import NoiseCtx

    torch.manual_seed(0)
    m = Model(Dimensions(tokens=60, mels=128, dims=128, head=2, layer=layer, act="gelu", n_type="AbbyNormal")).to(cuda)
    g = torch.Generator().manual_seed(3)
    B, S = 2, 101
    spec = torch.randn(B, 128, S, generator=g).to(cuda)
    pitch = (torch.rand(B, 1, S, generator=g) * 200).to(cuda)
    wav = (torch.randn(B, 1, S - 1, generator=g) * 0.1).to(cuda)
    m.set_noise(5, 7)
    steps = 6
    with prec.precision("fp32"):
        y = m.generate(spectrogram=spec, pitch=pitch, waveform=wav, max_new_tokens=steps)
        # naive: the reference loop, every block, full forward at each step
        with torch.no_grad():
            noise = NoiseCtx(5, 7, False)
            enc = m.enc.encode([pitch, spec, wav], noise, B)
            xa = {"a": enc[0], "b": enc[1], "c": enc[2]}
            yn = torch.ones(B, 1, dtype=torch.long, device=cuda)
            first_logits = None
            for _ in range(steps):
                logits = m.processor(yn, xa, noise, seq=True)
                if first_logits is None:
                    first_logits = logits
                nxt = logits[:, -1].argmax(-1, keepdim=True)
                yn = torch.cat((yn, nxt), 1)
                if bool((nxt == 2).all()):
                    break
            kv = m.processor.audio_cache(xa, noise, B)
            dl = m.processor.decode_logits(torch.ones(B, 1, dtype=torch.long, device=cuda), kv, noise)
    assert y.shape[0] == B and y.shape[1] <= steps + 1 and bool((y[:, 0] == 1).all())
    assert torch.equal(y, yn)
    assert torch.allclose(dl, first_logits, rtol=0, atol=1e-5 * float(first_logits.abs().max()))
