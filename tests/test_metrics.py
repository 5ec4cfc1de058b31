"""WER / compute_metrics (essentials.py:576-670) and the tokenizer glue (248-292): known answers, the
oracle's literal full-matrix restatement on random word sequences, and (when the reference's
tokenizer.json is present in this container) a decode round trip."""
import os
import random

import numpy as np
import pytest

from asrx import metrics
from oracle import metrics as om


@pytest.mark.parametrize("ref,hyp,dist", [
    ("", "", 0), ("a b c", "", 3), ("", "x y", 2), ("the cat sat", "the cat sat", 0),
    ("the cat sat", "the bat sat", 1),                # one substitution
    ("the cat sat on the mat", "the cat on the mat", 1),  # one deletion
    ("a b", "a x b", 1),                              # one insertion
    ("kitten sitting", "sitting kitten", 2),
    ("a b c d e f", "f e d c b a", 6),
])
def test_levenshtein_known_answers(ref, hyp, dist):
    assert metrics.levenshtein(ref.split(), hyp.split()) == dist
    assert om.levenshtein(ref.split(), hyp.split()) == dist


def test_wer_known_answers():
    # 1 substitution + 1 deletion over 3 + 4 reference words; case-insensitive
    assert metrics.wer_batch(["The Cat sat", "a b c d"], ["the bat SAT", "a b d"]) == pytest.approx(200 / 7)
    assert metrics.wer_batch([], []) == 0.0
    assert metrics.wer_batch([""], ["extra words"]) == 0.0  # no reference words -> 0 (essentials.py:602)


def test_wer_matches_oracle_random():
    rng = random.Random(0)
    vocab = [f"w{i}" for i in range(12)]
    refs, hyps = [], []
    for _ in range(200):
        refs.append(" ".join(rng.choice(vocab) for _ in range(rng.randint(0, 15))))
        hyps.append(" ".join(rng.choice(vocab) for _ in range(rng.randint(0, 15))))
    for r, h in zip(refs, hyps):
        assert metrics.levenshtein(r.split(), h.split()) == om.levenshtein(r.split(), h.split())
    assert metrics.wer_batch(refs, hyps) == om.wer_batch(refs, hyps)


class _Tok:
    """Minimal stand-in tokenizer: id i -> word 'w<i>'."""

    def batch_decode(self, ids_list):
        return [" ".join(f"w{i}" for i in ids) for ids in ids_list]


def test_compute_metrics_cleans_and_argmaxes():
    labels = np.array([[5, 6, 7, 2, 0, 0], [8, 9, 2, 0, 0, 0]])
    preds = np.array([[1, 5, 6, 9, 2, 0], [1, 8, 9, 2, 0, 0]])
    r = metrics.compute_metrics({"predictions": preds, "label_ids": labels}, tokenizer=_Tok())
    assert r["wer"] == pytest.approx(100 * 1 / 5)
    logits = np.eye(12)[preds]  # (B, T, V): argmaxed like the reference (essentials.py:633-634)
    r2 = metrics.compute_metrics({"predictions": (logits,), "label_ids": labels}, tokenizer=_Tok())
    assert r2["wer"] == r["wer"]
    assert metrics.clean_ids([1, 4, -100, 0, 2, 3]) == [4, 3]


TOK = "/root/reference/tokenizer.json"


@pytest.mark.skipif(not os.path.exists(TOK), reason="reference tokenizer.json not present")
def test_setup_tokenizer_round_trip():
    tok = metrics.setup_tokenizer(TOK)
    assert (tok.pad_token_id, tok.bos_token_id, tok.eos_token_id) == (0, 1, 2)
    ids = tok.encode("hello world this is a test")
    text = tok.batch_decode([[1] + ids + [2, 0, 0]])[0]
    assert metrics.wer_batch(["hello world this is a test"], [text]) == 0.0
