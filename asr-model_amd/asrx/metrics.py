"""Evaluation metrics of the reference (essentials.py:576-670) and its tokenizer glue (248-295), for
the greedy-decode WER of BASELINE configs[4].  Host-side text processing: the decoded ids come back
from the device once per batch (Model.generate), so there is nothing here for the GPU to do.

Same names, argument meaning and results as the reference:
  levenshtein(reference_words, hypothesis_words) -> int          essentials.py:576-592
  wer_batch(references, hypotheses) -> float (percent)           essentials.py:594-602
  compute_metrics(pred, tokenizer, model=None, ...) -> dict      essentials.py:612-670
  clean_ids / clean_batch                                        essentials.py:248-254
  setup_tokenizer(path) -> tokenizers.Tokenizer with the reference's encode/batch_decode/decode
                                                                 essentials.py:256-292
levenshtein keeps two DP rows instead of the reference's full matrix (same distance, O(n) memory).
"""
from __future__ import annotations

import os

import numpy as np

PAD, BOS, EOS = 0, 1, 2


def levenshtein(reference_words, hypothesis_words) -> int:
    m, n = len(reference_words), len(hypothesis_words)
    prev = list(range(n + 1))
    for q in range(1, m + 1):
        cur = [q] + [0] * n
        rq = reference_words[q - 1]
        for k in range(1, n + 1):
            if rq == hypothesis_words[k - 1]:
                cur[k] = prev[k - 1]
            else:
                cur[k] = min(prev[k - 1], cur[k - 1], prev[k]) + 1
        prev = cur
    return prev[n]


def wer_batch(references, hypotheses) -> float:
    total_errors = 0
    total_words = 0
    for ref, hyp in zip(references, hypotheses):
        ref_words = ref.lower().split()
        total_errors += levenshtein(ref_words, hyp.lower().split())
        total_words += len(ref_words)
    return (total_errors / total_words) * 100 if total_words > 0 else 0.0


def _tolist(ids):
    if hasattr(ids, "tolist"):
        return ids.tolist()
    return ids


def clean_ids(ids, pad_token_id=PAD, bos_token_id=BOS, eos_token_id=EOS):
    return [int(i) for i in _tolist(ids) if i not in (-100, pad_token_id, bos_token_id, eos_token_id)]


def clean_batch(batch_ids, pad_token_id=PAD, bos_token_id=BOS, eos_token_id=EOS):
    return [clean_ids(seq, pad_token_id, bos_token_id, eos_token_id) for seq in _tolist(batch_ids)]


def compute_metrics(pred, tokenizer=None, model=None, print_pred=False, num_samples=0, logits=None,
                    compute_result=False):
    """{"wer": WER %, "efficiency_score": (100 - WER) / trainable M params, per_layer_norms_<name>: |grad|}."""
    if isinstance(pred, dict):
        pred_ids, label_ids = pred["predictions"], pred["label_ids"]
    else:
        pred_ids, label_ids = pred.predictions, pred.label_ids
    if isinstance(pred_ids, tuple):
        pred_ids = pred_ids[0]
    pred_ids = np.asarray(_tolist(pred_ids)) if not isinstance(pred_ids, np.ndarray) else pred_ids
    if pred_ids.ndim == 3:
        pred_ids = np.argmax(pred_ids, axis=-1)

    def clean(ids):
        ids = _tolist(ids)
        if isinstance(ids[0], (list, tuple, np.ndarray)):
            return clean_batch(ids)
        return clean_ids(ids)

    label_ids = clean(label_ids)
    pred_ids = clean(pred_ids)
    pred_str = tokenizer.batch_decode(pred_ids)
    label_str = tokenizer.batch_decode(label_ids)
    if print_pred:
        for q in range(min(num_samples, len(pred_ids))):
            print(f"Pred tokens: {pred_ids[q]}")
            print(f"Label tokens: {label_ids[q]}")
            print(f"Pred: '{pred_str[q]}'")
            print(f"Label: '{label_str[q]}'")
            print("-" * 40)
    wer = wer_batch(label_str, pred_str)
    result = {"wer": float(wer), "efficiency_score": 0.0}
    if model is not None:
        trainable = sum(p.numel() for p in model.parameters() if p.requires_grad) / 1000000
        result["efficiency_score"] = float((100 - wer) / trainable if trainable > 0 else 0.0)
        for name, p in model.named_parameters():
            if p.grad is not None:
                result[f"per_layer_norms_{name}"] = float(p.grad.norm(2))
    return result


def setup_tokenizer(path: str):
    """HF `tokenizers` BPE from a tokenizer.json with the reference's wrappers (essentials.py:256-292):
    encode(text) -> ids, batch_decode / decode dropping pad/bos/eos/-100, pad/bos/eos ids 0/1/2."""
    from tokenizers import Tokenizer

    tok = Tokenizer.from_file(f"{path}")
    orig_encode, orig_decode = tok.encode, tok.decode

    def enc(text, add_special_tokens=True):
        ids = orig_encode(text).ids
        if not add_special_tokens:
            # the reference's list literal is ["<UNK>, <PAD>", "<BOS>", "<EOS>"] (one fused string)
            sp = [tok.token_to_id(t) for t in ["<UNK>, <PAD>", "<BOS>", "<EOS>"]]
            ids = [i for i in ids if i not in sp]
        return ids

    def bdec(ids_list, pad_token_id=PAD, bos_token_id=BOS, eos_token_id=EOS, skip_special_tokens=True):
        return [orig_decode(clean_ids(ids, pad_token_id, bos_token_id, eos_token_id)) for ids in _tolist(ids_list)]

    def dec(ids, pad_token_id=PAD, bos_token_id=BOS, eos_token_id=EOS):
        return orig_decode(clean_ids(ids, pad_token_id, bos_token_id, eos_token_id))

    def save_pretrained(save_dir):
        os.makedirs(save_dir, exist_ok=True)
        tok.save(f"{save_dir}/tokenizer.json")

    tok.encode, tok.batch_decode, tok.decode, tok.save_pretrained = enc, bdec, dec, save_pretrained
    tok.pad_token_id, tok.bos_token_id, tok.eos_token_id = PAD, BOS, EOS
    return tok
