"""The parity-metrics collector of the GPU suite (tests/model_parity.record): one JSON line per case with every
scalar metric, numpy / torch scalars converted, the per-parameter gradient table left out."""
import json

import numpy as np
import torch


def test_record_writes_json_lines(tmp_path):
    import model_parity as mp

    path = tmp_path / "parity.jsonl"
    res = {"logits_max": np.float64(1.5e-4), "argmax": 1.0, "loss": torch.tensor(2e-6), "grads": {"w": 1.0},
           "grads_all_global_worst": ("enc.conv1.0.weight", np.float32(3e-4)), "decisions": {"abby": 0.99, "n": 7},
           "replayed": np.int64(12)}
    mp.record("tiny_full", "fp32", res, path=str(path))
    mp.record("tiny_full", "bf16", {"argmax": 0.91}, path=str(path))
    lines = [json.loads(s) for s in path.read_text().splitlines()]
    assert [d["precision"] for d in lines] == ["fp32", "bf16"]
    d = lines[0]
    assert d["case"] == "tiny_full" and "grads" not in d
    assert d["logits_max"] == 1.5e-4 and d["replayed"] == 12 and abs(d["loss"] - 2e-6) < 1e-12
    assert d["decisions"] == {"abby": 0.99, "n": 7}
    assert d["grads_all_global_worst"][0] == "enc.conv1.0.weight"


def test_record_is_a_noop_without_a_target(monkeypatch):
    import model_parity as mp

    monkeypatch.delenv("ASRX_PARITY_LOG", raising=False)
    mp.record("x", "fp32", {"a": 1.0})  # nothing to write, nothing raised
