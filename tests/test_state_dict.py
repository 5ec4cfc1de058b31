"""Drop-in boundary (SURVEY.md §8(b) "Module tree / param names"): asrx.model.Model(Dimensions) has
the reference Model's state_dict keys and shapes, in order, so reference checkpoints load and
MaxFactor's name-based parameter groups (model.py:775-787) apply unchanged.  The expected lists are
committed fixtures generated from the module-tree restatement of the reference's constructors
(oracle/tree.py, tests/golden/make_keys.py)."""
import json
import os

import pytest
import torch

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name", ["reference_main", "tiny"])
def test_state_dict_matches_reference_tree(name):
    from asrx.config import CONFIGS
    from asrx.model import Model

    fx = json.load(open(os.path.join(HERE, f"state_dict_{name}.json")))
    with torch.device("meta"):
        model = Model(CONFIGS[name])
    got = [[k, list(v.shape)] for k, v in model.state_dict().items()]
    assert got == fx["state_dict"]
    assert CONFIGS[name].dims == fx["dimensions"]["dims"] and CONFIGS[name].head == fx["dimensions"]["head"]


def test_fixture_is_current():
    from oracle import tree

    fx = json.load(open(os.path.join(HERE, "state_dict_reference_main.json")))
    d = fx["dimensions"]
    spec = [[k, s] for k, s in tree.state_dict_spec(d["tokens"], d["mels"], d["dims"], d["head"], d["layer"])]
    assert spec == fx["state_dict"]


def test_reference_checkpoint_loads():
    """A state_dict saved from the reference tree (restated, random values) loads strictly."""
    from asrx.config import Dimensions
    from asrx.model import Model
    from oracle import tree

    ref = tree.model_skeleton(500, 128, 128, 2, 2)
    sd = {k: torch.randn(v.shape) if v.is_floating_point() else torch.zeros(v.shape, dtype=v.dtype)
          for k, v in ref.state_dict().items()}
    model = Model(Dimensions(tokens=500, mels=128, dims=128, head=2, layer=2, act="gelu", n_type="AbbyNormal"))
    model.load_state_dict(sd, strict=True)
    k = "processor.block.1.jump.layers.0.v_gate.mkey"
    assert torch.equal(model.state_dict()[k], sd[k])


@pytest.mark.parametrize("dims,head", [(384, 4), (192, 2), (1024, 4)])
def test_unsupported_head_dim_rejected_at_construction(dims, head):
    from asrx.config import Dimensions
    from asrx.model import Model

    with pytest.raises(ValueError, match="head dim"):
        with torch.device("meta"):
            Model(Dimensions(tokens=100, mels=128, dims=dims, head=head, layer=2, act="gelu", n_type="AbbyNormal"))
