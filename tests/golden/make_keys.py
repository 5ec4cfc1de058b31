"""Regenerate tests/golden/state_dict_*.json: the reference Model's state_dict (key, shape) list in
order, from the module-tree restatement of its constructors (oracle/tree.py, cited file:line there),
for the reference's own main() configuration (model.py:746) and the tiny BASELINE config.

    python tests/golden/make_keys.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT]

from oracle import tree  # noqa: E402

CASES = {"reference_main": (40000, 128, 512, 4, 4), "tiny": (40000, 128, 384, 6, 4)}

if __name__ == "__main__":
    for name, dims in CASES.items():
        spec = tree.state_dict_spec(*dims)
        with open(os.path.join(HERE, f"state_dict_{name}.json"), "w") as f:
            json.dump({"dimensions": dict(zip(("tokens", "mels", "dims", "head", "layer"), dims)), "state_dict": spec},
                      f, indent=0)
        print(name, len(spec))
