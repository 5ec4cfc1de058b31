"""Recorder of the model's hard decisions (for decision-aware parity tests; off by default).

The reference's forward takes discrete decisions from continuous values (SURVEY.md §7 "Hard parts"):
  * every AbbyNormal picks a normalisation mode per row: the argmax of gumbel_softmax(logits + cv,
    hard=True) (essentials.py:170);
  * every MSheath layer thresholds v_gate (STthreshold, model.py:330-334, 351) into ion in {0, 1} per
    position, and picks an action per sample from gumbel_softmax(policy, hard=True), forced to 1 when
    mean(ion) < 0.1 (model.py:476-482).
A 1-ulp difference in the value a decision is taken from can flip it, after which forward values and
gradients legitimately diverge.  When enabled, the HIP path records each decision keyed the way the
oracle restatement keys its noise (site key, sample id), so a test can report the agreement rates and
replay the HIP decisions inside the oracle (oracle/model.py Decisions).

Entries (all CPU tensors):
  ("abby", key, sid)          -> int64 (L, H) mode index per position (and head)
  ("cond", key, sid)          -> bool (L, H, d) mode 2's max-vs-avg choice per feature (rows in mode 2)
  ("ion", key, sid, layer)    -> float (L,) v_gate output of a sample at that MSheath layer
  ("action", key, sid, layer) -> (action, forced) of a sample at that layer
where key is the noise site key of the AbbyNormal call / of the MSheath call ("<site>.jump").
"""
from __future__ import annotations

_REC: dict | None = None


def enable():
    global _REC
    _REC = {}


def disable() -> dict:
    global _REC
    out, _REC = _REC, None
    return out or {}


def active() -> bool:
    return _REC is not None


def abby(key: int, sid_base: int, L: int, H: int, idx, cond=None):
    """idx: the kernel's (rows,) int32 mode index, rows ordered (sample, position, head); cond: (rows, d)
    uint8, mode 2's per-feature choice max > 2 avg (essentials.py:176-177) for the rows that picked mode 2
    (zero elsewhere) -- a discrete choice too, flipped by rounding when max is within ~1e-7 of 2 avg."""
    if _REC is None:
        return
    a = idx.detach().to("cpu").long().view(-1, L, H)
    c = cond.detach().to("cpu").bool().view(a.shape[0], L, H, -1) if cond is not None else None
    for s in range(a.shape[0]):
        _REC[("abby", int(key), sid_base + s)] = a[s].clone()
        if c is not None:
            _REC[("cond", int(key), sid_base + s)] = c[s].clone()


def msheath_layer(key: int, sid_base: int, layer: int, ion, rec_f32):
    """ion: (B, L) v_gate outputs; rec_f32: the control kernel's per-sample record viewed as float32
    (B, 8): [ys(3), action, low, jump_g, cg, act] (csrc/msheath.hip CtrlRec)."""
    if _REC is None:
        return
    ion = ion.detach().to("cpu").float()
    rec = rec_f32.detach().to("cpu").float()
    for s in range(ion.shape[0]):
        if rec[s, 7] > 0.5:  # the sample was at this layer
            _REC[("ion", int(key), sid_base + s, layer)] = ion[s].clone()
            _REC[("action", int(key), sid_base + s, layer)] = (int(rec[s, 3]), bool(rec[s, 4] > 0.5))
