"""Module-tree restatement of the reference's constructors (structure only: parameters and buffers,
no forward).  TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference cannot be imported here, so its state_dict key list is derived by
restating every __init__ on the Model's path with the same torch.nn building blocks, in the same
registration order (state_dict order = own parameters, own buffers, then children in registration
order; a shared submodule appears under every name it is registered at):

  Model            model.py:631-652        processor, enc
  processor        model.py:585-600        ln, token, pitch_tokens, position, blend, block; mask is a
                                           non-persistent buffer
  residual         model.py:559-573        ln, act_fn, attn, router, jump, mlp (mlp.0 / mlp.5 ARE ln)
  attention        model.py:234-249        q, kv, c, out, conv, ln, rot
  rotary           model.py:171-178        lin
  router           model.py:537-543        top, soft, alpha
  tgate            model.py:525-530        ga, cs
  MSheath          model.py:387-427        shared_head, mem_w, mem_gate, jump_s, layers, pnet, mlp_gate,
                                           mlp, mlp_ln
  v_gate           model.py:336-344        mkey, mval, mlp, tx, concat
  MPNet            model.py:375-382        net
  AudioEncoder     model.py:120-147        norm, local_norm, conv1, conv2, EncoderLayer, encoder
  ConvLite         model.py:93-106         point1, glu, depth, bn, swish, point2, dropout
  AbbyNormal       essentials.py:140-153   mode_router (get_norm's n_type="AbbyNormal", 193-219)
  LayerNorm        essentials.py:102-108   gamma, beta
  AdaptiveSpan     essentials.py:1219-1225 span_scale (BaseAttention 1164-1174 has no parameters)
  weight_norm      torch.nn.utils.parametrizations (model.py:6): parametrizations.weight.original0/1
"""
from __future__ import annotations

import torch
from torch import nn
from torch.nn.utils.parametrizations import weight_norm


def _abby(d):
    m = nn.Module()
    m.mode_router = nn.Sequential(nn.Linear(d, d), nn.SiLU(), nn.Linear(d, 3))
    return m


def _chan_ln(d):
    m = nn.Module()
    m.gamma = nn.Parameter(torch.ones(d))
    m.beta = nn.Parameter(torch.zeros(d))
    return m


def _conv_lite(d, k=15):
    m = nn.Module()
    m.point1 = nn.Conv1d(d, 2 * d, 1)
    m.glu = nn.GLU(dim=1)
    m.depth = nn.Conv1d(d, d, k, padding=(k - 1) // 2, groups=d)
    m.bn = nn.BatchNorm1d(d)
    m.swish = nn.SiLU()
    m.point2 = nn.Conv1d(d, d, 1)
    m.dropout = nn.Dropout(0.1)
    return m


def _encoder(mels, d, layer):
    m = nn.Module()
    m.norm = nn.Identity()
    m.local_norm = nn.Identity()
    act = nn.GELU()
    m.conv1 = nn.Sequential(nn.Conv1d(mels, d, 3, padding=1), m.norm)
    m.conv2 = nn.Sequential(nn.Conv1d(1, d, 3, padding=1), m.local_norm)
    m.EncoderLayer = nn.Identity()
    m.encoder = nn.ModuleList([nn.Sequential(act, weight_norm(nn.Conv1d(d, d, 3, padding=1)), _chan_ln(d), _conv_lite(d),
                                             act, nn.Conv1d(d, d, 3, padding=1, groups=d), act, nn.Dropout(0.1))
                               for _ in range(layer)])
    return m


def _attention(d, h):
    m = nn.Module()
    m.q = nn.Sequential(_abby(d), nn.Linear(d, d), nn.Identity())
    m.kv = nn.Sequential(_abby(d), nn.Linear(d, 2 * d), nn.Identity())
    m.c = nn.Sequential(_abby(d), nn.Linear(d, d), nn.Identity())
    m.out = nn.Sequential(nn.Identity(), nn.Linear(d, d))
    m.conv = nn.Identity()
    m.ln = _abby(d // h)
    m.rot = nn.Module()
    m.rot.lin = nn.Linear(d, (d // h) // 2)
    return m


def _v_gate(d):
    m = nn.Module()
    m.mkey = nn.Parameter(torch.randn(64, d))
    m.mval = nn.Parameter(torch.randn(64, 1))
    m.mlp = nn.Sequential(nn.Linear(d, d // 2), nn.SiLU(), nn.Linear(d // 2, 1))
    m.tx = nn.Parameter(torch.tensor(0.3), requires_grad=False)
    m.concat = nn.Linear(2, 1)
    return m


def _msheath(d, layer):
    m = nn.Module()
    m.shared_head = nn.Module()
    m.shared_head.span_scale = nn.Parameter(torch.tensor(1.0))
    m.mem_w = nn.Parameter(torch.zeros(1, 1, d))
    m.mem_gate = nn.Sequential(nn.Linear(d, 1), nn.Sigmoid())
    m.jump_s = nn.Parameter(torch.tensor([0.1, 0.05, 0.01]))
    m.layers = nn.ModuleList([nn.ModuleDict({"ln": nn.LayerNorm(d), "gate": nn.Sequential(nn.Linear(d, 1), nn.Sigmoid()),
                                             "v_gate": _v_gate(d), "adapter": nn.Linear(d, d) if i % 2 == 0 else None,
                                             "ranvier": None}) for i in range(layer)])
    m.pnet = nn.Module()
    m.pnet.net = nn.Sequential(nn.Linear(d, 128), nn.SiLU(), nn.Linear(128, 3))
    m.mlp_gate = nn.Sequential(nn.Linear(d, 1), nn.Sigmoid())
    m.mlp = nn.Sequential(nn.Linear(d, 4 * d), nn.SiLU(), nn.Linear(4 * d, d))
    m.mlp_ln = nn.LayerNorm(d)
    return m


def _residual(d, h, layer, n=3):
    m = nn.Module()
    m.ln = _abby(d)
    m.act_fn = nn.GELU()
    m.attn = _attention(d, h)
    m.router = nn.Module()
    m.router.top = nn.Linear(d * n, n)
    m.router.soft = nn.Sequential(nn.Linear(d * n, n), nn.Softmax(dim=-1))
    m.router.alpha = nn.Parameter(torch.ones(1))
    m.jump = _msheath(d, layer)
    tg = nn.Module()
    tg.ga = nn.ModuleList([nn.Sequential(nn.Linear(d, d), nn.Sigmoid()) for _ in range(n)])
    tg.cs = nn.Sequential(nn.Linear(d, n), nn.Softmax(dim=-1))
    m.mlp = nn.Sequential(m.ln, tg, nn.Linear(d, d * n), nn.GELU(), nn.Linear(d * n, d), m.ln)
    return m


def model_skeleton(tokens, mels, dims, head, layer, ctx=2048):
    """nn.Module with the reference Model's parameters and buffers (model.py:631-652)."""
    with torch.device("meta"):
        m = nn.Module()
        m.processor = nn.Module()
        p = m.processor
        p.ln = _abby(dims)
        p.token = nn.Embedding(tokens, dims)
        p.pitch_tokens = nn.Embedding(1024, dims)
        p.position = nn.Parameter(torch.ones(ctx, dims))
        p.blend = nn.Parameter(torch.tensor(0.5))
        p.block = nn.ModuleList([_residual(dims, head, layer) for _ in range(layer)])
        p.register_buffer("mask", torch.empty(ctx, ctx), persistent=False)
        m.enc = _encoder(mels, dims, layer)
    return m


def state_dict_spec(tokens, mels, dims, head, layer):
    """[(key, shape)] of the reference Model's state_dict in order."""
    return [(k, list(v.shape)) for k, v in model_skeleton(tokens, mels, dims, head, layer).state_dict().items()]
