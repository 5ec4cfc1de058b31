"""GEMM entry points over ``asrx_gemm`` (csrc/gemm.hip) for Linear / Conv1d forward and backward.

Layout vocabulary: activations are row-major (rows, features); weights are nn.Linear's (out, in).
"""
from __future__ import annotations

import torch

from . import lib, prec, probe

ACT = {"none": 0, "gelu": 1, "silu": 2, "sigmoid": 3, "relu": 4}


def gemm(A, B, C, *, M, N, K, lda, ldb, ldc, a_kc=True, b_kc=True, batch=1, sA=0, sB=0, sC=0,
         bias=None, Z=None, alpha=1.0, beta=0.0, act="none", conv_a=False, conv_b=False,
         conv_F=0, conv_C=0, splitk=1, precision=None):
    lib.require_gpu(A, B, C)
    p = prec.get() if precision is None else precision
    e0 = probe.begin("gemm")
    lib.call("asrx_gemm", p, lib.ptr(A), lda, sA, int(a_kc), int(conv_a), lib.ptr(B), ldb, sB,
             int(b_kc), int(conv_b), lib.ptr(C), ldc, sC, lib.ptr(bias), lib.ptr(Z), M, N, K, batch,
             float(alpha), float(beta), ACT[act], conv_F, conv_C, int(splitk), lib.stream())
    probe.end("gemm", e0, 2.0 * M * N * K * batch)
    return C


def _rows(x):
    return x.reshape(-1, x.shape[-1])


def linear_fwd(x, W, b=None, act="none", out=None, preact=None):
    """y = act(x @ W^T + b) for x (..., K), W (N, K)."""
    x2 = _rows(x)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    M, K = x2.shape
    N = W.shape[0]
    y = out if out is not None else torch.empty(*x.shape[:-1], N, device=x.device, dtype=torch.float32)
    gemm(x2, W, y, M=M, N=N, K=K, lda=K, ldb=K, ldc=N, a_kc=True, b_kc=True, bias=b, act=act,
         Z=preact)
    return y


def linear_dgrad(dy, W, out=None, beta=0.0):
    """dx = dy @ W for dy (..., N), W (N, K)."""
    d2 = _rows(dy)
    if not d2.is_contiguous():
        d2 = d2.contiguous()
    M, N = d2.shape
    K = W.shape[1]
    dx = out if out is not None else torch.empty(*dy.shape[:-1], K, device=dy.device, dtype=torch.float32)
    gemm(d2, W, dx, M=M, N=K, K=N, lda=N, ldb=K, ldc=K, a_kc=True, b_kc=False, beta=beta)
    return dx


def _splitk_for(m_rows: int, tiles: int) -> int:
    # enough workgroups to fill 256 CUs; each K-slice keeps >= 512 rows
    want = max(1, 512 // max(tiles, 1))
    return int(max(1, min(want, m_rows // 512)))


def linear_wgrad(dy, x, out=None, accumulate=False):
    """dW = dy^T @ x (N, K) summed over all rows; accumulates into `out` when accumulate=True."""
    d2 = _rows(dy)
    x2 = _rows(x)
    if not d2.is_contiguous():
        d2 = d2.contiguous()
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    M, N = d2.shape
    K = x2.shape[1]
    if out is None:
        out = torch.zeros(N, K, device=dy.device, dtype=torch.float32)
    elif not accumulate:
        out.zero_()
    tiles = ((N + 127) // 128) * ((K + 127) // 128)
    gemm(d2, x2, out, M=N, N=K, K=M, lda=N, ldb=K, ldc=K, a_kc=False, b_kc=False, beta=1.0,
         splitk=_splitk_for(M, tiles))
    return out
