"""The <= 4-output linear's backward (csrc/rowops.hip small_linear_bwd_kernel + small_linear_colsum_kernel; the
gate / mlp_gate / PolicyNet heads of model.py:441-505): parameter gradients are per-workgroup partials added in a
fixed order, so two runs -- eager, or replayed from a graph -- agree BIT FOR BIT; the partial buffer is allocated
on a stream's first use, which may come inside a graph capture (bench.py --graph captures on its own stream), and
must not invalidate the capture.  Values against a float64 product."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(lib, act, gy, y, x, W, dx, dW, db):
    dW.zero_()
    db.zero_()
    rows, K = x.shape
    lib.call("asrx_small_linear_bwd", gy.data_ptr(), y.data_ptr(), x.data_ptr(), W.data_ptr(), dx.data_ptr(),
             dW.data_ptr(), db.data_ptr(), rows, K, W.shape[0], act, 0.0, lib.stream())


@pytest.mark.parametrize("rows,K,N", [(1, 64, 1), (777, 384, 3), (20000, 384, 3), (200003, 128, 4)])
def test_small_linear_bwd_ordered_and_capturable(cuda, rows, K, N):
    from asrx import lib
    from asrx.gemm import ACT

    g = torch.Generator().manual_seed(rows + K + N)
    x = torch.randn(rows, K, generator=g).to(cuda)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = torch.randn(N, generator=g).to(cuda)
    y = torch.sigmoid(x @ W.t() + b)
    gy = torch.randn(rows, N, generator=g).to(cuda)
    act = ACT["sigmoid"]
    outs = []
    for _ in range(2):  # eager, twice
        o = (torch.empty_like(x), torch.empty_like(W), torch.empty_like(b))
        _run(lib, act, gy, y, x, W, *o)
        outs.append(o)
    # captured on a stream that has never run the kernel (its partial buffer is allocated inside the capture)
    o = (torch.empty_like(x), torch.empty_like(W), torch.empty_like(b))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=torch.cuda.Stream()):
        _run(lib, act, gy, y, x, W, *o)
    for _ in range(2):
        o[1].fill_(7.0)  # overwritten by the replay's zero + sums
        graph.replay()
        torch.cuda.synchronize()
        outs.append(tuple(t.clone() for t in o))
    for other in outs[1:]:
        for a, c in zip(outs[0], other):
            assert torch.equal(a, c)
    dz = (gy * y * (1 - y)).double()
    ref = (dz @ W.double(), dz.t() @ x.double(), dz.sum(0))
    for got, want, name in zip(outs[0], ref, ("dx", "dW", "db")):
        scale = float(want.abs().max()) + 1e-30
        err = float((got.double() - want).abs().max()) / scale
        assert err < 1e-4, (name, err)  # fp32 accumulation over up to 2e5 rows, against the largest entry
