"""Where the N > 1 path's per-step cost came from (profiles/r06_rccl_eager_init_ab.txt): runs bench.py (its arguments
follow, e.g. --dist-single) with torch.distributed.all_reduce stubbed out (GS_NOOP=1), with GradSync inactive
(GS_NOOP=3), and/or the process group created without device_id (GS_LAZY=1, what bench.py now does)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist


class _W:
    def wait(self):
        return True


mode = os.environ.get("GS_NOOP", "0")
if mode in ("1", "2"):
    real = dist.all_reduce

    def fake(t, *a, **k):
        return _W() if k.get("async_op") else None

    dist.all_reduce = fake
if mode == "3":  # process group up, GradSync inactive (no reduce, no stats, no comm-stream joins)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "asr-model_amd"))
    from asrx import dist as adist
    _init = adist.GradSync.__init__

    def init(self, *a, **k):
        k["reduce_single"] = False
        _init(self, *a, **k)
        self.active = False

    adist.GradSync.__init__ = init
if os.environ.get("GS_LAZY") == "1":  # no device_id: the communicator is created at the first collective
    _ipg = dist.init_process_group

    def ipg(*a, **k):
        k.pop("device_id", None)
        return _ipg(*a, **k)

    dist.init_process_group = ipg
import bench  # noqa: E402

sys.argv = ["bench.py"] + sys.argv[1:]
bench.main()
