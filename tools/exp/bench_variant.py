"""A/B helper: run bench.py in this process after asrx_set_gemm_variant(V) (env GEMM_VARIANT, default 5).
usage: GEMM_VARIANT=6 python tools/exp/bench_variant.py [bench args...]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "asr-model_amd")]
from asrx import lib  # noqa: E402

lib.load().asrx_set_gemm_variant(int(os.environ.get("GEMM_VARIANT", "5")))
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
