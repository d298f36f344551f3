"""Run bench.py with library debug options set (experiments; include/bgx.h
bgx_debug_option):   python tools/bench_with_options.py "NAME=V,NAME2=V" [bench args...]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mlp-ppo-2ply-p3_amd"), ROOT]
from bgx._lib import debug_option  # noqa: E402

for kv in filter(None, sys.argv[1].split(",")):
    k, v = kv.split("=", 1)
    debug_option(k, v)
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
