"""Work counters of the 2-ply doubles enumeration (library built with
-DBGX_COUNTERS into exp/libbgx_cnt.so; run with BGX_LIB=exp/libbgx_cnt.so)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mlp-ppo-2ply-p3_amd")]
import bgx  # noqa: E402
from bgx import _lib  # noqa: E402
from bgx.policy import PolicyNet  # noqa: E402
from bgx.search import ValueHead, two_ply  # noqa: E402

B = int(os.environ.get("CNT_B", "65536"))
dev = torch.device("cuda:0")
torch.manual_seed(0)
net = PolicyNet().to(dev)
eng = bgx.Engine(batch=B, max_moves=500, seed=77, dice="philox", auto_reset=True, device=dev)
eng.reset(want_obs=False)
for i in range(150):
    a, _, _ = net.act(net.rollout_inputs(eng), seed=5, step=i)
    eng.step(a, want_obs=False, want_info=False)
L = _lib.load()
f = L.bgx_debug_counters_search
f.argtypes = [ctypes.c_void_p]
c = (ctypes.c_ulonglong * 16)()
f(ctypes.cast(c, ctypes.c_void_p))
vh = ValueHead(PolicyNet(hidden_size=40).to(dev))
_, _, _, st = two_ply(eng, vh)
f(ctypes.cast(c, ctypes.c_void_p))
names = {0: "doubles calls", 1: "doubles cycles", 9: "phase-A cycles (until got4)", 10: "jobs reaching got4",
         6: "flat_leaves calls", 7: "flat_leaves leaves", 8: "committed unique", 13: "place_batch cycles",
         14: "depth-2 children (flat)", 15: "depth-3 children (flat)", 2: "commit calls",
         3: "dfs fresh depth-2", 5: "dfs fresh depth-3", 11: "sink push cycles", 12: "flat_leaves probe cycles (lane sum)"}
print(st)
for i in range(16):
    print(f"{i:2d} {names.get(i, '-'):32s} {c[i]:>16d}  per call {c[i] / max(c[0], 1):10.2f}")
