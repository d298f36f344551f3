"""Per-wave phase times of the rollout policy kernel (experiment; a -DBGX_POLICY_STAMPS build
of libbgx.so: python tools/build_variant.py scratch/libbgx_pstamp.so -DBGX_POLICY_STAMPS).

    BGX_LIB=scratch/libbgx_pstamp.so B=16384 python tools/policy_stamps.py

Stamps (s_memrealtime, 100 MHz): start, after the count-0 scan + record staging, after
GEMM1, after the output tiles; main waves (32 rows each) and the extra count-0 waves
separately: phase means and the kernel span."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mlp-ppo-2ply-p3_amd"))
import bgx  # noqa: E402
from bgx import _lib  # noqa: E402
from bgx.policy import PolicyNet  # noqa: E402

B = int(os.environ.get("B", 16384))
torch.manual_seed(0)
net = PolicyNet(hidden_size=128).cuda()
net.pack()
eng = bgx.Engine(batch=B, dice="philox", seed=3, auto_reset=True)
eng.reset()
for i in range(60):
    a, _, _ = net.act(eng, seed=1, step=i)
    eng.step(a)
rec = eng.records().clone()
L = _lib.load()
fn = L.bgx_debug_policy_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int32]
W = 8192
buf = np.zeros((W, 6), dtype=np.uint64)
out = {}
for rep in range(3):
    net.act(rec, seed=2, step=rep)
    torch.cuda.synchronize()
    fn(buf.ctypes.data_as(ctypes.c_void_p), W)          # read + clear
    net.act(rec, seed=2, step=10 + rep)
    torch.cuda.synchronize()
    fn(buf.ctypes.data_as(ctypes.c_void_p), W)
    used = buf[:, 4] != 0
    st = buf[used].astype(np.float64)
    t0 = st[:, 0].min()
    res = {}
    for name, flag in (("extra", 1), ("main", 2)):
        s = st[st[:, 4] == flag]
        if not len(s):
            continue
        res[name] = {"waves": int(len(s)),
                     "start_us_mean": float((s[:, 0] - t0).mean() / 100), "start_us_max": float((s[:, 0] - t0).max() / 100),
                     "stage_us": float((s[:, 1] - s[:, 0]).mean() / 100), "gemm1_us": float((s[:, 2] - s[:, 1]).mean() / 100),
                     "tiles_us": float((s[:, 3] - s[:, 2]).mean() / 100), "tiles_us_max": float((s[:, 3] - s[:, 2]).max() / 100),
                     "end_us_max": float((s[:, 3] - t0).max() / 100)}
    res["span_us"] = float((st[:, 3].max() - t0) / 100)
    out[f"rep{rep}"] = res
print(json.dumps(out))
