"""2-ply A/B in one process: env-var configs (read by bgx_two_ply on every call)
on one burned-in B = 65,536 engine.  Usage: python tools/exp_2ply.py 'K=V,K=V' ...
(an empty string = defaults).  Prints enumeration / evaluation ms per batch and
roots/s (median of 3 batches)."""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mlp-ppo-2ply-p3_amd")]
import bgx  # noqa: E402
from bgx.policy import PolicyNet  # noqa: E402
from bgx.search import ValueHead, two_ply, two_ply_timings  # noqa: E402

dev = torch.device("cuda:0")
H = int(os.environ.get("EXP_H", "40"))
torch.manual_seed(0)
net = PolicyNet().to(dev)
eng = bgx.Engine(batch=65536, max_moves=500, seed=1234, dice="philox", auto_reset=True, device=dev)
eng.reset(want_obs=False)
for i in range(160):
    a, _, _ = net.act(eng, seed=5, step=i)
    eng.step(a, want_obs=False, want_info=False)
torch.manual_seed(1)
vh = ValueHead(PolicyNet(hidden_size=H).to(dev))
ref = None
for cfg in sys.argv[1:]:
    keep = dict(os.environ)
    for kv in filter(None, cfg.split(",")):
        k, v = kv.split("=", 1)
        os.environ["BGX_2PLY_" + k] = v
    best, q, _, st = two_ply(eng, vh)
    torch.cuda.synchronize()
    if ref is None:
        ref = (best.clone(), q.clone(), st["leaves"])
    same = torch.equal(best, ref[0]) and torch.equal(q, ref[1]) and st["leaves"] == ref[2]
    en, ev, wall = [], [], []
    for _ in range(3):
        t0 = time.perf_counter()
        two_ply(eng, vh)
        torch.cuda.synchronize()
        wall.append(time.perf_counter() - t0)
        te, tv = two_ply_timings(eng)
        en.append(te)
        ev.append(tv)
    print(f"{cfg or 'default':40s} enum {statistics.median(en):7.2f} ms  eval {statistics.median(ev):6.2f} ms  "
          f"{65536 / statistics.median(wall) / 1e3:7.1f} k roots/s  same={same}", flush=True)
    os.environ.clear()
    os.environ.update(keep)
