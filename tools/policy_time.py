"""Standalone time of the rollout policy kernel (bgx_policy_act, MODE 0) on
self-play records: B lanes after some random-policy steps, skip on / off."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mlp-ppo-2ply-p3_amd"))
import bgx  # noqa: E402
from bgx.policy import PolicyNet  # noqa: E402

B = int(os.environ.get("B", 32768))
torch.manual_seed(0)
net = PolicyNet(hidden_size=128).cuda()
net.pack()
eng = bgx.Engine(batch=B, dice="philox", seed=3, auto_reset=True)
eng.reset()
for i in range(40):
    a, _, _ = net.act(eng, seed=1, step=i)
    eng.step(a)
rec = eng.records().clone()
cnt = (rec[:, 60].int() | (rec[:, 61].int() << 8))
print(f"B={B} count0 {float((cnt == 0).float().mean()):.3f} >32 {float((cnt > 32).float().mean()):.3f} "
      f">128 {float((cnt > 128).float().mean()):.3f}")
for sk in ("1", "0", "1", "0"):
    from bgx._lib import debug_option
    debug_option("BGX_POLICY_SKIP", sk)
    for _ in range(5):
        net.act(rec, seed=2, step=0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(50):
        net.act(rec, seed=2, step=k)
    e1.record()
    torch.cuda.synchronize()
    print(f"skip={sk}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us per launch")
