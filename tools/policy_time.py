"""Time bgx_policy_act alone on C3-shaped records (B = 65,536 lanes after a
burn-in of self-play): sampling vs greedy, with and without the logits output."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mlp-ppo-2ply-p3_amd"))
import torch, bgx
from bgx.policy import PolicyNet

B = int(os.environ.get("B", 65536))
torch.manual_seed(0)
net = PolicyNet(hidden_size=128).cuda()
eng = bgx.Engine(batch=B, dice="philox", seed=5, auto_reset=True)
eng.reset(want_obs=False)
for i in range(60):
    a, _, _ = net.act(eng.records(), seed=1, step=i)
    eng.step(a, want_obs=False)
rec = eng.records().clone()
for name, kw in (("sample", {}), ("greedy", {"greedy": True})):
    for _ in range(5):
        net.act(rec, seed=1, step=0, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(50):
        net.act(rec, seed=1, step=i, **kw)
    e1.record(); torch.cuda.synchronize()
    print(name, "%.1f us" % (e0.elapsed_time(e1) / 50 * 1000))
