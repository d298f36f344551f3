"""PPO update timing at the production batch (B = 65,536, T = 32): one rollout,
then update() x N; prints the median update seconds and the loss parts."""
import os, statistics, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mlp-ppo-2ply-p3_amd")]
from bgx.train import PPOTrainer  # noqa: E402
tr = PPOTrainer(batch=65536, horizon=32, seed=0)
tr.rollout()
torch.cuda.synchronize()
ts = []
for _ in range(int(os.environ.get("N", "4"))):
    time.sleep(0.05)                  # an idle gap that separates the updates in a kernel trace
    t0 = time.perf_counter()
    m = tr.update()
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print("update_s", round(statistics.median(ts), 5), m)
