"""Debug: 1-ply values of the H=128 evaluator vs torch, per hidden unit."""
import sys, os
import numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mlp-ppo-2ply-p3_amd"))
import bgx
from bgx.policy import PolicyNet
from bgx.search import ValueHead, one_ply

torch.manual_seed(0)
net = PolicyNet(hidden_size=128).cuda()
eng = bgx.Engine(batch=256, max_moves=500, dice="mt", auto_reset=True)
eng.seed(np.arange(256, dtype=np.uint32)); eng.reset()
rng = np.random.RandomState(2)
for _ in range(20):
    nm = eng.n_moves().cpu().numpy()
    eng.step(torch.from_numpy(np.array([rng.randint(k) if k else 0 for k in nm], np.int32)).cuda())
feats = eng.legal_features().float()
n = eng.n_moves().cpu().numpy()
mask = torch.zeros(feats.shape[:2], dtype=torch.bool, device="cuda")
for i in range(256): mask[i, :n[i]] = True

def run(tag):
    vh = ValueHead(net)
    _, _, vals = one_ply(eng, vh, want_values=True)
    with torch.no_grad():
        ref = net(feats.reshape(-1, 198))[1].reshape(vals.shape)
    err = (vals - ref).abs()[mask].max().item()
    print(tag, "maxerr", err, flush=True)
    return err

with torch.no_grad():
    W1 = net.fc1.weight.clone(); wv = net.value_head.weight.clone(); b1 = net.fc1.bias.clone()
    run("full")
    net.fc1.weight.copy_(W1.half().float()); run("W1 f16-exact (lo=0)")
    net.fc1.weight.copy_(W1)
    for u in [0, 1, 3, 4, 7, 8, 12, 15, 16, 20, 24, 31, 32, 33, 40, 63, 64, 96, 127]:
        w = torch.zeros_like(wv); w[0, u] = 1.0
        net.value_head.weight.copy_(w)
        run(f"unit {u}")
    net.value_head.weight.copy_(wv)
    net.fc1.bias.zero_(); run("b1=0")
