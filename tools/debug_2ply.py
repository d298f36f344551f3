import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mlp-ppo-2ply-p3_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np, torch, bgx, oracle as O
from bgx.policy import PolicyNet
from bgx.search import ValueHead, two_ply
ROLLS = [(a, b) for a in range(1, 7) for b in range(a, 7)]
PROBS = np.array([1 / 36 if a == b else 2 / 36 for a, b in ROLLS], np.float32)
mlp = dict(np.load(os.path.join(ROOT, "tests/golden/mlp.npz")))
net = PolicyNet(hidden_size=40).cuda()
net.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in mlp.items() if k.startswith("h40_") and not k.endswith(("logits", "values"))})
vh = ValueHead(net)
B = 48
eng = bgx.Engine(batch=B, max_moves=500, dice="mt", auto_reset=True)
eng.seed(np.arange(500, 500 + B, dtype=np.uint32)); eng.reset()
rng = np.random.RandomState(2)
for _ in range(25):
    nm = eng.n_moves().cpu().numpy()
    eng.step(torch.from_numpy(np.array([rng.randint(k) if k else 0 for k in nm], np.int32)).cuda())
best, bestq, q, stats = two_ply(eng, vh, want_q=True)
rec, mv, _ = eng.lanes(); rec = rec.cpu().numpy(); mv = mv.cpu().numpy().view(np.uint64)
q = q.cpu().numpy(); n_all = eng.n_moves().cpu().numpy()
def V(feats):
    with torch.no_grad(): return net(torch.from_numpy(np.asarray(feats, np.float32)).cuda())[1].cpu().numpy()
def Q(board, mover, move, sub_limit=4):
    subs = O.decode_move(int(move))[:sub_limit]
    aft = O.apply_move(board, mover, O.encode_move(subs)); opp = 1 - mover; acc = 0.0
    for r, roll in enumerate(ROLLS):
        reps, cnt = O.movegen(aft, opp, roll, cap=4096)
        leaf = [O.features(aft, mover)] if cnt == 0 else [O.features(O.apply_move(aft, opp, int(b)), mover) for b in reps]
        acc += float(PROBS[r]) * float(V(leaf).min())
    return acc
for i in range(4):
    n = int(n_all[i]); board, mover = rec[i, :52].view(np.int8), int(rec[i, 52])
    print("lane", i, "n", n, "mover", mover, "roll", rec[i,53], rec[i,54])
    for a in range(min(n, 6)):
        print("  a", a, O.decode_move(int(mv[i,a])), "kernel %.6f" % q[i,a], "full %.6f" % Q(board, mover, mv[i,a]), "first-sub %.6f" % Q(board, mover, mv[i,a], 1))
