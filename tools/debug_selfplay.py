import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mlp-ppo-2ply-p3_amd"), os.path.join(ROOT, "oracle")]
import numpy as np, torch, bgx, oracle as O
B, T = 512, 250
seeds = np.arange(1000, 1000 + B, dtype=np.uint32)
eng = bgx.Engine(batch=B, max_moves=500, dice="mt", auto_reset=True)
eng.seed(seeds)
envs = [O.Env(seed=int(s)) for s in seeds]
eng.reset(); [e.reset() for e in envs]
pol = np.random.RandomState(3)
for t in range(T):
    rec, mv, nt = eng.lanes(); rec = rec.cpu().numpy(); mv = mv.cpu().numpy().view(np.uint64)
    nm = (rec[:, 60].astype(int) | (rec[:, 61].astype(int) << 8))
    bad = []
    for i, e in enumerate(envs):
        b, st = e.state()
        if not np.array_equal(rec[i, :52].view(np.int8), b) or rec[i,52] != st[0] or (rec[i,53],rec[i,54]) != (st[1],st[2]) or nm[i] != st[3] or not np.array_equal(mv[i,:st[3]], e.legal()):
            bad.append(i)
    if bad:
        i = bad[0]; e = envs[i]; b, st = e.state()
        print("t", t, "bad lanes", bad[:10], len(bad))
        print("engine rec", rec[i, :64].tolist())
        print("oracle board", b.tolist(), "st", st.tolist())
        L = e.legal()
        print("n", nm[i], st[3])
        diff = [k for k in range(min(nm[i], st[3])) if mv[i,k] != L[k]]
        print("first diffs", diff[:5])
        for k in diff[:3]:
            print(k, O.decode_move(mv[i,k]), O.decode_move(L[k]))
        m2, n2 = O.movegen(rec[i, :52].view(np.int8), int(rec[i,52]), (int(rec[i,53]), int(rec[i,54])))
        print("oracle on engine board: n", n2, "match engine list", np.array_equal(m2[:nm[i]], mv[i,:nm[i]]))
        break
    acts = np.array([pol.randint(k) if k > 0 else 0 for k in nm], np.int32)
    if t % 17 == 5:
        acts[::7] = 499
    eng.step(torch.from_numpy(acts).cuda())
    for i, e in enumerate(envs):
        o, r, d, _ = e.step(int(acts[i]))
        if d: e.reset()
print("done")
