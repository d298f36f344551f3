"""Single-wave latency of the heaviest positions seen in self-play
(tools/monsters.npz, saved by tools/stamps.py): one bgx_movegen launch per
position, n = 1, so the time is one wave's critical path."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mlp-ppo-2ply-p3_amd")]
import numpy as np, torch, bgx

z = np.load(os.path.join(ROOT, "tools", "monsters.npz"))
recs, dur = z["recs"], z["dur"]
order = np.argsort(-dur)[:12]
eng = bgx.Engine(batch=64, dice="philox", seed=1)
res = []
for i in order:
    r = torch.from_numpy(recs[i:i + 1]).cuda()
    boards = r[:, :52].contiguous()
    pl = r[:, 52].contiguous()
    dice = r[:, 53:55].contiguous()
    for _ in range(2):
        eng.movegen(boards, pl, dice)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        nm, nt, _ = eng.movegen(boards, pl, dice)
    e1.record()
    torch.cuda.synchronize()
    res.append((int(i), int(dice[0, 0]), int(nt[0]), e0.elapsed_time(e1) / 5 * 1000, float(dur[i])))
    L = eng._lib
    if hasattr(L, "bgx_debug_counters"):
        import ctypes
        c = (ctypes.c_ulonglong * 16)()
        L.bgx_debug_counters(c)
        v = np.array(c[:], np.float64) / 7     # 7 launches
        names = ["dbl", "", "d2 batches", "d2 fresh", "d3 batches", "d3 fresh", "leaf batches", "leaf probes",
                 "committed", "", "", "d2 kids", "d3 kids"]
        print("   ", ", ".join("%s %.0f" % (names[k], v[k]) for k in (2, 3, 11, 4, 5, 12, 6, 7, 8)))
        print("    cycles(memtime): doubles %.0f  flat leaves %.0f (commit %.0f)  memo checks %.0f" % (v[1], v[14], v[13], v[15]))
for r in res:
    print("pos %2d dice %d-%d n_total %4d  movegen %7.1f us  (in-step wave %.1f us)" % (r[0], r[1], r[1], r[2], r[3], r[4]))
print("mean us", np.mean([r[3] for r in res]))
