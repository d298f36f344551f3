"""Diagnostics: per-wave start/end of k_step (BGX_STAMPS=1) -> residency profile."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mlp-ppo-2ply-p3_amd")]
import numpy as np, torch, bgx
from bgx._lib import debug_option
debug_option("BGX_STAMPS", 1)            # read at engine creation
from bgx.policy import PolicyNet
B = 65536
eng = bgx.Engine(batch=B, dice="philox", seed=5)
net = PolicyNet().cuda(); net.pack()
eng.reset(want_obs=False)
for i in range(160):
    rec = eng.records(); a, _, _ = net.act(rec, seed=1, step=i); eng.step(a, want_obs=False, want_info=False)
rec = eng.records(); a, _, _ = net.act(rec, seed=1, step=999)
eng.step(a, want_obs=False, want_info=False)
L = eng._lib; L.bgx_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
st = np.zeros((B, 2), np.uint64)
assert L.bgx_debug_stamps(eng._h, st.ctypes.data_as(ctypes.c_void_p)) == 0
rec = eng.records().cpu().numpy()
dbl = rec[:, 53] == rec[:, 54]
cur = rec[:, 52].astype(np.int64)
bd = rec[:, :48].view(np.int8).reshape(B, 2, 24)
pts = (bd[np.arange(B), cur] > 0).sum(1) + 2 * (rec[np.arange(B), 48 + cur] > 0)
t0 = st[:, 0].min(); s = (st[:, 0] - t0).astype(np.int64); e = (st[:, 1] - t0).astype(np.int64)
dur = e - s   # 100 MHz ticks
print("kernel span us %.1f" % (e.max() / 100))
print("dur us: nondbl median %.1f p99 %.1f max %.1f | dbl median %.1f p99 %.1f max %.1f" % (
    np.median(dur[~dbl]) / 100, np.percentile(dur[~dbl], 99) / 100, dur[~dbl].max() / 100,
    np.median(dur[dbl]) / 100, np.percentile(dur[dbl], 99) / 100, dur[dbl].max() / 100))
for k in range(0, 16):
    m = dbl & (pts == k)
    if m.sum():
        print("dbl pts=%2d n=%6d mean %.1f us median %.1f p99 %.1f" % (k, m.sum(), dur[m].mean() / 100,
              np.median(dur[m]) / 100, np.percentile(dur[m], 99) / 100))
print("nondbl mean %.1f" % (dur[~dbl].mean() / 100))
print("sum dur share: dbl %.2f" % (dur[dbl].sum() / dur.sum()))
T = e.max(); bins = 40
for k in range(0, bins, 2):
    a0, a1 = T * k // bins, T * (k + 1) // bins
    live = ((s < a1) & (e > a0)).sum()
    print("%5.0f-%5.0fus live waves %6d started %6d" % (a0 / 100, a1 / 100, live, ((s >= a0) & (s < a1)).sum()))
# which blockIdx ranges run late
late = np.argsort(-e)[:20]
print("latest-ending lanes", late, dur[late] / 100, dbl[late])

# slowest lanes over several steps: what are they? (saved for offline analysis)
rows = []
for k in range(12):
    rec0 = eng.records()
    pre = rec0.cpu().numpy()
    a, _, _ = net.act(rec0, seed=1, step=2000 + k)
    eng.step(a, want_obs=False, want_info=False)
    assert L.bgx_debug_stamps(eng._h, st.ctypes.data_as(ctypes.c_void_p)) == 0
    d = (st[:, 1] - st[:, 0]).astype(np.int64)
    r2, _, nt = eng.lanes()
    r2, nt = r2.cpu().numpy(), nt.cpu().numpy()
    span = (st[:, 1].max() - st[:, 0].min()) / 100
    for lane in np.argsort(-d)[:4]:
        rows.append((k, lane, d[lane] / 100, span, r2[lane, 53], r2[lane, 54], nt[lane], r2[lane, 62] & 1, r2[lane].copy()))
print("step lane dur_us span_us dice n_total ovf")
for r in rows:
    print(r[0], r[1], "%.1f %.1f" % (r[2], r[3]), r[4], r[5], r[6], r[7])
np.savez(os.path.join(ROOT, "gpurun_out", "slow_lanes.npz"), recs=np.stack([r[8] for r in rows]),
         dur=np.array([r[2] for r in rows]), ntot=np.array([r[6] for r in rows]))

# doubles cost table by (die, points occupied by the mover + 2*on-bar) over several steps
tab = {}
for k in range(8):
    rec0 = eng.records()
    a, _, _ = net.act(rec0, seed=1, step=3000 + k)
    eng.step(a, want_obs=False, want_info=False)
    assert L.bgx_debug_stamps(eng._h, st.ctypes.data_as(ctypes.c_void_p)) == 0
    d = (st[:, 1] - st[:, 0]).astype(np.int64) / 100.0
    r = eng.records().cpu().numpy()
    cur = r[:, 52].astype(np.int64)
    bd = r[:, :48].view(np.int8).reshape(B, 2, 24)
    pts = (bd[np.arange(B), cur] > 0).sum(1) + 2 * (r[np.arange(B), 48 + cur] > 0)
    dbl = r[:, 53] == r[:, 54]
    for i in np.nonzero(dbl)[0]:
        tab.setdefault((int(r[i, 53]), int(pts[i])), []).append(d[i])
print("die pts: n mean p90 p99 (us)")
for die in range(1, 7):
    row = []
    for p in range(0, 16):
        v = tab.get((die, p))
        if v and len(v) >= 20:
            row.append("%2d:%5.0f/%4.0f" % (p, np.mean(v), np.percentile(v, 99)))
    print(die, " ".join(row))
