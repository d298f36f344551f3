"""Prints the error metrics of tests/test_gpu_ppo_fused.py without asserting (debug aid)."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mlp-ppo-2ply-p3_amd"), os.path.join(ROOT, "tests")]
import test_gpu_ppo_fused as T  # noqa: E402
from bgx.train import ppo_row_plan  # noqa: E402
args = T._setup()
recs, h = args[0], args[-1]
perm, plan, row_plan = ppo_row_plan(recs)
dh, dy, gw2, gb2, sums = T._fused(*args, T.COEFS, perm, plan, row_plan)
rdh, rdy, rgw2, rgb2, rsums = T._reference(*args, T.COEFS)
print("sums", sums.tolist(), rsums.tolist())
print("dy rel", T._rel(dy, rdy), "dh rel", T._rel(dh, rdh), "gw2 rel", T._rel(gw2, rgw2), "gb2 rel", T._rel(gb2, rgb2))
print("gw2 vs own dy", T._rel(gw2, dy.float().t() @ h.float()), "gb2 vs own", T._rel(gb2, dy.float().sum(0)))
d = (dh.float() - rdh.float()).abs()
r, c = divmod(int(d.argmax()), dh.shape[1])
print("worst dh", r, c, float(dh[r, c]), float(rdh[r, c]))
print("row", r, "dh", dh[r, :16].tolist())
print("ref", rdh[r, :16].tolist())
ratio = None
for c0 in range(0, 128, 32):
    blk = dh[:64, c0:c0 + 32].float(); rb = rdh[:64, c0:c0 + 32].float()
    print("cols", c0, "rel", float((blk - rb).norm() / rb.norm()))
# permutation search: for column c of dh, which column of rdh matches best
best = []
for c in range(32):
    errs = [float((dh[:, c].float() - rdh[:, k].float()).norm()) for k in range(128)]
    best.append(min(range(128), key=lambda k: errs[k]))
print("col match", best)
gb = []
for c in range(32):
    errs = [float((gw2[:, c] - rgw2[:, k]).norm()) for k in range(128)]
    gb.append(min(range(128), key=lambda k: errs[k]))
print("gw2 col match", gb)
