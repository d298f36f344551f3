"""The fused fp16 output layer + loss head (csrc/bg_ppo_fused.hip: bgx_ppo_rows,
bgx_ppo_gw2) against the round-2 composition it replaces, on a real rollout:
hipBLASLt logits y = h W2h^T + b2h, the loss-head kernel bgx_ppo_head_ex (pinned to
torch autograd by test_gpu_train.py), dh = ReLU'(h) fp16(dy W2h), gW2 = dy^T h,
gb2 = column sums of dy (ppo_agent.py:268-305 under autocast)."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _setup(seed=7, batch=4096, horizon=8):
    from bgx.train import PPOTrainer, lane_returns
    from bgx.ppo import global_normalize
    tr = PPOTrainer(batch=batch, horizon=horizon, seed=seed)
    tr.rollout()
    b = tr.buf
    R = global_normalize(lane_returns(b["rewards"], b["dones"]).reshape(-1)).contiguous()
    adv = (R - b["values"].reshape(-1)).contiguous()
    recs = b["records"].reshape(-1, 64).contiguous()
    acts = b["actions"].reshape(-1).to(torch.int32).contiguous()
    old = b["logp"].reshape(-1).contiguous()
    net = tr.net
    A, Hd = net.action_head.weight.shape
    W2h = torch.zeros(512, Hd, dtype=torch.float16, device="cuda")
    b2h = torch.zeros(512, dtype=torch.float16, device="cuda")
    with torch.no_grad():
        W2h[:A] = net.action_head.weight.half(); W2h[A] = net.value_head.weight[0].half()
        b2h[:A] = net.action_head.bias.half(); b2h[A] = net.value_head.bias[0].half()
        from bgx.engine import encode_records
        h = torch.relu(F.linear(encode_records(recs, torch.float16), net.fc1.weight.half(), net.fc1.bias.half()))
    return recs, acts, old, R, adv, W2h, b2h, h.contiguous()


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _fused(recs, acts, old, R, adv, W2h, b2h, h, coefs, perm, plan, row_plan, want_dy=True):
    from bgx import _lib
    from bgx._lib import check
    L = _lib.load()
    m = recs.shape[0]
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    dh = torch.empty(m, 128, dtype=torch.float16, device="cuda")
    stats = torch.empty(m, 4, dtype=torch.float32, device="cuda")
    info = torch.empty(m, dtype=torch.int32, device="cuda")
    sums = torch.zeros(3, dtype=torch.float64, device="cuda")
    dy = torch.full((m, 512), float("nan"), dtype=torch.float16, device="cuda") if want_dy else None
    eps, cv, ce, gs = coefs
    check(L.bgx_ppo_rows(_p(h), _p(perm), _p(recs), _p(acts), _p(old), _p(R), _p(adv), m, 128, 500, _p(W2h), _p(b2h),
                         eps, cv, ce, gs, _p(dh), _p(stats), _p(info), _p(sums), _p(dy), _p(row_plan), 0, s),
          "bgx_ppo_rows")
    gw2 = torch.zeros(512, 128, dtype=torch.float32, device="cuda")
    gb2 = torch.zeros(512, dtype=torch.float32, device="cuda")
    ws = torch.empty(L.bgx_ppo_gw2_workspace(m) // 4, dtype=torch.float32, device="cuda")
    k1 = float(np.float32(gs) * np.float32(ce))
    check(L.bgx_ppo_gw2(_p(h), _p(perm), _p(stats), _p(info), m, 128, 500, _p(W2h), _p(b2h), k1, _p(plan), _p(ws),
                        _p(gw2), _p(gb2), s), "bgx_ppo_gw2")
    torch.cuda.synchronize()
    return dh, dy, gw2, gb2, sums


def _reference(recs, acts, old, R, adv, W2h, b2h, h, coefs):
    from bgx import _lib
    from bgx._lib import check
    L = _lib.load()
    m = recs.shape[0]
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    y = F.linear(h, W2h, b2h).contiguous()
    vals = y[:, 500].contiguous()
    dy = torch.empty_like(y)
    dval = torch.empty_like(vals)
    sums = torch.zeros(3, dtype=torch.float64, device="cuda")
    colsum = torch.empty(2048, 512, dtype=torch.float32, device="cuda")
    eps, cv, ce, gs = coefs
    check(L.bgx_ppo_head_ex(_p(y), 1, 512, _p(vals), _p(recs), _p(acts), _p(old), _p(R), _p(adv), m, 500, eps, cv, ce,
                            gs, _p(dy), 512, _p(dval), _p(sums), 1, _p(colsum), s), "bgx_ppo_head_ex")
    dh = (dy @ W2h) * (h > 0)
    gw2 = dy.float().t() @ h.float()
    gb2 = dy.float().sum(0)
    torch.cuda.synchronize()
    return dh, dy, gw2, gb2, sums


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


COEFS = (0.25, 0.5, 0.15, 16.0)      # eps_clip, value coef, entropy coef, per-row gradient scale


def test_fused_head_matches_round2_composition():
    from bgx.train import ppo_row_plan
    args = _setup()
    recs = args[0]
    perm, plan, row_plan = ppo_row_plan(recs)
    dh, dy, gw2, gb2, sums = _fused(*args, COEFS, perm, plan, row_plan)
    rdh, rdy, rgw2, rgb2, rsums = _reference(*args, COEFS)
    # loss sums: the same per-row formulas; fp32 log-sum-exp in another order
    m = recs.shape[0]
    assert torch.allclose(sums / m, rsums / m, rtol=1e-5, atol=1e-6), (sums / m, rsums / m)
    # dy: fp16 values of the same formulas (logits from MFMA vs hipBLASLt: an fp16
    # logit may differ by one ulp where the fp32 sums round differently)
    assert not torch.isnan(dy).any()
    d = (dy.float() - rdy.float()).abs()
    tol = rdy.float().abs() * 2e-3 + 1e-6
    assert float((d > tol).float().mean()) < 1e-3, float((d > tol).float().mean())
    assert _rel(dy, rdy) < 2e-3
    assert _rel(dh, rdh) < 2e-3
    assert _rel(gw2, rgw2) < 2e-3 and _rel(gb2, rgb2) < 2e-3
    # gW2 / gb2 from the recomputed dz == dy^T h of the rows kernel's own dy
    h = args[-1]
    assert _rel(gw2, dy.float().t() @ h.float()) < 1e-5
    assert _rel(gb2, dy.float().sum(0)) < 1e-5
    # masked columns (past the legal count of a row with legal moves) get exactly 0
    cnt = recs[:, 60].int() | (recs[:, 61].int() << 8)
    cols = torch.arange(500, device="cuda")[None, :]
    masked = (cols >= cnt[:, None]) & (cnt[:, None] > 0)
    assert bool((dy[:, :500][masked] == 0).all())
    assert bool((dy[:, 501:] == 0).all())


def test_fused_head_row_order_invariant():
    """Any row order gives the same dy / dh (per-row work) and the same gW2 up to
    the fp32 summation order: the sort only schedules."""
    from bgx.train import ppo_row_plan
    args = _setup(seed=3, batch=2048, horizon=5)
    recs = args[0]
    m = recs.shape[0]
    perm, plan, row_plan = ppo_row_plan(recs)
    a = _fused(*args, COEFS, perm, plan, row_plan)
    ident = torch.arange(m, dtype=torch.int32, device="cuda")
    ntiles = (m + 31) // 32
    tasks = (ntiles + 31) // 32
    plan2 = torch.tensor([tasks * i for i in range(17)] + [0] * 16, dtype=torch.int32, device="cuda")
    rev = torch.flip(ident, [0]).contiguous()
    # unsorted rows: every row tile through the 16-tile variant
    rp2 = torch.tensor([0, 0, 0, 0, 0, 0, 0, ntiles], dtype=torch.int32, device="cuda")
    for p2 in (ident, rev):
        b = _fused(*args, COEFS, p2, plan2, rp2)
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
        assert _rel(b[2], a[2]) < 1e-6 and _rel(b[3], a[3]) < 1e-6
        assert torch.allclose(a[4] / m, b[4] / m, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("m", [33, 4096 * 8 - 5, 1 << 18])
def test_gw1_from_records_matches_feature_gemm(m):
    """bgx_ppo_gw1 (gW1 / gb1 = dh^T [x | 1] with x generated on chip from the
    records) against the GEMM it replaces over the encoded fp16 feature rows
    (encode_records, pinned to the reference's features by G2), in fp64: the
    same fp16 operands, so only the fp32 accumulation order differs.  Ragged m
    (partial last row tile), records from a real rollout (every feature type:
    bar, off, one-hot, the ones column)."""
    from bgx import _lib
    from bgx._lib import check
    from bgx.engine import encode_records
    L = _lib.load()
    recs = _setup(seed=5, batch=4096, horizon=8)[0]
    reps = (m + recs.shape[0] - 1) // recs.shape[0]
    recs = recs.repeat(reps, 1)[:m].contiguous()
    g = torch.Generator(device="cuda").manual_seed(m)
    dh = (torch.randn(m, 128, device="cuda", generator=g) * 0.5).half()
    dh[torch.rand(m, 128, device="cuda", generator=g) < 0.4] = 0          # the ReLU mask's zeros
    gw1 = torch.zeros(128, 208, dtype=torch.float32, device="cuda")
    ws = torch.empty(L.bgx_ppo_gw1_workspace(m) // 4, dtype=torch.float32, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(2):                                                   # accumulates (+=)
        check(L.bgx_ppo_gw1(_p(dh), _p(recs), m, 128, _p(ws), _p(gw1), s), "bgx_ppo_gw1")
    x = encode_records(recs, torch.float16, width=208)
    x[:, 198] = 1.0
    ref = 2 * (dh.double().t() @ x.double())
    assert torch.equal(gw1[:, 199:], torch.zeros_like(gw1[:, 199:]))
    err = (gw1.double() - ref).abs()
    assert float(err.max()) <= 1e-5 * float(ref.abs().max()) + 1e-6, float(err.max())
    assert _rel(gw1.double(), ref) < 1e-6
    # deterministic: the same call gives the same bits
    gw1b = torch.zeros_like(gw1)
    for _ in range(2):
        check(L.bgx_ppo_gw1(_p(dh), _p(recs), m, 128, _p(ws), _p(gw1b), s), "bgx_ppo_gw1")
    assert torch.equal(gw1, gw1b)


def test_gather_rollout_matches_torch_indexing():
    """bgx_gather_rollout (the update's rows in plan order, one kernel) == torch
    indexing of the records and the four per-row fields, bit for bit."""
    from bgx.train import gather_rollout
    g = torch.Generator(device="cuda").manual_seed(3)
    m = 100_003
    recs = torch.randint(0, 256, (m, 64), dtype=torch.uint8, device="cuda", generator=g)
    acts = torch.randint(0, 500, (m,), dtype=torch.int32, device="cuda", generator=g)
    old, R, adv = (torch.randn(m, device="cuda", generator=g) for _ in range(3))
    perm = torch.randperm(m, device="cuda", generator=g).to(torch.int32)
    got = gather_rollout(perm, recs, acts, old, R, adv)
    pl = perm.long()
    for a, b in zip(got, (recs[pl], acts[pl], old[pl], R[pl], adv[pl])):
        assert torch.equal(a, b)


@pytest.mark.parametrize("m", [1, 31, 1024, 4097, 3 * 65536 + 77, (1 << 20) + 5])
def test_device_row_plan_matches_torch(m):
    """bgx_ppo_plan (stable counting sort by action-tile class + the k_ppo_gw2 / rows
    plan from the class totals, no host sync) equals the torch form it replaces
    (argsort stable + bincount + cumsum, ppo_row_plan_torch) exactly: legal counts 0
    (all 16 tiles), 1..500 and above n_actions, at sizes around the 1,024-row blocks."""
    from bgx.train import ppo_row_plan, ppo_row_plan_torch
    g = torch.Generator(device="cpu").manual_seed(m)
    recs = torch.randint(0, 256, (m, 64), dtype=torch.uint8, generator=g)
    kind = torch.randint(0, 10, (m,), generator=g)
    cnt = torch.where(kind == 0, torch.zeros(m, dtype=torch.int64),
                      torch.where(kind == 1, torch.randint(501, 2000, (m,), generator=g),
                                  torch.randint(1, 60, (m,), generator=g)))
    cnt = torch.where(kind == 2, torch.randint(60, 501, (m,), generator=g), cnt)
    recs[:, 60] = (cnt & 255).to(torch.uint8)
    recs[:, 61] = (cnt >> 8).to(torch.uint8)
    recs = recs.cuda()
    p1, pl1, rp1 = ppo_row_plan(recs)
    p2, pl2, rp2 = ppo_row_plan_torch(recs)
    assert torch.equal(p1, p2)
    assert torch.equal(pl1, pl2)
    assert torch.equal(rp1, rp2)


def test_device_row_plan_on_rollout():
    from bgx.train import ppo_row_plan, ppo_row_plan_torch
    recs = _setup(seed=5, batch=2048, horizon=6)[0]
    for a, b in zip(ppo_row_plan(recs), ppo_row_plan_torch(recs)):
        assert torch.equal(a, b)
