"""GPU-resident PPO trainer: rollout buffers are consistent with the engine and
the policy kernel, and an update runs end to end (finite losses, weights move)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_trainer_iteration():
    from bgx.train import PPOTrainer
    tr = PPOTrainer(batch=2048, horizon=12, seed=3, pinned=True, chunk=8192)
    w0 = [p.detach().clone() for p in tr.net.parameters()]
    m = tr.iteration()
    for k in ("policy_loss", "value_loss", "entropy", "total_loss"):
        assert np.isfinite(m[k]), (k, m)
    assert m["env_steps"] == 2048 * 12
    assert any(not torch.equal(a, b) for a, b in zip(w0, tr.net.parameters()))
    recs = tr.buf["records"]
    counts = (recs[..., 60].int() | (recs[..., 61].int() << 8))
    acts = tr.buf["actions"]
    assert bool(((acts < counts) | (counts == 0)).all())
    torch.cuda.synchronize()
    assert torch.equal(tr.pinned["actions"], acts.cpu())
    # rewards only on done steps, in {1, 1.5, 2} (no invalid actions are ever sampled)
    r, d = tr.buf["rewards"], tr.buf["dones"].bool()
    assert bool((r[~d] == 0).all()) and bool(torch.isin(r[d], torch.tensor([1.0, 1.5, 2.0], device="cuda")).all())
    m2 = tr.iteration()
    assert np.isfinite(m2["total_loss"])


def test_reference_returns_mode():
    from bgx.train import PPOTrainer
    tr = PPOTrainer(batch=256, horizon=8, seed=1, returns="reference")
    m = tr.iteration()
    assert np.isfinite(m["total_loss"])


@pytest.mark.parametrize("amp", [False, True])
def test_fused_loss_head_matches_torch(amp):
    """bgx_ppo_head (fused loss head) vs the torch formulation of ppo_epoch: same
    loss parts and parameter gradients (fp32: 1e-4 relative; fp16 autocast: the
    gradients pass through fp16 either way, 2e-2 relative on the largest)."""
    import copy
    from torch.amp import GradScaler
    from bgx.train import PPOTrainer, ppo_epoch, features_and_masks
    from bgx.ppo import global_normalize
    from bgx.train import lane_returns
    tr = PPOTrainer(batch=1024, horizon=6, seed=4)
    tr.rollout()
    buf = tr.buf
    R = global_normalize(lane_returns(buf["rewards"], buf["dones"]).reshape(-1))
    adv = R - buf["values"].reshape(-1)
    recs = buf["records"].reshape(-1, 64)
    f, legal = features_and_masks(recs, tr.A)
    data = [(f, legal, buf["actions"].reshape(-1), buf["logp"].reshape(-1), R, adv, recs)]
    N = recs.shape[0]
    res = {}
    for fused in (False, True):
        net = copy.deepcopy(tr.net)
        opt = torch.optim.Adam(net.parameters(), lr=1e-3)
        sc = GradScaler(device="cuda", enabled=amp)
        parts = ppo_epoch(net, opt, sc, data, N, 0.15, amp=amp, fused=fused, step=False)
        res[fused] = (parts, [p.grad.detach().float().clone() for p in net.parameters()])
    (p0, g0), (p1, g1) = res[False], res[True]
    assert torch.allclose(p0, p1, rtol=1e-4, atol=1e-6), (p0, p1)
    tol = 2e-2 if amp else 1e-4
    for a, b in zip(g0, g1):
        assert (a - b).abs().max() <= tol * a.abs().max() + 1e-7, ((a - b).abs().max(), a.abs().max())
