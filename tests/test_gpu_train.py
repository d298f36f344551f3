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
