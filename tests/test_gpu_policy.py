"""Fused policy kernel (bgx_policy_act) vs the reference BackgammonPolicyNetwork
(golden G5 logits/values) and torch fp32.  Tolerance: 1e-5 absolute on logits,
values and log-probs (BASELINE.json: MLP value outputs within 1e-5 fp32)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
TOL = 1e-5


@pytest.fixture(scope="module")
def bgx():
    import bgx as _bgx
    return _bgx


def _records(boards, players, counts=None):
    n = len(boards)
    r = np.zeros((n, 64), np.uint8)
    r[:, :52] = np.asarray(boards, np.int8).view(np.uint8)
    r[:, 52] = players
    c = np.full(n, 500) if counts is None else np.asarray(counts)
    r[:, 60] = c & 0xFF
    r[:, 61] = c >> 8
    return torch.from_numpy(r).cuda()


def _net(mlp, H):
    from bgx.policy import PolicyNet
    net = PolicyNet(hidden_size=H).cuda()
    sd = {k[len(f"h{H}_"):]: torch.from_numpy(v) for k, v in mlp.items()
          if k.startswith(f"h{H}_") and not k.endswith(("logits", "values"))}
    net.load_state_dict(sd)
    return net


@pytest.mark.parametrize("H", [128, 40])
def test_policy_logits_values_match_reference(bgx, golden, H):
    mlp, feat, mg = golden("mlp"), golden("features"), golden("movegen")
    idx = feat["obs_idx"][:600]
    rec = _records(mg["boards"][idx], feat["obs_player"][:600])
    net = _net(mlp, H)
    act, logp, val, logits = net.act(rec, seed=1, step=0, want_logits=True)
    lg = logits[:, :500].cpu().numpy()
    assert np.abs(lg - mlp[f"h{H}_logits"][:600]).max() < TOL
    assert np.abs(val.cpu().numpy() - mlp[f"h{H}_values"][:600]).max() < TOL
    assert np.abs(logits[:, 500].cpu().numpy() - mlp[f"h{H}_values"][:600]).max() < TOL


def test_policy_logp_and_greedy(bgx):
    from bgx.policy import PolicyNet, masked_probs
    torch.manual_seed(0)
    net = PolicyNet(hidden_size=128).cuda()
    eng = bgx.Engine(batch=4096, dice="philox", seed=5)
    eng.reset()
    for i in range(30):
        rec = eng.records()
        a, _, _ = net.act(rec, seed=3, step=i)
        eng.step(a)
    rec = eng.records()
    counts = (rec[:, 60].int() | (rec[:, 61].int() << 8))
    x = bgx.encode(rec[:, :52].contiguous(), rec[:, 52].contiguous())
    with torch.no_grad():
        lg, v = net(x)
    masks = (torch.arange(500, device="cuda")[None] < counts[:, None]).float()
    probs = masked_probs(lg, masks)
    a, logp, val = net.act(rec, seed=7, step=1)
    # zero legal moves: the reference softmaxes all 500 masked logits, any action passes
    assert torch.all((a < counts) | (counts == 0))
    legal = counts > 0
    ref_logp = torch.log(probs.gather(1, a.long()[:, None]).squeeze(1))
    assert (logp - ref_logp)[legal].abs().max().item() < 1e-4   # probs path goes through exp/log in fp32
    lsm = torch.log_softmax(lg + (masks + 1e-45).log(), -1).gather(1, a.long()[:, None]).squeeze(1)
    assert (logp - lsm).abs().max().item() < TOL
    assert (val - v).abs().max().item() < TOL
    g, _, _ = net.act(rec, greedy=True)
    assert torch.equal(g.long(), torch.argmax(probs, -1))


def test_policy_sampling_distribution(bgx):
    """Empirical action frequencies of one position vs softmax(masked) (chi-square)."""
    from bgx.policy import PolicyNet, masked_probs
    torch.manual_seed(1)
    net = PolicyNet(hidden_size=128).cuda()
    with torch.no_grad():
        net.action_head.weight.mul_(8.0)      # a peaked, non-uniform distribution
    eng = bgx.Engine(batch=64, dice="philox", seed=11)
    eng.reset()
    rec = eng.records()
    counts = (rec[:, 60].int() | (rec[:, 61].int() << 8)).cpu().numpy()
    lane = int(np.argmax(counts))
    n = int(counts[lane])
    N = 200_000
    reps = rec[lane:lane + 1].repeat(N, 1)
    a, _, _ = net.act(reps, seed=123, step=9)
    freq = np.bincount(a.cpu().numpy(), minlength=500)[:500] / N
    x = bgx.encode(rec[lane:lane + 1, :52].contiguous(), rec[lane:lane + 1, 52].contiguous())
    with torch.no_grad():
        lg, _ = net(x)
    mask = (torch.arange(500, device="cuda") < n).float()[None]
    p = masked_probs(lg, mask)[0].cpu().numpy()
    # illegal actions keep the reference's tiny mass exp(z - 103.28) (not -inf)
    pill = p[n:].sum()
    assert abs(freq[n:].sum() - pill) <= 6 * np.sqrt(pill / N) + 1e-5
    keep = p * N > 20
    chi2 = ((freq[keep] - p[keep]) ** 2 / p[keep]).sum() * N
    dof = int(keep.sum()) - 1
    assert chi2 < dof + 6 * np.sqrt(2 * dof) + 10, (chi2, dof)


def test_policy_sampling_no_legal_moves(bgx):
    """A row with no legal move samples from the softmax over all 500 masked
    logits (ppo_agent.py:160-170 with an all-zero mask).  The kernel draws such
    rows lane-parallel; rows with legal moves in the same waves are unaffected."""
    from bgx.policy import PolicyNet, masked_probs
    torch.manual_seed(2)
    net = PolicyNet(hidden_size=128).cuda()
    with torch.no_grad():
        net.action_head.weight.mul_(8.0)
    eng = bgx.Engine(batch=64, dice="philox", seed=13)
    eng.reset()
    rec = eng.records()
    N = 200_000
    reps = rec[:2].repeat(N // 2, 1).contiguous()
    reps[0::2, 60] = 0                         # even rows: no legal move
    reps[0::2, 61] = 0
    a, logp, _ = net.act(reps, seed=321, step=4)
    x = bgx.encode(rec[:1, :52].contiguous(), rec[:1, 52].contiguous())
    with torch.no_grad():
        lg, _ = net(x)
    p = masked_probs(lg, torch.zeros(1, 500, device="cuda"))[0].cpu().numpy()
    lsm = torch.log_softmax(lg + (torch.zeros(1, 500, device="cuda") + 1e-45).log(), -1)[0]
    az = a[0::2].long()
    # every logit carries the -103.28 mask here: |z| ~ 110, where one fp32 ulp is 7.6e-6
    assert (logp[0::2] - lsm[az]).abs().max().item() < 4 * TOL
    freq = np.bincount(az.cpu().numpy(), minlength=500)[:500] / (N // 2)
    keep = p * (N // 2) > 20
    chi2 = ((freq[keep] - p[keep]) ** 2 / p[keep]).sum() * (N // 2)
    dof = int(keep.sum()) - 1
    assert chi2 < dof + 6 * np.sqrt(2 * dof) + 10, (chi2, dof)
    c1 = int(rec[1, 60]) | (int(rec[1, 61]) << 8)
    assert c1 > 0 and torch.all(a[1::2] < c1)


def test_rollout_path_in_place(bgx):
    """The rollout path (PPOTrainer, bench C3): act(engine, out=, records_out=)
    reads the lane records in place and stores them; step(out=) writes rewards /
    dones into caller rows.  Same actions, log-probs, values, stored records,
    rewards, dones and final boards as the copying path, over 40 steps (Philox
    split dispatch with its side stream, double-buffered overflow counters);
    B = 3,000 leaves a ragged last 32-row wave in the policy kernel."""
    from bgx.policy import PolicyNet
    torch.manual_seed(5)
    net = PolicyNet(hidden_size=128).cuda()
    B = 3000
    e1 = bgx.Engine(batch=B, dice="philox", seed=21)
    e2 = bgx.Engine(batch=B, dice="philox", seed=21)
    e1.reset(want_obs=False)
    e2.reset(want_obs=False)
    kw = dict(device="cuda")
    rec_out = torch.empty(B, 64, dtype=torch.uint8, **kw)
    a2 = torch.empty(B, dtype=torch.int32, **kw)
    lp2, v2, r2 = (torch.empty(B, **kw) for _ in range(3))
    d2 = torch.empty(B, dtype=torch.uint8, **kw)
    for t in range(40):
        rec = e1.records()
        a1, lp1, v1 = net.act(rec, seed=9, step=t)
        net.act(e2, seed=9, step=t, out=(a2, lp2, v2), records_out=rec_out)
        assert torch.equal(rec, rec_out)
        assert torch.equal(a1, a2) and torch.equal(lp1, lp2) and torch.equal(v1, v2)
        _, r1, d1, _ = e1.step(a1, want_obs=False, want_info=False)
        e2.step(a2, want_obs=False, want_info=False, out=(r2, d2))
        assert torch.equal(r1, r2) and torch.equal(d1, d2)
    assert torch.equal(e1.records(), e2.records())
    assert e1.error() == 0 and e2.error() == 0


def _act_both(net, rec, seed, step, dbg):
    dbg.setenv("BGX_POLICY_SKIP", "1")
    on = [t.clone() for t in net.act(rec, seed=seed, step=step)]
    dbg.setenv("BGX_POLICY_SKIP", "0")
    off = [t.clone() for t in net.act(rec, seed=seed, step=step)]
    dbg.delenv("BGX_POLICY_SKIP")
    return on, off


def _assert_same(on, off, rec):
    assert torch.equal(on[0], off[0])                  # the sampled actions
    assert torch.equal(on[2], off[2])                  # values
    d = (on[1] - off[1]).abs()
    zero = (rec[:, 60].int() | rec[:, 61].int()) == 0
    assert d[~zero].max().item() <= 1e-6               # log-probs: summation order only
    # count-0 rows: every logit carries the -103.28 mask, |z| ~ 110, one fp32 ulp 7.6e-6
    # (as test_policy_sampling_no_legal_moves); their 4 waves' partial sums merge in LDS
    if zero.any():
        assert d[zero].max().item() < 4 * TOL


@pytest.mark.parametrize("heavy", ["64", "32", "1000"])
def test_policy_tile_skip_matches_full_pass(bgx, dbg, heavy):
    """The masked-action tile skip and the extra waves (bg_mlp.hip, k_policy_act MODE 0:
    rows with no legal move or more than BGX_POLICY_HEAVY legal actions gathered into
    workgroups that split the action tiles four ways; 1000 = count-0 rows only, the
    round-4 form) give the outputs of the full 16-tile pass: self-play positions
    (count-0 rows, doubles with hundreds of moves), a window with more gathered rows
    than the extra waves take, a ragged batch, and weights whose logit bound is too
    loose for any skip."""
    dbg.setenv("BGX_POLICY_HEAVY", heavy)
    from bgx.policy import PolicyNet
    torch.manual_seed(0)
    net = PolicyNet(hidden_size=128).cuda()
    eng = bgx.Engine(batch=8192, dice="philox", seed=11)
    eng.reset()
    zero_rows = 0
    for i in range(24):
        rec = eng.records()
        zero_rows += int((rec[:, 60].int() | rec[:, 61].int()).eq(0).sum())
        on, off = _act_both(net, rec, 7, i, dbg)
        _assert_same(on, off, rec)
        eng.step(on[0])
    assert zero_rows > 0
    rec = eng.records().clone()
    rec[300:420, 60:62] = 0                              # 120 count-0 rows in one 256-row window
    rec[1000:1010, 60] = 244                             # 500 legal actions
    rec[1000:1010, 61] = 1
    _assert_same(*_act_both(net, rec, 9, 0, dbg), rec)
    _assert_same(*_act_both(net, rec[:5000 - 17], 9, 1, dbg), rec[:5000 - 17])
    big = PolicyNet(hidden_size=128).cuda()
    with torch.no_grad():
        big.load_state_dict(net.state_dict())
        big.action_head.weight.mul_(40.0)
    _assert_same(*_act_both(big, rec, 9, 2, dbg), rec)
