"""PPO agent parity with the reference (golden G6: select_action + update() on
CPU) and the multi-rank exchange (gloo, world_size 2) — CPU only."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from bgx.ppo import BackgammonPPOAgent, allreduce_mean_, global_normalize


def test_agent_matches_reference_update(golden):
    g = golden("ppo")
    torch.manual_seed(3)
    agent = BackgammonPPOAgent(action_size=500, device=torch.device("cpu"))
    for k, v in agent.policy_network.state_dict().items():
        assert np.array_equal(v.numpy(), g["init_" + k]), k
    N, T = 8, 16
    obs = torch.from_numpy(g["obs"])
    masks = torch.from_numpy(g["masks"])
    torch.manual_seed(11)
    acts = []
    for t in range(T):
        a = agent.select_action(obs[t * N:(t + 1) * N], masks[t * N:(t + 1) * N])
        acts.append(a)
        for i in range(N):
            agent.memory[-N + i]["reward"] = torch.tensor([g["rewards"][t * N + i]])
            agent.memory[-N + i]["done"] = torch.tensor([bool(g["dones"][t * N + i])])
    assert np.array_equal(np.concatenate(acts), g["actions"])
    old_logp = torch.cat([m["action_log_prob"] for m in agent.memory]).detach().numpy()
    assert np.allclose(old_logp, g["old_logp"], atol=1e-6)
    agent.update()
    assert np.allclose([agent.last_policy_loss, agent.last_value_loss, agent.last_entropy_loss,
                        agent.last_total_loss], g["losses"], atol=1e-5)
    for k, v in agent.policy_network.state_dict().items():
        assert np.allclose(v.numpy(), g["final_" + k], atol=1e-6), k


def test_masked_softmax_semantics(golden):
    from bgx.policy import masked_probs
    g = golden("ppo")
    p = masked_probs(torch.from_numpy(g["sa_logits"]), torch.from_numpy(g["sa_masks"]))
    assert np.allclose(p.numpy(), g["sa_probs"], atol=1e-7)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=ws)
    torch.manual_seed(0)
    R = torch.randn(64)
    X = torch.randn(64, 198)
    lin = torch.nn.Linear(198, 7)
    shard = slice(rank * 32, (rank + 1) * 32)
    nr = global_normalize(R[shard])
    loss = (lin(X[shard]) ** 2).mean()
    loss.backward()
    grads = [p.grad.clone() for p in lin.parameters()]
    allreduce_mean_(grads)
    q.put((rank, nr.numpy(), [g.numpy() for g in grads]))
    torch.distributed.destroy_process_group()


def test_two_rank_allreduce_equals_full_batch():
    """world_size 2 (gloo): the all-reduced gradient and the global return
    normalisation equal the single-process values on the concatenated batch."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (nr, gr)) for r, nr, gr in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
    torch.manual_seed(0)
    R = torch.randn(64)
    X = torch.randn(64, 198)
    lin = torch.nn.Linear(198, 7)
    full = ((R - R.mean()) / (R.std() + 1e-5)).numpy()
    assert np.allclose(np.concatenate([res[0][0], res[1][0]]), full, atol=1e-5)
    (lin(X) ** 2).mean().backward()
    for g_ref, g0, g1 in zip([p.grad.numpy() for p in lin.parameters()], res[0][1], res[1][1]):
        assert np.allclose(g0, g_ref, atol=1e-6) and np.allclose(g1, g_ref, atol=1e-6)


def test_returns_functions_match_reference_quirk():
    from bgx.train import lane_returns, reference_returns
    rng = np.random.RandomState(0)
    T, B = 12, 5
    r = torch.from_numpy(rng.choice([0.0, 0.0, 1.0, -1.0, 1.5], size=(T, B)).astype(np.float32))
    d = torch.from_numpy((rng.rand(T, B) < 0.2).astype(np.uint8))
    agent = BackgammonPPOAgent(action_size=500, device=torch.device("cpu"))
    ref = np.array(agent.compute_returns(r.reshape(-1), d.reshape(-1).bool()), np.float32).reshape(T, B)
    assert np.allclose(reference_returns(r, d).numpy(), ref, atol=1e-5)
    lane = lane_returns(r, d).numpy()
    for b in range(B):
        R, exp = 0.0, np.zeros(T, np.float32)
        for t in range(T - 1, -1, -1):
            R = 0.0 if d[t, b] else R
            R = float(r[t, b]) + 0.99 * R
            exp[t] = R
        assert np.allclose(lane[:, b], exp, atol=1e-5)


def _epoch_inputs(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    feats = torch.rand(n, 198, generator=g)
    legal = torch.rand(n, 500, generator=g) < 0.1
    legal[:, 0] = True
    acts = torch.randint(0, 1, (n,), generator=g)
    old = torch.log(torch.rand(n, generator=g) * 0.5 + 0.25)
    ret = torch.randn(n, generator=g)
    adv = torch.randn(n, generator=g)
    return feats, legal, acts, old, ret, adv


def _fresh_net():
    from bgx.policy import PolicyNet
    torch.manual_seed(5)
    net = PolicyNet()
    # SGD(lr=1): the parameter change IS the (all-reduced, unscaled) gradient, so the
    # comparison below checks gradients (Adam's first step is ~lr*sign(g): ill-conditioned)
    opt = torch.optim.SGD(net.parameters(), lr=1.0)
    return net, opt, torch.amp.GradScaler(device="cpu")


@pytest.mark.parametrize("amp,rtol,atol", [(False, 1e-4, 1e-6), (True, 2e-2, 2e-3)])
def test_chunked_epoch_equals_full_batch(amp, rtol, atol):
    """Gradient accumulation over chunks == one full-batch gradient (fp32 tight;
    under the reference's autocast the tolerance is bf16's)."""
    from bgx.train import ppo_epoch
    data = _epoch_inputs(256)
    net1, opt1, sc1 = _fresh_net()
    ppo_epoch(net1, opt1, sc1, [data], 256, 0.15, amp=amp)
    net2, opt2, sc2 = _fresh_net()
    chunks = [tuple(x[i:i + 64] for x in data) for i in range(0, 256, 64)]
    ppo_epoch(net2, opt2, sc2, chunks, 256, 0.15, amp=amp)
    for a, b in zip(net1.parameters(), net2.parameters()):
        assert torch.allclose(a, b, atol=atol, rtol=rtol)


def _epoch_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=ws)
    from bgx.train import ppo_epoch
    data = _epoch_inputs(256)
    net, opt, sc = _fresh_net()
    shard = tuple(x[rank * 128:(rank + 1) * 128] for x in data)
    ppo_epoch(net, opt, sc, [shard], 128, 0.15, amp=False)
    q.put((rank, [p.detach().numpy().copy() for p in net.parameters()]))
    torch.distributed.destroy_process_group()


def test_two_rank_ppo_epoch_equals_full_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_epoch_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    from bgx.train import ppo_epoch
    net, opt, sc = _fresh_net()
    ppo_epoch(net, opt, sc, [_epoch_inputs(256)], 256, 0.15, amp=False)
    for i, p in enumerate(net.parameters()):
        assert np.allclose(res[0][i], p.detach().numpy(), atol=1e-5, rtol=1e-4)
        assert np.allclose(res[1][i], res[0][i])


def _norm_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=ws)
    R = _big_returns()
    n = R.numel() // ws
    q.put((rank, global_normalize(R[rank * n:(rank + 1) * n]).numpy()))
    torch.distributed.destroy_process_group()


def _big_returns():
    # discounted-return-like values: mostly small, a long tail toward +-2, offset mean
    g = torch.Generator().manual_seed(7)
    return (0.3 + 0.6 * torch.randn(1 << 21, generator=g) * torch.rand(1 << 21, generator=g)).float()


def test_two_rank_global_normalize_large():
    """2^21 returns over 2 ranks (gloo): the fp64 all-reduced (sum, sum of squares, n)
    normalisation equals the single-process (R - mean) / (std + 1e-5) within 1e-6."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_norm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    R = _big_returns()
    full = ((R - R.mean()) / (R.std() + 1e-5)).numpy()
    got = np.concatenate([res[0], res[1]])
    assert np.abs(got - full).max() < 1e-6


def test_episode_stats_match_reference_loop():
    """bgx.train.episode_stats == the reference loop's per-env accounting
    (train.py:55-99: episode_rewards += rewards; on done record the episode
    reward and win = winner == current_player, then zero), carried across two
    rollouts."""
    from bgx.train import episode_stats, EPISODE_STATS
    g = torch.Generator().manual_seed(3)
    T, B = 16, 37
    carry = torch.zeros(B, dtype=torch.float64)
    ref_acc = [0.0] * B
    for _ in range(2):
        dones = (torch.rand(T, B, generator=g) < 0.15).to(torch.uint8)
        win_r = torch.tensor([1.0, 1.5, 2.0])[torch.randint(0, 3, (T, B), generator=g)]
        rewards = torch.where(dones.bool(), win_r, torch.randint(0, 2, (T, B), generator=g) * 0.01)
        movers = torch.randint(0, 2, (T, B), generator=g, dtype=torch.uint8)
        got = dict(zip(EPISODE_STATS, episode_stats(rewards, dones, movers, carry).tolist()))
        want = dict.fromkeys(EPISODE_STATS, 0.0)
        for t in range(T):
            for i in range(B):
                ref_acc[i] += float(rewards[t, i])
                if dones[t, i]:
                    want["episodes"] += 1
                    want["episode_reward_sum"] += ref_acc[i]
                    want["wins"] += 1                       # winner == current_player on every win step
                    want["p1_wins"] += int(movers[t, i] == 0)
                    want["gammons"] += int(rewards[t, i] == 1.5)
                    want["backgammons"] += int(rewards[t, i] == 2.0)
                    ref_acc[i] = 0.0
        for k in EPISODE_STATS:
            assert got[k] == pytest.approx(want[k], abs=1e-9), k
        np.testing.assert_allclose(carry.numpy(), np.array(ref_acc), atol=1e-12)


def test_entropy_anneal_modes():
    """train.py never increments agent.total_episodes (it counts a module global,
    train.py:74), so ppo_agent.py:193-197 keeps the coefficient at 0.15; under
    train_single.py (agent.total_episodes += 1 per episode, :78) it anneals
    linearly to 0.01 over 400,000 episodes.  The reference agent class's own
    update_entropy_coef gives the train_single values for a counted episode total."""
    from bgx.train import entropy_coef_after_update
    from bgx.ppo import ENTROPY_COEF_START, ENTROPY_COEF_END, ENTROPY_ANNEAL_EPISODES
    agent = BackgammonPPOAgent(action_size=500, device=torch.device("cpu"))
    for eps in (0, 1, 65_536, 200_000, 399_999, 400_000, 10_000_000):
        assert entropy_coef_after_update("train", eps) == ENTROPY_COEF_START
        agent.total_episodes = eps
        agent.update_entropy_coef()
        assert entropy_coef_after_update("train_single", eps) == agent.entropy_coef
    assert entropy_coef_after_update("train_single", ENTROPY_ANNEAL_EPISODES // 2) == pytest.approx(0.08)
    assert entropy_coef_after_update("train_single", 10 ** 9) == pytest.approx(ENTROPY_COEF_END)
    import inspect
    from bgx.train import PPOTrainer
    assert inspect.signature(PPOTrainer).parameters["entropy_anneal"].default == "train"
