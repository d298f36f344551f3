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
