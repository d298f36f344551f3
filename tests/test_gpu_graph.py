"""C3 rollout steps captured in a HIP graph (bench.py's C3 path): replays equal
the same steps run eagerly (device step counter for the policy's noise, engines
joined before and at the end of the capture), and each replay draws fresh noise."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(bgx, seed):
    from bgx.policy import PolicyNet
    torch.manual_seed(0)
    net = PolicyNet(hidden_size=128).cuda()
    net.pack()
    eng = bgx.Engine(batch=4096, dice="philox", seed=seed, auto_reset=True)
    eng.reset(want_obs=False)
    for i in range(30):                                   # a mid-game population
        a, _, _ = net.act(eng, seed=1, step=i)
        eng.step(a, want_obs=False, want_info=False)
    torch.cuda.synchronize()
    return net, eng


@pytest.mark.parametrize("fork", [True, False])
def test_graph_replay_matches_eager_steps(fork):
    # fork=False: the captured engine runs each step on one stream (a linear graph,
    # bench.py's C3 layout) against eager forked steps: the same trajectories
    import bgx
    G = 4
    net, ea = _setup(bgx, 21)
    _, eb = _setup(bgx, 21)
    eb.set_fork(fork)
    assert torch.equal(ea.records(), eb.records())
    n = ea.batch
    bufs = [dict(act=torch.empty(n, dtype=torch.int32, device="cuda"),
                 logp=torch.empty(n, device="cuda"), val=torch.empty(n, device="cuda"),
                 rew=torch.empty(n, device="cuda"), done=torch.empty(n, dtype=torch.uint8, device="cuda"))
            for _ in range(2)]
    ctr = torch.full((1,), 1000, dtype=torch.int32, device="cuda")

    def one(e, b, i, step_ctr):
        net.act(e, seed=9, step=i, step_ctr=step_ctr, out=(b["act"], b["logp"], b["val"]))
        e.step(b["act"], want_obs=False, want_info=False, out=(b["rew"], b["done"]))

    cap = torch.cuda.Stream()
    with torch.cuda.stream(cap):
        eb.join()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        for i in range(G):
            one(eb, bufs[1], i, ctr)
        eb.join()
        net.advance_counter(ctr, G)
    torch.cuda.synchronize()
    for rep in range(3):                                  # replay r == eager steps 1000 + rG + i
        g.replay()
        for i in range(G):
            one(ea, bufs[0], 1000 + rep * G + i, None)
        torch.cuda.synchronize()
        assert int(ctr.item()) == 1000 + (rep + 1) * G
        assert torch.equal(ea.records(), eb.records()), rep
        for k in ("act", "val", "rew", "done"):
            assert torch.equal(bufs[0][k], bufs[1][k]), (rep, k)
        assert torch.equal(bufs[0]["logp"], bufs[1]["logp"]), rep
