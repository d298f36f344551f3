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
    # the update's record encoder == the board encoder (G2-pinned) on every rollout row
    from bgx.engine import encode, encode_records
    flat = recs.reshape(-1, 64)
    f32 = encode(flat[:, :52].contiguous(), flat[:, 52].contiguous())
    assert torch.equal(encode_records(flat), f32)
    assert torch.equal(encode_records(flat, torch.float16), f32.half())
    # 208-wide rows (the update's GEMM operand): the same features, then zeros
    for dt in (torch.float32, torch.float16):
        p208 = encode_records(flat, dt, width=208)
        assert p208.shape == (flat.shape[0], 208)
        assert torch.equal(p208[:, :198], f32.to(dt)) and not bool(p208[:, 198:].any())
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
    # the second rollout was replayed from HIP graphs, each carrying the pinned-host copy
    # of the previous slot pair (bgx.hostcopy): every field of every slot on the host
    assert tr._graphs is not None
    torch.cuda.synchronize()
    for k, v in tr.buf.items():
        assert torch.equal(tr.pinned[k], v.cpu()), k
    # episode metrics (train.py:64-99): every finished self-play episode is a win for
    # its last mover, and its reward is that win's reward (no other rewards occur)
    for _ in range(16):
        m3 = tr.iteration()
        if m3["episodes"] > 0:
            break
    assert m3["episodes"] > 0 and m3["win_rate"] == 1.0
    assert 0.0 <= m3["p1_win_rate"] <= 1.0 and 1.0 <= m3["avg_episode_reward"] <= 2.0
    assert m3["total_episodes"] == tr.total_episodes


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


def _records_from_fixture(g):
    n = len(g["counts"])
    rec = np.zeros((n, 64), np.uint8)
    rec[:, :52] = g["boards"].view(np.uint8)
    rec[:, 52] = g["players"]
    rec[:, 60] = g["counts"] & 0xFF
    rec[:, 61] = g["counts"] >> 8
    return torch.from_numpy(rec)


@pytest.mark.parametrize("variant", ["fp32", "fp16"])
def test_update_matches_reference(golden, variant):
    """PPOTrainer.update(returns="reference") on the reference agent's own batch
    (golden G6b / G6c: ppo_agent.py:218-305 run by importing the reference, 1,024
    rows, init weights, sampled actions and log-probs, old values) gives the
    reference's loss parts and post-update weights.

    fp32 (autocast off on both sides): losses and final weights within 1e-5
    (measured: 1e-7 and 8.5e-6, tools/ppo_parity_report.py).
    fp16 (the reference's CUDA autocast, emulated for the fixture by CPU fp16
    autocast + GradScaler; here the fused fp16 epoch: hipBLASLt fp16 GEMMs + the
    HIP loss head): losses within 1e-5 (measured 3.4e-7); fewer than 0.2 % of the
    entries of each weight update (final - init) differ by more than 1e-4
    (measured 0.07 % of fc1.weight, none elsewhere).  After 4 Adam steps a weight
    moves by up to 4e-3 (lr 1e-3, first steps ~ lr * sign(g)), and fp16 rounding
    differences between CPU and GPU GEMMs flip the sign of a few near-zero
    gradient entries, which moves those weights by ~2e-3."""
    from bgx.engine import encode, encode_records
    from bgx.train import PPOTrainer
    g = golden("ppo_" + variant)
    N, T = int(g["N"]), int(g["T"])
    tr = PPOTrainer(batch=N, horizon=T, hidden=128, returns="reference", amp=(variant == "fp16"))
    sd = {k[5:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("init_")}
    tr.net.load_state_dict(sd)
    rec = _records_from_fixture(g).cuda()
    assert torch.equal(encode(rec[:, :52].contiguous(), rec[:, 52].contiguous()).cpu(), torch.from_numpy(g["obs"]))
    assert torch.equal(encode_records(rec).cpu(), torch.from_numpy(g["obs"]))
    assert torch.equal(encode_records(rec, torch.float16).cpu(), torch.from_numpy(g["obs"]).half())
    tr.load_rollout(rec, torch.from_numpy(g["actions"]), torch.from_numpy(g["old_logp"]),
                    torch.from_numpy(g["old_v"]), torch.from_numpy(g["rewards"]), torch.from_numpy(g["dones"]))
    m = tr.update()
    got = np.array([m["policy_loss"], m["value_loss"], m["entropy"], m["total_loss"]])
    if variant == "fp32":
        assert np.abs(got - g["losses"]).max() < 1e-5, (got, g["losses"])
        for k, v in tr.net.state_dict().items():
            d = np.abs(v.cpu().numpy() - g["final_" + k]).max()
            assert d < 1e-5, (k, d)
    else:
        assert np.abs(got - g["losses"]).max() < 1e-5, (got, g["losses"])
        for k, v in tr.net.state_dict().items():
            du_ref = g["final_" + k] - g["init_" + k]
            du = v.cpu().numpy() - g["init_" + k]
            frac = np.mean(np.abs(du - du_ref) > 1e-4)
            assert frac < 2e-3, (k, frac)


def test_manual_fp16_epoch_large_batch():
    """The fused fp16 epoch at a production-sized batch (2^21 rows: GradScaler scale /
    n would put per-row fp16 gradients in the subnormal range) against the fp32
    torch epoch on the same data: relative Frobenius error of every gradient < 2e-3
    (measured 2.5e-4 .. 4.6e-4)."""
    import copy
    from torch.amp import GradScaler
    from bgx.train import PPOTrainer, ppo_epoch, features_and_masks, lane_returns
    from bgx.ppo import global_normalize
    tr = PPOTrainer(batch=65536, horizon=32, seed=9)
    tr.rollout()
    buf = tr.buf
    R = global_normalize(lane_returns(buf["rewards"], buf["dones"]).reshape(-1))
    adv = R - buf["values"].reshape(-1)
    recs = buf["records"].reshape(-1, 64)
    acts, old = buf["actions"].reshape(-1), buf["logp"].reshape(-1)
    N = recs.shape[0]

    def chunks(with_legal):
        for s in range(0, N, 1 << 19):
            e = s + (1 << 19)
            f, legal = features_and_masks(recs[s:e], tr.A)
            yield f, (legal if with_legal else None), acts[s:e], old[s:e], R[s:e], adv[s:e], recs[s:e]

    res = {}
    for amp in (False, True):
        net = copy.deepcopy(tr.net)
        opt = torch.optim.Adam(net.parameters(), lr=1e-3)
        sc = GradScaler(device="cuda")
        ppo_epoch(net, opt, sc, chunks(not amp), N, 0.15, amp=amp, fused=amp, step=False)
        res[amp] = [p.grad.detach().float() / sc.get_scale() for p in net.parameters()]
    for name, a, b in zip([n for n, _ in tr.net.named_parameters()], res[False], res[True]):
        rel = ((a - b).norm() / a.norm()).item()
        assert rel < 2e-3, (name, rel)


@pytest.mark.parametrize("hidden", [40, 128])
def test_fc1_from_records_matches_autocast_gemm(hidden):
    """bgx_fc1_records (fc1 forward of the fp16 epoch from the 64-byte records)
    == autocast's addmm relu(fp16(x) W1h^T + b1h) on the encoded features: the
    same fp16 operands and fp32 accumulation, so the outputs agree to the fp16
    rounding of an fp32 sum taken in another order (<= 1 ulp)."""
    import ctypes
    from bgx import _lib
    from bgx._lib import check
    from bgx.engine import encode_records
    from bgx.train import PPOTrainer
    tr = PPOTrainer(batch=2048, horizon=3, seed=5, hidden=hidden, chunk=8192)
    tr.rollout()
    rec = tr.buf["records"].reshape(-1, 64)[:5000].contiguous()        # ragged: not a multiple of 128
    L = _lib.load()
    torch.manual_seed(1)
    W1h = (torch.randn(hidden, 198, device="cuda") * 0.2).half()
    b1h = (torch.randn(hidden, device="cuda") * 0.1).half()
    pk = torch.empty(L.bgx_fc1_packed_size(hidden), dtype=torch.uint8, device="cuda")
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    check(L.bgx_fc1_pack(p(W1h), hidden, p(pk), s), "bgx_fc1_pack")
    h = torch.full((rec.shape[0], hidden), float("nan"), dtype=torch.float16, device="cuda")
    check(L.bgx_fc1_records(p(rec), rec.shape[0], p(pk), p(b1h), hidden, p(h), s), "bgx_fc1_records")
    x = encode_records(rec, torch.float16)
    ref32 = torch.relu(x.float() @ W1h.float().t() + b1h.float())
    assert torch.isfinite(h).all()
    ulp = torch.clamp(ref32.abs(), min=2.0 ** -6) * 2.0 ** -10   # floor 1.5e-5: fp32 sum-order noise near 0
    assert bool(((h.float() - ref32).abs() <= ulp * 1.01).all())
    blas = torch._addmm_activation(b1h, x, W1h.t())
    assert bool(((h.float() - blas.float()).abs() <= 2 * ulp).all())
    assert float((h == blas).float().mean()) > 0.99
    # bad arguments are refused, not run
    assert L.bgx_fc1_packed_size(130) < 0 and L.bgx_fc1_packed_size(42) < 0


def test_rollout_graphs_match_eager():
    """The trainer's rollout as HIP graphs (2 steps per graph per shard, captured at the
    end of the first rollout, the noise step from a device counter) fills the same
    buffers as the eager rollout, rollout after rollout, with 2 shards on 2 streams."""
    from bgx.train import PPOTrainer
    trs = [PPOTrainer(batch=32768, horizon=4, seed=7, shards=2, graphs=g) for g in (False, True)]
    assert trs[1].S == 2
    for it in range(3):
        for tr in trs:
            tr.rollout()
        torch.cuda.synchronize()
        assert (trs[1]._graphs is not None) and trs[0]._graphs is None
        for k in trs[0].buf:
            assert torch.equal(trs[0].buf[k], trs[1].buf[k]), (it, k)
        assert trs[0].step_counter == trs[1].step_counter == 4 * (it + 1)
    # the two shards draw different games and noise
    a = trs[0].buf["records"][:, :16384]
    b = trs[0].buf["records"][:, 16384:]
    assert not torch.equal(a, b)


def test_fused_head_bound_guard_redoes_update():
    """the fused head leaves a legal row's masked logits out of its
    log-sum-exp, exact while 2U + log(1e-45) < -30 (U bounds |logit|).  With the
    action head scaled up 60x the bound breaks: PPOTrainer must detect it, restore the
    weights / Adam / GradScaler state and redo the update on the exact epoch -- the
    result then equals a trainer that ran the exact epoch from the start."""
    from bgx.train import PPOTrainer
    trs = []
    for fused_head in (True, False):
        tr = PPOTrainer(batch=2048, horizon=4, seed=9, chunk=4096)
        with torch.no_grad():
            tr.net.action_head.weight.mul_(60.0)
        tr.fused_head = fused_head
        tr.rollout()
        trs.append(tr)
    # both trainers start from the same weights and rollout
    for a, b in zip(trs[0].net.parameters(), trs[1].net.parameters()):
        assert torch.equal(a, b)
    assert torch.equal(trs[0].buf["actions"], trs[1].buf["actions"])
    m0, m1 = trs[0].update(), trs[1].update()
    assert trs[0].fused_head is False                     # the guard fired
    for a, b in zip(trs[0].net.parameters(), trs[1].net.parameters()):
        assert torch.equal(a, b)
    # the loss parts are fp64 sums of per-workgroup partials (atomic order): equal to 1e-12
    assert m0.keys() == m1.keys() and all(m0[k] == pytest.approx(m1[k], rel=1e-12, abs=1e-12) for k in m0)
    # and the reference-scale network keeps the fused head
    tr = PPOTrainer(batch=2048, horizon=4, seed=9, chunk=4096)
    tr.iteration()
    assert tr.fused_head is True


def test_lane_returns_kernel_matches_torch_loop():
    """bgx_lane_returns (one thread per lane) == the torch per-step loop, bit for bit
    (same two fp32 roundings, no fma), on a real rollout with game ends."""
    from bgx.train import PPOTrainer, lane_returns, _lane_returns_torch
    tr = PPOTrainer(batch=4096, horizon=16, seed=2)
    for _ in range(12):                  # games last ~60 plies: roll on until some end in the window
        tr.rollout()
        r, d = tr.buf["rewards"], tr.buf["dones"]
        if int(d.sum()) > 0:
            break
    assert int(d.sum()) > 0
    assert torch.equal(lane_returns(r, d), _lane_returns_torch(r, d))
    g = torch.Generator(device="cuda").manual_seed(1)
    r2 = torch.randn(33, 1000, device="cuda", generator=g)
    d2 = (torch.rand(33, 1000, device="cuda", generator=g) < 0.1).to(torch.uint8)
    # arbitrary fp32 rewards: both against the fp64 recursion (rounding differences
    # between the kernel and torch's elementwise ops accumulate over the 33 steps)
    ref = _lane_returns_torch(r2.double(), d2)
    for got in (lane_returns(r2, d2), _lane_returns_torch(r2, d2)):
        assert torch.allclose(got.double(), ref, rtol=1e-5, atol=1e-5)


def test_adam_step_matches_torch():
    """bgx_adam_step (bgx.train.adam_step) == `scaler.step(opt); scaler.update()` with
    torch's fused Adam (ppo_agent.py:302-305): parameters, moments, step counters, the
    unscaled gradients, and the GradScaler scale / growth tracker, over steps that
    include a non-finite gradient (skipped step, scale backoff) and a growth event."""
    import copy
    from torch.amp import GradScaler
    from bgx.policy import PolicyNet
    from bgx.train import adam_step
    torch.manual_seed(3)
    net_a = PolicyNet(hidden_size=128).cuda()
    net_b = copy.deepcopy(net_a)
    opt_a = torch.optim.Adam(net_a.parameters(), lr=1e-3, fused=True)
    opt_b = torch.optim.Adam(net_b.parameters(), lr=1e-3, fused=True)
    sc_a, sc_b = GradScaler(device="cuda", growth_interval=3), GradScaler(device="cuda", growth_interval=3)
    g = torch.Generator(device="cuda").manual_seed(5)
    for it in range(8):
        sc_a.scale(torch.ones((), device="cuda"))
        sc_b.scale(torch.ones((), device="cuda"))
        assert torch.equal(sc_a._scale, sc_b._scale)
        for pa, pb in zip(net_a.parameters(), net_b.parameters()):
            gr = torch.randn(pa.shape, device="cuda", generator=g) * sc_a._scale * 1e-2
            if it == 4 and pa.dim() == 2 and pa.shape[0] == 500:
                gr[7, 3] = float("inf")
            pa.grad = gr.clone()
            pb.grad = gr.clone()
        sc_a.step(opt_a)
        sc_a.update()
        assert adam_step(opt_b, sc_b)
        torch.cuda.synchronize()
        assert torch.equal(sc_a._scale, sc_b._scale), it
        assert torch.equal(sc_a._growth_tracker, sc_b._growth_tracker), it
        for pa, pb in zip(net_a.parameters(), net_b.parameters()):
            sa, sb = opt_a.state[pa], opt_b.state[pb]
            assert torch.equal(sa["step"], sb["step"]), it
            for k in ("exp_avg", "exp_avg_sq"):
                assert torch.allclose(sa[k], sb[k], rtol=1e-6, atol=0), (it, k)
            assert torch.allclose(pa, pb, rtol=1e-6, atol=1e-9), it
            if it != 4:
                assert torch.allclose(pa.grad, pb.grad, rtol=1e-6, atol=0), it
    assert float(sc_a._scale) != 65536.0           # the backoff and growth both happened


def test_update_redone_after_skipped_step(monkeypatch):
    """The trainer's host copy of the GradScaler state (no get_scale() sync per epoch):
    a non-finite gradient in epoch 2 skips that step and backs the scale off on the
    device, the host copy then differs after the update, and the update is redone
    from its snapshot with per-epoch get_scale() -- the same weights, Adam state and
    scale as the exact path run directly."""
    import bgx.train as T
    res = []
    for hinted in (True, False):
        tr = T.PPOTrainer(batch=2048, horizon=4, seed=3, chunk=8192)
        tr.rollout()
        calls = {"n": 0}
        orig = T.adam_step

        def inj(opt, sc, orig=orig, calls=calls):
            calls["n"] += 1
            if calls["n"] % 4 == 2:                    # epoch 2 of every pass
                opt.param_groups[0]["params"][0].grad[0, 0] = float("inf")
            return orig(opt, sc)
        monkeypatch.setattr(T, "adam_step", inj)
        if not hinted:
            monkeypatch.setattr(T.PPOTrainer, "_scale_state", lambda self: None)
        tr.update()
        torch.cuda.synchronize()
        res.append(([p.detach().clone() for p in tr.net.parameters()],
                    [tr.opt.state[p]["exp_avg"].clone() for p in tr.net.parameters()],
                    float(tr.scaler._scale.item()), calls["n"]))
        monkeypatch.undo()
    (pa, ma, sa, na), (pb, mb, sb, nb) = res
    assert na == 8 and nb == 4                         # hinted: the first pass, then the redo
    assert sa == sb == 32768.0
    for a, b in zip(pa + ma, pb + mb):
        assert torch.allclose(a, b, rtol=1e-6, atol=0)


def test_graphed_update_redone_after_nonfinite(monkeypatch):
    """The graphed update's non-finite-step path: one clean update, then a
    rollout whose rewards hold an inf, so every epoch's gradient is non-finite.  The
    graphed trainer replays its captured epochs with the scale baked in at capture (the
    device skips each step and backs the scale off), finds the host hint stale after the
    update, restores its snapshot and redoes the update eagerly; the result equals, bit
    for bit, an eager trainer without the scale hint.  A third, clean update then runs
    on a recaptured graph (the scale changed) and still matches."""
    from bgx.train import PPOTrainer
    g = PPOTrainer(batch=8192, horizon=4, seed=21, update_graphs=True)
    e = PPOTrainer(batch=8192, horizon=4, seed=21, update_graphs=False)
    monkeypatch.setattr(e, "_scale_state", lambda: None)
    for it in range(3):
        for tr in (g, e):
            tr.rollout()
            if it == 1:
                tr.buf["rewards"][1, 7] = float("inf")
            tr.update()
        torch.cuda.synchronize()
        for a, b in zip(g.net.parameters(), e.net.parameters()):
            assert torch.equal(a, b), it
            assert torch.equal(g.opt.state[a]["exp_avg"], e.opt.state[b]["exp_avg"]), it
            assert torch.equal(g.opt.state[a]["exp_avg_sq"], e.opt.state[b]["exp_avg_sq"]), it
        assert float(g.scaler._scale.item()) == float(e.scaler._scale.item()), it
        assert all(torch.isfinite(p).all() for p in g.net.parameters())
    assert float(g.scaler._scale.item()) < 65536.0       # the non-finite steps backed the scale off
    assert g._ugraph is not None and g._ugraph_captures >= 1


def test_update_graph_recaptured_on_optimizer_change():
    """The captured update graph's key holds Adam's lr (passed by value to bgx_adam_step)
    and the addresses of the optimizer's state: changing lr between updates recaptures
    and the result equals an eager trainer with the same lr schedule."""
    from bgx.train import PPOTrainer
    trs = [PPOTrainer(batch=8192, horizon=4, seed=5, update_graphs=gr) for gr in (False, True)]
    for it in range(4):
        for tr in trs:
            if it == 2:
                tr.opt.param_groups[0]["lr"] = 3e-4
            tr.rollout()
            tr.update()
        torch.cuda.synchronize()
        for a, b in zip(trs[0].net.parameters(), trs[1].net.parameters()):
            assert torch.equal(a, b), it
    assert trs[1]._ugraph_captures == 2                  # at the second update, again after the lr change


@pytest.mark.parametrize("growth_interval", [2000, 3])
def test_update_graphs_match_eager(growth_interval):
    """The update's fused-head epoch replayed as a HIP graph (captured at the second
    update over persistent row buffers, recaptured when the GradScaler scale grows)
    gives bit-identical weights, Adam state, scale and loss parts to the eager epochs,
    update after update.  growth_interval 3: the scale grows inside an update, so the
    graph is recaptured between two of its epochs."""
    from bgx.train import PPOTrainer
    trs = [PPOTrainer(batch=8192, horizon=4, seed=21, update_graphs=g) for g in (False, True)]
    for tr in trs:
        tr.scaler._growth_interval = growth_interval
    for it in range(3):
        ms = []
        for tr in trs:
            tr.rollout()
            ms.append(tr.update())
        torch.cuda.synchronize()
        assert (trs[1]._ugraph is not None) == (it >= 1) and trs[0]._ugraph is None
        for a, b in zip(trs[0].net.parameters(), trs[1].net.parameters()):
            assert torch.equal(a, b), it
        for a, b in zip(trs[0].net.parameters(), trs[1].net.parameters()):
            assert torch.equal(trs[0].opt.state[a]["exp_avg_sq"], trs[1].opt.state[b]["exp_avg_sq"]), it
        assert float(trs[0].scaler._scale.item()) == float(trs[1].scaler._scale.item())
        # loss parts: fp64 sums of per-workgroup partials in atomic order
        assert all(ms[0][k] == pytest.approx(ms[1][k], rel=1e-12, abs=1e-12) for k in ms[0]), it


@pytest.mark.gpu
def test_episode_stats_kernel_matches_torch():
    """bgx_episode_stats (one HIP kernel per rollout) == bgx.train.episode_stats (the torch
    form, itself checked against the reference driver's loop on the CPU): the six sums and
    the updated per-lane carry, over two consecutive rollouts of a real trainer."""
    from bgx.train import PPOTrainer, episode_stats, episode_stats_records
    tr = PPOTrainer(batch=2048, horizon=24, seed=13, chunk=8192)
    c1 = torch.zeros(2048, dtype=torch.float64, device="cuda")
    c2 = c1.clone()
    for _ in range(2):
        tr.rollout()
        b = tr.buf
        a = episode_stats_records(b["rewards"], b["dones"], b["records"], c1)
        r = episode_stats(b["rewards"], b["dones"], b["records"][:, :, 52], c2)
        assert torch.equal(a, r), (a, r)
        assert torch.equal(c1, c2)
    assert float(a[0]) > 0
