"""Parity of the HIP engine (libbgx.so via the C ABI) against the reference's
golden fixtures and the CPU oracle.  Runs on the GPU box (pytest -m gpu)."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bgx():
    import bgx as _bgx
    assert torch.cuda.is_available()
    return _bgx


def _split_golden_moves(g):
    offs = g["offsets"]
    return [g["moves"][offs[i]:offs[i + 1]] for i in range(len(g["counts"]))]


@pytest.mark.parametrize("cap", [2048, 500])
def test_movegen_matches_reference(bgx, golden, cap):
    g = golden("movegen")
    n = len(g["counts"])
    eng = bgx.Engine(batch=n, max_moves=cap, dice="philox")
    nm, nt, mv = eng.movegen(torch.from_numpy(g["boards"]), torch.from_numpy(g["players"]),
                             torch.from_numpy(g["rolls"]), max_moves=cap)
    nm, nt, mv = nm.cpu().numpy(), nt.cpu().numpy(), mv.cpu().numpy().view(np.uint64)
    ref = _split_golden_moves(g)
    assert np.array_equal(nt, g["counts"])
    assert np.array_equal(nm, np.minimum(g["counts"], cap))
    for i in range(n):
        k = int(nm[i])
        assert np.array_equal(mv[i, :k], ref[i][:k]), i
    assert eng.error() == 0


@pytest.mark.parametrize("caps", [("4", "24"), ("1", "1")])
def test_movegen_overflow_tiers_vs_reference(bgx, golden, dbg, caps):
    """Positions through the overflow launch (k_movegen_over): the main table's cap of
    caps[0] unique afterstates sends almost every golden position to tier 1 (4,096-slot
    LDS table), whose cap of caps[1] sends most of those on to tier 2 (the workgroup's
    131,072-slot HBM table, in the same wave since round 6).  The lists equal the
    reference's golden ones, as without the caps."""
    dbg.setenv("BGX_MOVEGEN_CAP", caps[0])
    dbg.setenv("BGX_TIER1_CAP", caps[1])             # read at engine creation
    g = golden("movegen")
    n = len(g["counts"])
    eng = bgx.Engine(batch=n, max_moves=2048, dice="philox")
    nm, nt, mv = eng.movegen(torch.from_numpy(g["boards"]), torch.from_numpy(g["players"]),
                             torch.from_numpy(g["rolls"]), max_moves=2048)
    nm, nt, mv = nm.cpu().numpy(), nt.cpu().numpy(), mv.cpu().numpy().view(np.uint64)
    ref = _split_golden_moves(g)
    assert np.array_equal(nt, g["counts"])
    for i in range(n):
        k = int(nm[i])
        assert np.array_equal(mv[i, :k], ref[i][:k]), i
    assert eng.error() == 0


def test_movegen_random_positions_vs_oracle(bgx):
    rng = np.random.RandomState(7)
    n = 6000
    boards = np.zeros((n, 52), np.int8)
    for i in range(n):
        x = boards[i]
        for p in (0, 1):
            left = 15
            if rng.rand() < 0.15:
                x[48 + p] = rng.randint(1, 3); left -= x[48 + p]
            if rng.rand() < 0.3:
                x[50 + p] = rng.randint(0, left); left -= x[50 + p]
            pts = list(range(18, 24)) if (p == 0 and rng.rand() < 0.3) else (
                list(range(6)) if (p == 1 and rng.rand() < 0.3) else list(range(24)))
            while left > 0:
                q = pts[rng.randint(len(pts))]
                if x[(1 - p) * 24 + q] > 0:
                    pts = list(range(24))
                    continue
                k = min(left, rng.randint(1, 4)); x[p * 24 + q] += k; left -= k
    players = rng.randint(0, 2, n).astype(np.uint8)
    dice = rng.randint(1, 7, (n, 2)).astype(np.uint8)
    eng = bgx.Engine(batch=n, max_moves=600, dice="philox")
    nm, nt, mv = eng.movegen(torch.from_numpy(boards), torch.from_numpy(players), torch.from_numpy(dice))
    nm, nt, mv = nm.cpu().numpy(), nt.cpu().numpy(), mv.cpu().numpy().view(np.uint64)
    counts, ref = O.movegen_batch(boards, players, dice, 600)
    assert np.array_equal(nt, counts)
    for i in range(n):
        k = int(nm[i])
        assert np.array_equal(mv[i, :k], ref[i, :k]), i


def test_encode_matches_reference(bgx, golden):
    g, mg = golden("features"), golden("movegen")
    boards = torch.from_numpy(mg["boards"][g["obs_idx"]]).cuda()
    players = torch.from_numpy(g["obs_player"]).cuda()
    out = bgx.encode(boards, players).cpu().numpy()
    assert np.array_equal(out, g["obs"])
    # afterstate features through encode of the reference's afterstate boards
    pl = np.concatenate([np.full(ln, mg["players"][p], np.uint8) for p, ln in zip(g["aft_pos"], g["aft_lens"])])
    aft = bgx.encode(torch.from_numpy(g["aft_boards"]).cuda(), torch.from_numpy(pl).cuda()).cpu().numpy()
    assert np.array_equal(aft, g["aft"])


def _run_trace(bgx, g, games, match_length):
    eng = bgx.Engine(batch=len(games), max_moves=500, dice="mt", auto_reset=False, match_length=match_length)
    eng.seed(np.array(games, np.uint32))
    obs = eng.reset().cpu().numpy()
    for k, gi in enumerate(games):
        assert np.array_equal(obs[k], g["first_obs"][gi]), gi
    sels = [np.where(g["game"] == gi)[0] for gi in games]
    T = max(len(s) for s in sels)
    for t in range(T):
        rec, _, _ = eng.lanes()
        rec = rec.cpu().numpy()
        acts = np.zeros(len(games), np.int32)
        for k, s in enumerate(sels):
            if t < len(s):
                j = s[t]
                assert (rec[k, 53], rec[k, 54]) == (g["r0"][j], g["r1"][j]), (games[k], t)
                assert int(rec[k, 60]) | (int(rec[k, 61]) << 8) == g["n_legal"][j], (games[k], t)
                assert rec[k, 52] == g["mover"][j]
                acts[k] = g["action"][j]
        _, rew, done, info = eng.step(torch.from_numpy(acts).cuda())
        rew, done, info = rew.cpu().numpy(), done.cpu().numpy(), info.cpu().numpy()
        rec, _, _ = eng.lanes()
        rec = rec.cpu().numpy()
        for k, s in enumerate(sels):
            if t < len(s):
                j = s[t]
                assert rew[k] == g["reward"][j] and bool(done[k]) == bool(g["done"][j]), (games[k], t)
                assert ((info[k] >> 8) & 0xFF) - 1 == g["winner"][j]
                assert (info[k] >> 16) & 0xFF == g["score"][j]
                assert np.array_equal(rec[k, :52].view(np.int8), g["board_after"][j]), (games[k], t)
                assert rec[k, 52] == g["player_after"][j]


def test_env_traces_match_reference(bgx, golden):
    g = golden("traces")
    games = sorted(set(int(x) for x in g["game"]))
    _run_trace(bgx, g, [x for x in games if x % 5], 15)
    _run_trace(bgx, g, [x for x in games if x % 5 == 0], 3)


def test_vectorized_shared_stream_matches_reference(bgx, golden):
    g = golden("traces")
    n_env = g["vec_obs0"].shape[0]
    eng = bgx.Engine(batch=n_env, max_moves=500, dice="shared", auto_reset=True)
    eng.seed(np.full(n_env, 777, np.uint32))
    obs = eng.reset().cpu().numpy()
    assert np.array_equal(obs, g["vec_obs0"])
    for t in range(g["vec_actions"].shape[0]):
        assert np.array_equal(eng.n_moves().cpu().numpy(), g["vec_n_legal"][t])
        obs, rew, done, _ = eng.step(torch.from_numpy(g["vec_actions"][t].astype(np.int32)).cuda())
        assert np.array_equal(rew.cpu().numpy(), g["vec_rewards"][t])
        assert np.array_equal(done.cpu().numpy().astype(bool), g["vec_dones"][t])
        assert np.array_equal(obs.cpu().numpy(), g["vec_obs"][t]), t
        rec, _, _ = eng.lanes()
        assert np.array_equal(rec.cpu().numpy()[:, :52].view(np.int8), g["vec_boards"][t])


def test_selfplay_vs_oracle_per_lane(bgx):
    """512 lanes of random self-play, each lane checked step-by-step against an
    oracle env with the same seed (dice mode "mt")."""
    B, T = 512, 250
    seeds = np.arange(1000, 1000 + B, dtype=np.uint32)
    eng = bgx.Engine(batch=B, max_moves=500, dice="mt", auto_reset=True)
    eng.seed(seeds)
    envs = [O.Env(seed=int(s)) for s in seeds]
    obs = eng.reset().cpu().numpy()
    ref_obs = np.stack([e.reset() for e in envs])
    assert np.array_equal(obs, ref_obs)
    pol = np.random.RandomState(3)
    for t in range(T):
        nm = eng.n_moves().cpu().numpy()
        ref_n = np.array([e.state()[1][3] for e in envs])
        assert np.array_equal(nm, ref_n), t
        acts = np.array([pol.randint(k) if k > 0 else 0 for k in nm], np.int32)
        if t % 17 == 5:
            acts[::7] = 499          # invalid actions
        obs, rew, done, _ = eng.step(torch.from_numpy(acts).cuda())
        obs, rew, done = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()
        for i, e in enumerate(envs):
            o, r, d, _ = e.step(int(acts[i]))
            if d:
                o = e.reset()
            assert r == rew[i] and d == bool(done[i]), (t, i)
            assert np.array_equal(o, obs[i]), (t, i)
        rec, mv, _ = eng.lanes()
        rec, mv = rec.cpu().numpy(), mv.cpu().numpy().view(np.uint64)
        for i in range(0, B, 8):
            b, st = envs[i].state()
            assert np.array_equal(rec[i, :52].view(np.int8), b)
            assert np.array_equal(mv[i, :st[3]], envs[i].legal())


def test_afterstates_and_legal_features(bgx):
    B = 64
    eng = bgx.Engine(batch=B, max_moves=500, dice="mt", auto_reset=True)
    eng.seed(np.arange(B, dtype=np.uint32))
    eng.reset()
    pol = np.random.RandomState(1)
    for _ in range(30):
        nm = eng.n_moves().cpu().numpy()
        eng.step(torch.from_numpy(np.array([pol.randint(k) if k else 0 for k in nm], np.int32)).cuda())
    rec, mv, _ = eng.lanes()
    rec, mv = rec.cpu().numpy(), mv.cpu().numpy().view(np.uint64)
    aft = eng.afterstates().cpu().numpy()
    feats = eng.legal_features().cpu().numpy()
    for i in range(B):
        n = int(rec[i, 60]) | (int(rec[i, 61]) << 8)
        pl = int(rec[i, 52])
        for m in range(n):
            a = O.apply_move(rec[i, :52].view(np.int8), pl, int(mv[i, m]))
            assert np.array_equal(aft[i, m], a)
            assert np.array_equal(feats[i, m], O.features(a, pl))
        assert not aft[i, n:].any() and not feats[i, n:].any()


def test_large_batch_invariants(bgx):
    B = 65536
    eng = bgx.Engine(batch=B, max_moves=500, dice="philox", auto_reset=True)
    eng.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(40):
        nm = eng.n_moves()
        a = (torch.rand(B, device="cuda", generator=g) * nm.clamp(min=1).float()).to(torch.int32)
        eng.step(a)
    rec, _, _ = eng.lanes()
    rec = rec.to(torch.int32)
    tot0 = rec[:, :24].sum(1) + rec[:, 48] + rec[:, 50]
    tot1 = rec[:, 24:48].sum(1) + rec[:, 49] + rec[:, 51]
    assert bool((tot0 == 15).all()) and bool((tot1 == 15).all())
    both = (rec[:, :24] > 0) & (rec[:, 24:48] > 0)
    assert not bool(both.any())
    assert eng.error() == 0


def test_philox_split_dispatch_vs_oracle(bgx):
    """Philox mode runs the predicted-doubles prefix of the dispatch order and the
    light remainder (small table, no revisit memo) as separate launches: every
    lane's move list and apply must still equal the oracle's, whichever launch
    it ran in.  Each step: the oracle applies the chosen move to the previous
    record, and the new record's move list is recomputed from its board/dice."""
    B = 16384
    eng = bgx.Engine(batch=B, max_moves=500, dice="philox", seed=9, auto_reset=True)
    eng.reset()
    g = torch.Generator(device="cuda").manual_seed(1)
    checked_dbl = 0
    for t in range(24):
        prev, pmv, _ = eng.lanes()
        prev, pmv = prev.cpu().numpy(), pmv.cpu().numpy().view(np.uint64)
        nm = eng.n_moves()
        a = (torch.rand(B, device="cuda", generator=g) * nm.clamp(min=1).float()).to(torch.int32)
        eng.step(a, want_obs=False)
        if t < 4 or t % 5:
            continue
        rec, mv, nt = eng.lanes()
        rec, mv, nt = rec.cpu().numpy(), mv.cpu().numpy().view(np.uint64), nt.cpu().numpy()
        a = a.cpu().numpy()
        sel = np.arange(t, B, 11)
        boards = np.ascontiguousarray(rec[sel, :52]).view(np.int8)
        counts, ref = O.movegen_batch(boards, rec[sel, 52].copy(), rec[sel, 53:55].copy(), 500)
        for k, i in enumerate(sel):
            assert nt[i] == counts[k], (t, i)
            n = min(int(counts[k]), 500)
            assert np.array_equal(mv[i, :n], ref[k, :n]), (t, i)
            checked_dbl += int(rec[i, 53] == rec[i, 54])
            # the move applied this step, from the previous record (no game end, no pass)
            if prev[i, 55] == 0 and (int(prev[i, 60]) | (int(prev[i, 61]) << 8)) > 0:
                after = O.apply_move(prev[i, :52].view(np.int8), int(prev[i, 52]), int(pmv[i, a[i]]))
                if after[50 + int(prev[i, 52])] < 15:
                    assert np.array_equal(rec[i, :52].view(np.int8), after), (t, i)
    assert checked_dbl > 500
    assert eng.error() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("B", [16384, 1000])
def test_dispatch_order_does_not_change_results(bgx, dbg, B):
    """The dispatch order (class-sorted, XCD-aware 16-lane runs when B % 128 == 0,
    plain class sort otherwise, or no order at all with the run swizzle) only
    schedules: every variant must step every lane exactly once and give the same
    records, move lists and rewards."""
    variants = [{}, {"BGX_XCD": "0"}, {"BGX_ORDER": "0"}, {"BGX_ORDER": "0", "BGX_XCD": "0"}]
    engs = []
    for env in variants:
        for k in ("BGX_XCD", "BGX_ORDER"):
            dbg.delenv(k, raising=False)
        for k, v in env.items():
            dbg.setenv(k, v)
        e = bgx.Engine(batch=B, max_moves=500, dice="philox", seed=21, auto_reset=True)
        e.reset(want_obs=False)
        engs.append(e)
    g = torch.Generator(device="cuda").manual_seed(3)
    for _ in range(30):
        u = torch.rand(B, device="cuda", generator=g)
        outs = []
        for e in engs:
            a = (u * e.n_moves().clamp(min=1).float()).to(torch.int32)
            _, r, d, _ = e.step(a, want_obs=False)
            outs.append((r.clone(), d.clone()))
        for r, d in outs[1:]:
            assert torch.equal(r, outs[0][0]) and torch.equal(d, outs[0][1])
    rec0, mv0, nt0 = engs[0].lanes()
    n0 = (rec0[:, 60].long() | (rec0[:, 61].long() << 8))
    live = torch.arange(500, device="cuda")[None, :] < n0[:, None]     # entries past n are scratch
    for e in engs[1:]:
        rec, mv, nt = e.lanes()
        assert torch.equal(rec, rec0) and torch.equal(nt, nt0)
        assert torch.equal(torch.where(live, mv, 0), torch.where(live, mv0, 0))
        assert e.error() == 0
