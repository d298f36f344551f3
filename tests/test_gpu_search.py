"""1-ply / 2-ply search kernels vs a composition of the oracle (move lists,
afterstates, features) and the torch fp32 value head, at H = 40 (C2/C4) and at
the reference's H = 128 (agent/config.py:8; golden G5 weights).  Tolerance 1e-5
on V and Q.  2-ply leaves carry the root mover's one-hot (the reference's
evaluate_board(board, current_player), moves/expect_minmax.py:57-58, 100-143)."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-5
ROLLS = [(a, b) for a in range(1, 7) for b in range(a, 7)]
PROBS = np.array([1 / 36 if a == b else 2 / 36 for a, b in ROLLS], np.float32)


@pytest.fixture(scope="module", params=[40, 128])
def setup(golden, request):
    import bgx
    from bgx.policy import PolicyNet
    from bgx.search import ValueHead
    H = request.param
    mlp = golden("mlp")
    net = PolicyNet(hidden_size=H).cuda()
    pre = f"h{H}_"
    net.load_state_dict({k[len(pre):]: torch.from_numpy(v) for k, v in mlp.items()
                         if k.startswith(pre) and not k.endswith(("logits", "values"))})
    B = 48
    eng = bgx.Engine(batch=B, max_moves=500, dice="mt", auto_reset=True)
    eng.seed(np.arange(500, 500 + B, dtype=np.uint32))
    eng.reset()
    rng = np.random.RandomState(2)
    for _ in range(25):
        nm = eng.n_moves().cpu().numpy()
        eng.step(torch.from_numpy(np.array([rng.randint(k) if k else 0 for k in nm], np.int32)).cuda())
    return bgx, net, ValueHead(net), eng


def _V(net, feats):
    with torch.no_grad():
        return net(torch.from_numpy(np.asarray(feats, np.float32)).cuda())[1].cpu().numpy()


def test_one_ply(setup):
    bgx, net, vh, eng = setup
    from bgx.search import one_ply
    best, bestv, vals = one_ply(eng, vh, want_values=True)
    feats = eng.legal_features().cpu().numpy()
    n = eng.n_moves().cpu().numpy()
    best, vals = best.cpu().numpy(), vals.cpu().numpy()
    for i in range(eng.batch):
        if n[i] == 0:
            continue
        v = _V(net, feats[i, :n[i]])
        assert np.abs(vals[i, :n[i]] - v).max() < TOL
        assert best[i] == int(np.argmax(vals[i, :n[i]]))


def test_two_ply_vs_oracle_composition(setup):
    bgx, net, vh, eng = setup
    from bgx.search import two_ply
    best, bestq, q, stats = two_ply(eng, vh, want_q=True)
    rec, mv, _ = eng.lanes()
    rec, mv = rec.cpu().numpy(), mv.cpu().numpy().view(np.uint64)
    q, best = q.cpu().numpy(), best.cpu().numpy()
    n_all = eng.n_moves().cpu().numpy()
    leaves = 0
    checked = 0
    for i in range(eng.batch):
        n = int(n_all[i])
        board, mover = rec[i, :52].view(np.int8), int(rec[i, 52])
        opp = 1 - mover
        if n == 0:
            continue
        if checked < 10:
            Q = np.zeros(n, np.float32)
            for a in range(n):
                aft = O.apply_move(board, mover, int(mv[i, a]))
                acc = 0.0
                for r, roll in enumerate(ROLLS):
                    reps, cnt = O.movegen(aft, opp, roll, cap=4096)
                    if cnt == 0:
                        leaf = [O.features(aft, mover)]
                    else:
                        leaf = [O.features(O.apply_move(aft, opp, int(b)), mover) for b in reps]
                    acc += float(PROBS[r]) * float(_V(net, leaf).min())
                Q[a] = acc
            assert np.abs(q[i, :n] - Q).max() < TOL, i
            assert abs(Q[best[i]] - Q.max()) < TOL
            checked += 1
        for a in range(n):
            aft = O.apply_move(board, mover, int(mv[i, a]))
            for roll in ROLLS:
                leaves += max(O.movegen(aft, opp, roll, cap=4096)[1], 1)
    assert checked == 10
    assert stats["leaves"] == leaves
    assert stats["afterstates"] == int(n_all.sum()) and stats["jobs"] == 21 * int(n_all.sum())


@pytest.fixture(scope="module")
def targeted_roots():
    """>= 100 root positions picked from a seeded random-policy population
    (2,048 MT lanes, several game ages): 40 plain, 20 with the mover on the bar
    (bar entries), 20 in the bear-off (mover has borne off), 20 with a doubles
    roll.  Returns their 64-byte records."""
    import bgx
    eng = bgx.Engine(batch=2048, max_moves=500, dice="mt", auto_reset=True)
    eng.seed(np.arange(7000, 7000 + 2048, dtype=np.uint32))
    eng.reset()
    rng = np.random.RandomState(11)
    want = {"plain": 40, "bar": 20, "bearoff": 20, "doubles": 20}
    got = {k: [] for k in want}
    for t in range(1, 241):
        nm = eng.n_moves().cpu().numpy()
        eng.step(torch.from_numpy(np.array([rng.randint(k) if k else 0 for k in nm], np.int32)).cuda())
        if t % 20:
            continue
        rec = eng.records().cpu().numpy()
        for i in rng.permutation(len(rec))[:256]:
            r = rec[i]
            n, m = int(r[60]) | (int(r[61]) << 8), int(r[52])
            if n == 0 or n > 120 or r[55]:               # bounded oracle time per root
                continue
            cls = ("bar" if r[48 + m] > 0 else "bearoff" if r[50 + m] > 0 else
                   "doubles" if r[53] == r[54] else "plain")
            if len(got[cls]) < want[cls] and (cls != "plain" or t % 60 == 0):
                got[cls].append(r.copy())
        if all(len(got[k]) == want[k] for k in want):
            break
    assert all(len(got[k]) == want[k] for k in want), {k: len(v) for k, v in got.items()}
    return np.stack([r for k in want for r in got[k]])


def test_two_ply_targeted_roots_vs_oracle(setup, targeted_roots):
    """Q of every move of 100 targeted roots (bar entries, bear-offs, doubles,
    plain; replies with bar entries and doubles reply sets over 100 moves occur
    among their jobs) against the oracle composition bgo_two_ply_leaves + the
    torch fp32 value head: within 1e-5, same first argmax, exact leaf counts."""
    bgx, net, vh, _ = setup
    from bgx.search import two_ply
    R = targeted_roots
    eng = bgx.Engine(batch=len(R), max_moves=500, dice="mt", auto_reset=True)
    eng.set_lanes(torch.from_numpy(R))
    best, bestq, q, stats = two_ply(eng, vh, want_q=True)
    rec, mv, _ = eng.lanes()
    rec, mv = rec.cpu().numpy(), mv.cpu().numpy().view(np.uint64)
    q, best = q.cpu().numpy(), best.cpu().numpy()
    assert np.array_equal(rec[:, :60], R[:, :60])
    leaves = big = 0
    for i in range(len(R)):
        n = int(rec[i, 60]) | (int(rec[i, 61]) << 8)
        board, mover = rec[i, :52].view(np.int8), int(rec[i, 52])
        ref_moves, _ = O.movegen(board, mover, (int(rec[i, 53]), int(rec[i, 54])))
        assert np.array_equal(mv[i, :n], ref_moves[:500]), i
        Q = np.zeros(n, np.float32)
        for a in range(n):
            feats, counts = O.two_ply_leaves(board, mover, int(mv[i, a]))
            v = _V(net, feats)
            seg = np.minimum.reduceat(v, np.concatenate([[0], np.cumsum(counts)[:-1]]))
            Q[a] = float(np.dot(PROBS.astype(np.float64), seg.astype(np.float64)))
            leaves += int(counts.sum())
            big += int((counts[[0, 6, 11, 15, 18, 20]] > 100).sum())
        assert np.abs(q[i, :n] - Q).max() < TOL, i
        assert abs(Q[best[i]] - Q.max()) < TOL, i
    assert stats["leaves"] == leaves
    assert big >= 20, big                              # doubles reply sets over 100 moves


def test_two_ply_factored_matches_full_form(setup, dbg):
    """The factored evaluator (the root mover's part of X1 once per row, then the
    replier's k-blocks, block 12 and the hit deltas per leaf) against the full
    13-k-block form on every leaf (BGX_2PLY_UNFACTORED): Q within 1e-5, the same
    surviving-leaf count, the same choice wherever the best Q leads by more than 1e-5."""
    bgx, net, vh, eng = setup
    from bgx.search import two_ply
    best, bestq, q, st = two_ply(eng, vh, want_q=True)
    dbg.setenv("BGX_2PLY_UNFACTORED", "1")
    best2, bestq2, q2, st2 = two_ply(eng, vh, want_q=True)
    assert st2 == st
    n = eng.n_moves()
    col = torch.arange(q.shape[1], device="cuda")[None, :]
    m = col < n[:, None]
    assert float((q - q2)[m].abs().max()) < TOL
    qs = torch.where(m, q2, torch.full_like(q2, -1e30)).sort(dim=1, descending=True).values
    clear = (n > 0) & ((n == 1) | (qs[:, 0] - qs[:, 1] > TOL))
    assert torch.equal(best[clear], best2[clear])


def test_two_ply_pool_retry_rounds(setup, dbg):
    """A leaf pool far too small for one pass: lost jobs are re-run in later
    rounds; Q, the choice and the exact leaf count must not change."""
    bgx, net, vh, eng = setup
    from bgx.search import two_ply
    best, bestq, q, st = two_ply(eng, vh, want_q=True)
    dbg.setenv("BGX_2PLY_POOL", "65536")
    best2, bestq2, q2, st2 = two_ply(eng, vh, want_q=True)
    assert st2["leaves"] == st["leaves"]
    assert torch.equal(torch.nan_to_num(q2, 7.0), torch.nan_to_num(q, 7.0))
    assert torch.equal(best2, best) and torch.equal(bestq2, bestq)


@pytest.mark.parametrize("caps", ["6:3584", "6"])
@pytest.mark.parametrize("heavy", ["9:2", "9:0", "10:0"])
def test_two_ply_overflow_tiers(setup, dbg, caps, heavy):
    """Every reply enumeration forced out of its first LDS table: into the
    4,096-slot LDS tier ("6:3584") or on through it to the HBM-table tier ("6").
    Same Q, choice and leaf count as the normal path."""
    bgx, net, vh, _ = setup
    from bgx.search import two_ply
    eng = bgx.Engine(batch=3, max_moves=500, dice="mt", auto_reset=True)
    eng.seed(np.arange(900, 903, dtype=np.uint32))
    eng.reset()
    rng = np.random.RandomState(5)
    for _ in range(12):
        nm = eng.n_moves().cpu().numpy()
        eng.step(torch.from_numpy(np.array([rng.randint(k) if k else 0 for k in nm], np.int32)).cuda())
    best, bestq, q, st = two_ply(eng, vh, want_q=True)
    dbg.setenv("BGX_2PLY_HEAVY", heavy)
    dbg.setenv("BGX_2PLY_LDS_CAP", caps)
    best2, bestq2, q2, st2 = two_ply(eng, vh, want_q=True)
    assert eng.error() == 0
    assert st2["leaves"] == st["leaves"]
    assert torch.equal(torch.nan_to_num(q2, 7.0), torch.nan_to_num(q, 7.0))
    assert torch.equal(best2, best)


def test_two_ply_full_batch_paths_agree(dbg):
    """C4 at full size (B = 65,536 roots after 60 self-play steps): the doubles
    enumerator with its revisit memo inside a 512-slot table and with a
    1,024-slot table plus separate memo tables (different tier traffic, pruning
    and pool block order), and the replies of rows whose replier is on the bar as one
    table-free row walk or as 15 per-job walks, give bit-identical Q, the same choices
    and the same surviving-leaf counts; every choice is a legal move and every Q is
    finite."""
    import bgx
    from bgx.policy import PolicyNet
    from bgx.search import ValueHead, two_ply
    torch.manual_seed(0)
    net = PolicyNet().cuda()
    eng = bgx.Engine(batch=65536, max_moves=500, seed=77, dice="philox", auto_reset=True)
    eng.reset(want_obs=False)
    for i in range(60):
        a, _, _ = net.act(net.rollout_inputs(eng), seed=5, step=i)
        eng.step(a, want_obs=False, want_info=False)
    vh = ValueHead(PolicyNet(hidden_size=40).cuda())
    b1, q1, Q1, s1 = two_ply(eng, vh, want_q=True)
    dbg.setenv("BGX_2PLY_HEAVY", "10:0")
    b2, q2, Q2, s2 = two_ply(eng, vh, want_q=True)
    assert s1 == s2
    assert torch.equal(torch.nan_to_num(Q1, 7.0), torch.nan_to_num(Q2, 7.0))
    assert torch.equal(b1, b2) and torch.equal(q1, q2)
    # the rows whose replier is on the bar: the table-free row walk (nd_row_bar) against
    # the per-job walks it replaces
    dbg.delenv("BGX_2PLY_HEAVY")
    dbg.setenv("BGX_2PLY_BARROW", "0")
    b3, q3, Q3, s3 = two_ply(eng, vh, want_q=True)
    assert s1 == s3
    assert torch.equal(torch.nan_to_num(Q1, 7.0), torch.nan_to_num(Q3, 7.0))
    assert torch.equal(b1, b3) and torch.equal(q1, q3)
    n = eng.n_moves()
    assert bool(((b1 < n) | (n == 0)).all())
    has = n > 0
    assert bool(torch.isfinite(q1[has]).all())
    col = torch.arange(Q1.shape[1], device="cuda")[None, :]
    assert bool(torch.isfinite(Q1[col < n[:, None]]).all())
    assert s1["afterstates"] == int(n.sum()) and s1["jobs"] == 21 * s1["afterstates"]
    assert eng.error() == 0


def _leaf_reference(net, keys, tags, side, ml):
    """V of every valid pool leaf in fp64 (oracle.leaf_values)."""
    import oracle as O
    return O.leaf_values(net.fc1.weight.detach().cpu().double().numpy(), net.fc1.bias.detach().cpu().double().numpy(),
                         net.value_head.weight.detach().cpu().double().numpy().ravel(),
                         float(net.value_head.bias.detach().cpu()), keys, tags, side, ml)


@pytest.mark.parametrize("unfactored", [False, True])
def test_two_ply_every_leaf_vs_fp64(setup, dbg, tmp_path, unfactored):
    """Every surviving leaf of the 48-root batch (~534 k): the evaluator's V (the
    BGX_2PLY_DUMP test hook writes V per pool slot with the pool, row sides and max
    lengths) against an fp64 MLP on the leaf's own encoding, within 1e-6 -- the factored
    form (the mover's row part + replier k-blocks + hit deltas) and the full 13-k-block
    form.  This is the check that found the two-tiles-in-flight wide form wrong on
    columns 16-31 of its second tile (0.01-0.8 % of leaves, build-dependent)."""
    bgx, net, vh, eng = setup
    from bgx.search import two_ply
    pre = str(tmp_path / "d")
    dbg.setenv("BGX_2PLY_DUMP", pre)
    if unfactored:
        dbg.setenv("BGX_2PLY_UNFACTORED", "1")
    two_ply(eng, vh)
    keys = np.fromfile(pre + ".keys", np.uint32).reshape(-1, 4)
    tags = np.fromfile(pre + ".tags", np.uint32)
    v = np.fromfile(pre + ".v", np.float32)
    side = np.fromfile(pre + ".side", np.uint32).reshape(-1, 4)
    ml = np.fromfile(pre + ".ml", np.uint8)
    idx, vref = _leaf_reference(net, keys, tags, side, ml)
    assert len(idx) > 100_000
    err = np.abs(v[idx].astype(np.float64) - vref)
    assert err.max() < 1e-6, (int((err > 1e-6).sum()), idx[err > 1e-6][:16] % 64)


def test_two_ply_cross_stream_after_destroyed_engine():
    """The sequence that faulted in round 4 (profiles/r4_layout/r4v/fault.txt): a
    65,536-lane engine runs two_ply and is destroyed; two 32,768-lane engines are then
    stepped on the default stream and, with no host sync, two_ply runs on a fresh
    non-blocking stream.  The engine orders the call after its own steps (bgx.h "Stream
    ordering"), so Q, the choices and the surviving-leaf counts equal a same-stream
    call on the same lanes."""
    import bgx
    from bgx.policy import PolicyNet
    from bgx.search import ValueHead, two_ply
    torch.manual_seed(0)
    net = PolicyNet().cuda()
    vh = ValueHead(PolicyNet(hidden_size=40).cuda())

    def population(n, seed, steps):
        e = bgx.Engine(batch=n, max_moves=500, seed=seed, dice="philox", auto_reset=True)
        e.reset(want_obs=False)
        e.set_fork(False)
        for i in range(steps):
            a, _, _ = net.act(net.rollout_inputs(e), seed=5, step=i)
            e.step(a, want_obs=False, want_info=False)
        return e

    big = population(65536, 77, 20)
    two_ply(big, vh)
    del big
    torch.cuda.empty_cache()
    shards = [population(32768, 77 + 7919 * k, 60) for k in range(2)]
    side = [torch.cuda.Stream() for _ in shards]
    got = []
    for e, s in zip(shards, side):                # no sync: the steps may still be running
        with torch.cuda.stream(s):
            got.append(two_ply(e, vh, want_q=True))
    torch.cuda.synchronize()
    for e, (b1, q1, Q1, s1) in zip(shards, got):
        b2, q2, Q2, s2 = two_ply(e, vh, want_q=True)
        assert s1 == s2
        assert torch.equal(torch.nan_to_num(Q1, 7.0), torch.nan_to_num(Q2, 7.0))
        assert torch.equal(b1, b2) and torch.equal(q1, q2)
        assert e.error() == 0


def test_one_ply_selfplay_c2_batch():
    """C2 at its BASELINE batch (B = 4,096 games, value MLP 198->40->1, Philox dice):
    6 greedy 1-ply steps (one_ply then step).  At every step each choice is the FIRST
    argmax of that lane's afterstate values (backgammon_env.py:207-216 features with the
    mover's one-hot) and a legal move, and on a 64-lane sample the values of every
    afterstate equal an oracle + torch fp32 composition (O.apply_move, O.features, the
    torch value head) within 1e-5."""
    import bgx
    from bgx.policy import PolicyNet
    from bgx.search import ValueHead, one_ply
    torch.manual_seed(2)
    net = PolicyNet(hidden_size=40).cuda()
    vh = ValueHead(net)
    B = 4096
    eng = bgx.Engine(batch=B, max_moves=500, seed=123, dice="philox", auto_reset=True)
    eng.reset(want_obs=False)
    rng = np.random.RandomState(3)
    for t in range(6):
        best, bestv, vals = one_ply(eng, vh, want_values=True)
        n = eng.n_moves()
        rec, mv, _ = eng.lanes()
        col = torch.arange(vals.shape[1], device="cuda")[None, :]
        live = col < n[:, None].long()
        vm = torch.where(live, vals, torch.full_like(vals, -float("inf")))
        first = vm.argmax(dim=1).to(torch.int32)           # torch.argmax: the first maximum
        has = n > 0
        assert torch.equal(best[has], first[has]), t
        assert bool((best[~has] == 0).all())
        assert bool(torch.isfinite(vals[live]).all())
        assert torch.equal(bestv[has], vm.max(dim=1).values[has])
        recn, mvn, vn, nn = rec.cpu().numpy(), mv.cpu().numpy().view(np.uint64), vals.cpu().numpy(), n.cpu().numpy()
        for i in rng.choice(B, 64, replace=False):
            k = int(nn[i])
            if k == 0:
                continue
            board, mover = recn[i, :52].view(np.int8), int(recn[i, 52])
            feats = [O.features(O.apply_move(board, mover, int(mvn[i, a])), mover) for a in range(k)]
            ref = _V(net, feats)
            assert np.abs(vn[i, :k] - ref).max() < TOL, (t, i)
        eng.step(best, want_obs=False, want_info=False)
    assert eng.error() == 0
