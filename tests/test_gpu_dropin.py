"""The reference-API drop-in classes (bgx.BackgammonEnv, VectorizedBackgammonEnv,
get_all_possible_moves, ImmutableBoard, ...) against the reference's golden
traces: same calls, same numpy seeding, same results."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bgx():
    import bgx as _bgx
    return _bgx


def test_backgammon_env_trace(bgx, golden):
    g = golden("traces")
    for gi in [0, 1, 2, 3, 5, 7]:
        sel = np.where(g["game"] == gi)[0]
        env = bgx.BackgammonEnv(match_length=15 if gi % 5 else 3)
        env.seed(gi)
        obs = env.reset()
        assert np.array_equal(obs.numpy(), g["first_obs"][gi])
        for j in sel:
            assert env.roll_result == [int(g["r0"][j]), int(g["r1"][j])]
            assert int(env.action_mask.sum()) == g["n_legal"][j]
            assert int(env.current_player) == g["mover"][j]
            obs, rew, done, info = env.step(int(g["action"][j]))
            assert float(rew) == g["reward"][j] and done == bool(g["done"][j])
            assert int(info.get("winner", -1)) == g["winner"][j]
            assert np.array_equal(bgx.types.tensor_to52(env.board.tensor).numpy(), g["board_after"][j])


def test_env_public_turn_methods_trace(bgx, golden):
    """pass_turn / roll_dice / update_legal_moves (backgammon_env.py:198-251) as
    public methods: at every G4 row where the mover has no legal move the
    reference's step() runs exactly pass_turn(); roll_dice(); update_legal_moves()
    (:124-131), so the test calls the three instead of step() there and the rest
    of the reference game must follow unchanged.  Also checks the intermediate
    states: roll_dice alone leaves the legal moves stale (as the reference's
    attributes stay until update_legal_moves)."""
    g = golden("traces")
    games = sorted({int(x) for x in g["game"][g["kind"] == 1]})[:12]
    manual = 0
    for gi in games:
        sel = np.where(g["game"] == gi)[0]
        env = bgx.BackgammonEnv(match_length=15 if gi % 5 else 3)
        env.seed(gi)
        env.reset()
        for j in sel:
            assert env.roll_result == [int(g["r0"][j]), int(g["r1"][j])]
            assert int(env.action_mask.sum()) == g["n_legal"][j]
            assert int(env.current_player) == g["mover"][j]
            if g["kind"][j] == 1:                                # "No legal actions, turn passed"
                before = int(env.current_player)
                env.pass_turn()
                assert int(env.current_player) == 1 - before and int(env.action_mask.sum()) == 0
                env.roll_dice()
                assert int(env.action_mask.sum()) == 0             # stale until update_legal_moves
                env.update_legal_moves()
                manual += 1
                assert int(env.current_player) == g["player_after"][j]
            else:
                _, rew, done, _ = env.step(int(g["action"][j]))
                assert float(rew) == g["reward"][j] and done == bool(g["done"][j])
            assert np.array_equal(bgx.types.tensor_to52(env.board.tensor).numpy(), g["board_after"][j])
    assert manual >= 20


def test_vectorized_env_trace(bgx, golden):
    g = golden("traces")
    n_env = g["vec_obs0"].shape[0]
    np.random.seed(777)
    torch.manual_seed(777)
    venv = bgx.VectorizedBackgammonEnv(num_envs=n_env)
    obs = venv.reset()
    assert np.array_equal(obs.numpy(), g["vec_obs0"])
    for t in range(g["vec_actions"].shape[0]):
        assert np.array_equal(venv.get_action_masks().sum(1).numpy().astype(int), g["vec_n_legal"][t])
        obs, rew, done, infos = venv.step(g["vec_actions"][t])
        assert np.array_equal(obs.numpy(), g["vec_obs"][t])
        assert np.array_equal(rew.numpy(), g["vec_rewards"][t])
        assert np.array_equal(done.numpy(), g["vec_dones"][t])
    # numpy's global stream advanced exactly as the reference's did
    assert len(infos) == n_env


def test_get_all_possible_moves_api(bgx, golden):
    g = golden("movegen")
    offs = g["offsets"]
    for i in list(range(0, len(g["counts"]), 37)) + [len(g["counts"]) - 1]:
        board = bgx.ImmutableBoard(bgx.types.tensor_from52(torch.from_numpy(g["boards"][i])))
        mv = bgx.get_all_possible_moves(bgx.Player(int(g["players"][i])), board, [int(x) for x in g["rolls"][i]])
        enc = np.array([bgx.types.encode_move(m) for m in mv], np.uint64)
        assert len(mv) == g["counts"][i]
        assert np.array_equal(enc, g["moves"][offs[i]:offs[i + 1]])


def test_legal_board_features_and_features(bgx, golden):
    f, mg = golden("features"), golden("movegen")
    row = 0
    for pos, ln in list(zip(f["aft_pos"], f["aft_lens"]))[:40]:
        board = bgx.ImmutableBoard(bgx.types.tensor_from52(torch.from_numpy(mg["boards"][pos])))
        p = bgx.Player(int(mg["players"][pos]))
        mv = bgx.get_all_possible_moves(p, board, [int(x) for x in mg["rolls"][pos]])
        feats = bgx.generate_all_board_features(board, p, mv)
        assert np.array_equal(feats.numpy(), f["aft"][row:row + ln])
        row += ln
    env = bgx.BackgammonEnv()
    env.seed(3)
    env.reset()
    lbf = env.legal_board_features
    n = int(env.action_mask.sum())
    ref = bgx.generate_all_board_features(env.board, env.current_player, env.legal_moves)
    assert lbf.shape == (500, 198) and torch.equal(lbf[:n], ref) and not lbf[n:].any()


def test_env_legal_moves_and_render(bgx, golden, capsys):
    """env.legal_moves (backgammon_env.py:198-243, FullMove lists in reference
    order) along seeded games, and render() on the lane's board (golden G7)."""
    from bgx.types import render_board
    g = golden("misc")
    seeds = g["lm_seed"]
    for s in np.unique(seeds):
        sel = np.where(seeds == s)[0]
        env = bgx.BackgammonEnv()
        env.seed(int(s))
        pol = np.random.RandomState(500 + int(s) - 100)
        env.reset()
        for j in sel:
            want = g["lm_moves"][g["lm_off"][j]:g["lm_off"][j + 1]]
            lm = env.legal_moves
            got = [sum((int(m.start) | (int(m.end) << 5) | (int(bool(m.hits_blot)) << 10) | (1 << 15)) << (16 * i)
                       for i, m in enumerate(fm.sub_move_commands)) for fm in lm]
            assert got == [int(v) for v in want], (s, j)
            assert all(fm.player == env.current_player for fm in lm)
            n = len(lm)
            _, _, done, _ = env.step(int(pol.randint(n)) if n else 0)
            if done:
                env.reset()
        env.render()
        assert capsys.readouterr().out == render_board(env.board)
