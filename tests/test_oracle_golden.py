"""Pin the CPU oracle (oracle/bgoracle.c) against fixtures generated from the
reference itself (tests/golden/make_golden.py).  CPU only."""
import numpy as np

import oracle as O


def test_movegen_matches_reference(golden):
    g = golden("movegen")
    offs = g["offsets"]
    bad = 0
    for i in range(len(g["counts"])):
        ref = g["moves"][offs[i]:offs[i + 1]]
        got, n = O.movegen(g["boards"][i], int(g["players"][i]), g["rolls"][i], cap=4096)
        if n != g["counts"][i] or not np.array_equal(got, ref):
            bad += 1
    assert bad == 0, f"{bad} positions differ"
    assert g["counts"].max() > 500  # truncation case present


def test_known_answers():
    # SURVEY.md §8c known-answer tests (measured on the reference)
    for roll, n in (((3, 1), 16), ((6, 5), 7), ((4, 4), 52), ((1, 1), 42), ((2, 6), 14)):
        assert O.movegen(O.INITIAL_BOARD52, 0, roll)[1] == n
    first = O.decode_move(O.movegen(O.INITIAL_BOARD52, 0, (2, 6))[0][0])
    assert first == [(0, 6, 0), (0, 2, 0)]


def test_features_match_reference(golden):
    g, mg = golden("features"), golden("movegen")
    for k, i in enumerate(g["obs_idx"]):
        f = O.features(mg["boards"][i], int(g["obs_player"][k]))
        assert np.array_equal(f, g["obs"][k])
    # afterstate boards (apply) and afterstate features (mover's one-hot)
    row = 0
    for pos, ln in zip(g["aft_pos"], g["aft_lens"]):
        moves, n = O.movegen(mg["boards"][pos], int(mg["players"][pos]), mg["rolls"][pos], cap=4096)
        assert n == ln
        for m in moves:
            a = O.apply_move(mg["boards"][pos], int(mg["players"][pos]), int(m))
            assert np.array_equal(a, g["aft_boards"][row])
            assert np.array_equal(O.features(a, int(mg["players"][pos])), g["aft"][row])
            row += 1
    assert row == len(g["aft"])


def test_dice_stream(golden):
    g = golden("dice")
    for s in g["seeds"]:
        mt = O.MT(int(s))
        assert [mt.die() for _ in range(g["dice"].shape[1])] == list(g["dice"][s])


def test_env_traces(golden):
    g = golden("traces")
    games = np.unique(g["game"])
    for gi in games:
        sel = np.where(g["game"] == gi)[0]
        env = O.Env(seed=int(gi), match_length=15 if gi % 5 else 3)
        obs = env.reset()
        assert np.array_equal(obs, g["first_obs"][gi])
        for j in sel:
            b, st = env.state()
            assert (st[1], st[2]) == (g["r0"][j], g["r1"][j])
            assert st[3] == g["n_legal"][j]
            assert st[0] == g["mover"][j]
            obs, rew, done, info = env.step(int(g["action"][j]))
            assert rew == g["reward"][j] and done == g["done"][j]
            assert info[1] == g["winner"][j] and info[2] == g["score"][j]
            b, st = env.state()
            assert np.array_equal(b, g["board_after"][j]), (gi, j)
            assert st[0] == g["player_after"][j]


def test_vectorized_trace_shared_stream(golden):
    """VectorizedBackgammonEnv (vec_bg_env.py:28-49): N envs share numpy's ONE global
    stream, consumed in lane order; done -> env.reset() immediately."""
    g = golden("traces")
    n_env = g["vec_obs0"].shape[0]
    shared = O.MT(777)
    envs = [O.Env(seed=0) for _ in range(n_env)]
    for e in envs:
        e.share_rng(shared)
    obs0 = np.stack([e.reset() for e in envs])
    assert np.array_equal(obs0, g["vec_obs0"])
    for t in range(g["vec_actions"].shape[0]):
        for i, e in enumerate(envs):
            assert e.state()[1][3] == g["vec_n_legal"][t, i]
            obs, rew, done, _ = e.step(int(g["vec_actions"][t, i]))
            if done:
                obs = e.reset()
            assert rew == g["vec_rewards"][t, i] and done == g["vec_dones"][t, i]
            assert np.array_equal(obs, g["vec_obs"][t, i])
            assert np.array_equal(e.state()[0], g["vec_boards"][t, i])
