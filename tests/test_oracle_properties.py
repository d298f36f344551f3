"""Property tests (hypothesis) of the CPU oracle's rules on arbitrary legal
positions: random checker layouts for both players, either player to move, any
roll.  The move LISTS are pinned by the golden fixtures (test_oracle_golden.py);
these are the rule invariants the reference's code implies for every position:

* every move keeps 15 checkers per side and never leaves a point held by both
  players (move_checker, immutable_board.py:42-89);
* afterstates are pairwise distinct (add_unique_board, handle_moves.py:313-341);
* all surviving moves have the same sub-move count, the maximum
  (filter_full_moves_by_max_submoves, get_all_moves.py:73-94);
* a player with checkers on the bar starts every move with an entry
  (get_moves_bar, move_logic.py:95-137);
* doubles moves use at most 4 sub-moves, others at most 2.
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

import oracle as O


@st.composite
def positions(draw):
    board = np.zeros(52, np.int8)
    # P1: 15 checkers over points 0..23, bar (24) and off (25)
    for _ in range(15):
        s = draw(st.integers(0, 25))
        if s < 24:
            board[s] += 1
        elif s == 24:
            board[48] += 1
        else:
            board[50] += 1
    free = [p for p in range(24) if board[p] == 0] + [24, 25]
    for _ in range(15):
        s = draw(st.sampled_from(free))
        if s < 24:
            board[24 + s] += 1
        elif s == 24:
            board[49] += 1
        else:
            board[51] += 1
    for side in (0, 1):                      # a finished game has nothing to move
        if board[50 + side] == 15:
            board[50 + side] -= 1
            board[48 + side] += 1
    player = draw(st.integers(0, 1))
    a, b = draw(st.integers(1, 6)), draw(st.integers(1, 6))
    return board, player, (a, b)


def _subs(v: int):
    return [(v >> (16 * i)) & 0xFFFF for i in range(4) if (v >> (16 * i)) & 0x8000]


@settings(max_examples=400, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(positions())
def test_move_rule_invariants(pos):
    board, player, roll = pos
    moves, n = O.movegen(board, player, roll, cap=8192)
    assert n == len(moves)
    lens = {len(_subs(int(m))) for m in moves}
    assert len(lens) <= 1
    if lens:
        assert 1 <= lens.pop() <= (4 if roll[0] == roll[1] else 2)
    seen = set()
    for m in moves:
        after = O.apply_move(board, player, int(m))
        for side in (0, 1):
            pts = after[24 * side:24 * side + 24].astype(int)
            assert (pts >= 0).all()
            assert pts.sum() + int(after[48 + side]) + int(after[50 + side]) == 15
        assert not ((after[:24] > 0) & (after[24:48] > 0)).any()
        key = after.tobytes()
        assert key not in seen
        seen.add(key)
        if board[48 + player] > 0:           # bar checkers enter first
            assert (_subs(int(m))[0] & 31) == 24


@pytest.mark.parametrize("seed", range(3))
def test_env_conservation(seed):
    """Seeded random self-play on the oracle env: 15 checkers a side after every
    step; rewards 0 / -1 (invalid) inside a game, 1 / 1.5 / 2 at its end."""
    env = O.Env(seed=seed)
    env.reset()
    rng = np.random.RandomState(seed)
    for _ in range(600):
        _, meta = env.state()
        n = int(meta[3])
        _, r, done, _ = env.step(rng.randint(n) if n else 0)
        board, _ = env.state()
        b = np.asarray(board, np.int64)
        assert b[:24].sum() + b[48] + b[50] == 15 and b[24:48].sum() + b[49] + b[51] == 15
        if done:
            assert r in (1.0, 1.5, 2.0)
            env.reset()
        else:
            assert r in (0.0, -1.0)
