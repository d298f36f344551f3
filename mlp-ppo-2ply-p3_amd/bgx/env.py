"""Drop-in BackgammonEnv / VectorizedBackgammonEnv (environment/backgammon_env.py,
environment/vec_bg_env.py) on the HIP engine.

Dice come from numpy's GLOBAL legacy RandomState exactly like the reference
(backgammon_env.py:245-246): before each reset/step the engine imports
np.random's MT19937 state and afterwards writes the advanced state back, so a
script that calls np.random.seed(s) / env.seed(s) sees the reference's games
bit for bit.  (The high-throughput path is bgx.Engine, which keeps per-lane
streams on the device.)
"""
from __future__ import annotations

import types as _pytypes
from typing import Dict, List

import numpy as np
import torch

from .engine import Engine
from .types import (ImmutableBoard, Player, decode_move, tensor_from52, board_to_string,  # noqa: F401
                    render_board, FullMove)

REWARD_INVALID_ACTION = -1.0     # backgammon_env.py:23-28
REWARD_PASS = 0.0
REWARD_HIT = 0.01
REWARD_WIN_NORMAL = 1.0
REWARD_WIN_GAMMON = 1.5
REWARD_WIN_BACKGAMMON = 2.0

_KIND_INFO = {1: "No legal actions, turn passed", 2: "Invalid action"}


def _push_numpy(eng: Engine, lane: int = 0):
    st = np.random.get_state()
    arr = np.empty(625, np.uint32)
    arr[:624] = st[1]
    arr[624] = st[2]
    eng.mt_state(lane, arr)


def _pull_numpy(eng: Engine, lane: int = 0):
    arr = eng.mt_state(lane)
    st = np.random.get_state()
    np.random.set_state(("MT19937", arr[:624].copy(), int(arr[624]), st[3], st[4]))


def _info_dict(v: int) -> dict:
    mover = Player(v & 0xFF)
    winner = ((v >> 8) & 0xFF) - 1
    score = (v >> 16) & 0xFF
    kind = (v >> 24) & 0xFF
    d = {"current_player": mover}
    if winner >= 0:
        d.update({"winner": Player(winner), "game_score": score})
    if kind in _KIND_INFO:
        d["info"] = _KIND_INFO[kind]
    return d


class _LaneView:
    """Read-only per-lane state (board, current_player, roll_result, legal_moves, ...)."""

    def __init__(self, eng: Engine, lane: int, device):
        self._eng, self._lane, self.device = eng, lane, torch.device(device)
        self._rec = None

    def _invalidate(self):
        self._rec = None

    def _record(self) -> np.ndarray:
        if self._rec is None:
            self._rec = self._eng.record(self._lane)
        return self._rec

    @property
    def board(self) -> ImmutableBoard:
        t = torch.from_numpy(self._record()[:52].view(np.int8).copy())
        return ImmutableBoard(tensor_from52(t).to(self.device))

    @property
    def current_player(self) -> Player:
        return Player(int(self._record()[52]))

    @property
    def roll_result(self):
        r = self._record()
        return [int(r[53]), int(r[54])]

    @property
    def game_over(self) -> bool:
        return bool(self._record()[55])

    @property
    def match_over(self) -> bool:
        return bool(self._record()[56])

    @property
    def player_scores(self) -> Dict[Player, int]:
        r = self._record()
        return {Player.PLAYER1: int(r[57]), Player.PLAYER2: int(r[58])}

    @property
    def n_legal(self) -> int:
        r = self._record()
        return int(r[60]) | (int(r[61]) << 8)

    @property
    def action_mask(self) -> torch.Tensor:
        m = torch.zeros(self._eng.max_moves, dtype=torch.float32)
        m[: self.n_legal] = 1.0
        return m.to(self.device)

    @property
    def legal_moves(self) -> List[FullMove]:
        n = self.n_legal
        if n == 0:
            return []
        _, mv, _ = self._eng.lanes(self._lane, 1)
        p = self.current_player
        return [decode_move(v, p) for v in mv[0, :n].cpu().numpy().view(np.uint64)]

    @property
    def legal_board_features(self) -> torch.Tensor:
        """[max_legal_moves, 198]: afterstate features, zero padded (backgammon_env.py:207-243)."""
        return self._eng.legal_features(self._lane, 1)[0].to(self.device)


class BackgammonEnv(_LaneView):
    """environment/backgammon_env.py:35-405 on one engine lane."""

    metadata = {"render.modes": ["human"]}

    def __init__(self, match_length=15, max_legal_moves=500, device=None):
        self.match_length = match_length
        self.max_legal_moves = max_legal_moves
        dev = torch.device(device) if device is not None else torch.device("cpu")
        eng = Engine(batch=1, max_moves=max_legal_moves, dice="mt", auto_reset=False, match_length=match_length)
        super().__init__(eng, 0, dev)
        self.observation_space = _pytypes.SimpleNamespace(shape=(198,), low=-1.0, high=1.0, dtype=np.float32)
        self.action_space = _pytypes.SimpleNamespace(n=max_legal_moves)
        self.current_match_winner = None

    def seed(self, seed=None):                       # backgammon_env.py:357-363
        torch.manual_seed(seed)
        if seed is not None:
            np.random.seed(seed)

    def reset(self):
        if self.match_over:
            self.current_match_winner = None
        _push_numpy(self._eng)
        obs = self._eng.reset()
        _pull_numpy(self._eng)
        self._invalidate()
        return obs[0].clone().to(self.device)

    def step(self, action):
        a = int(action)
        if not -self.max_legal_moves <= a < self.max_legal_moves:
            raise IndexError(f"index {a} is out of bounds for dimension 0 with size {self.max_legal_moves}")
        _push_numpy(self._eng)
        obs, rew, done, info = self._eng.step(torch.tensor([a], dtype=torch.int32, device=self._eng.device))
        _pull_numpy(self._eng)
        self._invalidate()
        info_d = _info_dict(int(info[0]))
        if info_d.get("info") == "Invalid action":
            print(f"Invalid action selected: {a}. Assigned reward: {float(rew[0])}")
        if "winner" in info_d and self.match_over:
            self.current_match_winner = info_d["winner"]
        return (obs[0].clone().to(self.device), torch.tensor(float(rew[0]), device=self.device),
                bool(done[0]), info_d)

    def get_observation(self):
        return self.board.get_board_features(self.current_player).to(self.device)

    # The reference's step() calls these three in turn (backgammon_env.py:129-131,
    # 186-188); here step() does the same on the device.  As public methods they
    # edit the lane's record the way the reference edits its attributes:
    # roll_dice and pass_turn leave legal_moves / action_mask stale until
    # update_legal_moves() re-enumerates them.
    def _write_record(self, rec: np.ndarray, regen: bool):
        self._eng.set_lanes(torch.from_numpy(np.ascontiguousarray(rec, dtype=np.uint8))[None], 0, regen=regen)
        self._invalidate()

    def update_legal_moves(self):                   # :198-243
        self._write_record(self._record(), regen=True)

    def roll_dice(self):                            # :245-246, numpy's global stream
        rec = self._record().copy()
        rec[53] = np.random.randint(1, 7)
        rec[54] = np.random.randint(1, 7)
        self._write_record(rec, regen=False)

    def pass_turn(self):                            # :248-251
        rec = self._record().copy()
        rec[52] ^= 1
        self._write_record(rec, regen=False)

    def check_for_gammon(self, player: Player) -> bool:        # :365-373
        return int(self.board.tensor[3, 1 - int(player)]) == 0

    def check_for_backgammon(self, player: Player) -> bool:    # :375-405
        t = self.board.tensor
        opp = 1 - int(player)
        if int(t[3, opp]) > 0:
            return False
        lo = 18 if player == Player.PLAYER1 else 0
        return bool((t[opp, lo:lo + 6] > 0).any()) or int(t[2, opp]) > 0

    def render(self, mode="human"):
        """backgammon_env.py:253-355's board drawing, with the bar / off lookup
        that raises IndexError in the reference fixed (types.render_board)."""
        if mode != "human":
            raise NotImplementedError("Only 'human' mode is supported")
        print(render_board(self.board), end="")

    def close(self):
        pass


class VectorizedBackgammonEnv:
    """environment/vec_bg_env.py:7-71: N lanes, auto-reset on done, one shared
    numpy dice stream consumed in lane order (engine dice mode "shared")."""

    def __init__(self, num_envs=1, match_length=15, max_legal_moves=500, device=None):
        self.num_envs = num_envs
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self._eng = Engine(batch=num_envs, max_moves=max_legal_moves, dice="shared", auto_reset=True,
                           match_length=match_length)
        self.envs = [_LaneView(self._eng, i, self.device) for i in range(num_envs)]
        self.observation_space = _pytypes.SimpleNamespace(shape=(198,), low=-1.0, high=1.0, dtype=np.float32)
        self.action_space = _pytypes.SimpleNamespace(n=max_legal_moves)

    def _invalidate(self):
        for e in self.envs:
            e._invalidate()

    def reset(self):
        _push_numpy(self._eng)
        obs = self._eng.reset()
        _pull_numpy(self._eng)
        self._invalidate()
        return obs.clone().to(self.device)

    def step(self, actions):
        a = torch.as_tensor(np.asarray(actions), dtype=torch.int32)
        _push_numpy(self._eng)
        obs, rew, done, info = self._eng.step(a.to(self._eng.device))
        _pull_numpy(self._eng)
        self._invalidate()
        infos = [_info_dict(int(v)) for v in info.cpu().numpy()]
        return (obs.clone().to(self.device), rew.clone().to(self.device),
                done.to(torch.bool).to(self.device), infos)

    def get_action_masks(self):
        return self._eng.action_masks().to(self.device)

    def get_legal_board_features(self):
        return self._eng.legal_features().to(self.device)

    def render(self):
        for i in range(self.num_envs):
            print(f"--- env {i}")
            print(board_to_string(self.envs[i].board))

    def close(self):
        pass
