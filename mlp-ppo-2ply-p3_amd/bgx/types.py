"""Reference data types (players/player.py, moves/move_types.py, board/*.py) and
the board-level API (immutable_board.py, moves/get_all_moves.py, ai/batching.py,
moves/get_all_dice_rolls.py) backed by the HIP kernels.

Boards keep the reference's (4,24) int8 tensor representation; the kernels use
the 52-byte form (p1[24] p2[24] bar[2] off[2]).  Every computation runs on the
GPU through libbgx.so; CPU tensors are moved to the GPU and results moved back.
"""
from __future__ import annotations

from dataclasses import dataclass
from enum import IntEnum
from typing import List

import numpy as np
import torch


class Player(IntEnum):                       # players/player.py:6-12
    PLAYER1 = 0
    PLAYER2 = 1


class Position(IntEnum):                     # moves/move_types.py:9-35
    P_0 = 0; P_1 = 1; P_2 = 2; P_3 = 3; P_4 = 4; P_5 = 5; P_6 = 6; P_7 = 7  # noqa: E702
    P_8 = 8; P_9 = 9; P_10 = 10; P_11 = 11; P_12 = 12; P_13 = 13; P_14 = 14  # noqa: E702
    P_15 = 15; P_16 = 16; P_17 = 17; P_18 = 18; P_19 = 19; P_20 = 20  # noqa: E702
    P_21 = 21; P_22 = 22; P_23 = 23; BAR = 24; BEAR_OFF = 25  # noqa: E702


class BoardState(IntEnum):                   # board/board_state.py:6-10
    NORMAL = 0
    ON_BAR = 1
    BEAR_OFF = 2
    GAME_OVER = 3


@dataclass(frozen=True)
class SubMove:                               # moves/move_types.py:38-42
    start: Position
    end: Position
    hits_blot: bool


@dataclass
class FullMove:                              # moves/move_types.py:45-48
    sub_move_commands: List[SubMove]
    player: Player


def decode_move(v: int, player: Player) -> FullMove:
    """uint64 engine move (include/bgx.h) -> FullMove."""
    v = int(v) & (2**64 - 1)
    subs = []
    for i in range(4):
        s = (v >> (16 * i)) & 0xFFFF
        if not s & 0x8000:
            break
        subs.append(SubMove(Position(s & 31), Position((s >> 5) & 31), bool((s >> 10) & 1)))
    return FullMove(sub_move_commands=subs, player=Player(player))


def encode_move(m: FullMove) -> int:
    v = 0
    for i, s in enumerate(m.sub_move_commands):
        v |= (int(s.start) | (int(s.end) << 5) | (int(bool(s.hits_blot)) << 10) | (1 << 15)) << (16 * i)
    return v


def tensor_to52(t: torch.Tensor) -> torch.Tensor:
    """(...,4,24) int8 -> (...,52) int8."""
    return torch.cat([t[..., 0, :], t[..., 1, :], t[..., 2, :2], t[..., 3, :2]], dim=-1).to(torch.int8)


def tensor_from52(x: torch.Tensor) -> torch.Tensor:
    """(...,52) int8 -> (...,4,24) int8."""
    shape = x.shape[:-1]
    out = torch.zeros(*shape, 4, 24, dtype=torch.int8, device=x.device)
    out[..., 0, :] = x[..., :24]
    out[..., 1, :] = x[..., 24:48]
    out[..., 2, :2] = x[..., 48:50]
    out[..., 3, :2] = x[..., 50:52]
    return out


def _gpu() -> torch.device:
    return torch.device("cuda", torch.cuda.current_device())


_UTIL = {}


def util_engine(n: int):
    """A per-device engine used only for stateless ops (movegen on posed boards)."""
    from .engine import Engine
    dev = _gpu()
    e = _UTIL.get(dev.index)
    if e is None or e.batch < n:
        e = Engine(batch=max(n, 1024), max_moves=4096, dice="philox", device=dev)
        _UTIL[dev.index] = e
    return e


@dataclass(frozen=True)
class ImmutableBoard:                        # board/immutable_board.py:16-246
    tensor: torch.Tensor

    @staticmethod
    def initial_board(device=None) -> "ImmutableBoard":
        t = torch.zeros((4, 24), dtype=torch.int8, device=device)
        t[0, 0], t[0, 11], t[0, 16], t[0, 18] = 2, 5, 3, 5
        t[1, 23], t[1, 12], t[1, 7], t[1, 5] = 2, 5, 3, 5
        return ImmutableBoard(t)

    def move_checker(self, player: Player, sub_move: SubMove) -> "ImmutableBoard":
        """immutable_board.py:42-89 (copy-on-write sub-move apply, with the
        reference's 'return the board unchanged' on invalid sub-moves)."""
        t = self.tensor.clone()
        me, opp = int(player), 1 - int(player)
        s, e = int(sub_move.start), int(sub_move.end)
        if s == Position.BAR:
            if t[2, me] <= 0:
                return self
            t[2, me] -= 1
        else:
            if t[me, s] <= 0:
                return self
            t[me, s] -= 1
        if sub_move.hits_blot:
            if e >= 24 or t[opp, e] <= 0:
                return self
            t[opp, e] -= 1
            t[2, opp] += 1
        if e == Position.BEAR_OFF:
            t[3, me] += 1
        else:
            t[me, e] += 1
        return ImmutableBoard(t)

    def get_board_features(self, current_player: Player) -> torch.Tensor:
        """immutable_board.py:171-212 via the HIP encoder."""
        return get_board_features_batch_from_tensors(self.tensor[None], current_player)[0]


def execute_sub_move_on_board(board: ImmutableBoard, sub_move: SubMove, player: Player) -> ImmutableBoard:
    return board.move_checker(player, sub_move)


def execute_full_move_on_board_copy(board: ImmutableBoard, full_move: FullMove) -> ImmutableBoard:
    nb = board
    for s in full_move.sub_move_commands:
        nb = nb.move_checker(full_move.player, s)
    return nb


def board_hash(board: ImmutableBoard) -> int:
    return hash(board.tensor.detach().cpu().numpy().tobytes())


def board_to_string(board: ImmutableBoard) -> str:          # immutable_board.py:249-267
    t = board.tensor.cpu()
    lines = []
    for i in range(24):
        a, b = int(t[0, i]), int(t[1, i])
        cell = "!" if a > 0 and b > 0 else ("●" * a if a > 0 else ("○" * b if b > 0 else "-"))
        lines.append(f"{i}: {cell}")
    return "\n".join(lines)


_TOKENS = ("●", "○")                                          # backgammon_env.py:15-18


def render_board(board: ImmutableBoard) -> str:
    """The text of BackgammonEnv.render (backgammon_env.py:253-355) with its bar /
    off lookup fixed: the reference reads tensor[player, BAR=24] on a (4,24)
    tensor and raises IndexError; here bar = tensor[2, p] and off = tensor[3, p].
    Returns the printed text (render() prints it)."""
    t = board.tensor.cpu()
    out = []
    cnt, col = [0] * 24, [" "] * 24
    for i in range(24):
        a, b = int(t[0, i]), int(t[1, i])
        if a > 0 and b > 0:
            out.append(f"Invalid board state at point {i}: Both players have checkers.")
            col[i] = "?"
        elif a > 0 or b > 0:
            cnt[i], col[i] = (a, _TOKENS[0]) if a > 0 else (b, _TOKENS[1])

    def half(points, p):
        bar, off = int(t[2, p]), int(t[3, p])
        tok = _TOKENS[p]
        for lvl in range(max(max(cnt[q] for q in points), bar, off)):
            cells = [f"{col[q] if cnt[q] > lvl else ' ':^3}" for q in points]
            mid = f"{tok if bar > lvl else ' ':^3}"
            end = f"{tok if off > lvl else ' ':^3}"
            out.append("|  " + " | ".join(cells[:6]) + f" | {mid} | " + " | ".join(cells[6:]) + f" | {end} |")

    rule = "|------------------------------------|     |-----------------------------------|     |"
    out.append("| 12 | 13 | 14 | 15 | 16 | 17 | BAR | 18 | 19 | 20 | 21 | 22 | 23 | OFF |")
    out.append(f"|------------Outer Board-------------|     |-----------P={_TOKENS[1]} Home Board----------|     |")
    half(list(range(12, 24)), 1)
    out.append(rule)
    half(list(range(11, -1, -1)), 0)
    out.append(f"|------------Outer Board-------------|     |-----------P={_TOKENS[0]} Home Board----------|     |")
    out.append("| 11 | 10 | 9  | 8  | 7  | 6  | BAR | 5  | 4  | 3  | 2  | 1  | 0  | OFF |\n")
    return "\n".join(out) + "\n"


def get_all_possible_moves(player: Player, board: ImmutableBoard, roll_result) -> List[FullMove]:
    """moves/get_all_moves.py:9-70 on the HIP move generator (complete list, no truncation)."""
    e = util_engine(1)
    b = tensor_to52(board.tensor).reshape(1, 52).to(e.device)
    p = torch.tensor([int(player)], dtype=torch.uint8, device=e.device)
    d = torch.tensor([[int(roll_result[0]), int(roll_result[1])]], dtype=torch.uint8, device=e.device)
    nm, nt, mv = e.movegen(b, p, d, max_moves=4096)
    n = int(nt[0])
    if n > 4096:
        raise RuntimeError(f"{n} legal moves exceed the 4096-move buffer")
    return [decode_move(v, player) for v in mv[0, :n].cpu().numpy().view(np.uint64)]


def filter_full_moves_by_max_submoves(full_moves: List[FullMove]) -> List[FullMove]:   # get_all_moves.py:73-94
    if not full_moves:
        return []
    m = max(len(x.sub_move_commands) for x in full_moves)
    return [x for x in full_moves if len(x.sub_move_commands) == m]


def get_board_features_batch_from_tensors(board_tensors: torch.Tensor, current_player: Player) -> torch.Tensor:
    """ai/batching.py:78-147: (N,4,24) int8 -> (N,198) f32 on the HIP encoder."""
    from .engine import encode
    dev = board_tensors.device
    b = tensor_to52(board_tensors).to(_gpu())
    p = torch.full((b.shape[0],), int(current_player), dtype=torch.uint8, device=b.device)
    return encode(b, p).to(dev)


def generate_all_board_features(board: ImmutableBoard, current_player: Player, legal_moves: List[FullMove],
                                roll_result=None) -> torch.Tensor:
    """ai/batching.py:10-75 (afterstate features of every legal move)."""
    if not legal_moves:
        return torch.empty((0, 198), dtype=torch.float32, device=board.tensor.device)
    lens = {len(m.sub_move_commands) for m in legal_moves}
    if len(lens) != 1:
        raise ValueError("Inconsistent number of SubMoves (M) in batch.")
    boards = torch.stack([execute_full_move_on_board_copy(board, m).tensor for m in legal_moves])
    return get_board_features_batch_from_tensors(boards, current_player)


def get_all_dice_rolls_tensor():
    """moves/get_all_dice_rolls.py:5-34: the 21 distinct rolls and their probabilities."""
    rolls, counts = [], []
    for a in range(1, 7):
        for b in range(a, 7):
            rolls.append([a, b])
            counts.append(1 if a == b else 2)
    return torch.tensor(rolls, dtype=torch.int32), torch.tensor(counts, dtype=torch.float32) / 36
