"""ctypes wrapper around the CPU parity oracle (``oracle/libbgoracle.so``).

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg as the *checker*.  The product package
(``mlp-ppo-2ply-p3_amd/bgx``) never imports this module.

The oracle restates the reference's rules (see ``bgoracle.c``); parity of the
oracle itself is pinned against fixtures generated from the reference
(``tests/golden/``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libbgoracle.so")
_lib = None

MOVE_DTYPE = np.uint64


def build() -> str:
    """Compile the oracle with make (gcc); returns the library path."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        L.bgo_movegen.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, ctypes.c_int, P]
        L.bgo_movegen.restype = ctypes.c_int
        L.bgo_apply_move.argtypes = [P, ctypes.c_int, ctypes.c_uint64]
        L.bgo_features.argtypes = [P, ctypes.c_int, P]
        L.bgo_features_batch.argtypes = [P, P, ctypes.c_int, P]
        L.bgo_movegen_batch.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int, P, P]
        L.bgo_two_ply_leaves.argtypes = [P, ctypes.c_int, ctypes.c_uint64, P, ctypes.c_int, P]
        L.bgo_two_ply_leaves.restype = ctypes.c_int
        L.bgo_mt_seed.argtypes = [P, ctypes.c_uint32]
        L.bgo_mt_next.argtypes = [P]
        L.bgo_mt_next.restype = ctypes.c_uint32
        L.bgo_roll_die.argtypes = [P]
        L.bgo_roll_die.restype = ctypes.c_int
        L.bgo_mt_size.restype = ctypes.c_int
        L.bgo_env_size.restype = ctypes.c_int
        L.bgo_env_init.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_uint32]
        L.bgo_env_free.argtypes = [P]
        L.bgo_env_reset.argtypes = [P, P]
        L.bgo_env_step.argtypes = [P, ctypes.c_int, P, P, P, P]
        L.bgo_env_state.argtypes = [P, P, P]
        L.bgo_env_legal.argtypes = [P, P]
        L.bgo_env_share_rng.argtypes = [P, P]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def movegen(board52, player: int, roll, cap: int = 4096):
    """Ordered legal moves (encoded uint64) and the untruncated count."""
    b = np.ascontiguousarray(board52, dtype=np.int8)
    out = np.zeros(cap, dtype=np.uint64)
    nu = ctypes.c_int(0)
    n = lib().bgo_movegen(_p(b), int(player), int(roll[0]), int(roll[1]), _p(out), cap, ctypes.byref(nu))
    return out[: min(n, cap)].copy(), n


def movegen_batch(boards52, players, dice, cap: int):
    b = np.ascontiguousarray(boards52, dtype=np.int8)
    p = np.ascontiguousarray(players, dtype=np.uint8)
    d = np.ascontiguousarray(dice, dtype=np.uint8)
    n = b.shape[0]
    counts = np.zeros(n, dtype=np.int32)
    out = np.zeros((n, cap), dtype=np.uint64)
    lib().bgo_movegen_batch(_p(b), _p(p), _p(d), n, cap, _p(counts), _p(out))
    return counts, out


def apply_move(board52, player: int, move: int):
    b = np.array(board52, dtype=np.int8, copy=True)
    lib().bgo_apply_move(_p(b), int(player), ctypes.c_uint64(int(move)))
    return b


def features(board52, player: int):
    b = np.ascontiguousarray(board52, dtype=np.int8)
    out = np.zeros(198, dtype=np.float32)
    lib().bgo_features(_p(b), int(player), _p(out))
    return out


def features_batch(boards52, players):
    b = np.ascontiguousarray(boards52, dtype=np.int8)
    p = np.ascontiguousarray(players, dtype=np.uint8)
    out = np.zeros((b.shape[0], 198), dtype=np.float32)
    lib().bgo_features_batch(_p(b), _p(p), b.shape[0], _p(out))
    return out


def two_ply_leaves(board52, mover: int, move: int, cap: int = 1 << 16):
    """Leaf features [rows, 198] of one root move over the 21 rolls and the leaf
    count per roll (bgo_two_ply_leaves)."""
    b = np.ascontiguousarray(board52, dtype=np.int8)
    while True:
        out = np.empty((cap, 198), dtype=np.float32)
        counts = np.zeros(21, dtype=np.int32)
        n = lib().bgo_two_ply_leaves(_p(b), int(mover), ctypes.c_uint64(int(move)), _p(out), cap, _p(counts))
        if n >= 0:
            return out[:n], counts
        cap *= 4


class MT:
    """numpy-legacy MT19937 restatement (np.random.seed(s); np.random.randint(1,7))."""

    def __init__(self, seed: int):
        self._buf = ctypes.create_string_buffer(lib().bgo_mt_size())
        lib().bgo_mt_seed(self._buf, seed & 0xFFFFFFFF)

    def next_u32(self) -> int:
        return lib().bgo_mt_next(self._buf)

    def die(self) -> int:
        return lib().bgo_roll_die(self._buf)


class Env:
    """CPU restatement of BackgammonEnv (environment/backgammon_env.py:35-405)."""

    def __init__(self, seed: int, match_length: int = 15, max_moves: int = 500):
        self._buf = ctypes.create_string_buffer(lib().bgo_env_size())
        self.max_moves = max_moves
        lib().bgo_env_init(self._buf, match_length, max_moves, seed & 0xFFFFFFFF)

    def __del__(self):
        try:
            lib().bgo_env_free(self._buf)
        except Exception:
            pass

    def share_rng(self, mt: "MT"):
        """Draw dice from a shared stream (VectorizedBackgammonEnv semantics)."""
        self._shared = mt
        lib().bgo_env_share_rng(self._buf, mt._buf)

    def reset(self):
        obs = np.zeros(198, dtype=np.float32)
        lib().bgo_env_reset(self._buf, _p(obs))
        return obs

    def step(self, action: int):
        obs = np.zeros(198, dtype=np.float32)
        rew = np.zeros(1, dtype=np.float32)
        done = np.zeros(1, dtype=np.int32)
        info = np.zeros(4, dtype=np.int32)
        lib().bgo_env_step(self._buf, int(action), _p(obs), _p(rew), _p(done), _p(info))
        return obs, float(rew[0]), bool(done[0]), info

    def state(self):
        b = np.zeros(52, dtype=np.int8)
        st = np.zeros(9, dtype=np.int32)
        lib().bgo_env_state(self._buf, _p(b), _p(st))
        return b, st

    def legal(self):
        _, st = self.state()
        out = np.zeros(max(int(st[3]), 1), dtype=np.uint64)
        lib().bgo_env_legal(self._buf, _p(out))
        return out[: int(st[3])]


def decode_move(v: int):
    """uint64 move -> [(start, end, hit), ...] (16 bits per sub-move)."""
    v = int(v)
    subs = []
    for i in range(4):
        s = (v >> (16 * i)) & 0xFFFF
        if not s & 0x8000:
            break
        subs.append((s & 31, (s >> 5) & 31, (s >> 10) & 1))
    return subs


def encode_move(subs) -> int:
    v = 0
    for i, (a, b, h) in enumerate(subs):
        v |= (a | (b << 5) | (int(h) << 10) | (1 << 15)) << (16 * i)
    return v


INITIAL_BOARD52 = np.zeros(52, dtype=np.int8)
for _k, _v in {0: 2, 11: 5, 16: 3, 18: 5}.items():
    INITIAL_BOARD52[_k] = _v
for _k, _v in {23: 2, 12: 5, 7: 3, 5: 5}.items():
    INITIAL_BOARD52[24 + _k] = _v

def leaf_values(W1, b1, w2, b2, keys, tags, side, ml):
    """V in fp64 of every valid 2-ply leaf-pool slot, from the evaluator's own inputs read
    back from the device (bgx_debug_option BGX_2PLY_DUMP: the 16-byte keys -- the replier's
    nibbles, bar, off, hit mask --, the tags, the rows' mover sides and the jobs' final max
    lengths), encoded as immutable_board.py:171-212 with the root mover's one-hot (DESIGN.md
    §5) and put through relu(F W1^T + b1) w2 + b2.  Returns (slot indices, V)."""
    keys = np.asarray(keys); tags = np.asarray(tags); side = np.asarray(side); ml = np.asarray(ml)
    used = tags != 0xFFFFFFFF
    job = (tags & 0x1FFFFFFF).astype(np.int64)
    valid = used & (ml[np.where(used, job, 0)] == (tags >> 29))
    idx = np.nonzero(valid)[0]
    k, jb = keys[idx], job[idx]
    rs = side[jb // 21]
    q = ((rs[:, 3] >> 8) & 1).astype(np.int64)
    hits = k[:, 3] >> 8

    def nib(lo, hi):
        v = np.zeros((len(lo), 24), np.int64)
        for p in range(16):
            v[:, p] = (lo >> np.uint64(4 * p)) & np.uint64(15)
        for p in range(8):
            v[:, 16 + p] = (hi >> np.uint32(4 * p)) & np.uint32(15)
        return v
    qn = nib(k[:, 0].astype(np.uint64) | (k[:, 1].astype(np.uint64) << np.uint64(32)), k[:, 2])
    hb = np.stack([(hits >> p) & 1 for p in range(24)], 1).astype(np.int64)
    mn = nib(rs[:, 0].astype(np.uint64) | (rs[:, 1].astype(np.uint64) << np.uint64(32)), rs[:, 2]) - hb
    bars = [k[:, 3] & 15, (rs[:, 3] & 15) + hb.sum(1)]
    offs = [(k[:, 3] >> 4) & 15, (rs[:, 3] >> 4) & 15]
    F = np.zeros((len(idx), 198))
    for P in range(2):
        rep = (q == P)[:, None]
        cnt = np.where(rep, qn, mn)
        F[:, 98 * P + 0:96 + 98 * P:4] = cnt >= 1
        F[:, 98 * P + 1:96 + 98 * P:4] = cnt >= 2
        F[:, 98 * P + 2:96 + 98 * P:4] = cnt >= 3
        F[:, 98 * P + 3:96 + 98 * P:4] = np.where(cnt >= 3, (cnt - 3) / 2.0, 0)
        F[:, 96 + 98 * P] = np.where(q == P, bars[0], bars[1]) / 2.0
        F[:, 97 + 98 * P] = np.where(q == P, offs[0], offs[1]) / 15.0
    F[np.arange(len(idx)), 196 + (1 - q)] = 1.0        # the root mover's one-hot
    return idx, np.maximum(F @ np.asarray(W1, np.float64).T + np.asarray(b1, np.float64), 0) @ np.asarray(w2, np.float64) + b2
