"""1-ply greedy and 2-ply expectimax move selection over engine lanes
(the reference's intended moves/expect_minmax.py, which is
commented out there).  V = value_head(relu(fc1 x)) of a
BackgammonPolicyNetwork (policy_network.py:54-56), H <= 128 (C2/C4 use H = 40;
the reference trains H = 128, agent/config.py:8).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import check
from .engine import Engine, _ptr


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


class ValueHead:
    """Packed (fc1, value_head) of a policy network for the search kernels."""

    def __init__(self, net):
        L = _lib.load()
        self.hidden = net.fc1.out_features
        n = L.bgx_value_packed_size(self.hidden)
        if n < 0:
            raise ValueError(f"value search supports hidden <= 128 (got {self.hidden})")
        dev = net.fc1.weight.device
        ps = [t.detach().float().contiguous() for t in (net.fc1.weight, net.fc1.bias, net.value_head.weight,
                                                         net.value_head.bias)]
        self.packed = torch.empty(n, dtype=torch.float32, device=dev)
        check(L.bgx_value_pack(*[_ptr(t) for t in ps], self.hidden, _ptr(self.packed), _stream(dev)),
              "bgx_value_pack")
        self.bias = float(net.value_head.bias.detach().float().cpu()[0])


def one_ply(eng: Engine, vh: ValueHead, want_values: bool = False):
    """First argmax over each lane's afterstates of V(afterstate, mover one-hot)."""
    L = _lib.load()
    B, dev = eng.batch, eng.device
    best = torch.empty(B, dtype=torch.int32, device=dev)
    bestv = torch.empty(B, dtype=torch.float32, device=dev)
    vals = torch.full((B, eng.max_moves), float("nan"), dtype=torch.float32, device=dev) if want_values else None
    check(L.bgx_one_ply(eng._h, _ptr(vh.packed), vh.hidden, vh.bias, _ptr(best), _ptr(bestv), _ptr(vals),
                        _stream(dev)), "bgx_one_ply")
    return (best, bestv, vals) if want_values else (best, bestv)


def two_ply(eng: Engine, vh: ValueHead, want_q: bool = False):
    """2-ply expectimax for every lane: returns (best int32[B], best Q f32[B],
    Q f32[B, max_moves] or None, stats {leaves, jobs, afterstates})."""
    L = _lib.load()
    B, dev = eng.batch, eng.device
    best = torch.empty(B, dtype=torch.int32, device=dev)
    bestq = torch.empty(B, dtype=torch.float32, device=dev)
    q = torch.full((B, eng.max_moves), float("nan"), dtype=torch.float32, device=dev) if want_q else None
    stats = (ctypes.c_uint64 * 3)()
    check(L.bgx_two_ply(eng._h, _ptr(vh.packed), vh.hidden, vh.bias, _ptr(best), _ptr(bestq), _ptr(q),
                        ctypes.cast(stats, ctypes.c_void_p), _stream(dev)), "bgx_two_ply")
    return best, bestq, q, {"leaves": int(stats[0]), "jobs": int(stats[1]), "afterstates": int(stats[2])}


def two_ply_timings(eng: Engine):
    """(enumeration ms, evaluation ms) of the last two_ply call's first round,
    timed with HIP events on the caller's stream."""
    L = _lib.load()
    ms = (ctypes.c_float * 2)()
    check(L.bgx_two_ply_timings(eng._h, ctypes.cast(ms, ctypes.c_void_p)), "bgx_two_ply_timings")
    return float(ms[0]), float(ms[1])
