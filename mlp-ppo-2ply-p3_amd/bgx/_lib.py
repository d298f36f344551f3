"""ctypes binding of libbgx.so (the C ABI in include/bgx.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950) and
must be present: there is no CPU fallback for the product path.
"""
from __future__ import annotations

import ctypes
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# BGX_LIB overrides the library path (A/B experiments between builds)
LIB_PATH = os.environ.get("BGX_LIB") or os.path.join(_HERE, "libbgx.so")

BGX_OK, BGX_EINVAL, BGX_EDEVICE, BGX_ENOMEM, BGX_EOVERFLOW, BGX_ESTATE = 0, -1, -2, -3, -4, -5
DICE_MT_LANE, DICE_MT_SHARED, DICE_PHILOX = 0, 1, 2

# (name, restype, argtypes) for every symbol declared in include/bgx.h
_P = ctypes.c_void_p
_I32 = ctypes.c_int32
SIGNATURES = {
    "bgx_engine_create": (ctypes.c_int, [ctypes.c_int, _I32, _I32, ctypes.c_uint64, _I32, _I32, _I32,
                                         ctypes.POINTER(_P)]),
    "bgx_engine_destroy": (ctypes.c_int, [_P]),
    "bgx_engine_set_fork": (ctypes.c_int, [_P, _I32, _P]),
    "bgx_engine_seed": (ctypes.c_int, [_P, _P, ctypes.c_uint64]),
    "bgx_engine_mt_state": (ctypes.c_int, [_P, _I32, _P, _I32]),
    "bgx_engine_buffers": (ctypes.c_int, [_P, _P]),
    "bgx_reset": (ctypes.c_int, [_P, _P, _P, _P]),
    "bgx_step": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P]),
    "bgx_movegen": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _P, _P, _P, _P]),
    "bgx_encode": (ctypes.c_int, [_P, _P, _I32, _P, _P]),
    "bgx_encode_records": (ctypes.c_int, [_P, _I32, _I32, _P, _P]),
    "bgx_encode_records_ex": (ctypes.c_int, [_P, _I32, _I32, _I32, _P, _P]),
    "bgx_afterstates": (ctypes.c_int, [_P, _I32, _I32, _P, _P]),
    "bgx_legal_features": (ctypes.c_int, [_P, _I32, _I32, _P, _P]),
    "bgx_action_masks": (ctypes.c_int, [_P, _P, _P, _P]),
    "bgx_copy_lanes": (ctypes.c_int, [_P, _I32, _I32, _P, _P, _P, _P]),
    "bgx_set_lanes": (ctypes.c_int, [_P, _I32, _I32, _P, _P]),
    "bgx_set_lanes_ex": (ctypes.c_int, [_P, _I32, _I32, _P, _I32, _P]),
    "bgx_engine_error": (ctypes.c_int, [_P, _P]),
    "bgx_policy_packed_size": (ctypes.c_int, [_I32, _I32]),
    "bgx_policy_pack": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I32, _I32, _P, _P]),
    "bgx_policy_act": (ctypes.c_int, [_P, _I32, _P, _I32, _I32, ctypes.c_uint64, ctypes.c_uint32, _I32, _P, _P, _P,
                                      _P, _P]),
    "bgx_policy_act_rec": (ctypes.c_int, [_P, _I32, _P, _I32, _I32, ctypes.c_uint64, ctypes.c_uint32, _I32, _P, _P,
                                          _P, _P, _P, _P]),
    "bgx_policy_act_ctr": (ctypes.c_int, [_P, _I32, _P, _I32, _I32, ctypes.c_uint64, ctypes.c_uint32, _P, _I32, _P,
                                          _P, _P, _P, _P, _P]),
    "bgx_counter_add": (ctypes.c_int, [_P, ctypes.c_uint32, _P]),
    "bgx_engine_join": (ctypes.c_int, [_P, _P]),
    "bgx_value_packed_size": (ctypes.c_int, [_I32]),
    "bgx_value_pack": (ctypes.c_int, [_P, _P, _P, _P, _I32, _P, _P]),
    "bgx_one_ply": (ctypes.c_int, [_P, _P, _I32, ctypes.c_float, _P, _P, _P, _P]),
    "bgx_two_ply": (ctypes.c_int, [_P, _P, _I32, ctypes.c_float, _P, _P, _P, _P, _P]),
    "bgx_two_ply_timings": (ctypes.c_int, [_P, _P]),
    "bgx_ppo_head": (ctypes.c_int, [_P, _I32, ctypes.c_int64, _P, _P, _P, _P, _P, _P, _I32, _I32, ctypes.c_float,
                                    ctypes.c_float, ctypes.c_float, ctypes.c_float, _P, ctypes.c_int64, _P, _P, _P]),
    "bgx_ppo_head_ex": (ctypes.c_int, [_P, _I32, ctypes.c_int64, _P, _P, _P, _P, _P, _P, _I32, _I32, ctypes.c_float,
                                       ctypes.c_float, ctypes.c_float, ctypes.c_float, _P, ctypes.c_int64, _P, _P, _I32,
                                       _P, _P]),
    "bgx_relu_backward": (ctypes.c_int, [_P, _P, _I32, _I32, _P, _I32, _P]),
    "bgx_fc1_packed_size": (ctypes.c_int, [_I32]),
    "bgx_fc1_pack": (ctypes.c_int, [_P, _I32, _P, _P]),
    "bgx_fc1_records": (ctypes.c_int, [_P, _I32, _P, _P, _I32, _P, _P]),
    "bgx_fc1_records_ex": (ctypes.c_int, [_P, _I32, _P, _P, _I32, _P, _P, _P]),
    "bgx_ppo_rows": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _I32, _I32, _I32, _P, _P, ctypes.c_float,
                                    ctypes.c_float, ctypes.c_float, ctypes.c_float, _P, _P, _P, _P, _P, _P, _P, _I32, _P]),
    "bgx_ppo_gw2_workspace": (ctypes.c_int64, [_I32]),
    "bgx_ppo_gw2": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _I32, _P, _P, ctypes.c_float, _P, _P, _P, _P, _P]),
    "bgx_ppo_gw1_workspace": (ctypes.c_int64, [_I32]),
    "bgx_ppo_gw1": (ctypes.c_int, [_P, _P, _I32, _I32, _P, _P, _P]),
    "bgx_copy_regions": (ctypes.c_int, [_P, _I32, _I32, _P]),
    "bgx_host_device_ptr": (ctypes.c_int, [_P, ctypes.POINTER(_P)]),
    "bgx_lane_returns": (ctypes.c_int, [_P, _P, _I32, _I32, ctypes.c_float, _P, _P]),
    "bgx_ppo_epoch_prep": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I32, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                          _P, _P]),
    "bgx_ppo_epoch_grads": (ctypes.c_int, [_P, _P, _P, _I32, _I32, ctypes.c_float, _P, _P, _P, _P, _P, _P, _P, _P,
                                           ctypes.c_float, _P, _P, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                           _P, _P]),
    "bgx_episode_stats_workspace": (ctypes.c_int64, [_I32]),
    "bgx_episode_stats": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _P, _P, _P]),
    "bgx_adam_step": (ctypes.c_int, [_I32, _P, _P, _P, _P, _P, _P, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                     ctypes.c_double, _P, _P, ctypes.c_float, ctypes.c_float, _I32, _P, _P]),
    "bgx_gather_rollout": (ctypes.c_int, [_P, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "bgx_ppo_plan_workspace": (ctypes.c_int64, [_I32]),
    "bgx_ppo_plan": (ctypes.c_int, [_P, _I32, _I32, _P, _P, _P, _P, _P]),
    "bgx_ppo_plan_rows": (ctypes.c_int, [_P, _I32, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "bgx_debug_option": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p]),
    "bgx_last_error": (ctypes.c_char_p, []),
    "bgx_build_id": (ctypes.c_char_p, []),
}

_PKG = os.path.dirname(_HERE)
_CSRC = os.path.join(_PKG, "csrc")
_HEADER = os.path.join(os.path.dirname(_PKG), "include", "bgx.h")
BUILD_ID_TAG = b"bgx-build-id:"


def source_hash(flags: str = "") -> str:
    """sha256 over every file under csrc/, include/bgx.h and the compile flags:
    the build id compiled into libbgx.so (bgx_build_id())."""
    h = hashlib.sha256()
    files = sorted(os.path.join(_CSRC, f) for f in os.listdir(_CSRC)
                   if f.endswith((".hip", ".h", ".cpp"))) + [_HEADER]
    for f in files:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(flags.encode())
    return h.hexdigest()


def embedded_build_id(path: str = LIB_PATH):
    """The build id stored in a built library file (read from its bytes, no load)."""
    if not os.path.exists(path):
        return None
    data = open(path, "rb").read()
    i = data.find(BUILD_ID_TAG)
    return data[i + len(BUILD_ID_TAG):i + len(BUILD_ID_TAG) + 64].decode() if i >= 0 else None


class BgxRegion(ctypes.Structure):
    _fields_ = [("src", _P), ("dst", _P), ("width", ctypes.c_int64), ("rows", ctypes.c_int64),
                ("spitch", ctypes.c_int64), ("dpitch", ctypes.c_int64)]


MAX_COPY_REGIONS = 8           # include/bgx.h BGX_MAX_COPY_REGIONS


class BgxBuffers(ctypes.Structure):
    _fields_ = [("lanes", _P), ("moves", _P), ("n_total", _P), ("batch", _I32), ("max_moves", _I32)]


_lib = None


class BgxError(RuntimeError):
    pass


def load():
    """Load libbgx.so; raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise BgxError(f"{LIB_PATH} missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


STATUS_NAMES = {BGX_EINVAL: "BGX_EINVAL", BGX_EDEVICE: "BGX_EDEVICE", BGX_ENOMEM: "BGX_ENOMEM",
                BGX_EOVERFLOW: "BGX_EOVERFLOW", BGX_ESTATE: "BGX_ESTATE"}


def check(rc: int, what: str):
    if rc != BGX_OK:
        msg = load().bgx_last_error()
        raise BgxError(f"{what} failed: status {rc} {STATUS_NAMES.get(rc, '')} ({msg.decode() if msg else ''})")


def debug_option(name: str, value=None):
    """bgx_debug_option: set (value str/int) or unset (None) one of the library's named
    debug options (include/bgx.h: the exact alternative paths the tests compare, and
    diagnostics).  The library never reads the environment."""
    check(load().bgx_debug_option(name.encode(), None if value is None else str(value).encode()),
          f"bgx_debug_option({name})")


class debug_options:
    """Context manager: set debug options for a block, unset them after."""

    def __init__(self, **opts):
        self.opts = opts

    def __enter__(self):
        for k, v in self.opts.items():
            debug_option(k, v)
        return self

    def __exit__(self, *exc):
        for k in self.opts:
            debug_option(k, None)
        return False
