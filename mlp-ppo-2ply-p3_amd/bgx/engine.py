"""Device-resident batch of backgammon games (the HIP engine behind the C ABI).

`Engine` owns B game lanes on one GPU.  Every method enqueues HIP kernels on the
current torch stream of the engine's device and returns torch tensors; nothing
here synchronises the host except the explicit `error()` check.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import check

DICE_MODES = {"mt": _lib.DICE_MT_LANE, "shared": _lib.DICE_MT_SHARED, "philox": _lib.DICE_PHILOX}

# lane record byte offsets (bg_engine.hip)
R_CUR, R_ROLL0, R_ROLL1, R_OVER, R_MATCH, R_S0, R_S1, R_NEED, R_NM0, R_NM1, R_FLAGS = \
    52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class Engine:
    """B concurrent BackgammonEnv lanes (backgammon_env.py:35-405) on one GPU.

    dice: "mt"      lane i draws from numpy-legacy MT19937 seeded seeds[i]
                    (== a reference BackgammonEnv after env.seed(seeds[i]))
          "shared"  one MT19937 stream consumed in lane order
                    (== reference VectorizedBackgammonEnv after np.random.seed(s))
          "philox"  Philox4x32-10 per lane (speed mode)
    auto_reset: True = VectorizedBackgammonEnv.step semantics (vec_bg_env.py:35-36),
                False = BackgammonEnv.step semantics (backgammon_env.py:119-121).
    """

    def __init__(self, batch: int, max_moves: int = 500, seed: int = 0, dice: str = "philox",
                 auto_reset: bool = True, match_length: int = 15, device=None):
        self._lib = _lib.load()
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if dev.type != "cuda":
            raise ValueError("bgx.Engine needs a GPU device (HIP); there is no CPU fallback")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.batch = int(batch)
        self.max_moves = int(max_moves)
        self.dice = dice
        self.auto_reset = bool(auto_reset)
        h = ctypes.c_void_p()
        check(self._lib.bgx_engine_create(dev.index, self.batch, self.max_moves, int(seed) & (2**64 - 1),
                                          DICE_MODES[dice], int(self.auto_reset), int(match_length),
                                          ctypes.byref(h)), "bgx_engine_create")
        self._h = h
        kw = dict(device=dev)
        self.obs = torch.zeros(self.batch, 198, dtype=torch.float32, **kw)
        self.reward = torch.zeros(self.batch, dtype=torch.float32, **kw)
        self.done = torch.zeros(self.batch, dtype=torch.uint8, **kw)
        self.info = torch.zeros(self.batch, dtype=torch.int32, **kw)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                torch.cuda.synchronize(self.device)
                self._lib.bgx_engine_destroy(h)
            except Exception:
                pass
            self._h = None

    def lanes_ptr(self) -> int:
        """Device address of the engine's lane records (uint8[B][64], the
        bgx_buffers.lanes layout that records() copies): a consumer on the
        engine's stream may read them in place (e.g. PolicyNet.act(engine))."""
        if getattr(self, "_lanes_ptr", None) is None:
            b = _lib.BgxBuffers()
            check(self._lib.bgx_engine_buffers(self._h, ctypes.byref(b)), "bgx_engine_buffers")
            self._lanes_ptr = int(b.lanes)
        return self._lanes_ptr

    # ------------------------------------------------------------ plumbing --
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def seed(self, seeds=None, philox_seed: int = 0):
        """Per-lane MT seeds (BackgammonEnv.seed, backgammon_env.py:357-363)."""
        import numpy as np
        if seeds is None:
            seeds = np.arange(self.batch, dtype=np.uint32)
        arr = np.ascontiguousarray(np.broadcast_to(np.asarray(seeds, dtype=np.uint64) & 0xFFFFFFFF,
                                                   (self.batch,)).astype(np.uint32))
        torch.cuda.synchronize(self.device)
        check(self._lib.bgx_engine_seed(self._h, arr.ctypes.data_as(ctypes.c_void_p), int(philox_seed)),
              "bgx_engine_seed")

    def mt_state(self, lane: int = 0, state=None):
        """Get (state=None) or set the MT19937 state (uint32[625] = key + pos) of a
        lane / of the shared stream: numpy RandomState.get_state() compatible."""
        import numpy as np
        buf = np.zeros(625, dtype=np.uint32) if state is None else np.ascontiguousarray(state, dtype=np.uint32)
        check(self._lib.bgx_engine_mt_state(self._h, int(lane), buf.ctypes.data_as(ctypes.c_void_p),
                                            0 if state is None else 1), "bgx_engine_mt_state")
        return buf

    # ----------------------------------------------------------------- env --
    def reset(self, lane_mask: torch.Tensor | None = None, want_obs: bool = True) -> torch.Tensor:
        m = None
        if lane_mask is not None:
            m = lane_mask.to(device=self.device, dtype=torch.uint8).contiguous()
        check(self._lib.bgx_reset(self._h, _ptr(m), _ptr(self.obs) if want_obs else None, self._stream()),
              "bgx_reset")
        return self.obs

    def step(self, actions: torch.Tensor, want_obs: bool = True, want_info: bool = True, out=None):
        """Advance every lane by one BackgammonEnv.step; returns (obs, reward, done, info)
        views of engine-owned buffers (overwritten by the next step).  want_obs=False
        skips the fp32 observation write (rollouts that keep int8 boards); `out` =
        (reward f32[B], done u8[B]) tensors the step writes instead (rows of a
        device-resident rollout buffer)."""
        a = actions
        if not (isinstance(a, torch.Tensor) and a.device == self.device and a.dtype == torch.int32
                and a.is_contiguous()):
            a = torch.as_tensor(a).to(device=self.device, dtype=torch.int32).contiguous()
        reward, done = self.reward, self.done
        if out is not None:
            reward, done = out
            if (reward.dtype != torch.float32 or done.dtype != torch.uint8 or reward.device != self.device
                    or done.device != self.device or not reward.is_contiguous() or not done.is_contiguous()
                    or reward.numel() != self.batch or done.numel() != self.batch):
                raise ValueError("step: out must be contiguous (float32[B], uint8[B]) on the engine's device")
        check(self._lib.bgx_step(self._h, _ptr(a), _ptr(self.obs) if want_obs else None, _ptr(reward),
                                 _ptr(done), _ptr(self.info) if want_info else None, self._stream()),
              "bgx_step")
        return self.obs, reward, done, self.info

    def join(self):
        """Order the current stream after the engine's side-stream work (the next
        step's dispatch order, launched asynchronously by step): call it before a
        HIP graph capture of steps and as the capture's last call (bgx_engine_join)."""
        check(self._lib.bgx_engine_join(self._h, self._stream()), "bgx_engine_join")

    def set_fork(self, fork: bool):
        """fork=True (default): a Philox step's light launch and the next dispatch order
        run on the engine's side stream beside the heavy launch; False: all of a step
        on the current stream, so a HIP graph of steps is one linear chain (several
        engines on their own streams then fill the hardware queues one each; bench.py
        C3).  Same results either way (bgx_engine_set_fork)."""
        check(self._lib.bgx_engine_set_fork(self._h, int(bool(fork)), self._stream()), "bgx_engine_set_fork")

    # --------------------------------------------------------------- state --
    def lanes(self, lane0: int = 0, n: int | None = None):
        """(records uint8[n,64], moves int64[n,max_moves], n_total int32[n]) copies."""
        n = self.batch - lane0 if n is None else n
        rec = torch.empty(n, 64, dtype=torch.uint8, device=self.device)
        mv = torch.empty(n, self.max_moves, dtype=torch.int64, device=self.device)
        nt = torch.empty(n, dtype=torch.int32, device=self.device)
        check(self._lib.bgx_copy_lanes(self._h, lane0, n, _ptr(rec), _ptr(mv), _ptr(nt), self._stream()),
              "bgx_copy_lanes")
        return rec, mv, nt

    def record(self, lane: int):
        """One lane's 64-byte record as a host numpy array (synchronises)."""
        r = torch.empty(1, 64, dtype=torch.uint8, device=self.device)
        check(self._lib.bgx_copy_lanes(self._h, int(lane), 1, _ptr(r), None, None, self._stream()),
              "bgx_copy_lanes")
        return r.cpu().numpy()[0]

    def records(self, out: torch.Tensor | None = None) -> torch.Tensor:
        """Lane records only (uint8[B,64]: board52, mover, roll, flags, legal count)."""
        if out is None:
            out = torch.empty(self.batch, 64, dtype=torch.uint8, device=self.device)
        check(self._lib.bgx_copy_lanes(self._h, 0, self.batch, _ptr(out), None, None, self._stream()),
              "bgx_copy_lanes")
        return out

    def set_lanes(self, records: torch.Tensor, lane0: int = 0, regen: bool = True):
        """Overwrite lane records [lane0, lane0 + n); regen: re-enumerate their legal
        moves for the stored player / roll (update_legal_moves), else leave the
        stored moves as they are (roll_dice / pass_turn, bgx_set_lanes_ex)."""
        r = records.to(device=self.device, dtype=torch.uint8).contiguous()
        if r.dim() != 2 or r.shape[1] != 64:
            raise ValueError(f"set_lanes: records must be [n, 64] bytes, got {tuple(r.shape)}")
        check(self._lib.bgx_set_lanes_ex(self._h, lane0, r.shape[0], _ptr(r), int(bool(regen)), self._stream()),
              "bgx_set_lanes_ex")

    def n_moves(self, out: torch.Tensor | None = None) -> torch.Tensor:
        """Legal-action count per lane (int16[B]); mask = arange(max_moves) < count."""
        if out is None:
            out = torch.empty(self.batch, dtype=torch.int16, device=self.device)
        check(self._lib.bgx_action_masks(self._h, _ptr(out), None, self._stream()), "bgx_action_masks")
        return out

    def action_masks(self) -> torch.Tensor:
        """float[B, max_moves] (VectorizedBackgammonEnv.get_action_masks, vec_bg_env.py:51-56)."""
        out = torch.empty(self.batch, self.max_moves, dtype=torch.float32, device=self.device)
        check(self._lib.bgx_action_masks(self._h, None, _ptr(out), self._stream()), "bgx_action_masks")
        return out

    def afterstates(self, lane0: int = 0, n: int | None = None) -> torch.Tensor:
        n = self.batch - lane0 if n is None else n
        out = torch.empty(n, self.max_moves, 52, dtype=torch.int8, device=self.device)
        check(self._lib.bgx_afterstates(self._h, lane0, n, _ptr(out), self._stream()), "bgx_afterstates")
        return out

    def legal_features(self, lane0: int = 0, n: int | None = None) -> torch.Tensor:
        n = self.batch - lane0 if n is None else n
        out = torch.empty(n, self.max_moves, 198, dtype=torch.float32, device=self.device)
        check(self._lib.bgx_legal_features(self._h, lane0, n, _ptr(out), self._stream()), "bgx_legal_features")
        return out

    def error(self) -> int:
        v = ctypes.c_int32(0)
        check(self._lib.bgx_engine_error(self._h, ctypes.byref(v)), "bgx_engine_error")
        return v.value

    # ------------------------------------------------------ stateless ops --
    def movegen(self, boards52: torch.Tensor, players: torch.Tensor, dice: torch.Tensor, max_moves: int | None = None):
        """get_all_possible_moves on n positions (n <= batch).  Returns
        (n_moves int16[n], n_total int32[n], moves int64[n, max_moves])."""
        cap = self.max_moves if max_moves is None else int(max_moves)
        b = boards52.to(device=self.device, dtype=torch.int8).contiguous()
        p = players.to(device=self.device, dtype=torch.uint8).contiguous()
        d = dice.to(device=self.device, dtype=torch.uint8).contiguous()
        n = b.shape[0]
        nm = torch.empty(n, dtype=torch.int16, device=self.device)
        nt = torch.empty(n, dtype=torch.int32, device=self.device)
        mv = torch.zeros(n, cap, dtype=torch.int64, device=self.device)
        check(self._lib.bgx_movegen(self._h, _ptr(b), _ptr(p), _ptr(d), n, cap, _ptr(nm), _ptr(nt), _ptr(mv),
                                    self._stream()), "bgx_movegen")
        return nm, nt, mv


def encode_records(records: torch.Tensor, dtype=torch.float32, width: int = 198) -> torch.Tensor:
    """get_board_features of n 64-byte lane records (board bytes 0..51, player to
    move at 52) as fp32, or fp16 = the fp32 features rounded (autocast's cast).
    width 208: rows padded with 10 zero columns (16-byte aligned GEMM operand)."""
    if records.dim() != 2 or records.shape[1] != 64 or records.element_size() != 1:
        raise ValueError(f"encode_records: records must be [n, 64] bytes, got {tuple(records.shape)} {records.dtype}")
    if dtype not in (torch.float32, torch.float16):
        raise ValueError(f"encode_records: dtype must be float32 or float16, got {dtype}")
    if width not in (198, 208):
        raise ValueError(f"encode_records: width must be 198 or 208, got {width}")
    L = _lib.load()
    r = records.contiguous()
    out = torch.empty(r.shape[0], width, dtype=dtype, device=r.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(r.device).cuda_stream)
    check(L.bgx_encode_records_ex(_ptr(r), r.shape[0], 0 if dtype == torch.float32 else 1, width, _ptr(out), s),
          "bgx_encode_records_ex")
    return out


def encode(boards52: torch.Tensor, players: torch.Tensor) -> torch.Tensor:
    """ImmutableBoard.get_board_features for a batch (immutable_board.py:171-212)."""
    L = _lib.load()
    b = boards52.to(dtype=torch.int8).contiguous()
    p = players.to(device=b.device, dtype=torch.uint8).contiguous()
    out = torch.empty(b.shape[0], 198, dtype=torch.float32, device=b.device)
    s = ctypes.c_void_p(torch.cuda.current_stream(b.device).cuda_stream)
    check(L.bgx_encode(_ptr(b), _ptr(p), b.shape[0], _ptr(out), s), "bgx_encode")
    return out
