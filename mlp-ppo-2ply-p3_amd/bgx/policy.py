"""BackgammonPolicyNetwork (agent/policy_network.py:6-75) and the rollout-side
policy step (select_action, agent/ppo_agent.py:138-191) over engine lanes.

The module keeps the reference's parameter names (fc1, action_head, value_head)
so state_dicts load both ways.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

import ctypes

from . import _lib
from ._lib import check
from .engine import encode, _ptr

# log(0 + 1e-45) in fp32: the reference masks with logits + log(mask + 1e-45)
# (ppo_agent.py:166), i.e. -103.27893 for illegal actions, not -inf.
MASK_LOG = float(torch.log(torch.tensor(1e-45, dtype=torch.float32)))


class PolicyNet(nn.Module):
    """198 -> H -> {action logits [A], value [1]} with ReLU (policy_network.py:44-75)."""

    def __init__(self, input_size: int = 198, hidden_size: int = 128, action_size: int = 500):
        super().__init__()
        self.fc1 = nn.Linear(input_size, hidden_size)
        self.action_head = nn.Linear(hidden_size, action_size)
        self.value_head = nn.Linear(hidden_size, 1)

    def forward(self, x):
        x = F.relu(self.fc1(x))
        return self.action_head(x), self.value_head(x).squeeze(-1)

    # ---------------------------------------------------------- rollout --
    @staticmethod
    def rollout_inputs(eng) -> torch.Tensor:
        """The lanes' 64-byte records (int8 board + mover + legal count): the
        rollout stores these instead of fp32 observations."""
        return eng.records()

    # ---------------------------------------------------- HIP fast path --
    @torch.no_grad()
    def pack(self, inplace: bool = False) -> torch.Tensor:
        """Pack the weights into the MFMA operand layout of bgx_policy_act (call
        after every optimizer step).  `inplace`: rewrite the previous pack's buffer
        (its address is baked into captured HIP graphs of act)."""
        L = _lib.load()
        H, A = self.fc1.out_features, self.action_head.out_features
        n = L.bgx_policy_packed_size(H, A)
        if n < 0:
            raise ValueError(f"unsupported policy shape H={H} A={A}")
        dev = self.fc1.weight.device
        ps = [t.detach().float().contiguous() for t in (self.fc1.weight, self.fc1.bias, self.action_head.weight,
                                                         self.action_head.bias, self.value_head.weight,
                                                         self.value_head.bias)]
        prev = getattr(self, "_packed", None)
        if inplace and prev is not None and prev.numel() == n and prev.device == dev:
            out = prev
        else:
            out = torch.empty(n, dtype=torch.float32, device=dev)
        s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        check(L.bgx_policy_pack(*[_ptr(t) for t in ps], H, A, _ptr(out), s), "bgx_policy_pack")
        self._packed = out
        return out

    @torch.no_grad()
    def act(self, records: torch.Tensor, seed: int = 0, step: int = 0, greedy: bool = False,
            packed: torch.Tensor | None = None, want_logits: bool = False, out=None,
            records_out: torch.Tensor | None = None, step_ctr: torch.Tensor | None = None):
        """select_action (ppo_agent.py:138-191) for every lane in ONE fused HIP
        kernel (encode -> MLP on MFMA -> masked softmax -> sample).  Returns
        (action int32[B], log_prob f32[B], value f32[B][, logits]); `out` =
        (action, log_prob, value) tensors to write instead (e.g. rows of a
        device-resident rollout buffer).  `records` may be a bgx.Engine: its
        lane records are read in place; `records_out` (uint8[B, 64]) then
        receives the kernel's copy of them (the rollout's stored state).
        `step_ctr` (int32[1] on the device): the noise's step is step + step_ctr[0]
        read when the kernel runs, so a captured HIP graph replays with fresh draws
        (advance it with `advance_counter`)."""
        L = _lib.load()
        packed = packed if packed is not None else getattr(self, "_packed", None)
        if packed is None:
            packed = self.pack()
        H, A = self.fc1.out_features, self.action_head.out_features
        if isinstance(records, torch.Tensor):
            # the kernel reads 64 bytes per row with 16-byte loads: anything else would read
            # past the allocation or decode garbage
            if (records.dtype not in (torch.uint8, torch.int8) or records.dim() != 2 or records.shape[1] != 64
                    or records.device.type != "cuda"):
                raise ValueError(f"act: records must be a uint8/int8 [n, 64] tensor on the GPU, got "
                                 f"{records.dtype} {tuple(records.shape)} on {records.device}")
            if records.device != packed.device:
                raise ValueError("act: records and the packed weights are on different devices")
            r = records.contiguous()
            rptr, n, dev = r.data_ptr(), r.shape[0], r.device
        else:                                              # a bgx.Engine: lane records in place
            rptr, n, dev = records.lanes_ptr(), records.batch, records.device
        if records_out is not None and (records_out.dtype != torch.uint8 or records_out.device != dev
                                        or not records_out.is_contiguous() or records_out.numel() != n * 64):
            raise ValueError("act: records_out must be a contiguous uint8[n, 64] tensor on the records' device")
        if out is not None:
            act, logp, val = out
            for t, dt in zip(out, (torch.int32, torch.float32, torch.float32)):
                if t.dtype != dt or t.device != dev or not t.is_contiguous() or t.numel() != n:
                    raise ValueError("act: out tensors must be contiguous int32/f32/f32 [n] on the records' device")
        else:
            act = torch.empty(n, dtype=torch.int32, device=dev)
            logp = torch.empty(n, dtype=torch.float32, device=dev)
            val = torch.empty(n, dtype=torch.float32, device=dev)
        logits = torch.empty(n, 32 * ((A + 32) // 32), dtype=torch.float32, device=dev) if want_logits else None
        s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        if step_ctr is not None and (step_ctr.dtype != torch.int32 or step_ctr.device != dev or step_ctr.numel() != 1):
            raise ValueError("act: step_ctr must be an int32[1] tensor on the records' device")
        check(L.bgx_policy_act_ctr(ctypes.c_void_p(rptr), n, _ptr(packed), H, A, int(seed) & (2**64 - 1),
                                   int(step) & 0xFFFFFFFF, _ptr(step_ctr), int(bool(greedy)), _ptr(act), _ptr(logp),
                                   _ptr(val), _ptr(logits), _ptr(records_out), s),
              "bgx_policy_act_ctr")
        if want_logits:
            return act, logp, val, logits
        return act, logp, val

    @staticmethod
    def advance_counter(step_ctr: torch.Tensor, v: int):
        """step_ctr[0] += v on the current stream (bgx_counter_add; graph-capturable)."""
        L = _lib.load()
        s = ctypes.c_void_p(torch.cuda.current_stream(step_ctr.device).cuda_stream)
        check(L.bgx_counter_add(_ptr(step_ctr), int(v) & 0xFFFFFFFF, s), "bgx_counter_add")

    @torch.no_grad()
    def act_torch(self, records: torch.Tensor, generator=None):
        """Same step composed from torch ops on encoded features (a slower
        reference composition used by tests)."""
        B = records.shape[0]
        boards = records[:, :52].contiguous()
        cur = records[:, 52].contiguous()
        counts = records[:, 60].to(torch.int32) | (records[:, 61].to(torch.int32) << 8)
        x = encode(boards, cur)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits, value = self(x)
        logits = logits.float()
        A = logits.shape[1]
        legal = torch.arange(A, device=logits.device)[None, :] < counts[:, None]
        masked = torch.where(legal, logits, logits + MASK_LOG)
        logp_all = torch.log_softmax(masked, dim=-1)
        act = torch.multinomial(logp_all.exp(), 1, generator=generator).squeeze(1)
        logp = logp_all.gather(1, act[:, None]).squeeze(1)
        return act.to(torch.int32), logp, value.float()


def masked_probs(logits: torch.Tensor, masks: torch.Tensor) -> torch.Tensor:
    """softmax(logits + log(mask + 1e-45)) exactly as ppo_agent.py:166-167."""
    return torch.softmax(logits + (masks + 1e-45).log(), dim=-1)


__all__ = ["PolicyNet", "masked_probs", "MASK_LOG", "math"]
