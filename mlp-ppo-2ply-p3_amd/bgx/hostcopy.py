"""Rollout rows mirrored into pinned host memory (the reference keeps its rollout
memory on the host, agent/ppo_agent.py:175-187).

`HostMirror` pairs device rollout buffers [T, B, ...] with pinned host buffers of
the same layout and copies any slot range x lane range of EVERY field with one
kernel launch (bgx_copy_regions: one strided 2-D region per field), so a HIP graph
of rollout steps carries the copy of its slots as a single node on a forked
stream.  Round 3 copied each field of each step with torch's copy_, i.e. six
runtime copies per step that ROCm ran as blit kernels (`__amd_rocclr_copyBuffer`)
on the compute queue, outside any graph.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import check


def host_device_ptr(t: torch.Tensor) -> int:
    """Device address of a pinned host tensor's storage (bgx_host_device_ptr)."""
    if t.device.type != "cpu" or not t.is_pinned():
        raise ValueError("host_device_ptr: needs a pinned host tensor")
    out = ctypes.c_void_p()
    check(_lib.load().bgx_host_device_ptr(ctypes.c_void_p(t.data_ptr()), ctypes.byref(out)), "bgx_host_device_ptr")
    return int(out.value)


class HostMirror:
    def __init__(self, dev_bufs: dict):
        if len(dev_bufs) > _lib.MAX_COPY_REGIONS:
            raise ValueError(f"HostMirror: at most {_lib.MAX_COPY_REGIONS} fields")
        shapes = {tuple(v.shape[:2]) for v in dev_bufs.values()}
        if len(shapes) != 1:
            raise ValueError("HostMirror: every field must be [T, B, ...] with the same T, B")
        self.T, self.B = shapes.pop()
        for k, v in dev_bufs.items():
            # bgx_copy_regions moves 16-byte chunks: every lane range's bytes must be a
            # multiple of 16 (uint8 fields: B a multiple of 16)
            row = (v[0, 0].numel() if v.dim() > 2 else 1) * v.element_size()
            if (self.B * row) % 16 or v.data_ptr() % 16:
                raise ValueError(f"HostMirror: field {k!r} has {self.B * row} bytes per slot; the pinned-host "
                                 f"copy needs a multiple of 16 (batch a multiple of 16)")
        self.dev = dev_bufs
        self.host = {k: torch.empty(v.shape, dtype=v.dtype).pin_memory() for k, v in dev_bufs.items()}
        self._hptr = {k: host_device_ptr(t) for k, t in self.host.items()}
        self._lib = _lib.load()

    def copy(self, t0: int, nslots: int, lo: int = 0, hi: int | None = None, stream=None):
        """Slots [t0, t0 + nslots) x lanes [lo, hi) of every field to the host
        buffers, one launch on `stream` (default: the current stream)."""
        hi = self.B if hi is None else hi
        if not (0 <= t0 and t0 + nslots <= self.T and 0 <= lo < hi <= self.B):
            raise ValueError("HostMirror.copy: slot or lane range out of bounds")
        regs = (_lib.BgxRegion * len(self.dev))()
        for i, (k, v) in enumerate(self.dev.items()):
            row = v[0, 0].numel() * v.element_size()           # bytes per lane
            off = (t0 * self.B + lo) * row
            regs[i] = _lib.BgxRegion(v.data_ptr() + off, self._hptr[k] + off, (hi - lo) * row, nslots,
                                     self.B * row, self.B * row)
        dev = next(iter(self.dev.values())).device
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        check(self._lib.bgx_copy_regions(ctypes.cast(regs, ctypes.c_void_p), len(self.dev), 0,
                                         ctypes.c_void_p(s.cuda_stream)), "bgx_copy_regions")
