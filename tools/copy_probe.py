"""Device -> pinned host copy bandwidth on the box: bgx_copy_regions (kernel stores
across PCIe) at several workgroup counts, against torch's copy_ (the runtime's own
path), for a 5.3 MB rollout slot pair and a 64 MB block."""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mlp-ppo-2ply-p3_amd"))
from bgx import _lib  # noqa: E402
from bgx.hostcopy import host_device_ptr  # noqa: E402

L = _lib.load()
for nbytes in (5308416, 64 << 20):
    src = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda")
    dst = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    dptr = host_device_ptr(dst)
    s = torch.cuda.current_stream()

    def kcopy(wg):
        reg = (_lib.BgxRegion * 1)(_lib.BgxRegion(src.data_ptr(), dptr, nbytes, 1, nbytes, nbytes))
        assert L.bgx_copy_regions(ctypes.cast(reg, ctypes.c_void_p), 1, wg, ctypes.c_void_p(s.cuda_stream)) == 0

    def run(fn, n=20):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return nbytes * n / (time.perf_counter() - t0) / 1e9
    for wg in (16, 64, 256, 1024):
        print(f"{nbytes / 1e6:7.1f} MB  bgx_copy_regions wg={wg:5d}: {run(lambda: kcopy(wg)):6.1f} GB/s")
    print(f"{nbytes / 1e6:7.1f} MB  torch copy_ non_blocking  : {run(lambda: dst.copy_(src, non_blocking=True)):6.1f} GB/s")
    assert torch.equal(dst, src.cpu())
