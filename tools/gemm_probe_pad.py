"""Probe the PPO update's per-chunk GEMMs at 2^20 rows with the feature width
K = 198 (396-byte rows, not 16-byte aligned) against K padded to 200 / 208
(zero columns: identical results), plus the 512-wide head GEMMs, to see which
shapes hipBLASLt runs far below their HBM/MFMA bounds."""
import torch
torch.manual_seed(0)
M = 1 << 20
dev = "cuda"


def t(f, n=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


H = 128
b1 = torch.randn(H, device=dev, dtype=torch.half)
for K in (198, 200, 208, 256):
    x = torch.randn(M, K, device=dev, dtype=torch.half)
    W1 = torch.randn(H, K, device=dev, dtype=torch.half)
    dh = torch.randn(M, H, device=dev, dtype=torch.half)
    S = 64
    fwd = t(lambda: torch._addmm_activation(b1, x, W1.t()))
    wg = t(lambda: torch.bmm(dh.view(S, M // S, H).transpose(1, 2), x.view(S, M // S, K),
                             out_dtype=torch.float32).sum(0))
    print(f"K={K}: fc1 fwd (bias+relu) {fwd:7.1f} us   gW1 split-64 {wg:7.1f} us")
h = torch.randn(M, H, device=dev, dtype=torch.half)
W2 = torch.randn(512, H, device=dev, dtype=torch.half)
b2 = torch.randn(512, device=dev, dtype=torch.half)
dy = torch.randn(M, 512, device=dev, dtype=torch.half)
print(f"head fwd F.linear {t(lambda: torch.nn.functional.linear(h, W2, b2)):7.1f} us")
print(f"head fwd addmm    {t(lambda: torch.addmm(b2, h, W2.t())):7.1f} us")
print(f"dh = dy @ W2      {t(lambda: dy @ W2):7.1f} us")
for S in (32, 64, 128):
    print(f"gW2 split-{S}     {t(lambda: torch.bmm(dy.view(S, M // S, 512).transpose(1, 2), h.view(S, M // S, H), out_dtype=torch.float32).sum(0)):7.1f} us")
