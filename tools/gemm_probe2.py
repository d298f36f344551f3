"""Forward / backward GEMM shapes of the fp16 PPO epoch at 2^20 rows with padded K:
F.linear(x [M,K], W [128,K]) (+ fused relu via _addmm_activation), dy @ W2 (K = 512),
and the split-K weight gradient of fc1 (dh^T x) per K."""
import torch
import torch.nn.functional as F
torch.manual_seed(0)
M = 1 << 20


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
    return e0.elapsed_time(e1) / n


for K in (198, 200, 208, 224, 256):
    x = torch.randn(M, K, device="cuda", dtype=torch.half)
    W = torch.randn(128, K, device="cuda", dtype=torch.half)
    b = torch.randn(128, device="cuda", dtype=torch.half)
    dh = torch.randn(M, 128, device="cuda", dtype=torch.half)
    lin = t(lambda: F.linear(x, W, b))
    linr = t(lambda: torch.relu(F.linear(x, W, b)))
    fused = t(lambda: torch._addmm_activation(b, x, W.t()))
    wg = t(lambda: torch.bmm(dh.view(64, M // 64, 128).transpose(1, 2), x.view(64, M // 64, K),
                             out_dtype=torch.float32).sum(0))
    print(f"K={K}: linear {lin:.3f} ms  linear+relu {linr:.3f}  addmm_activation {fused:.3f}  wgrad {wg:.3f}", flush=True)
h = torch.randn(M, 128, device="cuda", dtype=torch.half)
for N in (512, 504):
    W2 = torch.randn(N, 128, device="cuda", dtype=torch.half)
    b2 = torch.randn(N, device="cuda", dtype=torch.half)
    dy = torch.randn(M, N, device="cuda", dtype=torch.half)
    print(f"N={N}: y = linear(h) {t(lambda: F.linear(h, W2, b2)):.3f} ms  dh = dy @ W2 {t(lambda: dy @ W2):.3f}  "
          f"wgrad {t(lambda: torch.bmm(dy.view(64, M // 64, N).transpose(1, 2), h.view(64, M // 64, 128), out_dtype=torch.float32).sum(0)):.3f}",
          flush=True)
    for S in (16, 32, 128):
        print(f"   wgrad split {S}: {t(lambda: torch.bmm(dy.view(S, M // S, N).transpose(1, 2), h.view(S, M // S, 128), out_dtype=torch.float32).sum(0)):.3f}")
