"""Probe hipBLASLt shapes of the PPO update's GEMMs at 1M rows (weight
gradients are K = 1M reductions): plain vs manual split-K (bmm + sum)."""
import torch
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


for N, K in ((500, 128), (128, 198)):
    G = torch.randn(M, N, device="cuda", dtype=torch.half)
    H = torch.randn(M, K, device="cuda", dtype=torch.half)
    ref = (G.float().t() @ H.float())
    print(N, K, "plain G^T H %.3f ms" % t(lambda: G.t() @ H), " H^T G %.3f" % t(lambda: H.t() @ G))
    for S in (8, 16, 32, 64, 128):
        f = lambda: torch.bmm(G.view(S, M // S, N).transpose(1, 2), H.view(S, M // S, K)).float().sum(0)
        f32 = lambda: torch.baddbmm(torch.empty(0, device="cuda"), G.view(S, M // S, N).transpose(1, 2),
                                    H.view(S, M // S, K)).sum(0) if False else None
        err = (f() - ref).abs().max().item() / ref.abs().max().item()
        print("  split %3d: %.3f ms  rel err %.2e" % (S, t(f), err))
