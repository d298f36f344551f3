"""Is the C3 rollout step host-bound?  Enqueue time of K steps (2 shards, the
bench's launch sequence without timing events) vs the time until the GPU is done."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mlp-ppo-2ply-p3_amd"))
import bgx  # noqa: E402
from bgx.policy import PolicyNet  # noqa: E402

dev = torch.device("cuda", 0)
S, B, K, ring = 2, 65536, 400, 32
Bs = B // S
engs = [bgx.Engine(batch=Bs, max_moves=500, seed=1234 + 104729 * k, dice="philox", auto_reset=True, device=dev)
        for k in range(S)]
for e in engs:
    e.reset(want_obs=True)
torch.manual_seed(0)
net = PolicyNet(hidden_size=128, action_size=500).to(dev)
net.pack()
streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
bufs = [{"records": torch.empty(ring, Bs, 64, dtype=torch.uint8, device=dev),
         "act": torch.empty(ring, Bs, dtype=torch.int32, device=dev),
         "logp": torch.empty(ring, Bs, dtype=torch.float32, device=dev),
         "value": torch.empty(ring, Bs, dtype=torch.float32, device=dev),
         "reward": torch.empty(ring, Bs, dtype=torch.float32, device=dev),
         "done": torch.empty(ring, Bs, dtype=torch.uint8, device=dev)} for _ in range(S)]


def step(i):
    for k in range(S):
        e, st, b, slot = engs[k], streams[k], bufs[k], i % ring
        with torch.cuda.stream(st):
            net.act(e, seed=4242 + k, step=i, out=(b["act"][slot], b["logp"][slot], b["value"][slot]),
                    records_out=b["records"][slot])
            e.step(b["act"][slot], want_obs=False, want_info=False, out=(b["reward"][slot], b["done"][slot]))


for i in range(100):
    step(i)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    for i in range(K):
        step(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"enqueue {1e6 * (t1 - t0) / K:.1f} us/step, total {1e6 * (t2 - t0) / K:.1f} us/step "
          f"-> {B * K / (t2 - t0) / 1e6:.1f} M env steps/s")
# host cost split: policy act vs engine step (enqueue only)
for name, fn in (("act", lambda i: net.act(engs[0], seed=1, step=i, out=(bufs[0]["act"][0], bufs[0]["logp"][0],
                                                                         bufs[0]["value"][0]))),
                 ("step", lambda i: engs[0].step(bufs[0]["act"][0], want_obs=False, want_info=False,
                                                 out=(bufs[0]["reward"][0], bufs[0]["done"][0])))):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(200):
        fn(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"{name}: enqueue {1e6 * (t1 - t0) / 200:.1f} us/call")
