"""Why does a 20-step C3 window run slower than a 1,000-step one?  The bench's C3
setup (2 shards on 2 streams, 2-step HIP graphs per shard); timed like bench.py
(synchronize, host clock, K steps, synchronize), repeated:
  aligned-20    both shards start the window together (as after bench.py's barrier)
  free-1000     one long window
  shifted-20    shard 1 starts each window after shard 0's first graph has run half
                way (an event recorded after shard 0's first policy kernel)
Prints ms/step per mode."""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mlp-ppo-2ply-p3_amd"))
import bgx  # noqa: E402
from bgx.graphs import capture  # noqa: E402
from bgx.policy import PolicyNet  # noqa: E402

dev = torch.device("cuda", 0)
S, B, ring, G = 2, 65536, 32, 2
Bs = B // S
engs = [bgx.Engine(batch=Bs, max_moves=500, seed=1234 + 104729 * k, dice="philox", auto_reset=True, device=dev)
        for k in range(S)]
for e in engs:
    e.reset(want_obs=False)
torch.manual_seed(0)
net = PolicyNet(hidden_size=128, action_size=500).to(dev)
net.pack()
streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
kw = dict(device=dev)
bufs = [{"records": torch.empty(ring, Bs, 64, dtype=torch.uint8, **kw),
         "act": torch.empty(ring, Bs, dtype=torch.int32, **kw), "logp": torch.empty(ring, Bs, **kw),
         "value": torch.empty(ring, Bs, **kw), "reward": torch.empty(ring, Bs, **kw),
         "done": torch.empty(ring, Bs, dtype=torch.uint8, **kw)} for _ in range(S)]
ctrs = [torch.zeros(1, dtype=torch.int32, **kw) for _ in range(S)]
for i in range(150):
    for k in range(S):
        with torch.cuda.stream(streams[k]):
            b = bufs[k]
            net.act(engs[k], seed=4242 + k, step=i, out=(b["act"][0], b["logp"][0], b["value"][0]))
            engs[k].step(b["act"][0], want_obs=False, want_info=False, out=(b["reward"][0], b["done"][0]))
for k in range(S):
    with torch.cuda.stream(streams[k]):
        engs[k].join()
torch.cuda.synchronize()
caps = [torch.cuda.Stream(dev) for _ in range(S)]


def body(k, g0):
    e, b = engs[k], bufs[k]
    for i in range(g0, g0 + G):
        net.act(e, seed=4242 + k, step=i, step_ctr=ctrs[k], out=(b["act"][i], b["logp"][i], b["value"][i]),
                records_out=b["records"][i])
        e.step(b["act"][i], want_obs=False, want_info=False, out=(b["reward"][i], b["done"][i]))
    e.join()
    PolicyNet.advance_counter(ctrs[k], ring)


graphs = [[capture("probe", lambda k=k, g0=g0: body(k, g0), caps[k]) for k in range(S)] for g0 in range(0, ring, G)]
torch.cuda.synchronize()
r = [0]


gpu_ms, enq_ms = {}, {}


def window(steps, shift=False, tag=None):
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(S)]
    for k in range(S):
        ev[k][0].record(streams[k])
    t0 = time.perf_counter()
    for j in range(steps // G):
        row = graphs[r[0] % len(graphs)]
        r[0] += 1
        with torch.cuda.stream(streams[0]):
            row[0].replay()
        if shift and j == 0:
            sev = torch.cuda.Event()
            sev.record(streams[0])
            streams[1].wait_event(sev)
        with torch.cuda.stream(streams[1]):
            row[1].replay()
    t1 = time.perf_counter()
    for k in range(S):
        ev[k][1].record(streams[k])
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) * 1e3 / steps
    if tag:
        g = max(ev[k][0].elapsed_time(ev[k2][1]) for k in range(S) for k2 in range(S))
        gpu_ms.setdefault(tag, []).append(g / steps)
        enq_ms.setdefault(tag, []).append((t1 - t0) * 1e3 / steps)
    return el


for _ in range(3):
    window(20)
res = {}
for rep in range(3):
    for mode, steps, sh in (("aligned-20", 20, False), ("shifted-20", 20, True), ("aligned-100", 100, False),
                            ("free-1000", 1000, False)):
        res.setdefault(mode, []).append(window(steps, sh, mode) if mode != "aligned-20" else
                                        statistics.median(window(20, tag=mode) for _ in range(10)))
for m, v in res.items():
    print(f"{m:12s} ms/step {statistics.median(v):.4f}  ({', '.join(f'{x:.4f}' for x in v)})  "
          f"GPU events {statistics.median(gpu_ms[m]):.4f}  host enqueue {statistics.median(enq_ms[m]):.4f}")
