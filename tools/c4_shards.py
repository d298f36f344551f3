"""C4 as game shards: 2-ply root decisions/s for B = 65,536 roots as one engine, against
S engines of B/S roots each driven by its own host thread on its own stream (a
bgx_two_ply call synchronises its stream twice -- the row count after the scan and
the pool counters after the evaluation -- so one host thread would serialise the
shards; ctypes drops the GIL inside the call).  One shard's enumeration can then run
beside another's evaluation.

    python tools/c4_shards.py [--shards 2] [--batches 3] [--hidden 40]
"""
import argparse
import json
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mlp-ppo-2ply-p3_amd"))
import bgx  # noqa: E402
from bgx.policy import PolicyNet  # noqa: E402
from bgx.search import ValueHead, two_ply  # noqa: E402


def population(n, seed, dev, steps, net):
    e = bgx.Engine(batch=n, max_moves=500, seed=seed, dice="philox", auto_reset=True, device=dev)
    e.reset(want_obs=False)
    e.set_fork(False)
    for i in range(steps):
        a, _, _ = net.act(e, seed=5, step=i)
        e.step(a, want_obs=False, want_info=False)
    return e


def run(engs, vh, batches, dev):
    streams = [torch.cuda.Stream(dev) for _ in engs]
    for s in streams:               # the populations were stepped on the current stream
        s.wait_stream(torch.cuda.current_stream(dev))
    for e, s in zip(engs, streams):                  # warm: workspace sizing, code load
        with torch.cuda.stream(s):
            two_ply(e, vh)
    torch.cuda.synchronize(dev)
    leaves = [0] * len(engs)

    def worker(k):
        torch.cuda.set_device(dev)
        with torch.cuda.stream(streams[k]):
            for _ in range(batches):
                _, _, _, st = two_ply(engs[k], vh)
                leaves[k] += st["leaves"]
    t0 = time.perf_counter()
    if len(engs) == 1:
        worker(0)
    else:
        th = [threading.Thread(target=worker, args=(k,)) for k in range(len(engs))]
        for t in th:
            t.start()
        for t in th:
            t.join()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    roots = sum(e.batch for e in engs) * batches
    return {"shards": len(engs), "roots_per_s": roots / el, "seconds": el, "leaves": sum(leaves)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--shards", default="2", help="comma-separated shard counts")
    ap.add_argument("--batches", type=int, default=3)
    ap.add_argument("--hidden", type=int, default=40)
    ap.add_argument("--age", type=int, default=180)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = PolicyNet(hidden_size=128, action_size=500).to(dev)
    net.pack()
    torch.manual_seed(1)
    vh = ValueHead(PolicyNet(hidden_size=a.hidden).to(dev))
    out = []
    one = [population(a.batch, 77, dev, a.age, net)]
    out.append(run(one, vh, a.batches, dev))
    del one
    torch.cuda.empty_cache()
    for S in [int(x) for x in a.shards.split(",")]:
        sh = [population(a.batch // S, 77 + 7919 * k, dev, a.age, net) for k in range(S)]
        out.append(run(sh, vh, a.batches, dev))
        del sh
        torch.cuda.empty_cache()
    print(json.dumps({"tool": "tools/c4_shards.py", "hidden": a.hidden, "runs": out}))


if __name__ == "__main__":
    main()
