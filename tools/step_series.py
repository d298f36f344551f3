"""C3 step time against game age: the bench's headline step (B = 65,536 games as
--shards shards on their own streams, linear env steps unless --fork, 2-step HIP
graphs per shard, policy + masked sampling + env.step + rollout rows to the HBM
ring) from a fresh reset to --steps steps, timed in windows of --window steps with
HIP events (the shards are joined
only at window boundaries, as bench.py's timed region is).  Separates the
population's game-age effect from box-to-box effects.

    python tools/step_series.py --steps 1200 --window 20 > gpurun_out/series.json
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mlp-ppo-2ply-p3_amd"))
import bgx  # noqa: E402
from bgx.graphs import capture  # noqa: E402
from bgx.policy import PolicyNet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1200)
    ap.add_argument("--window", type=int, default=20)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--shards", type=int, default=4)
    ap.add_argument("--fork", action="store_true", help="fork each step's light launch (bench.py --fork-steps)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    S, B, ring, G = args.shards, args.batch, 32, 2
    Bs = B // S
    engs = [bgx.Engine(batch=Bs, max_moves=500, seed=args.seed + 104729 * k, dice="philox", auto_reset=True,
                       device=dev) for k in range(S)]
    for e in engs:
        e.reset(want_obs=False)
        e.set_fork(args.fork)
    torch.manual_seed(0)
    net = PolicyNet(hidden_size=128, action_size=500).to(dev)
    net.pack()
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
    kw = dict(device=dev)
    bufs = [{"records": torch.empty(ring, Bs, 64, dtype=torch.uint8, **kw),
             "act": torch.empty(ring, Bs, dtype=torch.int32, **kw),
             "logp": torch.empty(ring, Bs, dtype=torch.float32, **kw),
             "value": torch.empty(ring, Bs, dtype=torch.float32, **kw),
             "reward": torch.empty(ring, Bs, dtype=torch.float32, **kw),
             "done": torch.empty(ring, Bs, dtype=torch.uint8, **kw)} for _ in range(S)]
    ctrs = [torch.zeros(1, dtype=torch.int32, **kw) for _ in range(S)]
    caps = [torch.cuda.Stream(dev) for _ in range(S)]
    for k in range(S):
        with torch.cuda.stream(streams[k]):
            engs[k].join()
    torch.cuda.synchronize(dev)

    def graph_steps(k, g0):
        e, b = engs[k], bufs[k]
        for i in range(g0, g0 + G):
            net.act(e, seed=4242 + k, step=i, step_ctr=ctrs[k], out=(b["act"][i], b["logp"][i], b["value"][i]),
                    records_out=b["records"][i])
            e.step(b["act"][i], want_obs=False, want_info=False, out=(b["reward"][i], b["done"][i]))
        e.join()
        PolicyNet.advance_counter(ctrs[k], ring)
    # the capture records launches only: the games are still at age 0 afterwards
    graphs = [[capture("series", lambda k=k, g0=g0: graph_steps(k, g0), caps[k]) for k in range(S)]
              for g0 in range(0, ring, G)]
    torch.cuda.synchronize(dev)
    out, r = [], 0
    for w0 in range(0, args.steps, args.window):
        for st in streams[1:]:
            streams[0].wait_stream(st)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(streams[0])
        for st in streams[1:]:
            st.wait_stream(streams[0])
        for _ in range(args.window // G):
            row = graphs[r % len(graphs)]
            r += 1
            for k in range(S):
                with torch.cuda.stream(streams[k]):
                    row[k].replay()
        for st in streams[1:]:
            streams[0].wait_stream(st)
        b.record(streams[0])
        out.append((w0, a, b))
        if len(out) % 10 == 0:
            torch.cuda.synchronize(dev)
            print(f"[series] {w0 + args.window} steps", file=sys.stderr, flush=True)
    torch.cuda.synchronize(dev)
    rows = [{"age": w0, "ms_per_step": a.elapsed_time(b) / args.window,
             "env_steps_per_s": B * args.window / (a.elapsed_time(b) * 1e-3)} for w0, a, b in out]
    print(json.dumps({"tool": "tools/step_series.py", "batch": B, "shards": S, "fork": args.fork, "window": args.window,
                      "steps": args.steps, "time": time.strftime("%Y-%m-%d %H:%M:%S"), "series": rows}))


if __name__ == "__main__":
    main()
