"""A/B of PPO iteration variants in one process (experiments): for each variant (a
comma-separated list of bgx.train module attributes set to 0/1), a fresh PPOTrainer
(B = 65,536, T = 32) runs 1 warm + N timed iterations; prints the mean rollout / update
seconds and env steps/s.  Variants alternate over ROUNDS rounds.

    python tools/ppo_ab.py "PPO_GW1_SIDE=0" "PPO_GW1_SIDE=1"
"""
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mlp-ppo-2ply-p3_amd")]
import bgx.train as T  # noqa: E402


def run(spec, n):
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=")
        setattr(T, k, type(getattr(T, k))(int(v)))
    tr = T.PPOTrainer(batch=65536, horizon=32, seed=11)
    tr.iteration()
    torch.cuda.synchronize()
    ms, t0 = [], time.perf_counter()
    for _ in range(n):
        ms.append(tr.iteration())
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"variant": spec, "steps_per_s_M": round(65536 * 32 * n / el / 1e6, 1),
            "rollout_ms": round(1e3 * statistics.mean(m["rollout_s"] for m in ms), 3),
            "update_ms": round(1e3 * statistics.mean(m["update_s"] for m in ms), 3),
            "loss": round(ms[-1]["total_loss"], 6)}


def main():
    n = int(os.environ.get("N", "6"))
    for r in range(int(os.environ.get("ROUNDS", "2"))):
        for spec in sys.argv[1:]:
            print(json.dumps(dict(run(spec, n), round=r)), flush=True)


if __name__ == "__main__":
    main()
