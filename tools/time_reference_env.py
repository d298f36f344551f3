"""Time the REFERENCE Python env (build container only: /root/reference is never
shipped) and the C port beside it on the same host, as the bridge ratio that
bench.py's cpu_baseline.reference_python reports.

  python tools/time_reference_env.py [--procs 8] [--seconds 30]

Each process: BackgammonEnv (environment/backgammon_env.py) seeded with its index,
torch.set_num_threads(1), a random legal policy, auto-reset on done.  The port
(oracle/bgoracle.c via oracle.py) runs the same loop.  Writes
profiles/cpu_reference_timing.json."""
import argparse
import json
import multiprocessing as mp
import os
import platform
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def _import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    m = types.ModuleType("src")
    m.__path__ = [REF + "/src"]
    sys.modules["src"] = m
    gym = types.ModuleType("gym")
    sp = types.ModuleType("gym.spaces")
    gym.Env = type("Env", (), {"close": lambda self: None})
    sp.Box = lambda low, high, shape, dtype: types.SimpleNamespace(shape=shape)
    sp.Discrete = lambda n: types.SimpleNamespace(n=n)
    gym.spaces = sp
    sys.modules.update({"gym": gym, "gym.spaces": sp})
    import src.moves  # noqa: F401  (before src.board: circular import)
    from src.environment.backgammon_env import BackgammonEnv
    return BackgammonEnv


def _ref_worker(k, seconds, q):
    import numpy as np
    import torch
    torch.set_num_threads(1)
    BackgammonEnv = _import_reference()
    env = BackgammonEnv()
    env.seed(k)
    env.reset()
    rng = np.random.RandomState(1000 + k)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        n = int(env.action_mask.sum().item())
        _, _, done, _ = env.step(int(rng.randint(n)) if n else 0)
        steps += 1
        if done:
            env.reset()
    q.put(steps / (time.perf_counter() - t0))


def _port_worker(k, seconds, q):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from port_bench import run
    q.put(run(seconds, k)[0])


def timed(worker, procs, seconds):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(k, seconds, q)) for k in range(procs)]
    for p in ps:
        p.start()
    rates = [q.get(timeout=seconds * 4 + 120) for _ in ps]
    for p in ps:
        p.join()
    return sum(rates)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--seconds", type=float, default=30.0)
    a = ap.parse_args()
    ref = timed(_ref_worker, a.procs, a.seconds)
    port = timed(_port_worker, a.procs, a.seconds / 3)
    out = {"reference_env_steps_per_s": ref, "port_env_steps_per_s": port, "port_over_reference": port / ref,
           "processes": a.procs, "seconds_reference": a.seconds, "seconds_port": a.seconds / 3,
           "host_cpus": os.cpu_count(), "host": platform.processor() or platform.machine(),
           "policy": "random legal, auto-reset on done, one env per process, torch.set_num_threads(1)",
           "script": "tools/time_reference_env.py (build container; the reference never travels)"}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "cpu_reference_timing.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))
