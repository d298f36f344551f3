"""Timing loop of the C port (oracle/bgoracle.c) for the CPU baseline: a random
legal policy stepping one BackgammonEnv with auto-reset.  Test / baseline
infrastructure only (bench.py's cpu_baseline leg, tools/time_reference_env.py)."""
import time

import numpy as np

import oracle as O


def run(seconds: float, seed: int = 0):
    """Returns (env steps/s, steps) of one process running for ~`seconds`."""
    O.build()
    env = O.Env(seed=seed)
    env.reset()
    rng = np.random.RandomState(seed)
    steps = 0
    t0 = time.perf_counter()
    while True:
        for _ in range(200):
            n = int(env.state()[1][3])
            _, _, done, _ = env.step(rng.randint(n) if n else 0)
            if done:
                env.reset()
            steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return steps / el, steps


def _worker(args):
    seconds, seed = args
    return run(seconds, seed)


def run_parallel(seconds: float, procs: int):
    """`procs` spawned processes, one env each: (summed env steps/s, total steps)."""
    import multiprocessing as mp
    with mp.get_context("spawn").Pool(procs) as pool:
        res = pool.map(_worker, [(seconds, k) for k in range(procs)])
        # let the workers exit on their own: leaving the with-block while they are
        # alive terminates them with SIGTERM (abort dumps under rocprofv3)
        pool.close()
        pool.join()
    return sum(r[0] for r in res), sum(r[1] for r in res)
