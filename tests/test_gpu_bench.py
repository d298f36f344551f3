"""bench.py's N-rank path on the one-GPU box: `python bench.py --gpus 2` starts
two ranks itself (torch.distributed.run child; BGX_DIST_BACKEND=gloo so both
share GPU 0) and rank 0 prints the line.  Checks n_gpus, the value as the sum
over ranks over the max-over-ranks time, the PPO iteration over both ranks with
identical weights after the all-reduced update, and the host_mirror leg.
RCCL itself (backend nccl, one rank per GPU) runs only on a multi-GPU node."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo():
    env = dict(os.environ, BGX_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "5", "--warmup", "2",
           "--burn-in", "5", "--batch", "8192", "--two-ply-batches", "1", "--c2-steps", "4", "--horizon", "4",
           "--mirror-steps", "4", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]           # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["dist_backend"] == "gloo"
    pr = line["per_rank"]
    assert [p["rank"] for p in pr] == [0, 1]
    assert all(p["env_steps"] == 8192 * 5 for p in pr)
    el = max(p["seconds"] for p in pr)
    assert line["value"] == pytest.approx(sum(p["env_steps"] for p in pr) / el, rel=1e-9)
    assert line["config"]["global_batch"] == 2 * 8192
    ppo = line["ppo_iteration"]
    assert ppo["ranks"] == 2 and ppo["weights_identical_across_ranks"] is True
    assert all(v == v for v in ppo["losses_last"].values())
    assert line["host_mirror"]["env_steps_per_s"] > 0
    assert line["two_ply"]["root_decisions_per_s"] > 0 and line["one_ply_selfplay"]["env_steps_per_s"] > 0
