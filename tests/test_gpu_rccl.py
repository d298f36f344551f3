"""The RCCL path and the HIP-graph capture failure path, on the one-GPU box.

* `bench.py` under a ONE-rank "nccl" process group (BGX_DIST_FORCE=1): RCCL's
  communicator init (device_id: eager, so its watchdog thread is alive), the
  barrier / all-reduce / all-gather of the timing and the weight check, the PPO
  gradient all-reduce (bgx.ppo.allreduce_mean_ runs whenever a group exists) and
  every HIP-graph capture (C2, C3, the trainer's rollout) beside the watchdog.
  The driver's multi-GPU runs (`bench.py --gpus N`) go through this same code
  with N ranks.
* A capture that fails is terminal (bgx/graphs.py): BGX_INJECT_CAPTURE_FAILURE
  makes the capture at one site fail for real (a stream synchronize inside it);
  the process must print the error and exit with status 3 -- no eager
  continuation over engine host state that advanced through steps that never
  ran, and no SIGSEGV in teardown (round 3's gpurun_out/r3h)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "4", "--warmup", "2", "--burn-in", "4", "--batch", "8192", "--no-cpu-baseline"]


def _bench(extra, env_extra, timeout=300):
    env = dict(os.environ, OMP_NUM_THREADS="4", **env_extra)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + SMALL + extra, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_one_rank_rccl_with_graphs():
    r = _bench(["--two-ply-batches", "1", "--c2-steps", "4", "--horizon", "4", "--mirror-steps", "4"],
               {"BGX_DIST_FORCE": "1", "BGX_DIST_BACKEND": "nccl"})
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["dist_backend"] == "nccl"
    assert line["config"]["hip_graph"] is not None                 # C3 replayed from graphs
    assert line["one_ply_selfplay"]["hip_graph"] is True           # C2 too
    ppo = line["ppo_iteration"]                                    # trainer graphs + RCCL all-reduce
    assert ppo["weights_identical_across_ranks"] is True and "nccl" in ppo["collective"]
    assert all(v == v for v in ppo["losses_last"].values())
    assert line["per_rank"][0]["env_steps"] == 8192 * 4


@pytest.mark.parametrize("site,extra", [
    ("c3", ["--two-ply-batches", "0", "--c2-steps", "0", "--horizon", "0", "--mirror-steps", "0"]),
    ("trainer", ["--no-graphs", "--two-ply-batches", "0", "--c2-steps", "0", "--horizon", "4", "--mirror-steps", "0"]),
])
def test_capture_failure_is_terminal(site, extra):
    r = _bench(extra, {"BGX_INJECT_CAPTURE_FAILURE": site}, timeout=240)
    assert r.returncode == 3, (r.returncode, r.stderr[-3000:])
    assert f"HIP graph capture failed at {site}" in r.stderr, r.stderr[-3000:]
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
