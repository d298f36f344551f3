"""C5 rehearsal short of an 8-GPU node: 2 ranks (torch.distributed.run, gloo,
both on the one GPU) run PPOTrainer.iteration() on their own game shards; the
workers (tests/_c5_worker.py) check weights identical on both ranks after the
update, the global return normalisation against the concatenated single-process
formula, and the distributed epoch against one single-process epoch over the
concatenated batch."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_trainer_iteration(tmp_path):
    out = str(tmp_path / "c5")
    env = dict(os.environ, BGX_DIST_BACKEND="gloo", C5_OUT=out, OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "tests", "_c5_worker.py")]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    res = [json.load(open(f"{out}.{k}.json")) for k in range(2)]
    for x in res:
        assert x["world_size"] == 2
        assert x["init_identical"] and x["final_identical"] and x["weights_moved"] and x["losses_finite"]
        assert x["norm_max_abs_err"] < 1e-6
    assert res[0]["epoch_rel_err"] < 1e-4, res[0]
