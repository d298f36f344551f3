"""bench.py's multi-GPU entry (CPU): `python bench.py --gpus N` with no
WORLD_SIZE starts N ranks under torch.distributed.run as a child process
before anything touches the GPU, and a rank refuses a --gpus / WORLD_SIZE
mismatch.  The launched ranks themselves run in tests/test_gpu_bench.py."""
import importlib.util
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_gpus_flag_launches_ranks(monkeypatch):
    b = _bench()
    seen = {}

    def fake_run(cmd, env=None, **kw):
        seen["cmd"], seen["env"] = cmd, env
        return subprocess.CompletedProcess(cmd, 0)

    monkeypatch.setattr(b.subprocess, "run", fake_run)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "20", "--warmup", "3"])
    with pytest.raises(SystemExit) as ex:
        b.main()
    assert ex.value.code == 0
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "20", "--warmup", "3"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert not torch.cuda.is_initialized()            # the parent never touched the GPU


def test_rank_refuses_world_size_mismatch(monkeypatch):
    b = _bench()
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        b.dist_init(4)


def test_enumeration_issue_roofline_from_committed_counters():
    """two_ply.roofline_issue is reproducible from the committed profile: the
    enumerators' SQ instruction totals per batch over an enumeration window, priced
    against each pipe's chip capacity (VALU 2 cycles on 1,024 SIMDs, the rest one per
    cycle on 256 CUs, 2.4 GHz); the busiest pipe is the roofline."""
    import json
    b = _bench()
    summ = json.load(open(os.path.join(ROOT, "profiles", "latest_summary.json")))
    enums = summ["two_ply_enum"]
    r = b.enum_roofline(enums, 4, 26.5, "test")
    valu = sum(e["totals"]["SQ_INSTS_VALU"] for e in enums) / 4
    assert r["pipes"]["VALU"]["frac"] == pytest.approx(valu * 2 / 1024 / 2.4e9 / 26.5e-3)
    assert r["frac"] == max(p["frac"] for p in r["pipes"].values()) and 0 < r["frac"] < 1
    assert r["pipe"] in ("SALU", "VALU")
