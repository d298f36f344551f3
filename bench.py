"""bench.py — self-play env steps/sec on MI355X (BASELINE.json metric).

Default workload (N=1 line): BASELINE config C3 — B=65,536 concurrent games per
GPU, one PPO rollout step per iteration = policy forward (BackgammonPolicyNetwork
198->128->{500 logits, 1 value}) + masked-softmax sampling + env.step on every
lane + rollout row (int8 lane boards, action, log-prob, value, reward, done)
stored to a device ring in HBM.  The `host_mirror` sub-object times the same
step with every row also copied to pinned host memory (PCIe-inclusive, the
reference's host-side rollout, ppo_agent.py:175-187).  `value` = env steps/s
summed over ranks.

  python bench.py --gpus N --steps K --warmup W [--workload c3|c1]

Multi-GPU: one process per GPU, independent game shards (weak scaling), no
collective on the rollout path; barrier + max-over-ranks timing.  Launched as
`torch.distributed.run ... bench.py --gpus N` (the driver) each rank reads
RANK / LOCAL_RANK / WORLD_SIZE; `python bench.py --gpus N` with no WORLD_SIZE
in the environment starts the N ranks itself (torch.distributed.run as a child
process; this parent never touches the GPU) and exits with their status.
Backend "nccl" (= RCCL over xGMI); BGX_DIST_BACKEND=gloo lets several ranks
share one GPU for rehearsals.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "mlp-ppo-2ply-p3_amd")]

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
BF16_PEAK_TFLOPS = 2500.0      # dense bf16 MFMA (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c3", choices=["c3", "c1"])
    ap.add_argument("--horizon", type=int, default=32,
                    help="also time full PPO iterations (T rollout steps + update); 0 = skip")
    ap.add_argument("--two-ply-batches", type=int, default=2,
                    help="C4: timed 2-ply expectimax passes over all B root positions (0 = skip)")
    ap.add_argument("--c4-shards", type=int, default=4,
                    help="C4 (H = 40): the B roots as S engines on S streams and host threads, so one shard's "
                         "reply enumeration runs beside another's evaluation (S=1 1.61 M, S=4 1.82 M, S=8 1.82 M "
                         "root decisions/s; DESIGN.md §8 Round 5)")
    ap.add_argument("--c2-steps", type=int, default=50,
                    help="C2: timed greedy 1-ply self-play steps at B=4096 (0 = skip)")
    ap.add_argument("--c2-shards", type=int, default=4,
                    help="C2: the 4,096 games as S engines on S streams, each replayed as its own HIP graph of "
                         "linear steps (S=1 43.2 M, S=2 50.0 M, S=4 51.5-52.0 M env steps/s; profiles/r4_layout/r4r)")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--shards", type=int, default=4,
                    help="the B games of a GPU as S engines of B/S lanes on S streams, so one shard's policy "
                         "kernel runs beside another's env step.  With --fork-steps off each shard's graph is one "
                         "linear chain on its own hardware queue (HIP's 4): S=2 341 M, S=4 382 M, S=8 280 M env "
                         "steps/s at 1,000 steps (DESIGN.md §8 Round 4)")
    ap.add_argument("--fork-steps", action="store_true",
                    help="C3: fork each env step's light launch onto the engine's side stream (round 3's layout, "
                         "best at S=2: 362 M at 1,000 steps but 313 M at 20, its graphs' internal streams share "
                         "hardware queues with the other shard's)")
    ap.add_argument("--burn-in", type=int, default=150,
                    help="untimed steps before warmup so the game population reaches its steady mix "
                         "(openings are cheaper than mid-game positions)")
    ap.add_argument("--host-mirror", action="store_true",
                    help="C3 headline with every rollout row also copied to pinned host memory (PCIe-inclusive)")
    ap.add_argument("--mirror-steps", type=int, default=64,
                    help="steps of the host_mirror sub-object (C3 + pinned-host copy of every row; 0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graphs", action="store_true", help="C2 and C3 with eager launches instead of HIP graphs")
    ap.add_argument("--graph-steps", type=int, default=2,
                    help="C3: rollout steps per HIP graph (even: the engine's host state is a 2-step fixed point; "
                         "the timed steps replay K // G graphs, the rest run eagerly)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    return ap.parse_args()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int) -> int:
    """`python bench.py --gpus N` without a launcher: run this same command as N
    ranks under torch.distributed.run (one process per GPU) in a child process
    and return its exit status.  Called before anything touches the GPU; the
    ranks' stdout is this process's stdout, so rank 0's JSON line is the output."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # dmabuf IPC only on this driver (RCCL)
    return subprocess.run(cmd, env=env).returncode


def dist_init(gpus: int):
    """One process per GPU.  BGX_DIST_FORCE=1 (tests) initialises the process group
    even at WORLD_SIZE=1, so RCCL's init, all-reduce, all-gather and barrier, and
    the HIP-graph captures beside its watchdog thread, run on a one-GPU box."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if ws != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws}")
    ndev = torch.cuda.device_count()
    backend = os.environ.get("BGX_DIST_BACKEND", "nccl")
    if ws > 1 and backend == "nccl" and ws > ndev:
        raise SystemExit(f"bench.py: {ws} RCCL ranks need {ws} GPUs, {ndev} visible "
                         "(BGX_DIST_BACKEND=gloo rehearses several ranks on one GPU)")
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(ndev, 1)
    torch.cuda.set_device(local)
    if ws > 1 or os.environ.get("BGX_DIST_FORCE") == "1":
        import torch.distributed as dist
        if ws == 1:                                 # a one-rank group: rendezvous on this host
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        # "nccl" is RCCL on ROCm (one rank per GPU); BGX_DIST_BACKEND=gloo lets
        # several ranks share one GPU for functional rehearsals of the N>1 path
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        return rank, ws, local, backend
    return rank, ws, local, None


def _dist_on() -> bool:
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def gather_ranks(x, ws: int) -> list:
    """Every rank's list of floats, in rank order (a CUDA tensor: RCCL and gloo)."""
    if not _dist_on():
        return [x]
    import torch.distributed as dist
    t = torch.tensor(x, dtype=torch.float64, device="cuda")
    out = [torch.empty_like(t) for _ in range(ws)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def barrier(ws):
    if _dist_on():
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, ws: int) -> float:
    if not _dist_on():
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, ws: int) -> float:
    if not _dist_on():
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def cpu_baseline(seconds: float):
    """The oracle (C restatement of the reference env, oracle/bgoracle.c) stepping a
    random legal policy on the GPU box's host cores: one process per core on the
    cores this job may use (at most 16, the box's CPU share per GPU), plus a
    1-core run.  The reference's own Python env cannot run on the box; its timing
    on the build container (tools/time_reference_env.py, with the port timed
    beside it as the bridge ratio) is attached from profiles/."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import port_bench
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    procs = max(1, min(16, avail))
    one, one_steps = port_bench.run(seconds, 0)
    multi, multi_steps = port_bench.run_parallel(seconds, procs)
    out = {"value": multi, "unit": "env steps/s", "cores": procs, "kind": "port",
           "sample": f"{multi_steps} random-policy BackgammonEnv.step calls of the C oracle (oracle/bgoracle.c), "
                     f"{procs} processes x 1 thread, {seconds:.0f} s",
           "cores_available": avail, "host_cpus": os.cpu_count(),
           "cores_note": ("16 processes: the GPU box's CPU share per GPU is 16 (its OMP_NUM_THREADS / MAX_JOBS "
                          f"are {os.environ.get('OMP_NUM_THREADS', '?')}; the pool's rules size worker pools to that "
                          "share); the affinity mask and cpu_count show the whole machine's CPUs, which the other "
                          "GPUs' jobs share.  The port scales linearly per process (single_core x cores ~= value)"),
           "single_core": {"value": one, "steps": one_steps, "seconds": seconds}}
    ref = os.path.join(ROOT, "profiles", "cpu_reference_timing.json")
    if os.path.exists(ref):
        r = json.load(open(ref))
        out["reference_python"] = {
            "value": r["reference_env_steps_per_s"], "unit": "env steps/s", "cores": r["processes"],
            "where": "build container (the reference never travels to the GPU box)",
            "port_same_host": r["port_env_steps_per_s"], "port_over_reference": r["port_over_reference"],
            "estimated_here": multi / r["port_over_reference"], "estimated_here_cores": procs,
            "estimate_note": "the reference env on this host's cores, estimated as this host's port rate / the "
                             "port:reference ratio measured on the build container",
            "source": "profiles/cpu_reference_timing.json (tools/time_reference_env.py)"}
    return out


def ppo_iteration_bench(B: int, horizon: int, ws: int, dev, iters: int = 4, streams=None):
    """Full PPO iterations (rollout of `horizon` steps on B lanes + 4-epoch update
    with the gradient all-reduce across ranks): env steps/s INCLUDING the update.
    `streams`: the C3 leg's shard streams, reused when the shard counts match."""
    from bgx.train import PPOTrainer
    group = None
    kw = {"chunk": int(os.environ["BGX_PPO_CHUNK"])} if os.environ.get("BGX_PPO_CHUNK") else {}
    tr = PPOTrainer(batch=B, horizon=horizon, seed=11, device=dev, process_group=group, streams=streams, **kw)
    tr.iteration()                                   # warm
    torch.cuda.synchronize(dev)
    barrier(ws)
    t0 = time.perf_counter()
    ms = [tr.iteration() for _ in range(iters)]
    torch.cuda.synchronize(dev)
    barrier(ws)
    el = max_over_ranks(time.perf_counter() - t0, ws)
    steps = sum_over_ranks(float(B * horizon * iters), ws)
    out = {"config": f"PPO iteration: B={B}/GPU x T={horizon} rollout + 4-epoch full-batch update "
                     f"(chunked, features re-encoded from int8 records), grad all-reduce over {ws} rank(s)",
           "ranks": ws, "env_steps_per_s_incl_update": steps / el, "seconds_per_iteration": el / iters,
           "rollout_s": sum(m["rollout_s"] for m in ms) / iters, "update_s": sum(m["update_s"] for m in ms) / iters,
           "losses_last": {k: ms[-1][k] for k in ("policy_loss", "value_loss", "entropy", "total_loss")}}
    if _dist_on():  # data parallel: the all-reduced update leaves every rank on the same weights
        import torch.distributed as dist
        flat = torch.cat([p.detach().reshape(-1) for p in tr.net.parameters()])
        allw = [torch.empty_like(flat) for _ in range(ws)]
        dist.all_gather(allw, flat)
        out["weights_identical_across_ranks"] = all(torch.equal(allw[0], w) for w in allw)
        out["collective"] = ("one flat fp32 gradient all-reduce per optimizer step (4 per update) + the "
                             "(sum r, sum r^2, n) return-normalisation all-reduce, backend "
                             + dist.get_backend())
    return out


def one_ply_selfplay_bench(B: int, steps: int, ws: int, rank: int, dev, shards: int = 4, graphs: bool = True,
                           streams=None):
    """C2: B games per GPU, greedy 1-ply self-play with the value head
    MLP(198->40->1): every step = V over each lane's legal afterstates (mover's
    one-hot, as legal_board_features) -> first argmax -> env.step.  The B games
    run as `shards` engines on their own streams: at this batch each launch is
    bound by its slowest lane, so one shard's search runs beside the other's
    step.  `streams`: the C3 leg's shard streams (one hardware queue each), reused
    when the shard counts match: fresh pool streams can share a hardware queue (HIP
    maps streams to its 4 queues round-robin as they are created), which serialised
    two shards (31 vs 52 M env steps/s once the C4 leg had taken pool streams)."""
    import bgx
    from bgx.policy import PolicyNet
    from bgx.search import ValueHead, one_ply
    torch.manual_seed(2)
    vh = ValueHead(PolicyNet(hidden_size=40).to(dev))
    S = shards if B % shards == 0 else 1
    engs = [bgx.Engine(batch=B // S, max_moves=500, seed=123 + rank + 7919 * k, dice="philox", auto_reset=True,
                       device=dev) for k in range(S)]
    if streams is None or len(streams) != S:
        streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
    for e in engs:
        e.reset(want_obs=False)
        e.set_fork(False)          # one stream per step: 43.1 vs 38.9 M forked (profiles/r4_layout/r4o)
    torch.cuda.synchronize(dev)

    def step():
        for e, st in zip(engs, streams):
            with torch.cuda.stream(st):
                best, _ = one_ply(e, vh)
                e.step(best, want_obs=False, want_info=False)

    for _ in range(20):                                # burn-in + warm
        step()
    torch.cuda.synchronize(dev)
    # At B = 4,096 a step is a dozen short launches (1-ply pass, split env step,
    # dispatch order, overflow tiers): replayed as one HIP graph of two steps (the
    # engine alternates its overflow-counter set every step, so a pair of steps
    # is a fixed point of its host state).  Every launch reads its state from the
    # device, so the replays are the same steps as the eager calls.
    graph = None
    if graphs:
        from bgx.graphs import capture
        # each shard's engine is joined before its capture and as the capture's last
        # call (no side-stream work held unjoined: hipErrorStreamCaptureUnjoined);
        # one graph per shard, replayed on the shard's stream
        caps = [torch.cuda.Stream(dev) for _ in range(S)]
        for k in range(S):
            caps[k].wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(caps[k]):
                engs[k].join()
                for _ in range(2):
                    best, _ = one_ply(engs[k], vh)
                    engs[k].step(best, want_obs=False, want_info=False)
                engs[k].join()
        torch.cuda.synchronize(dev)

        def two_steps(k):
            for _ in range(2):
                best, _ = one_ply(engs[k], vh)
                engs[k].step(best, want_obs=False, want_info=False)
            engs[k].join()
        # a failed capture ends the process
        graph = [capture("c2", lambda k=k: two_steps(k), caps[k]) for k in range(S)]
        torch.cuda.synchronize(dev)
    barrier(ws)
    t0 = time.perf_counter()
    if graph is not None:
        for _ in range(steps // 2):
            for k in range(S):
                with torch.cuda.stream(streams[k]):
                    graph[k].replay()
        steps = steps // 2 * 2
    else:
        for _ in range(steps):
            step()
    torch.cuda.synchronize(dev)
    barrier(ws)
    el = max_over_ranks(time.perf_counter() - t0, ws)
    return {"config": f"C2: B={B} games/GPU as {S} shard(s), 1-ply greedy self-play, value MLP 198->40->1 "
                      "(argmax over afterstates)",
            "env_steps_per_s": sum_over_ranks(float(B * steps), ws) / el, "ms_per_step": el * 1e3 / steps,
            "steps": steps, "shards": S, "hip_graph": graph is not None}


def two_ply_shards(eng, shards: int):
    """The C4 roots of `eng` as `shards` engines of B/S lanes holding the same positions
    (records copied, legal moves regenerated: the same rows and leaves as one engine)."""
    import bgx
    if shards <= 1 or eng.batch % shards:
        return [eng]
    n = eng.batch // shards
    rec = eng.records()
    out = []
    for k in range(shards):
        e = bgx.Engine(batch=n, max_moves=eng.max_moves, seed=1000 + k, dice="philox", auto_reset=True,
                       device=eng.device)
        e.set_lanes(rec[k * n:(k + 1) * n])
        out.append(e)
    torch.cuda.synchronize(eng.device)
    return out


def two_ply_bench(engs, batches: int, ws: int, dev, hidden: int = 40, streams=None):
    """C4: 2-ply expectimax over the 21 rolls for every lane's current position
    (B roots per GPU), value head MLP(198->H->1) on MFMA.  The roots run
    as len(engs) game shards, each on its own stream driven by its own host thread (a
    bgx_two_ply call synchronises its stream after the row scan and after the pool
    pass; ctypes drops the GIL inside it), so one shard's reply enumeration runs beside
    another's evaluation.  Shard k > 0 starts k/S of a batch later.  `streams`: given
    streams instead of fresh pool streams (the bench passes none: the C3 leg's streams
    gave 1.73-1.80 M against 1.80-1.84 M on fresh ones)."""
    import threading
    from bgx.policy import PolicyNet
    from bgx.search import ValueHead, two_ply, two_ply_timings
    torch.manual_seed(1)
    vnet = PolicyNet(hidden_size=hidden).to(dev)
    vh = ValueHead(vnet)
    S = len(engs)
    if streams is None or len(streams) != S:
        streams = [torch.cuda.Stream(dev) for _ in range(S)]
    for st in streams:
        st.wait_stream(torch.cuda.current_stream(dev))
    t_warm = 0.0
    for e, st in zip(engs, streams):               # warm (workspace sizing, code load)
        with torch.cuda.stream(st):
            t = time.perf_counter()
            two_ply(e, vh)
            t_warm = max(t_warm, time.perf_counter() - t)
    torch.cuda.synchronize(dev)
    barrier(ws)
    res = [dict(leaves=0, jobs=0, enum_ms=0.0, eval_ms=0.0) for _ in range(S)]
    errs = []

    def worker(k):
        try:
            torch.cuda.set_device(dev)
            if k:
                time.sleep(t_warm * k / S)
            with torch.cuda.stream(streams[k]):
                for _ in range(batches):
                    _, _, _, st = two_ply(engs[k], vh)
                    te, tv = two_ply_timings(engs[k])
                    r = res[k]
                    r["leaves"] += st["leaves"]
                    r["jobs"] += st["jobs"]
                    r["enum_ms"] += te
                    r["eval_ms"] += tv
        except Exception as ex:                   # re-raised in the main thread
            errs.append(ex)

    t0 = time.perf_counter()
    if S == 1:
        worker(0)
    else:
        th = [threading.Thread(target=worker, args=(k,)) for k in range(S)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    torch.cuda.synchronize(dev)
    if errs:
        raise errs[0]
    barrier(ws)
    el = max_over_ranks(time.perf_counter() - t0, ws)
    B = sum(e.batch for e in engs)
    leaves = sum(r["leaves"] for r in res)
    jobs = sum(r["jobs"] for r in res)
    # per-shard HIP-event phase times, averaged over the shards (they overlap)
    enum_ms = sum(r["enum_ms"] for r in res) / S
    eval_ms = sum(r["eval_ms"] for r in res) / S
    roots = sum_over_ranks(float(B * batches), ws)
    leaves_all = sum_over_ranks(float(leaves), ws)
    flop_per_leaf = 2 * 198 * hidden + 2 * hidden
    nt = (hidden + 15) // 16
    # k_eval (the MFMA kernel): algorithmic FLOPs of one shard's leaves / its HIP-event time
    eval_tflops = (leaves / S) * flop_per_leaf / (eval_ms / batches * 1e-3) / batches / 1e12 if eval_ms > 0 else None
    # evaluator tile forms: narrow = 16 units (hi + lo rows) per 32-row tile,
    # wide (nt > 4) = 32 units per tile with hi and lo as two k-blocks of one accumulator
    wide = nt > 4
    units = 32 * ((nt + 1) // 2) if wide else 16 * nt
    tiles = (f"H as {(nt + 1) // 2} 32-unit tiles, hi and lo as two k-blocks" if wide
             else f"H as {nt} 16-unit hi+lo tiles")
    return {"config": f"C4: B={B} roots/GPU as {S} shard(s) on {S} streams / host threads, 2-ply expectimax over "
                      f"21 rolls, value MLP 198->{hidden}->1 "
                      "(W1 split hi+lo on f16 MFMA, exact f16 features; fp32-equivalent); leaves encoded with "
                      "the root mover's one-hot, min over replies",
            "hidden": hidden, "batches": batches, "shards": S,
            "root_decisions_per_s": roots / el, "leaf_evals_per_s": leaves_all / el,
            "leaves_per_root": leaves_all / roots, "reply_enumerations": jobs * ws, "seconds": el,
            "enumeration_ms_per_batch": enum_ms / batches, "evaluation_ms_per_batch": eval_ms / batches,
            "roofline": {"kernel": f"k_eval<{nt}>: leaf pool -> f16-exact features -> W1 hi+lo on "
                                   "v_mfma_f32_32x32x16_f16 -> value head -> per-job min (HIP events)",
                         "bound": "mfma", "achieved": eval_tflops, "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": eval_tflops / BF16_PEAK_TFLOPS if eval_tflops else None,
                         "flop_per_leaf": flop_per_leaf,
                         "issued_over_algorithmic": _issued_over_algorithmic(nt, leaves_all / roots, flop_per_leaf),
                         "issued_unfactored_bound": 2 * (units / hidden) * (208 / 198),
                         "note": f"issued_over_algorithmic: SQ_INSTS_MFMA of a whole-batch k_eval<{nt}> dispatch "
                                 "(profiles/latest_summary.json) x 32,768 FLOP per v_mfma_f32_32x32x16_f16 / (65,536 "
                                 "roots x leaves per root x FLOP per leaf); the factored evaluator runs 7 + (hit "
                                 "blocks) of the 13 k-blocks per leaf.  issued_unfactored_bound: algorithmic x 2 (W1 "
                                 f"hi+lo for fp32 accuracy) x {units}/{hidden} ({tiles}) x 208/198 (K padding, bias)"}}


def _issued_over_algorithmic(nt: int, leaves_per_root: float, flop_per_leaf: int):
    """Issued / algorithmic MFMA FLOPs of k_eval<nt> from the committed PMC pass (None
    without one): its largest dispatch is one engine's whole 65,536-root batch."""
    try:
        summ = json.load(open(os.path.join(ROOT, "profiles", "latest_summary.json")))
        e = next(x for x in summ.get("two_ply_eval", []) if x["kernel"] == f"k_eval<{nt}>")
        return e["SQ_INSTS_MFMA_max_dispatch"] * 32768 / (65536 * leaves_per_root * flop_per_leaf)
    except Exception:
        return None


EVAL_PMC_ARGS = ("--steps 2 --warmup 1 --burn-in 150 --horizon 0 --no-cpu-baseline --two-ply-batches 1 "
                 "--c2-steps 0 --mirror-steps 0")


def enum_roofline(enums, batches_profiled: int, enum_ms: float, src) -> dict:
    """The 2-ply reply enumeration (k_enum*: the two enumerators side by side on two
    streams, then the overflow tiers) priced against instruction issue, like the env
    step's roofline_issue: wave-instructions per batch by pipe (SQ_INSTS_* totals of the
    committed enum1 pass / the batches that pass ran) over the live enumeration window
    of this run, against each pipe's chip capacity.  The wave-time split of each
    enumerator (enum2 pass) says where the rest of its time goes."""
    model = {"VALU": ("SQ_INSTS_VALU", 2, 1024), "SALU": ("SQ_INSTS_SALU", 1, 256), "LDS": ("SQ_INSTS_LDS", 1, 256),
             "SMEM": ("SQ_INSTS_SMEM", 1, 256), "VMEM": ("SQ_INSTS_VMEM", 1, 256), "BRANCH": ("SQ_INSTS_BRANCH", 1, 256)}
    t = enum_ms * 1e-3
    pipes = {}
    for p, (c, cyc, units) in model.items():
        n = sum(e["totals"].get(c, 0.0) for e in enums) / batches_profiled
        pipes[p] = {"wave_insts_per_batch": n, "achieved_G_per_s": n / t / 1e9, "peak_G_per_s": units * 2.4 / cyc,
                    "frac": n * cyc / units / 2.4e9 / t}
    top = max(pipes, key=lambda p: pipes[p]["frac"])
    return {"kernel": "reply enumeration: " + " + ".join(e["kernel"] for e in enums if e["totals"].get("SQ_INSTS_VALU", 0) > 1e6),
            "bound": "issue", "pipe": top, "achieved": pipes[top]["achieved_G_per_s"], "peak": pipes[top]["peak_G_per_s"],
            "unit": "G wave-instructions/s", "frac": pipes[top]["frac"], "pipes": pipes, "enumeration_ms": enum_ms,
            "wave_time_split": {e["kernel"]: e["wave_time_split"] for e in enums if e.get("wave_time_split")
                                and e["totals"].get("SQ_INSTS_VALU", 0) > 1e6},
            "counters_source": src, "batches_profiled": batches_profiled}


def policy_roofline(pairs, rows: int, prof, src) -> dict:
    """C3's policy kernel (k_policy_act: encoder + 198->128->{500,1} MLP on split-f16 MFMA +
    masked log-softmax + Gumbel-max sample) priced against the dense MFMA peak: algorithmic
    FLOPs per row 2(198*128 + 128*501) over its HIP-event time per shard launch (eager steps
    after the timed region, the policy launch of each shard step).  The committed PMC passes
    of the same kernel (tools/profile.sh pol1/pol2 -> profiles/latest_summary.json "policy")
    give what the hardware issued: MFMA busy and VALU issue fractions, wave-time split."""
    ms = sum(a.elapsed_time(b) for a, b in pairs) / len(pairs)
    flop_row = 2 * (198 * 128 + 128 * 501)
    ach = rows * flop_row / (ms * 1e-3) / 1e12
    out = {"kernel": "k_policy_act<4,0> (one 32-row wave per MFMA tile column, rollout specialisation)",
           "bound": "mfma", "achieved": ach, "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
           "frac": ach / BF16_PEAK_TFLOPS, "flop_per_row": flop_row, "rows_per_launch": rows, "kernel_ms": ms}
    if prof:
        p = prof[0]
        out["pmc"] = {"mfma_busy_frac": p.get("mfma_busy_frac_at_2p4GHz"),
                      "valu_issue_frac": p.get("valu_issue_frac_at_2p4GHz"),
                      "wave_time_split": p.get("wave_time_split"), "avg_ns_profiled": p.get("avg_ns_c3"),
                      "source": "profiles/latest_summary.json policy (" + str(src) + ")"}
    return out


def issue_roofline(sq: dict, lanes: int, kern_ms: float, src) -> dict:
    """The env step's real bound: instruction issue, not HBM.  Wave-instructions per
    lane-step by pipe (SQ_INSTS_* of the C3 step alone, profiles/latest_summary.json,
    tools/profile.sh passes sqi/sqc) x the lanes of one shard step, over the live
    HIP-event time of that step, against each pipe's chip capacity (VALU: 2 cycles per
    wave64 instruction on each of 1,024 SIMD-32s; SALU, LDS, SMEM, VMEM, branch: one
    instruction per cycle on each of 256 CUs; 2.4 GHz).  frac = the busiest pipe's
    utilisation.  The wave-time split says where the rest of each wave's time goes."""
    ins, model, ghz = sq["instructions_per_lane_step"], sq["pipe_model"], sq["clock_ghz"]
    t = kern_ms * 1e-3
    pipes = {}
    for p, m in model.items():
        n = ins.get(m["counter"], 0.0) * lanes
        pipes[p] = {"wave_insts_per_lane_step": ins.get(m["counter"], 0.0),
                    "achieved_G_per_s": n / t / 1e9, "peak_G_per_s": m["units"] * ghz / m["cycles_per_inst"],
                    "frac": n * m["cycles_per_inst"] / m["units"] / (ghz * 1e9) / t}
    top = max(pipes, key=lambda p: pipes[p]["frac"])
    return {"kernel": "env step (same launches and HIP-event window as `roofline`)", "bound": "issue",
            "pipe": top, "achieved": pipes[top]["achieved_G_per_s"], "peak": pipes[top]["peak_G_per_s"],
            "unit": "G wave-instructions/s", "frac": pipes[top]["frac"], "pipes": pipes,
            "wave_time_split": sq.get("wave_time_split"), "lanes_per_launch": lanes, "kernel_ms": kern_ms,
            "counters_source": src}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    rank, ws, local, backend = dist_init(args.gpus)
    dev = torch.device("cuda", local)
    import bgx
    from bgx.policy import PolicyNet

    B = args.batch
    S = max(1, args.shards)
    assert B % S == 0
    Bs = B // S
    engs = [bgx.Engine(batch=Bs, max_moves=500, seed=1234 + 7919 * rank + 104729 * k, dice="philox", auto_reset=True,
                       device=dev) for k in range(S)]
    for e in engs:
        e.reset(want_obs=True)
        e.set_fork(args.fork_steps)
    eng = engs[0]
    torch.manual_seed(0)
    net = PolicyNet(hidden_size=128, action_size=500).to(dev)
    net.pack()
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
    # Rollout storage: a device-resident ring of T rollout rows per shard (the
    # PPOTrainer layout, bgx/train.py): records, actions, log-probs, values,
    # rewards, dones — 81 B per lane-step written straight into HBM by the
    # kernels.  --host-mirror additionally streams every row to pinned host
    # memory on a side stream (the reference keeps its rollout in host lists);
    # that copy runs as blit kernels that share the CUs with the policy kernel.
    ring = 32
    kw = dict(device=dev)
    bufs = [{
        "records": torch.empty(ring, Bs, 64, dtype=torch.uint8, **kw),
        "act": torch.empty(ring, Bs, dtype=torch.int32, **kw),
        "logp": torch.empty(ring, Bs, dtype=torch.float32, **kw),
        "value": torch.empty(ring, Bs, dtype=torch.float32, **kw),
        "reward": torch.empty(ring, Bs, dtype=torch.float32, **kw),
        "done": torch.empty(ring, Bs, dtype=torch.uint8, **kw),
    } for _ in range(S)]
    want_mirror = args.host_mirror or args.mirror_steps > 0
    from bgx.hostcopy import HostMirror
    mirrors = [HostMirror(b) for b in bufs] if want_mirror else None     # pinned twins of the rings
    copy_streams = [torch.cuda.Stream(dev) for _ in range(S)] if want_mirror else None
    counts = [torch.empty(Bs, dtype=torch.int16, device=dev) for _ in range(S)]
    gen = torch.Generator(device=dev).manual_seed(99 + rank)
    ev_pairs, pol_pairs = [], []
    state = {"i": 0, "mirror": args.host_mirror}

    def shard_step(k, i, timed):
        e, st = engs[k], streams[k]
        with torch.cuda.stream(st):
            if args.workload == "c1":
                e.n_moves(out=counts[k])
                act = (torch.rand(Bs, device=dev, generator=gen) * counts[k].clamp(min=1).float()).to(torch.int32)
                if timed:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                e.step(act, want_obs=False, want_info=False)
                if timed:
                    e1.record(st)
                    ev_pairs.append((e0, e1))
                return
            b, slot = bufs[k], i % ring
            # fused HIP policy step on the engine's lane records in place; it also
            # stores them (int8 boards, no fp32 obs round trip) as the rollout row
            if timed:
                p0, p1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                p0.record(st)
            net.act(e, seed=4242 + rank * 16 + k, step=i,
                    out=(b["act"][slot], b["logp"][slot], b["value"][slot]), records_out=b["records"][slot])
            if timed:
                p1.record(st)
                pol_pairs.append((p0, p1))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
            e.step(b["act"][slot], want_obs=False, want_info=False, out=(b["reward"][slot], b["done"][slot]))
            if timed:
                e1.record(st)
                ev_pairs.append((e0, e1))
            if state["mirror"]:                                   # pinned-host mirror (side stream)
                cs = copy_streams[k]
                cs.wait_stream(st)
                mirrors[k].copy(slot, 1, stream=cs)                # every field of the slot, one launch
                if slot == ring - 1:
                    st.wait_stream(cs)                            # the ring wraps: rows must be on the host

    def step(timed: bool):
        i = state["i"]
        state["i"] += 1
        for k in range(S):
            shard_step(k, i, timed)

    def sync_all():
        torch.cuda.synchronize(dev)

    for _ in range(args.burn_in):
        step(False)
    # warmup + a sample of legal-move counts for the algorithmic byte count
    nm_sum, nm_n = 0.0, 0
    for w in range(args.warmup):
        step(False)
        if w >= args.warmup // 2:
            sync_all()
            nm_sum += sum(float(e.n_moves(out=counts[k]).float().mean().item()) for k, e in enumerate(engs)) / S
            nm_n += 1
    mean_moves = nm_sum / max(nm_n, 1)
    # C3 as HIP graphs: one rollout step is ~20 launches and event waits over the two
    # shards' streams and the engines' side streams, ~150 us of host time per step in
    # eager mode (tools/c3_host_probe.py) -- close to the GPU's own step time.  Each
    # shard's G steps are captured as a graph of their own (one graph per group of ring
    # slots) and the shards' graphs replay on their own streams, side by side (one
    # capture holding both shards' streams crashes the runtime at the end of capture).
    # The policy's noise step is read from a per-shard device counter that each replay
    # advances, so a replay is G fresh rollout steps.  Each engine is joined before the
    # capture and at its end, so a graph holds no unjoined side-stream work and the
    # engine's host state (overflow-counter parity, pending dispatch order) is the same
    # before and after it (G even).  tests/test_gpu_graph.py: replays == eager steps.
    G = args.graph_steps
    graphs = []                                         # graphs[g][k]: slots [gG, gG + G) of shard k
    if not args.no_graphs and args.workload == "c3" and G >= 2 and G % 2 == 0 and ring % G == 0:
        from bgx.graphs import capture
        ctrs = [torch.zeros(1, dtype=torch.int32, device=dev) for _ in range(S)]
        caps = [torch.cuda.Stream(dev) for _ in range(S)]
        for k in range(S):
            with torch.cuda.stream(streams[k]):
                engs[k].join()
        torch.cuda.synchronize(dev)

        def graph_steps(k, g0):
            e, b = engs[k], bufs[k]
            for i in range(g0, g0 + G):
                net.act(e, seed=4242 + rank * 16 + k, step=i, step_ctr=ctrs[k],
                        out=(b["act"][i], b["logp"][i], b["value"][i]), records_out=b["records"][i])
                e.step(b["act"][i], want_obs=False, want_info=False, out=(b["reward"][i], b["done"][i]))
            e.join()
            PolicyNet.advance_counter(ctrs[k], ring)
        for g0 in range(0, ring, G):              # a failed capture ends the process (bgx/graphs.py)
            graphs.append([capture("c3", lambda k=k, g0=g0: graph_steps(k, g0), caps[k]) for k in range(S)])
        torch.cuda.synchronize(dev)
        for row in graphs:                          # untimed: first replays upload the graphs
            for k in range(S):
                with torch.cuda.stream(streams[k]):
                    row[k].replay()
        torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    barrier(ws)
    torch.cuda.synchronize(dev)
    # the timed region on the device clock too: a HIP event on every shard's stream before
    # its first and after its last timed step (the roofline's step window)
    tev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(S)]
    t0 = time.perf_counter()
    for k in range(S):
        tev[k][0].record(streams[k])
    if graphs:
        for r in range(args.steps // G):
            row = graphs[r % len(graphs)]
            for k in range(S):
                with torch.cuda.stream(streams[k]):
                    row[k].replay()
        for _ in range(args.steps % G):
            step(False)
    else:
        for _ in range(args.steps):
            step(True)
    for k in range(S):
        tev[k][1].record(streams[k])
    t_enq = time.perf_counter() - t0             # host time to enqueue the timed steps
    torch.cuda.synchronize(dev)
    barrier(ws)
    torch.cuda.synchronize(dev)
    el_rank = time.perf_counter() - t0
    # device span of the timed region: first shard start to last shard end
    dev_span_ms = max(tev[0][0].elapsed_time(tev[k][1]) for k in range(S))
    if graphs:
        # the roofline's kernel time: HIP events around bgx_step in eager steps right
        # after the timed replays (events cannot be timed inside a graph)
        for _ in range(16):
            step(True)
        torch.cuda.synchronize(dev)
    el = max_over_ranks(el_rank, ws)
    per_rank = gather_ranks([float(B * args.steps), el_rank], ws)
    total_steps = sum(r[0] for r in per_rank)
    value = total_steps / el
    kern_ms = sum(a.elapsed_time(b) for a, b in ev_pairs) / len(ev_pairs)
    # algorithmic bytes per lane-step of the env-step kernel:
    # record in+out 128, action 4, chosen move 8, new move list 8*n, reward 4, done 1, rng ctr 8+8
    bytes_per_lane = 128 + 4 + 8 + 8 * mean_moves + 4 + 1 + 16
    achieved = Bs * bytes_per_lane / (kern_ms * 1e-3) / 1e9    # one shard's env step per window
    # HBM bytes per env step of one shard (all kernels bgx_step launches: both k_step
    # launches, the order sort, the overflow tiers) from the committed rocprofv3 PMC
    # passes (tools/profile.sh -> profiles/latest_summary.json; (FETCH_SIZE + WRITE_SIZE)
    # x 1024: the step's 64-B record / 4-8-B scalar reads are single 64-B requests that
    # FETCH_SIZE counts exactly, calibrated in profiles/r2_fetch_calibration.json)
    traffic, traffic_src, prof_kernels, sq, summ, prof_ok = None, None, None, None, None, False
    prof = os.path.join(ROOT, "profiles", "latest_summary.json")
    if os.path.exists(prof):
        try:
            summ = json.load(open(prof))
            prof_ok = True
            env = summ.get("env_step")
            if env and env["hbm_bytes_per_step"] > 0:
                traffic, traffic_src = env["hbm_bytes_per_step"], summ.get("command")
                prof_kernels = {k["name"]: round(k["avg_ns"] / 1e3, 1) for k in env["kernels"]}
            sq = (env or {}).get("sq")
        except Exception:
            traffic = None
    line = {
        "metric": "self-play env steps/sec (whole node) + 2-ply evals/sec at batch=65536",
        "value": value,
        "unit": "env steps/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8 boards / fp32-equivalent policy MLP (split-f16 MFMA)",
        "data": "synthetic self-play (Philox dice), random-init BackgammonPolicyNetwork weights",
        "burn_in": args.burn_in,
        "config": {"workload": (f"C3: B={B} games/GPU PPO rollout step (policy 198->128->{{500,1}} + masked "
                                "sample + env.step, rollout rows stored to an HBM ring"
                                + (" + pinned-host mirror" if args.host_mirror else "") + ")")
                   if args.workload == "c3" else
                   f"C1-on-GPU: B={B} games/GPU random legal policy env.step",
                   "global_batch": B * ws, "games_per_gpu": B, "max_legal_moves": 500,
                   "parallelism": f"dp{ws} (independent game shards)", "shards_per_gpu": S,
                   "streams_per_gpu": S, "step_fork": bool(args.fork_steps),
                   "hip_graph": ({"steps_per_graph": G, "replays": args.steps // G, "eager_steps": args.steps % G}
                                 if graphs else None)},
        "roofline": {"kernel": "env step = k_step<0,9,0,false,1> (predicted-doubles prefix) then "
                               "k_step<0,8,0,true,1> (the rest) + k_order_count/scatter + k_movegen_over tiers, "
                               "one wave per game, "
                               + ("the light launch on the engine's side stream (event fork-join)" if args.fork_steps
                                  else "both launches on the shard's stream")
                               + f"; {S} shards' steps overlap on {S} streams",
                     "bound": "hbm", "achieved": B * bytes_per_lane / (dev_span_ms / args.steps * 1e-3) / 1e9,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": B * bytes_per_lane / (dev_span_ms / args.steps * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "window": "the timed region on the device clock (HIP events on every shard's stream before the "
                               "first and after the last timed step) / steps: the shards' env-step launches overlap "
                               "each other and the policy kernels, so the step window is the launches' union",
                     "window_ms": dev_span_ms / args.steps, "algorithmic_bytes_per_step": B * bytes_per_lane,
                     "traffic": traffic * S if traffic else None,
                     "traffic_unit": f"bytes per env step of all {S} shards (PMC, profiles/latest_summary.json)",
                     "traffic_per_lane_step": traffic / Bs if traffic else None,
                     "traffic_over_algorithmic": traffic / (Bs * bytes_per_lane) if traffic else None,
                     "traffic_source": traffic_src, "lanes_per_step": B, "bytes_per_lane_step": bytes_per_lane,
                     "mean_legal_moves": mean_moves,
                     "per_shard_eager": {"achieved": achieved, "frac": achieved / HBM_PEAK_GBS, "kernel_ms": kern_ms,
                                         "lanes_per_launch": Bs, "algorithmic_bytes_per_step": Bs * bytes_per_lane,
                                         "note": "one shard's env-step bytes / HIP events around its bgx_step in 16 "
                                                 "eager steps right after the timed region, the other shards' "
                                                 "kernels sharing the GPU"},
                     "rocprof_avg_us": prof_kernels,
                     "rocprof_note": "per-launch averages of the C3 step's kernels from the committed kernel trace "
                                     "(profiles/latest_summary.json env_step); under 4-shard overlap a launch's "
                                     "duration includes the time it shares the CUs with the other shards"},
    }
    # the same bytes chip-wide: every shard's env-step bytes over the whole step window
    # (ms_per_step), while the per-shard figure above divides one shard's bytes by one
    # shard's event window with the other shards' kernels sharing the GPU
    ms_step = el * 1e3 / args.steps
    chip = B * bytes_per_lane / (ms_step * 1e-3) / 1e9
    line["roofline"]["chip_wide_wall"] = {"achieved": chip, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                          "frac": chip / HBM_PEAK_GBS, "window_ms": ms_step,
                                          "note": "all shards' algorithmic env-step bytes / ms_per_step (host clock)"}
    line["host_enqueue_ms"] = t_enq * 1e3
    line["per_rank"] = [{"rank": k, "env_steps": r[0], "seconds": r[1]} for k, r in enumerate(per_rank)]
    if backend is not None:
        line["dist_backend"] = backend
    if args.mirror_steps > 0 and not args.host_mirror and args.workload == "c3":
        # north_star's "rollout into pinned host buffers": the same C3 step with every
        # rollout row also copied to pinned host memory.  Graph form (default): each
        # shard's 2-step graph also carries, on a forked copy stream, ONE bgx_copy_regions
        # launch for the previous slot pair of every field (bgx.hostcopy), so the copy of
        # pair p overlaps the steps of pair p + 1; eager form (--no-graphs, and a short
        # comparison run): one copy launch per step and shard after the step.
        mirror = {"config": "C3 as the headline + every rollout row (64-B record, action, log-prob, value, reward, "
                            "done: 81 B per lane-step) copied to pinned host memory",
                  "host_bytes_per_step_per_gpu": B * 81}
        torch.cuda.synchronize(dev)
        if graphs:
            # the headline's graphs, each shard's replayed pair followed by ONE copy launch of
            # that pair's rows (bgx_copy_regions, all 6 fields), on the shard's stream (linear
            # shards) or on its copy stream (--fork-steps); the copy of one shard's pair runs
            # beside the other shards' steps.  The copy streams are joined
            # only when the ring wraps (before a pair's slots are overwritten).  (Round 4 first
            # captured the copy inside each graph as a forked branch: the graph's join then held
            # every pair to its copy, 179 M vs 248 M env steps/s for the eager form.)
            nrep = max(1, args.mirror_steps // G)
            for k in range(S):                      # the eager timing steps left side-stream work
                with torch.cuda.stream(streams[k]):
                    engs[k].join()
            torch.cuda.synchronize(dev)
            barrier(ws)
            t0 = time.perf_counter()
            # linear shards (the default): the copy on the shard's own stream right after its
            # pair (4 shards = HIP's 4 hardware queues; per-shard copy streams would share
            # queues with the other shards' steps: 255 vs 167 M env steps/s, gpurun_out r4n)
            own = not args.fork_steps
            for r in range(nrep):
                g = r % len(graphs)
                for k in range(S):
                    with torch.cuda.stream(streams[k]):
                        if own:
                            graphs[g][k].replay()
                            mirrors[k].copy(g * G, G, stream=streams[k])
                            continue
                        if g == 0 and r > 0:
                            streams[k].wait_stream(copy_streams[k])     # the ring wraps
                        graphs[g][k].replay()
                        copy_streams[k].wait_stream(streams[k])
                        mirrors[k].copy(g * G, G, stream=copy_streams[k])
            for k in range(S):
                streams[k].wait_stream(copy_streams[k])
            torch.cuda.synchronize(dev)
            barrier(ws)
            elm = max_over_ranks(time.perf_counter() - t0, ws)
            msteps = nrep * G
            mirror.update({"env_steps_per_s": sum_over_ranks(float(B * msteps), ws) / elm,
                           "ms_per_step": elm * 1e3 / msteps, "steps": msteps,
                           "form": f"the headline's HIP graphs ({G} steps per shard), each replayed pair followed by "
                                   "one copy launch (6 fields) on the shard's "
                                   + ("stream" if own else "copy stream")})
        state["mirror"] = True                       # eager form: one copy launch per step and shard
        esteps = args.mirror_steps if not graphs else min(args.mirror_steps, 16)
        for _ in range(2):
            step(False)
        torch.cuda.synchronize(dev)
        barrier(ws)
        t0 = time.perf_counter()
        for _ in range(esteps):
            step(False)
        for cs in copy_streams:
            torch.cuda.current_stream(dev).wait_stream(cs)
        torch.cuda.synchronize(dev)
        barrier(ws)
        elm = max_over_ranks(time.perf_counter() - t0, ws)
        state["mirror"] = False
        eager = {"env_steps_per_s": sum_over_ranks(float(B * esteps), ws) / elm, "ms_per_step": elm * 1e3 / esteps,
                 "steps": esteps}
        if graphs:
            mirror["eager"] = eager
        else:
            mirror.update(eager)
            mirror["form"] = "eager launches, one copy launch (6 fields) per step and shard"
        line["host_mirror"] = mirror
    if pol_pairs:
        line["roofline_policy"] = policy_roofline(pol_pairs, Bs, (summ or {}).get("policy") if prof_ok else None,
                                                  (summ or {}).get("pmc_command") if prof_ok else None)
    if sq and sq.get("instructions_per_lane_step") and args.workload == "c3":
        line["roofline_issue"] = issue_roofline(sq, Bs, kern_ms, summ.get("pmc_command"))
        # chip-wide: every lane-step of the whole GPU over the device step window (the per-CU
        # scalar unit's real load; the object above prices one shard over its own event window)
        cw = issue_roofline(sq, B, dev_span_ms / args.steps, summ.get("pmc_command"))
        line["roofline_issue"]["chip_wide"] = {k: cw[k] for k in ("pipe", "achieved", "peak", "unit", "frac", "pipes")}
        line["roofline_issue"]["chip_wide"]["window_ms"] = dev_span_ms / args.steps
    if args.two_ply_batches > 0:
        eng2 = engs[0] if S == 1 else bgx.Engine(batch=B, max_moves=500, seed=77 + rank, dice="philox",
                                                 auto_reset=True, device=dev)
        if S > 1:                                  # full-batch positions for C4: a short self-play burn-in
            eng2.reset(want_obs=False)
            for i in range(args.burn_in + args.warmup + args.steps):   # the same game age as shard 0's
                a2, _, _ = net.act(eng2, seed=5, step=i)
                eng2.step(a2, want_obs=False, want_info=False)
        c4 = two_ply_shards(eng2, args.c4_shards)
        line["two_ply"] = two_ply_bench(c4, args.two_ply_batches, ws, dev)
        if len(c4) > 1:
            # the evaluator's roofline from one whole-batch engine (its HIP-event phases are
            # not shared with another shard's enumeration); the shards' own per-shard figure,
            # taken while the other shards' kernels share the GPU, is kept beside it
            one = two_ply_bench([eng2], 1, ws, dev)
            line["two_ply"]["roofline_per_shard_overlapped"] = line["two_ply"]["roofline"]
            line["two_ply"]["roofline"] = dict(one["roofline"], source="one engine of all B roots, 1 batch")
            line["two_ply"]["one_engine"] = {k: one[k] for k in ("root_decisions_per_s", "enumeration_ms_per_batch",
                                                                "evaluation_ms_per_batch", "leaves_per_root")}
        del c4
        # the same roots with the reference's H = 128 value head (agent/config.py:8)
        # (one engine: its phase times are those of a whole B-root batch)
        line["two_ply_h128"] = two_ply_bench([eng2], 1, ws, dev, hidden=128)
        enums = (summ or {}).get("two_ply_enum") if prof_ok else None
        if enums:
            # tools/profile.sh's enum passes run --two-ply-batches 1 with the default 4 shards:
            # a warm and a timed batch in each of the three legs (H = 40 as shards and as one
            # engine, H = 128 as one engine) -- 6 enumerations of the B roots (round 5 divided
            # by 4); priced over the whole-batch enumeration window of the one-engine H = 128
            # leg (the enumeration does not depend on H)
            line["two_ply"]["roofline_issue"] = enum_roofline(
                enums, 6, line["two_ply_h128"]["enumeration_ms_per_batch"],
                summ.get("enum_command", "python bench.py " + EVAL_PMC_ARGS))
        if eng2 is not engs[0]:             # its 2-ply leaf pool and workspaces (~11 GB) go back
            del eng2
            import gc
            gc.collect()
            torch.cuda.synchronize(dev)
            torch.cuda.empty_cache()
    if args.c2_steps > 0:
        line["one_ply_selfplay"] = one_ply_selfplay_bench(4096, args.c2_steps, ws, rank, dev, args.c2_shards,
                                                          not args.no_graphs, streams=streams)
    if args.horizon > 0 and args.workload in ("c3", "ppo"):
        # the trainer's shards on the C3 leg's streams (one hardware queue each)
        tr_shards = 4 if B >= 65536 and B % 1024 == 0 else (2 if B >= 32768 and B % 256 == 0 else 1)
        line["ppo_iteration"] = ppo_iteration_bench(B, args.horizon, ws, dev,
                                                    streams=streams if len(streams) == tr_shards else None)
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if _dist_on():
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
