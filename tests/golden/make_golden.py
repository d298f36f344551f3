"""Generate the golden fixtures in tests/golden/ by importing the REFERENCE.

Run ONLY in the build container (the reference lives at /root/reference and is
never shipped):  python tests/golden/make_golden.py

The reference is pure Python with no tests of its own, so these
fixtures are its outputs on seeded inputs.  Import shims
stub the uninstalled `gym` base class and the cloud/logging deps of the PPO
agent (boto3, botocore, tensorboardX); none of them touch the rules or the
arithmetic.  Output files (all data, no reference source):

  movegen.npz    G1  boards/player/roll -> ordered legal-move lists (+ counts)
  features.npz   G2  observation + afterstate features (fp32)
  dice.npz       G3  env.seed(s) + env.roll_dice() streams
  traces.npz     G4  full seeded random-policy game traces (single env)
  mlp.npz        G5  BackgammonPolicyNetwork weights + inputs -> logits/values
  ppo.npz        G6  one select_action + one update() on a fixed batch (CPU)
  ppo_fp32.npz   G6b the reference update() with autocast disabled (fp32), 1,024 rows
  ppo_fp16.npz   G6c the reference update() under fp16 autocast + GradScaler (the
                     reference's CUDA numerics, emulated by CPU fp16 autocast)
  misc.npz       G7  get_all_dice_rolls_tensor(), board_to_string / render text,
                     env.legal_moves along seeded single-env games

  python tests/golden/make_golden.py [name ...]   (default: every file)
"""
from __future__ import annotations

import os
import sys
import time
import types

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _shim():
    sys.path.insert(0, REF)
    for name, path in (("src", REF + "/src"), ("src.agent", REF + "/src/agent")):
        m = types.ModuleType(name)
        m.__path__ = [path]
        sys.modules[name] = m
    gym = types.ModuleType("gym")
    sp = types.ModuleType("gym.spaces")
    gym.Env = type("Env", (), {"close": lambda self: None})
    sp.Box = lambda low, high, shape, dtype: types.SimpleNamespace(shape=shape)
    sp.Discrete = lambda n: types.SimpleNamespace(n=n)
    gym.spaces = sp
    sys.modules.update({"gym": gym, "gym.spaces": sp})
    # cloud / logging deps of ppo_agent.py (never used by the PPO arithmetic)
    boto3 = types.ModuleType("boto3")
    boto3.client = lambda *a, **k: None
    botocore = types.ModuleType("botocore")
    bcfg = types.ModuleType("botocore.config")
    bcfg.Config = lambda *a, **k: None
    botocore.config = bcfg
    botocore.exceptions = types.SimpleNamespace(ClientError=Exception)
    tbx = types.ModuleType("tensorboardX")
    rw = types.ModuleType("tensorboardX.record_writer")
    rw.RecordWriter = type("RecordWriter", (), {"__init__": lambda self, *a, **k: None})
    rw.S3RecordWriter = type("S3RecordWriter", (), {"__init__": lambda self, *a, **k: None})
    tbx.record_writer = rw

    class _SW:
        def __init__(self, *a, **k):
            pass

        def add_scalar(self, *a, **k):
            pass

        def close(self):
            pass

    tbx.SummaryWriter = _SW
    sys.modules.update({"boto3": boto3, "botocore": botocore, "botocore.config": bcfg,
                        "tensorboardX": tbx, "tensorboardX.record_writer": rw})
    import src.moves  # noqa: F401  (before src.board: circular import)


_shim()
import torch  # noqa: E402
from src.board.immutable_board import (ImmutableBoard, execute_full_move_on_board_copy)  # noqa: E402
from src.moves.get_all_moves import get_all_possible_moves  # noqa: E402
from src.players.player import Player  # noqa: E402
from src.ai.batching import generate_all_board_features  # noqa: E402
from src.environment.backgammon_env import BackgammonEnv  # noqa: E402
from src.environment.vec_bg_env import VectorizedBackgammonEnv  # noqa: E402
from src.agent.policy_network import BackgammonPolicyNetwork  # noqa: E402

torch.set_num_threads(1)


def b52(board: ImmutableBoard) -> np.ndarray:
    t = board.tensor.cpu().numpy().astype(np.int8)
    return np.concatenate([t[0], t[1], t[2, :2], t[3, :2]]).astype(np.int8)


def from52(x: np.ndarray) -> ImmutableBoard:
    t = torch.zeros((4, 24), dtype=torch.int8)
    t[0] = torch.from_numpy(x[:24].astype(np.int8))
    t[1] = torch.from_numpy(x[24:48].astype(np.int8))
    t[2, 0], t[2, 1], t[3, 0], t[3, 1] = int(x[48]), int(x[49]), int(x[50]), int(x[51])
    return ImmutableBoard(t)


def enc(full_move) -> int:
    v = 0
    for i, s in enumerate(full_move.sub_move_commands):
        v |= (int(s.start) | (int(s.end) << 5) | (int(bool(s.hits_blot)) << 10) | (1 << 15)) << (16 * i)
    return v


ALL_ROLLS = [(a, b) for a in range(1, 7) for b in range(1, 7)]


def random_board(rng: np.random.RandomState) -> np.ndarray:
    """A random position with 15 checkers a side (no shared points)."""
    x = np.zeros(52, dtype=np.int8)
    kind = rng.randint(4)   # 0 generic, 1 mover bearing off, 2 bar-heavy, 3 race
    for p in (0, 1):
        home = list(range(18, 24)) if p == 0 else list(range(6))
        left = 15
        if kind == 2 and rng.rand() < 0.7:
            bar = rng.randint(1, 4)
            x[48 + p] = bar
            left -= bar
        if kind in (1, 3) and rng.rand() < 0.8:
            off = rng.randint(0, 15)
            x[50 + p] = off
            left -= off
        pts = home if (kind == 1 or (kind == 3 and rng.rand() < 0.5)) else list(range(24))
        while left > 0:
            q = pts[rng.randint(len(pts))]
            if x[(1 - p) * 24 + q] > 0:
                if rng.rand() < 0.2:
                    pts = list(range(24))
                continue
            k = min(left, rng.randint(1, 4))
            x[p * 24 + q] += k
            left -= k
    return x


def edge_boards():
    """Hand-built edge positions (bar/blocked entry, bear-off farthest/exact, ...)."""
    out = []

    def mk(p1, p2, bar=(0, 0), off=(0, 0)):
        x = np.zeros(52, dtype=np.int8)
        for k, v in p1.items():
            x[k] = v
        for k, v in p2.items():
            x[24 + k] = v
        x[48], x[49] = bar
        x[50], x[51] = off
        return x

    init = b52(ImmutableBoard.initial_board(torch.device("cpu")))
    out.append(init)
    out.append(mk({20: 1}, {5: 15}, off=(14, 0)))                       # last checker
    out.append(mk({18: 1, 20: 1}, {5: 15}, off=(13, 0)))
    out.append(mk({18: 2, 19: 2, 21: 3, 23: 1}, {3: 2, 0: 13}, off=(7, 0)))
    out.append(mk({0: 2, 11: 5, 16: 3}, {0: 0, 1: 2, 2: 2, 3: 2, 4: 2, 5: 2, 12: 5}, bar=(5, 0)))  # closed board
    out.append(mk({0: 2, 11: 5, 16: 3, 18: 3}, {1: 2, 3: 2, 5: 2, 12: 5, 7: 2}, bar=(2, 2)))
    out.append(mk({i: 1 for i in range(0, 22, 2)} | {22: 4}, {i: 1 for i in range(1, 24, 2)} | {23: 4}))
    out.append(mk({5: 2, 6: 2, 7: 2, 8: 2, 9: 2, 10: 2, 12: 3}, {4: 1, 11: 1, 13: 1, 14: 1, 20: 11}))
    out.append(mk({19: 3, 22: 2}, {0: 2, 1: 2, 2: 2, 3: 3, 4: 3, 5: 3}, off=(10, 0)))
    out.append(mk({23: 15}, {0: 15}))
    out.append(mk({18: 15}, {5: 15}))
    out.append(mk({17: 1, 23: 14}, {6: 1, 0: 14}))
    # mirrored P2-centric cases
    out.append(mk({18: 15}, {3: 1}, off=(0, 14)))
    out.append(mk({18: 15}, {5: 1, 3: 1}, off=(0, 13)))
    out.append(mk({20: 2, 22: 2}, {0: 2, 1: 2, 4: 3, 5: 1}, off=(11, 7)))
    return out


def gen_movegen():
    t0 = time.time()
    rows = []   # (board52, player, r0, r1)
    for x in edge_boards():
        for p in (0, 1):
            for r in ALL_ROLLS:
                rows.append((x, p, r[0], r[1]))
    rng = np.random.RandomState(12345)
    for _ in range(1500):
        x = random_board(rng)
        p = rng.randint(2)
        r = ALL_ROLLS[rng.randint(36)]
        rows.append((x, p, r[0], r[1]))
    # positions with > 500 moves (truncation)
    spread = np.zeros(52, dtype=np.int8)
    spread[:15] = 1
    spread[24 + 23] = 15
    rows.append((spread, 0, 1, 1))
    rows.append((spread, 0, 2, 2))
    sp2 = np.zeros(52, dtype=np.int8)
    sp2[24 + 9:24 + 24] = 1
    sp2[0] = 15
    rows.append((sp2, 1, 1, 1))
    boards, players, rolls, counts, offsets, moves = [], [], [], [], [0], []
    for (x, p, a, b) in rows:
        fm = get_all_possible_moves(Player(p), from52(x), [int(a), int(b)])
        boards.append(x)
        players.append(p)
        rolls.append((a, b))
        counts.append(len(fm))
        moves.extend(enc(m) for m in fm)
        offsets.append(len(moves))
    print(f"G1 movegen: {len(rows)} positions, {len(moves)} moves, max {max(counts)} "
          f"({time.time() - t0:.1f}s)")
    return dict(boards=np.array(boards, np.int8), players=np.array(players, np.uint8),
                rolls=np.array(rolls, np.uint8), counts=np.array(counts, np.int32),
                offsets=np.array(offsets, np.int64), moves=np.array(moves, np.uint64))


def gen_traces(n_games=40):
    """G4: BackgammonEnv.seed(s); random legal policy from a separate RandomState."""
    t0 = time.time()
    recs = {k: [] for k in ("game", "step", "mover", "r0", "r1", "n_legal", "action", "reward",
                            "done", "winner", "score", "kind", "board_after", "player_after")}
    first_obs = []
    for g in range(n_games):
        env = BackgammonEnv(match_length=15 if g % 5 else 3, max_legal_moves=500)
        env.seed(g)
        pol = np.random.RandomState(10_000 + g)
        obs = env.reset()
        first_obs.append(obs.numpy().copy())
        games_done = 0
        step = 0
        while games_done < (2 if g % 4 == 0 else 1):
            n = int(env.action_mask.sum().item())
            r0, r1 = env.roll_result
            if n > 0:
                u = pol.rand()
                a = int(pol.randint(n)) if u > 0.03 else int(n + pol.randint(3))   # some invalid actions
            else:
                a = int(pol.randint(500))
            mover = int(env.current_player)
            obs, rew, done, info = env.step(a)
            kind = 3 if (done and float(rew) == 0.0) else (
                1 if info.get("info", "").startswith("No legal") else (2 if info.get("info") == "Invalid action" else 0))
            recs["game"].append(g)
            recs["step"].append(step)
            recs["mover"].append(mover)
            recs["r0"].append(r0)
            recs["r1"].append(r1)
            recs["n_legal"].append(n)
            recs["action"].append(a)
            recs["reward"].append(float(rew))
            recs["done"].append(bool(done))
            recs["winner"].append(int(info["winner"]) if "winner" in info else -1)
            recs["score"].append(int(info.get("game_score", 0)))
            recs["kind"].append(kind)
            recs["board_after"].append(b52(env.board))
            recs["player_after"].append(int(env.current_player))
            step += 1
            if done and kind != 3:
                games_done += 1
        # single-env semantics: one more step after game over resets the game
        _ = env.step(0)
    out = {k: np.array(v) for k, v in recs.items()}
    out["first_obs"] = np.array(first_obs, np.float32)
    print(f"G4 traces: {n_games} games, {len(recs['game'])} steps ({time.time() - t0:.1f}s)")
    return out


def gen_vec_trace(num_envs=4, steps=150):
    """G4b: VectorizedBackgammonEnv with auto-reset.  The reference's envs share ONE
    global numpy stream, consumed env-by-env in lane order each step."""
    np.random.seed(777)
    torch.manual_seed(777)
    venv = VectorizedBackgammonEnv(num_envs=num_envs)
    pol = np.random.RandomState(4242)
    obs0 = venv.reset().numpy().copy()
    acts, rews, dones, obs, boards, nleg = [], [], [], [], [], []
    for _ in range(steps):
        masks = venv.get_action_masks().numpy()
        n = masks.sum(1).astype(int)
        a = np.array([pol.randint(k) if k > 0 else 0 for k in n], np.int64)
        o, r, d, _info = venv.step(a)
        acts.append(a)
        nleg.append(n)
        rews.append(r.numpy().copy())
        dones.append(d.numpy().copy())
        obs.append(o.numpy().copy())
        boards.append(np.stack([b52(e.board) for e in venv.envs]))
    print(f"G4b vec trace: {num_envs} envs x {steps} steps")
    return dict(obs0=obs0, actions=np.array(acts), n_legal=np.array(nleg), rewards=np.array(rews),
                dones=np.array(dones), obs=np.array(obs, np.float32), boards=np.array(boards, np.int8))


def gen_features(mg):
    t0 = time.time()
    idx = np.arange(0, len(mg["counts"]), 7)[:400]
    obs, obs_player = [], []
    aft_rows, aft_pos = [], []
    for i in idx:
        x, p = mg["boards"][i], int(mg["players"][i])
        b = from52(x)
        for cp in (0, 1):
            obs.append(b.get_board_features(Player(cp)).numpy())
            obs_player.append(cp)
        if mg["counts"][i] > 0 and len(aft_pos) < 120:
            fm = get_all_possible_moves(Player(p), b, [int(v) for v in mg["rolls"][i]])
            f = generate_all_board_features(b, Player(p), fm, [int(v) for v in mg["rolls"][i]]).numpy()
            aft_rows.append(f)
            aft_pos.append(i)
    aft = np.concatenate(aft_rows).astype(np.float32)
    lens = np.array([len(r) for r in aft_rows], np.int32)
    # afterstate boards for the same positions (execute_full_move_on_board_copy)
    aft_boards = []
    for i in aft_pos:
        b = from52(mg["boards"][i])
        fm = get_all_possible_moves(Player(int(mg["players"][i])), b, [int(v) for v in mg["rolls"][i]])
        aft_boards.extend(b52(execute_full_move_on_board_copy(b, m)) for m in fm)
    print(f"G2 features: {len(obs)} obs, {len(aft)} afterstate rows ({time.time() - t0:.1f}s)")
    return dict(obs_idx=np.repeat(idx, 2), obs_player=np.array(obs_player, np.uint8),
                obs=np.array(obs, np.float32), aft_pos=np.array(aft_pos, np.int64), aft_lens=lens,
                aft=aft, aft_boards=np.array(aft_boards, np.int8))


def gen_dice():
    streams = []
    for s in range(8):
        env = BackgammonEnv()
        env.seed(s)
        d = []
        for _ in range(500):
            env.roll_dice()
            d.extend(env.roll_result)
        streams.append(d)
    print("G3 dice: 8 seeds x 1000 dice")
    return dict(seeds=np.arange(8), dice=np.array(streams, np.uint8))


def gen_mlp(feat):
    out = {}
    x = torch.from_numpy(np.concatenate([feat["obs"][:600], feat["aft"][:424]]))
    out["x"] = x.numpy()
    for H, seed in ((40, 0), (128, 1)):
        torch.manual_seed(seed)
        net = BackgammonPolicyNetwork(input_size=198, hidden_size=H, action_size=500)
        with torch.no_grad():
            logits, values = net(x)
        for k, v in net.state_dict().items():
            out[f"h{H}_{k}"] = v.numpy()
        out[f"h{H}_logits"] = logits.numpy()
        out[f"h{H}_values"] = values.numpy()
    print("G5 mlp: H in {40,128}, 1024 rows")
    return out


def gen_ppo(feat, mg):
    """G6: select_action + update() of the reference agent on CPU."""
    import src.agent.ppo_agent as pa
    torch.manual_seed(3)
    agent = pa.BackgammonPPOAgent(action_size=500, device=torch.device("cpu"))
    init_sd = {k: v.clone().numpy() for k, v in agent.policy_network.state_dict().items()}
    N, T = 8, 16
    obs_all = torch.from_numpy(feat["obs"][: N * T])
    counts = np.minimum(mg["counts"][: N * T], 500)
    masks_all = torch.zeros(N * T, 500)
    for i, c in enumerate(counts):
        masks_all[i, : max(int(c), 1)] = 1.0
    rng = np.random.RandomState(9)
    rewards = rng.choice([0.0, 0.0, 0.0, 1.0, -1.0, 1.5], size=N * T).astype(np.float32)
    dones = (rng.rand(N * T) < 0.15)
    torch.manual_seed(11)
    actions = []
    for t in range(T):
        a = agent.select_action(obs_all[t * N:(t + 1) * N], masks_all[t * N:(t + 1) * N])
        actions.append(a)
        for i in range(N):
            agent.memory[-N + i]["reward"] = torch.tensor([rewards[t * N + i]])
            agent.memory[-N + i]["done"] = torch.tensor([bool(dones[t * N + i])])
    old_logp = torch.cat([m["action_log_prob"] for m in agent.memory]).detach().numpy()
    old_v = torch.cat([m["state_value"] for m in agent.memory]).detach().numpy()
    agent.update()
    out = dict(obs=obs_all.numpy(), masks=masks_all.numpy(), rewards=rewards, dones=dones,
               actions=np.concatenate(actions).astype(np.int64), old_logp=old_logp, old_v=old_v,
               losses=np.array([agent.last_policy_loss, agent.last_value_loss,
                                agent.last_entropy_loss, agent.last_total_loss], np.float64))
    for k, v in init_sd.items():
        out["init_" + k] = v
    for k, v in agent.policy_network.state_dict().items():
        out["final_" + k] = v.numpy()
    # select_action distribution on fixed logits (masked softmax with log(mask+1e-45))
    lg = torch.randn(6, 500, generator=torch.Generator().manual_seed(5))
    mk = masks_all[:6]
    out["sa_logits"] = lg.numpy()
    out["sa_masks"] = mk.numpy()
    out["sa_probs"] = torch.softmax(lg + (mk + 1e-45).log(), dim=-1).numpy()
    print("G6 ppo: select_action x16 + update() on 128 samples")
    return out


def gen_ppo_batch(mg, mode: str, N=16, T=64):
    """G6b/G6c: the reference agent's update() on a 1,024-row batch built from
    G1 positions, autocast switched to fp32 (mode "fp32") or fp16 ("fp16", the
    dtype CUDA autocast uses).  Rows carry their board + player + legal count
    (mask = 1 for the first n, all-zero when n == 0, as backgammon_env.py:207-243),
    so the GPU trainer can rebuild them as 64-byte records."""
    import src.agent.ppo_agent as pa
    from torch.amp import autocast as _ac
    if mode == "fp32":
        pa.autocast = lambda device_type, **k: _ac(device_type, enabled=False)
    else:
        pa.autocast = lambda device_type, **k: _ac(device_type, dtype=torch.float16)
    rows = np.arange(N * T) * 2 % len(mg["counts"])
    boards = mg["boards"][rows]
    players = mg["players"][rows]
    counts = np.minimum(mg["counts"][rows], 500).astype(np.int32)
    obs = torch.stack([from52(boards[i]).get_board_features(Player(int(players[i]))) for i in range(N * T)]).float()
    masks = torch.zeros(N * T, 500)
    for i, c in enumerate(counts):
        masks[i, :int(c)] = 1.0
    torch.manual_seed(21)
    agent = pa.BackgammonPPOAgent(action_size=500, device=torch.device("cpu"))
    init_sd = {k: v.clone().numpy() for k, v in agent.policy_network.state_dict().items()}
    rng = np.random.RandomState(31)
    rewards = rng.choice([0.0] * 8 + [1.0, -1.0, 1.5, 2.0, -1.5], size=N * T).astype(np.float32)
    dones = rng.rand(N * T) < 0.1
    torch.manual_seed(41)
    actions = []
    for t in range(T):
        a = agent.select_action(obs[t * N:(t + 1) * N], masks[t * N:(t + 1) * N])
        actions.append(a)
        for i in range(N):
            agent.memory[-N + i]["reward"] = torch.tensor([rewards[t * N + i]])
            agent.memory[-N + i]["done"] = torch.tensor([bool(dones[t * N + i])])
    old_logp = torch.cat([m["action_log_prob"] for m in agent.memory]).detach().numpy()
    old_v = torch.cat([m["state_value"] for m in agent.memory]).detach().numpy()
    agent.update()
    pa.autocast = _ac
    out = dict(N=N, T=T, boards=boards, players=players, counts=counts, obs=obs.numpy(), rewards=rewards,
               dones=dones, actions=np.concatenate(actions).astype(np.int64), old_logp=old_logp, old_v=old_v,
               losses=np.array([agent.last_policy_loss, agent.last_value_loss,
                                agent.last_entropy_loss, agent.last_total_loss], np.float64),
               entropy_coef=agent.entropy_coef)
    for k, v in init_sd.items():
        out["init_" + k] = v
    for k, v in agent.policy_network.state_dict().items():
        out["final_" + k] = v.numpy()
    print(f"G6 ppo ({mode}): update() on {N * T} rows, losses {out['losses']}")
    return out


class _FixedBarOff:
    """render() indexes board.tensor[player, BAR=24] / [player, BEAR_OFF=25] on a
    (4,24) tensor and raises IndexError.  This read-only view maps
    those two indices to the bar / off channels (tensor[2, p], tensor[3, p]), the
    evident intent, so the fixed layout can be captured; the reference code runs
    unmodified."""

    def __init__(self, t):
        self.t = t

    def __getitem__(self, ix):
        if isinstance(ix, tuple) and len(ix) == 2 and isinstance(ix[1], int) and ix[1] >= 24:
            return self.t[2 if ix[1] == 24 else 3, ix[0]]
        return self.t[ix]


def gen_misc(mg):
    """G7: dice-roll table, board_to_string / render text, env.legal_moves."""
    import contextlib
    import io
    from src.moves.get_all_dice_rolls import get_all_dice_rolls_tensor
    from src.board.immutable_board import board_to_string
    rolls, probs = get_all_dice_rolls_tensor()
    out = dict(rolls=rolls.numpy(), probs=probs.numpy())
    idx = list(range(0, len(edge_boards()) * 72, 72)) + list(range(1100, 1400, 10))
    strs, rend = [], []
    env = BackgammonEnv()
    for i in idx:
        b = from52(mg["boards"][i])
        strs.append(board_to_string(b))
        env.board = types.SimpleNamespace(tensor=_FixedBarOff(b.tensor))
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            env.render()
        rend.append(buf.getvalue())
    out.update(str_idx=np.array(idx, np.int64), board_strings=np.array(strs), render=np.array(rend))
    # legal_moves along seeded games (single env, random legal policy)
    lm_seed, lm_step, lm_moves, lm_off = [], [], [], [0]
    for s in range(6):
        env = BackgammonEnv()
        env.seed(100 + s)
        pol = np.random.RandomState(500 + s)
        env.reset()
        for step in range(60):
            mv = [enc(m) for m in env.legal_moves]
            lm_seed.append(100 + s)
            lm_step.append(step)
            lm_moves.extend(mv)
            lm_off.append(len(lm_moves))
            n = len(mv)
            _, _, done, _ = env.step(int(pol.randint(n)) if n else 0)
            if done:
                env.reset()
    out.update(lm_seed=np.array(lm_seed), lm_step=np.array(lm_step), lm_moves=np.array(lm_moves, np.uint64),
               lm_off=np.array(lm_off, np.int64))
    print(f"G7 misc: 21 rolls, {len(idx)} board strings / renders, {len(lm_step)} legal_moves lists")
    return out


def main():
    want = set(sys.argv[1:])
    if want:
        mg = dict(np.load(os.path.join(OUT, "movegen.npz")))
        if "ppo_fp32" in want:
            np.savez_compressed(os.path.join(OUT, "ppo_fp32.npz"), **gen_ppo_batch(mg, "fp32"))
        if "ppo_fp16" in want:
            np.savez_compressed(os.path.join(OUT, "ppo_fp16.npz"), **gen_ppo_batch(mg, "fp16"))
        if "misc" in want:
            np.savez_compressed(os.path.join(OUT, "misc.npz"), **gen_misc(mg))
        return
    mg = gen_movegen()
    np.savez_compressed(os.path.join(OUT, "movegen.npz"), **mg)
    feat = gen_features(mg)
    np.savez_compressed(os.path.join(OUT, "features.npz"), **feat)
    np.savez_compressed(os.path.join(OUT, "dice.npz"), **gen_dice())
    tr = gen_traces()
    tr.update({"vec_" + k: v for k, v in gen_vec_trace().items()})
    np.savez_compressed(os.path.join(OUT, "traces.npz"), **tr)
    np.savez_compressed(os.path.join(OUT, "mlp.npz"), **gen_mlp(feat))
    np.savez_compressed(os.path.join(OUT, "ppo.npz"), **gen_ppo(feat, mg))
    np.savez_compressed(os.path.join(OUT, "ppo_fp32.npz"), **gen_ppo_batch(mg, "fp32"))
    np.savez_compressed(os.path.join(OUT, "ppo_fp16.npz"), **gen_ppo_batch(mg, "fp16"))
    np.savez_compressed(os.path.join(OUT, "misc.npz"), **gen_misc(mg))


if __name__ == "__main__":
    main()
