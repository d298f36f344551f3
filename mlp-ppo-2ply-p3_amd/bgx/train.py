"""GPU-resident PPO self-play trainer (the reference's train.py:30-123 loop,
ppo_agent.py:218-366 update) on the bgx engine.

Rollout: every step the fused policy kernel (bgx_policy_act) samples an
action for all B lanes from their 64-byte lane records, the engine steps them,
and the step's records / actions / log-probs / values / rewards / dones are
kept in device buffers [T, B] (records are int8 boards: 64 B per sample instead
of the reference's 792-byte fp32 observation); optionally mirrored to pinned
host memory on a side stream.

Update: returns, global normalisation, advantages = R_hat - V_old, then
NUM_EPOCHS full-batch epochs exactly like ppo_agent.py:268-305 (autocast +
GradScaler + Adam, clip 0.25, 0.5*MSE, -c_ent*H) but computed in chunks with
gradient accumulation (features re-encoded from the stored records by the HIP
encoder) and ONE all-reduce of the gradients per epoch across ranks.

Entropy coefficient (`entropy_anneal`): the reference's update always calls
update_entropy_coef (ppo_agent.py:193-197), which anneals by
`agent.total_episodes`.  Its vectorised driver train.py never increments that
counter (it counts a module-global `total_episodes`, train.py:74), so under
train.py the coefficient stays at ENTROPY_COEF_START = 0.15 for the whole run;
train_single.py increments `agent.total_episodes` per episode (train_single.py:78)
and the coefficient anneals to 0.01 over 400,000 episodes.  PPOTrainer restates
train.py, so `entropy_anneal="train"` (constant 0.15) is the default;
`"train_single"` anneals by the episodes finished in the rollouts.

Returns: `returns="lane"` (default) discounts within each game lane;
`returns="reference"` reproduces the reference's quirk of discounting over the
flat step-major memory in which the environments are interleaved
(ppo_agent.py:206-216).

    python -m bgx.train --batch 65536 --horizon 64 --updates 10 [--metrics m.jsonl]
    torchrun --nproc-per-node 8 -m bgx.train ...            (one process per GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F
from torch.amp import GradScaler, autocast
from torch.distributions import Categorical

import ctypes

from . import _lib
from ._lib import check
from .engine import Engine, encode_records
from .graphs import capture
from .hostcopy import HostMirror
from .policy import PolicyNet, MASK_LOG
from .ppo import (EPS_CLIP, GAMMA, LEARNING_RATE, NUM_EPOCHS, VALUE_LOSS_COEF, ENTROPY_COEF_START,
                  ENTROPY_COEF_END, ENTROPY_ANNEAL_EPISODES, allreduce_mean_, global_normalize, _world)


def lane_returns(rewards: torch.Tensor, dones: torch.Tensor, gamma: float = GAMMA) -> torch.Tensor:
    """R_t = r_t + gamma * R_{t+1}, reset at done, per lane; [T, B].  On the GPU one HIP
    kernel (bgx_lane_returns, the same fp32 roundings as the torch loop below, which
    stays as the CPU path and the tests' reference)."""
    if rewards.is_cuda and rewards.dtype == torch.float32 and dones.dtype == torch.uint8:
        r, d = rewards.contiguous(), dones.contiguous()
        out = torch.empty_like(r)
        T, B = r.shape[0], r[0].numel()
        check(_lib.load().bgx_lane_returns(ctypes.c_void_p(r.data_ptr()), ctypes.c_void_p(d.data_ptr()), T, B,
                                           float(gamma), ctypes.c_void_p(out.data_ptr()),
                                           ctypes.c_void_p(torch.cuda.current_stream(r.device).cuda_stream)),
              "bgx_lane_returns")
        return out
    return _lane_returns_torch(rewards, dones, gamma)


def _lane_returns_torch(rewards: torch.Tensor, dones: torch.Tensor, gamma: float = GAMMA) -> torch.Tensor:
    T = rewards.shape[0]
    out = torch.empty_like(rewards)
    R = torch.zeros_like(rewards[0])
    for t in range(T - 1, -1, -1):
        R = torch.where(dones[t].bool(), torch.zeros_like(R), R)
        R = rewards[t] + gamma * R
        out[t] = R
    return out


EPISODE_STATS = ("episodes", "episode_reward_sum", "wins", "p1_wins", "gammons", "backgammons")


def episode_stats_records(rewards: torch.Tensor, dones: torch.Tensor, records: torch.Tensor,
                          carry: torch.Tensor) -> torch.Tensor:
    """episode_stats with the movers read from the [T, B, 64] rollout records (byte 52).
    On the GPU one HIP kernel walks each lane's T steps (bgx_episode_stats: the same sums,
    exact in fp64 in any order) instead of ~25 torch launches over [T, B]."""
    if (rewards.is_cuda and rewards.dtype == torch.float32 and dones.dtype == torch.uint8
            and records.dtype == torch.uint8 and carry.dtype == torch.float64 and carry.is_contiguous()
            and rewards.is_contiguous() and dones.is_contiguous() and records.is_contiguous()):
        T, B = rewards.shape
        L = _lib.load()
        ws = torch.empty(max(int(L.bgx_episode_stats_workspace(B)) // 8, 1), dtype=torch.float64, device=rewards.device)
        out = torch.empty(len(EPISODE_STATS), dtype=torch.float64, device=rewards.device)
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        check(L.bgx_episode_stats(p(rewards), p(dones), p(records), p(carry), T, B, p(ws), p(out),
                                  ctypes.c_void_p(torch.cuda.current_stream(rewards.device).cuda_stream)),
              "bgx_episode_stats")
        return out
    return episode_stats(rewards, dones, records[:, :, 52], carry)


def episode_stats(rewards: torch.Tensor, dones: torch.Tensor, movers: torch.Tensor,
                  carry: torch.Tensor) -> torch.Tensor:
    """The reference loop's per-env episode accounting (train.py:55-99) over a
    [T, B] rollout, on the device without a per-step loop.

    `carry` [B] (fp64) is each lane's reward accumulated in its unfinished
    episode (`episode_rewards`, train.py:58) and is updated in place.  Returns
    the sums named by EPISODE_STATS as one fp64 tensor: finished episodes,
    their summed episode rewards (train.py:73), wins as the reference counts
    them (`info["winner"] == info["current_player"]`, train.py:74-77: the
    mover of a winning step, i.e. a done with a positive reward), wins by
    PLAYER1 (`log_metrics`' "1 if Player1 wins", ppo_agent.py:494), and
    gammon / backgammon wins (rewards 1.5 / 2.0, backgammon_env.py:26-28).
    `movers` [T, B] is the player to move before each step (record byte 52).
    """
    T, B = rewards.shape
    d = dones.bool()
    r = rewards.double()
    seg = torch.cumsum(d, 0, dtype=torch.int64) - d.long()      # episodes finished before step t
    idx = seg + torch.arange(B, device=r.device, dtype=torch.int64) * (T + 1)
    sums = torch.zeros(B * (T + 1), dtype=torch.float64, device=r.device)
    sums.scatter_add_(0, idx.reshape(-1), r.reshape(-1))
    sums = sums.view(B, T + 1)
    sums[:, 0] += carry
    n = d.sum(0, dtype=torch.int64)
    open_ep = sums.gather(1, n[:, None]).squeeze(1)
    finished = sums.sum(1) - open_ep
    carry.copy_(open_ep)
    return torch.stack([n.sum().double(), finished.sum(),
                        (d & (r > 0)).sum().double(), (d & (r > 0) & (movers == 0)).sum().double(),
                        (d & (r == 1.5)).sum().double(), (d & (r == 2.0)).sum().double()])


def reference_returns(rewards: torch.Tensor, dones: torch.Tensor, gamma: float = GAMMA) -> torch.Tensor:
    """ppo_agent.py:206-216 over the flat step-major memory (envs interleaved)."""
    flat_r = rewards.reshape(-1).double().cpu().numpy()
    flat_d = dones.reshape(-1).cpu().numpy()
    out = [0.0] * len(flat_r)
    R = 0.0
    for k in range(len(flat_r) - 1, -1, -1):
        if flat_d[k]:
            R = 0.0
        R = flat_r[k] + gamma * R
        out[k] = R
    return torch.tensor(out, dtype=torch.float32, device=rewards.device).view_as(rewards)


def entropy_coef_after_update(mode: str, total_episodes: int) -> float:
    """update_entropy_coef (ppo_agent.py:193-197) as each reference driver feeds it:
    train.py leaves agent.total_episodes at 0 (it increments a module global,
    train.py:74), so the coefficient stays at the start value; train_single.py
    counts every episode into it (train_single.py:78)."""
    episodes = total_episodes if mode == "train_single" else 0
    progress = min(1.0, episodes / ENTROPY_ANNEAL_EPISODES)
    return ENTROPY_COEF_START - progress * (ENTROPY_COEF_START - ENTROPY_COEF_END)


def features_and_masks(records: torch.Tensor, n_actions: int):
    feats = encode_records(records)
    counts = records[:, 60].to(torch.int32) | (records[:, 61].to(torch.int32) << 8)
    legal = torch.arange(n_actions, device=records.device)[None, :] < counts[:, None]
    return feats, legal


def _is_policy_mlp(net) -> bool:
    """The manual fp16 epoch needs exactly relu(fc1) -> {action_head, value_head}."""
    return (isinstance(net, PolicyNet) and type(net).forward is PolicyNet.forward
            and all(getattr(net, k).bias is not None for k in ("fc1", "action_head", "value_head"))
            and net.fc1.out_features % 8 == 0 and net.fc1.out_features <= 256)     # bgx_relu_backward


class _PPOHead(torch.autograd.Function):
    """The loss head of ppo_epoch on the HIP kernel bgx_ppo_head: forward computes
    the per-row losses' sums AND the gradients w.r.t. logits and values (already
    multiplied by `gscale` = GradScaler scale / n_total); backward hands them out.
    Call .backward() on the (zero) output directly: the incoming gradient is
    taken to be 1."""

    @staticmethod
    def forward(ctx, logits, values, records, actions, old_logp, returns, adv, coefs, sums):
        eps, c_v, c_e, gscale = coefs
        if logits.dtype not in (torch.float16, torch.float32) or values.dtype != logits.dtype:
            raise TypeError(f"bgx_ppo_head: logits/values must be fp16 or fp32 alike, got {logits.dtype}/{values.dtype}")
        logits, values = logits.contiguous(), values.contiguous()
        n, A = logits.shape
        dlog = torch.empty_like(logits)
        dval = torch.empty_like(values)
        L = _lib.load()
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        check(L.bgx_ppo_head(p(logits), 0 if logits.dtype == torch.float32 else 1, A, p(values),
                             p(records), p(actions), p(old_logp), p(returns), p(adv), n, A, eps, c_v, c_e, gscale,
                             p(dlog), A, p(dval), p(sums),
                             ctypes.c_void_p(torch.cuda.current_stream(logits.device).cuda_stream)), "bgx_ppo_head")
        ctx.save_for_backward(dlog, dval)
        return logits.new_zeros((), dtype=torch.float32)

    @staticmethod
    def backward(ctx, g):
        dlog, dval = ctx.saved_tensors
        return dlog, dval, None, None, None, None, None, None, None


def ppo_epoch(net: nn.Module, optimizer, scaler, chunks, n_total: int, entropy_coef: float, group=None,
              amp: bool = True, fused: bool | None = None, step: bool = True, sync: bool = True, guard=None,
              fused_head: bool = True, scale_hint=None, parts=None):
    """One full-batch PPO epoch (ppo_agent.py:268-305) over `chunks` =
    iterable of (features, legal_mask, actions, old_logp, returns, advantages
    [, records]), with gradient accumulation and one all-reduce.  Returns loss
    parts (sync=False with `parts` given: added on the device to that fp64 [4] tensor, which
    is returned).  fused (default: on the GPU when the chunks carry their 64-byte
    records): the loss head runs as one HIP kernel (bgx_ppo_head) instead of the
    torch formulation below, which stays as its reference (tests compare them)."""
    optimizer.zero_grad(set_to_none=True)
    acc = torch.zeros(4, dtype=torch.float64)
    dev = next(net.parameters()).device
    dev_type = dev.type
    if fused is None:
        fused = dev_type == "cuda"
    if fused:
        return _ppo_epoch_fused(net, optimizer, scaler, chunks, n_total, entropy_coef, group, amp, step, sync, guard,
                                fused_head, scale_hint, parts)
    for feats, legal, actions, old_logp, returns, adv, *_ in chunks:
        w = feats.shape[0] / n_total
        with autocast(device_type=dev_type, enabled=amp):
            logits, values = net(feats)
            masked = torch.where(legal, logits.float(), logits.float() + MASK_LOG)
            # torch.distributions.Categorical(probs) as ppo_agent.py:273-291: log_prob and
            # entropy on log(clamp(probs, eps, 1 - eps))
            dist_ = Categorical(torch.softmax(masked, dim=-1))
            new_logp = dist_.log_prob(actions.long())
            ratios = torch.exp(new_logp - old_logp)
            surr1 = ratios * adv
            surr2 = torch.clamp(ratios, 1 - EPS_CLIP, 1 + EPS_CLIP) * adv
            policy_loss = -torch.min(surr1, surr2).mean()
            value_loss = nn.functional.mse_loss(values.float().squeeze(-1), returns)
            entropy = dist_.entropy().mean()
            loss = policy_loss + VALUE_LOSS_COEF * value_loss - entropy_coef * entropy
        scaler.scale(loss * w).backward()
        acc += torch.tensor([policy_loss.item(), value_loss.item(), entropy.item(), loss.item()],
                            dtype=torch.float64) * w
    if step:
        allreduce_mean_([p.grad for p in net.parameters() if p.grad is not None], group)
        scaler.step(optimizer)
        scaler.update()
    return acc


PPO_COLSUM_BLOCKS = 2048       # include/bgx.h BGX_PPO_COLSUM_BLOCKS
RELU_BLOCKS = 1024             # bgx_relu_backward's grid (rows of its column-sum partials)


def _wgrad(g: torch.Tensor, x: torch.Tensor, splits: int = 64) -> torch.Tensor:
    """g^T x (fp16 [m, N], [m, K]) -> fp32 [N, K]: the weight gradient of a
    linear layer, a K = m reduction.  hipBLASLt runs this shape (m = 2^20,
    N x K = 512 x 128) at ~70 TFLOP/s; as `splits` batched GEMMs over row slices
    (fp32 partials: no fp16 overflow however many rows a slice sums) plus an
    fp32 sum of the partials it runs 7-10x faster (tools/gemm_probe.py)."""
    m = g.shape[0]
    if m % splits or m < 64 * splits:
        return torch.mm(g.t(), x, out_dtype=torch.float32)
    return torch.bmm(g.view(splits, m // splits, -1).transpose(1, 2), x.view(splits, m // splits, -1),
                     out_dtype=torch.float32).sum(0)


# Rows per update of the reference (T_HORIZON x NUM_ENVS, agent/config.py:4-6).  The
# manual fp16 epoch writes per-row gradients at GradScaler scale / min(n, REF_ROWS):
# the per-row fp16 magnitudes of the reference's own update, whatever the batch
# (scale / n at 4M rows would push them into fp16's subnormal range); the remaining
# factor min(n, REF_ROWS) / n is applied in fp32 to the summed weight gradients.
REF_ROWS = 4096

# Feature row width of the manual fp16 epoch: 208 = 198 features + 10 zero columns,
# so fc1's weight-gradient GEMM reads 16-byte aligned rows (396-byte rows keep
# hipBLASLt off its vector-load kernels; tools/gemm_probe_pad.py).  The zero columns
# meet zero weight columns: every product is unchanged.
FEAT_W = 208


def _ppo_epoch_amp_manual(net, chunks, n_total, coefs, sums):
    """The fp16-autocast epoch's forward and backward written out (the same
    fp16 GEMMs, fp32 accumulation): [action_head; value_head] as ONE GEMM
    padded to 512 outputs (hipBLASLt: 0.35 vs 0.74 ms at 2^20 x 500), the loss
    head kernel reading the logits / writing their gradient in place (row stride
    512), ReLU backward on the stored activations, and split-K weight
    gradients (_wgrad).  Gradients land in p.grad as fp32, as autograd's would."""
    eps, c_v, c_e, gscale = coefs              # gscale = GradScaler scale / n_total
    row_scale = gscale * n_total / min(n_total, REF_ROWS)
    post = min(n_total, REF_ROWS) / n_total    # fp32 factor back to scale / n_total
    W1, b1 = net.fc1.weight, net.fc1.bias
    Wa, ba = net.action_head.weight, net.action_head.bias
    wv, bv = net.value_head.weight, net.value_head.bias
    A, Hd = Wa.shape
    Ap = (A + 1 + 31) // 32 * 32
    dev = W1.device
    with torch.no_grad():
        W1h, b1h = W1.half(), b1.half()
        F_in = W1.shape[1]
        Kw = None                                   # padded feature width of the chunks, if any
        W2h = torch.zeros(Ap, Hd, dtype=torch.float16, device=dev)
        b2h = torch.zeros(Ap, dtype=torch.float16, device=dev)
        W2h[:A] = Wa.half(); W2h[A] = wv[0].half()
        b2h[:A] = ba.half(); b2h[A] = bv[0].half()
        gW1 = torch.zeros_like(W1); gb1 = torch.zeros_like(b1)
        gW2 = torch.zeros(Ap, Hd, dtype=torch.float32, device=dev)
        gb2 = torch.zeros(Ap, dtype=torch.float32, device=dev)
        L = _lib.load()
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        colsum = torch.empty(PPO_COLSUM_BLOCKS, 512, dtype=torch.float32, device=dev)
        fc1_rec = L.bgx_fc1_packed_size(Hd) > 0        # else the GEMM over the feature rows
        if fc1_rec:                                 # W1h in the record kernel's fragment order
            w1pack = torch.empty(L.bgx_fc1_packed_size(Hd), dtype=torch.uint8, device=dev)
            check(L.bgx_fc1_pack(p(W1h), Hd, p(w1pack), stream), "bgx_fc1_pack")
        hsum = torch.empty(RELU_BLOCKS, Hd, dtype=torch.float32, device=dev)
        for feats, legal, actions, old_logp, returns, adv, records, *_ in chunks:
            x = feats.half()
            if x.shape[1] != F_in and Kw is None:   # zero-padded rows: zero weight columns to match
                Kw = x.shape[1]
                W1h = torch.nn.functional.pad(W1h, (0, Kw - F_in))
                gW1 = torch.zeros(W1.shape[0], Kw, dtype=torch.float32, device=dev)
            if fc1_rec:                             # fc1 forward from the 64-byte records (no feature read)
                h = torch.empty(x.shape[0], Hd, dtype=torch.float16, device=dev)
                rec = records.contiguous()
                check(L.bgx_fc1_records(p(rec), rec.shape[0], p(w1pack), p(b1h), Hd, p(h), stream),
                      "bgx_fc1_records")
            else:                                   # bias + ReLU in the GEMM epilogue (relu commutes with
                h = torch._addmm_activation(b1h, x, W1h.t())     # the fp16 rounding)
            y = F.linear(h, W2h, b2h)                      # [m, Ap]: logits | value | 0
            m = y.shape[0]
            vals = y[:, A].contiguous()
            dy = torch.empty_like(y)
            dval = torch.empty_like(vals)
            # dy = [dlogits | dvalue | 0] written by the kernel, with its column sums
            check(L.bgx_ppo_head_ex(p(y), 1, Ap, p(vals), p(records.contiguous()),
                                    p(actions.to(torch.int32).contiguous()), p(old_logp.float().contiguous()),
                                    p(returns.float().contiguous()), p(adv.float().contiguous()), m, A, eps, c_v,
                                    c_e, row_scale, p(dy), Ap, p(dval), p(sums), 1, p(colsum), stream),
                  "bgx_ppo_head_ex")
            gW2 += _wgrad(dy, h)
            gb2 += colsum.sum(0)[:Ap]
            dh = dy @ W2h
            # relu backward (grad where out > 0) in place + the bias gradient's column sums
            check(L.bgx_relu_backward(p(dh), p(h), m, Hd, p(hsum), RELU_BLOCKS, stream), "bgx_relu_backward")
            gW1 += _wgrad(dh, x)
            gb1 += hsum.sum(0)
        if post != 1.0:
            for t in (gW1, gb1, gW2, gb2):
                t.mul_(post)
    W1.grad, b1.grad = (gW1 if Kw is None else gW1[:, :F_in].contiguous()), gb1
    Wa.grad, ba.grad = gW2[:A].contiguous(), gb2[:A].contiguous()
    wv.grad, bv.grad = gW2[A:A + 1].contiguous(), gb2[A:A + 1].contiguous()


PPO_GW2_TASK_TILES = 32        # include/bgx.h BGX_PPO_GW2_TASK_TILES
FEAT_BIAS_COL = 198            # the ones column of the 208-wide rows: gW1[:, 198] = gb1


def ppo_row_plan(records: torch.Tensor, n_actions: int = 500, out=None):
    """ppo_row_plan_torch on the GPU as three HIP launches (bgx_ppo_plan: a stable
    counting sort by class plus the plan from the class totals), no host sync; the
    torch form on the CPU.  out: (perm int32[m], plan int32[33], row_plan int32[8])
    to write into (the graphed update's persistent buffers)."""
    if not records.is_cuda:
        return ppo_row_plan_torch(records, n_actions)
    m = records.shape[0]
    L = _lib.load()
    dev = records.device
    rec = records.contiguous()
    ws = torch.empty(max(int(L.bgx_ppo_plan_workspace(m)) // 4, 1), dtype=torch.int32, device=dev)
    if out is not None:
        perm, plan, row_plan = out
    else:
        perm = torch.empty(m, dtype=torch.int32, device=dev)
        plan = torch.empty(33, dtype=torch.int32, device=dev)
        row_plan = torch.empty(8, dtype=torch.int32, device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    check(L.bgx_ppo_plan(p(rec), m, n_actions, p(ws), p(perm), p(plan), p(row_plan),
                         ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "bgx_ppo_plan")
    return perm, plan, row_plan


def ppo_row_plan_torch(records: torch.Tensor, n_actions: int = 500):
    """Row order and work plan of bgx_ppo_rows / bgx_ppo_gw2 for one chunk of
    rollout rows (computed once per update; the records do not change across
    epochs).  A row needs the 32-action tiles holding its legal columns
    (ceil(cnt / 32); all 16 when cnt = 0, every action then being masked by the
    same constant); rows are sorted by that count (stable).  plan = the k_ppo_gw2
    task prefix per action tile (17) and the first row tile (in sorted order) that
    reaches each action tile (16); row_plan = the row tiles [lo, hi) of the
    bgx_ppo_rows variants for at most 1, 2, 4 and 16 leading action tiles.  Device
    tensors only: no host sync."""
    m = records.shape[0]
    cnt = records[:, 60].to(torch.int32) | (records[:, 61].to(torch.int32) << 8)
    lim = torch.where(cnt == 0, torch.full_like(cnt, n_actions), cnt.clamp(max=n_actions))
    cls = ((lim + 31) // 32).to(torch.uint8)
    perm = torch.argsort(cls, stable=True).to(torch.int32)
    cum = torch.cumsum(torch.bincount(cls, minlength=17), 0)
    start = torch.div(cum[:16], 32, rounding_mode="floor")
    start[15] = 0                                     # the value column's tile: every row
    ntiles = (m + 31) // 32
    # tasks of tile o: the kTS-aligned row groups that hold a row tile >= start[o]
    tasks = (ntiles + PPO_GW2_TASK_TILES - 1) // PPO_GW2_TASK_TILES - torch.div(start, PPO_GW2_TASK_TILES,
                                                                                rounding_mode="floor")
    pre = torch.cat([torch.zeros(1, dtype=tasks.dtype, device=tasks.device), torch.cumsum(tasks, 0)])
    # row tiles whose last (largest) row needs <= k tiles: cum[k] // 32, all of them at cum[k] == m
    e = torch.where(cum[[1, 2, 4]] >= m, torch.full_like(cum[[1, 2, 4]], ntiles), cum[[1, 2, 4]] // 32)
    z = torch.zeros(1, dtype=e.dtype, device=e.device)
    nt = torch.full_like(z, ntiles)
    row_plan = torch.stack([z[0], e[0], e[0], e[1], e[1], e[2], e[2], nt[0]]).to(torch.int32).contiguous()
    return perm, torch.cat([pre, start]).to(torch.int32).contiguous(), row_plan


def gather_rollout(perm, recs, acts, old, R, adv, out=None):
    """Rows perm[i] of the records and the four per-row fields, in one HIP kernel on the
    GPU (bgx_gather_rollout; torch's index gathers of the [m, 64] records ran at ~1 TB/s),
    the torch gathers elsewhere.  Returns (records, actions, old_logp, returns, adv),
    written into `out` when given."""
    acts, old, R, adv = (acts.to(torch.int32).contiguous(), old.float().contiguous(), R.float().contiguous(),
                         adv.float().contiguous())
    recs = recs.contiguous()
    if not recs.is_cuda:
        pl = perm.long()
        return recs[pl].contiguous(), acts[pl], old[pl], R[pl], adv[pl]
    m = perm.shape[0]
    if out is None:
        out = (torch.empty_like(recs), torch.empty_like(acts), torch.empty_like(old), torch.empty_like(R),
               torch.empty_like(adv))
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    check(_lib.load().bgx_gather_rollout(p(perm.to(torch.int32).contiguous()), m, p(recs), p(acts), p(old), p(R), p(adv),
                                         *[p(t) for t in out],
                                         ctypes.c_void_p(torch.cuda.current_stream(recs.device).cuda_stream)),
          "bgx_gather_rollout")
    return out


def plan_rollout(recs, acts, old, R, adv, n_actions: int = 500, out_rows=None, out_plan=None):
    """ppo_row_plan + gather_rollout in one pass on the GPU (bgx_ppo_plan_rows: the rows
    written straight to their plan-order positions).  Returns ((records, actions,
    old_logp, returns, adv) in plan order, plan, row_plan); out_rows / out_plan (the
    graphed update's persistent buffers; out_plan = (perm, plan, row_plan), perm unused)
    to write into."""
    if not recs.is_cuda:
        perm, plan, row_plan = ppo_row_plan_torch(recs, n_actions)
        return gather_rollout(perm, recs, acts, old, R, adv), plan, row_plan
    acts, old, R, adv = (acts.to(torch.int32).contiguous(), old.float().contiguous(), R.float().contiguous(),
                         adv.float().contiguous())
    rec = recs.contiguous()
    m, dev = rec.shape[0], rec.device
    L = _lib.load()
    ws = torch.empty(max(int(L.bgx_ppo_plan_workspace(m)) // 4, 1), dtype=torch.int32, device=dev)
    rows = out_rows if out_rows is not None else (torch.empty_like(rec), torch.empty_like(acts), torch.empty_like(old),
                                                  torch.empty_like(R), torch.empty_like(adv))
    if out_plan is not None:
        _, plan, row_plan = out_plan
    else:
        plan = torch.empty(33, dtype=torch.int32, device=dev)
        row_plan = torch.empty(8, dtype=torch.int32, device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    check(L.bgx_ppo_plan_rows(p(rec), m, n_actions, p(ws), p(acts), p(old), p(R), p(adv), *[p(t) for t in rows], None,
                              p(plan), p(row_plan), ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
          "bgx_ppo_plan_rows")
    return rows, plan, row_plan


def _fused_head_ok(net) -> bool:
    """The fused output layer + loss head (csrc/bg_ppo_fused.hip) is built for the
    reference's shape (H = 128, 500 actions); other shapes take the manual epoch
    (hipBLASLt head GEMM + bgx_ppo_head_ex + dy W2h + ReLU backward + split-K gW2)."""
    return net.fc1.out_features == 128 and net.action_head.out_features == 500


# The fused head computes, for a row with cnt >= 1 legal actions, only the action tiles
# holding its legal columns: the masked logits z + log(1e-45) (ppo_agent.py:166) are left
# out of the log-sum-exp and their gradients are 0.  That equals the reference exactly
# while every masked term lies e^-30 below the row's sum, i.e. while 2U + log(1e-45) <
# -30 with U a bound on |z|: U = max_a |Wa_h[a]| max_row |h| + max_a |ba_h[a]|.  The fc1
# kernel reports max_row |h|^2 (bgx_fc1_records_ex); PPOTrainer checks the bound after
# each update and redoes an update that broke it on the exact round-2 epoch.
MASK_SHORTCUT_LIMIT = -MASK_LOG - 30.0


def _ptr_or_none(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _fused_fast(net) -> bool:
    """The fused epoch's one-launch prologue / epilogue apply (bgx_ppo_epoch_prep / _grads):
    198 input features and fp32 contiguous parameters."""
    params = (net.fc1.weight, net.fc1.bias, net.action_head.weight, net.action_head.bias, net.value_head.weight,
              net.value_head.bias)
    return net.fc1.weight.shape[1] == 198 and all(t.dtype == torch.float32 and t.is_contiguous() for t in params)


def _ppo_epoch_amp_fused(net, chunks, n_total, coefs, sums, guard=None, parts=None, entropy_coef=0.0):
    """The fp16-autocast epoch with the output layer and loss head fused
    (bgx_ppo_rows + bgx_ppo_gw2): fc1 from the records (bgx_fc1_records), then per
    row the logits, the loss head, dy and dh = ReLU'(h) fp16(dy W2h) on MFMA without
    the [n, 512] logits in HBM; gW2 / gb2 = dy^T [h | 1] from per-row statistics;
    gW1 / gb1 = dh^T [x | 1] with x generated from the records on chip (bgx_ppo_gw1:
    no feature rows in HBM).  Same fp16 operands, fp32 accumulation and per-row
    gradient scaling as _ppo_epoch_amp_manual; gradients land in p.grad as fp32.
    The chunks' feature entries are not read.  `guard` (a device bool, optional) is
    set when the masked-action shortcut's bound (MASK_SHORTCUT_LIMIT) does not hold.
    `parts` (fp64 [4], fast path only): the prologue zeroes `sums` and the epilogue adds this
    epoch's loss parts to `parts` (the torch form's arithmetic), so no small torch kernels run
    around the epoch."""
    eps, c_v, c_e, gscale = coefs
    row_scale = gscale * n_total / min(n_total, REF_ROWS)
    post = min(n_total, REF_ROWS) / n_total
    W1, b1 = net.fc1.weight, net.fc1.bias
    Wa, ba = net.action_head.weight, net.action_head.bias
    wv, bv = net.value_head.weight, net.value_head.bias
    A, Hd = Wa.shape
    F_in = W1.shape[1]
    dev = W1.device
    k1 = float(np.float32(row_scale) * np.float32(c_e))      # the kernel's fp32 gscale * c_entropy
    params = (W1, b1, Wa, ba, wv, bv)
    # one launch for the casts, the packed fc1 fragments and the zeroed accumulators (and
    # one for the gradient hand-off below) instead of ~20 small torch kernels per epoch
    fast = _fused_fast(net)
    if parts is not None and not fast:
        raise ValueError("loss-part accumulation needs the fast fused epoch")
    with torch.no_grad():
        L = _lib.load()
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        w1pack = torch.empty(L.bgx_fc1_packed_size(Hd), dtype=torch.uint8, device=dev)
        if fast:
            b1h = torch.empty(Hd, dtype=torch.float16, device=dev)
            W2h = torch.empty(512, Hd, dtype=torch.float16, device=dev)
            b2h = torch.empty(512, dtype=torch.float16, device=dev)
            gW1 = torch.empty(Hd, 208, dtype=torch.float32, device=dev)
            gW2 = torch.empty(512, Hd, dtype=torch.float32, device=dev)
            gb2 = torch.empty(512, dtype=torch.float32, device=dev)
            hmax2 = torch.empty(1, dtype=torch.float32, device=dev) if guard is not None else None
            bound = torch.empty(2, 512, dtype=torch.float32, device=dev) if guard is not None else None
            check(L.bgx_ppo_epoch_prep(*[p(t) for t in params], Hd, A, p(w1pack), p(b1h), p(W2h), p(b2h), p(gW1),
                                       p(gW2), p(gb2), _ptr_or_none(hmax2), _ptr_or_none(bound),
                                       _ptr_or_none(sums if parts is not None else None), stream),
                  "bgx_ppo_epoch_prep")
        else:
            W1h, b1h = W1.half(), b1.half()
            W2h = torch.zeros(512, Hd, dtype=torch.float16, device=dev)
            b2h = torch.zeros(512, dtype=torch.float16, device=dev)
            W2h[:A] = Wa.half(); W2h[A] = wv[0].half()
            b2h[:A] = ba.half(); b2h[A] = bv[0].half()
            gW1 = torch.zeros(Hd, 208, dtype=torch.float32, device=dev)
            gW2 = torch.zeros(512, Hd, dtype=torch.float32, device=dev)
            gb2 = torch.zeros(512, dtype=torch.float32, device=dev)
            check(L.bgx_fc1_pack(p(W1h), Hd, p(w1pack), stream), "bgx_fc1_pack")
            hmax2 = torch.zeros(1, dtype=torch.float32, device=dev) if guard is not None else None
        for _feats, _legal, actions, old_logp, returns, adv, records, *extra in chunks:
            prep = extra[0] if extra else {}
            rec = records.contiguous()
            m = rec.shape[0]
            perm, plan, row_plan = prep["plan"] if "plan" in prep else ppo_row_plan(rec, A)
            h = torch.empty(m, Hd, dtype=torch.float16, device=dev)
            check(L.bgx_fc1_records_ex(p(rec), m, p(w1pack), p(b1h), Hd, p(h), _ptr_or_none(hmax2), stream),
                  "bgx_fc1_records_ex")
            dh = torch.empty(m, Hd, dtype=torch.float16, device=dev)
            stats = torch.empty(m, 4, dtype=torch.float32, device=dev)
            info = torch.empty(m, dtype=torch.int32, device=dev)
            acts = actions.to(torch.int32).contiguous()
            old, ret, ad = old_logp.float().contiguous(), returns.float().contiguous(), adv.float().contiguous()
            pp = None if perm is None else p(perm)             # None: rows already in plan order
            check(L.bgx_ppo_rows(p(h), pp, p(rec), p(acts), p(old), p(ret), p(ad), m, Hd, A, p(W2h), p(b2h),
                                 eps, c_v, c_e, row_scale, p(dh), p(stats), p(info), p(sums), None, None, p(row_plan), 0,
                                 stream),
                  "bgx_ppo_rows")
            ws = torch.empty(L.bgx_ppo_gw2_workspace(m) // 4, dtype=torch.float32, device=dev)
            check(L.bgx_ppo_gw2(p(h), pp, p(stats), p(info), m, Hd, A, p(W2h), p(b2h), k1, p(plan), p(ws),
                                p(gW2), p(gb2), stream), "bgx_ppo_gw2")
            # dh is in the order of rec (bgx_ppo_rows writes it in the original row order)
            ws1 = torch.empty(L.bgx_ppo_gw1_workspace(m) // 4, dtype=torch.float32, device=dev)
            check(L.bgx_ppo_gw1(p(dh), p(rec), m, Hd, p(ws1), p(gW1), stream), "bgx_ppo_gw1")
        if fast:
            grads = [torch.empty_like(t) for t in params]
            check(L.bgx_ppo_epoch_grads(p(gW1), p(gW2), p(gb2), Hd, A, float(post), *[p(g) for g in grads],
                                        _ptr_or_none(bound), _ptr_or_none(hmax2), float(MASK_SHORTCUT_LIMIT),
                                        _ptr_or_none(guard), p(sums), float(n_total), float(VALUE_LOSS_COEF),
                                        float(entropy_coef), _ptr_or_none(parts), stream), "bgx_ppo_epoch_grads")
            W1.grad, b1.grad, Wa.grad, ba.grad, wv.grad, bv.grad = grads
            return
        if post != 1.0:
            for t in (gW1, gW2, gb2):
                t.mul_(post)
        if guard is not None:
            U = W2h[:A].float().norm(dim=1).max() * hmax2[0].sqrt() + b2h[:A].float().abs().max()
            guard |= 2.0 * U > MASK_SHORTCUT_LIMIT
    W1.grad, b1.grad = gW1[:, :F_in].contiguous(), gW1[:, FEAT_BIAS_COL].contiguous()
    Wa.grad, ba.grad = gW2[:A].contiguous(), gb2[:A].contiguous()
    wv.grad, bv.grad = gW2[A:A + 1].contiguous(), gb2[A:A + 1].contiguous()


def adam_step(optimizer, scaler) -> bool:
    """`scaler.step(optimizer); scaler.update()` (ppo_agent.py:302-305) for a fused
    torch.optim.Adam as ONE HIP call (bgx_adam_step: the inf check, the Adam step and the
    scale update over every tensor's elements in one flat launch each; torch's fused path
    runs ~4 multi-tensor workgroups over a 90 k-parameter net plus a dozen small ops).
    The optimizer state and the GradScaler state are torch's own tensors, updated as
    torch would (tests/test_gpu_train.py::test_adam_step_matches_torch).  Returns False
    (nothing done) for a configuration it does not restate: the caller then runs torch's."""
    if not isinstance(optimizer, torch.optim.Adam) or len(optimizer.param_groups) != 1:
        return False
    grp = optimizer.param_groups[0]
    if (grp.get("weight_decay", 0) or grp.get("amsgrad") or grp.get("maximize") or grp.get("capturable")
            or grp.get("differentiable") or not grp.get("fused") or torch.is_tensor(grp["lr"])):
        return False
    ps = [p for p in grp["params"] if p.grad is not None]
    if not ps or len(ps) > 8 or any(p.dtype != torch.float32 or p.grad.dtype != torch.float32 or not p.is_cuda
                                    or not p.is_contiguous() or not p.grad.is_contiguous() for p in ps):
        return False
    dev = ps[0].device
    for p in ps:                                     # torch's lazy state (fused: fp32 device step)
        st = optimizer.state[p]
        if len(st) == 0:
            st["step"] = torch.zeros((), dtype=torch.float32, device=dev)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
    found = getattr(optimizer, "_bgx_found", None)
    if found is None or found.device != dev:
        found = optimizer._bgx_found = torch.zeros(1, dtype=torch.int32, device=dev)
    use_scale = scaler is not None and scaler.is_enabled()
    if use_scale:
        scale, tracker = scaler._scale, scaler._growth_tracker
        if scale is None or tracker is None:
            return False
    n = len(ps)
    arr = lambda ts: ctypes.cast((ctypes.c_void_p * n)(*[t.data_ptr() for t in ts]), ctypes.c_void_p)
    st = [optimizer.state[p] for p in ps]
    numels = (ctypes.c_int64 * n)(*[p.numel() for p in ps])
    b1, b2 = grp["betas"]
    check(_lib.load().bgx_adam_step(
        n, arr(ps), arr([p.grad for p in ps]), arr([s["exp_avg"] for s in st]), arr([s["exp_avg_sq"] for s in st]),
        arr([s["step"] for s in st]), ctypes.cast(numels, ctypes.c_void_p), float(grp["lr"]), float(b1), float(b2),
        float(grp["eps"]), ctypes.c_void_p(scale.data_ptr() if use_scale else None),
        ctypes.c_void_p(tracker.data_ptr() if use_scale else None),
        float(scaler._growth_factor) if use_scale else 2.0, float(scaler._backoff_factor) if use_scale else 0.5,
        int(scaler._growth_interval) if use_scale else 1, ctypes.c_void_p(found.data_ptr()),
        ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "bgx_adam_step")
    return True


def _ppo_epoch_fused(net, optimizer, scaler, chunks, n_total, entropy_coef, group, amp, step, sync=True, guard=None,
                     fused_head=True, scale_hint=None, parts=None):
    """scale_hint (PPOTrainer.update): {"scale", "tracker"}, the host's copy of the
    GradScaler state, used instead of get_scale() (a host sync per epoch that left the
    GPU idle while the next epoch's launches were issued) and advanced as a finite
    step advances it; the trainer checks it against the device state after the
    update and redoes the update with per-epoch get_scale() when a skipped
    (non-finite) step made them differ."""
    dev = next(net.parameters()).device
    if scaler.is_enabled():
        if getattr(scaler, "_scale", None) is None:
            scaler.scale(torch.ones((), device=dev))      # initialises the scale tensor lazily
        scale = scale_hint["scale"] if scale_hint is not None else scaler.get_scale()
    else:
        scale = 1.0
    coefs = (EPS_CLIP, VALUE_LOSS_COEF, float(entropy_coef), float(scale) / n_total)
    manual = amp and _is_policy_mlp(net)
    # `parts` (fp64 [4] accumulator, sync=False only): the fast fused epoch adds its loss parts
    # on the device inside its own epilogue launch (and its prologue zeroes the sums)
    in_kernel = (parts is not None and not sync and manual and fused_head and _fused_head_ok(net)
                 and _fused_fast(net))
    if in_kernel and (parts.device != dev or parts.dtype != torch.float64 or parts.numel() != 4):
        raise ValueError("parts must be a float64 [4] tensor on the parameters' device")
    sums = (torch.empty if in_kernel else torch.zeros)(3, dtype=torch.float64, device=dev)
    if manual:
        if fused_head and _fused_head_ok(net):
            _ppo_epoch_amp_fused(net, chunks, n_total, coefs, sums, guard, parts=parts if in_kernel else None,
                                 entropy_coef=entropy_coef)
        else:
            _ppo_epoch_amp_manual(net, chunks, n_total, coefs, sums)
        chunks = ()
    for feats, legal, actions, old_logp, returns, adv, records, *_ in chunks:
        with autocast(device_type=dev.type, enabled=amp):
            logits, values = net(feats)
        out = _PPOHead.apply(logits, values, records.contiguous(), actions.to(torch.int32).contiguous(),
                             old_logp.float().contiguous(), returns.float().contiguous(), adv.float().contiguous(),
                             coefs, sums)
        out.backward()
    if step:
        allreduce_mean_([p.grad for p in net.parameters() if p.grad is not None], group)
        if not adam_step(optimizer, scaler):
            scaler.step(optimizer)
            scaler.update()
        if scale_hint is not None and scaler.is_enabled():     # _amp_update_scale_ without a non-finite
            t = scale_hint["tracker"] + 1
            if t == scaler._growth_interval:
                scale_hint["scale"] = float(np.float32(scale_hint["scale"] * scaler._growth_factor))
                t = 0
            scale_hint["tracker"] = t
    if not sync:        # loss parts stay on the device (fp64, same arithmetic): no host sync per epoch
        if in_kernel:
            return parts
        m = sums / n_total
        e = torch.cat([m, (m[0] + VALUE_LOSS_COEF * m[1] - entropy_coef * m[2]).reshape(1)])
        if parts is not None:
            parts += e
            return parts
        return e
    pol, val, ent = (sums / n_total).tolist()
    tot = pol + VALUE_LOSS_COEF * val - entropy_coef * ent
    return torch.tensor([pol, val, ent, tot], dtype=torch.float64)


class PPOTrainer:
    def __init__(self, batch: int = 65536, horizon: int = 64, hidden: int = 128, n_actions: int = 500,
                 seed: int = 0, device=None, process_group=None, pinned: bool = False, returns: str = "lane",
                 chunk: int = 1 << 21, fused: bool | None = None, amp: bool = True,
                 entropy_anneal: str = "train", shards: int | None = None, graphs: bool | None = None,
                 fork: bool | None = None, streams=None, update_graphs: bool | None = None):
        if entropy_anneal not in ("train", "train_single"):
            raise ValueError(f"entropy_anneal must be 'train' or 'train_single', got {entropy_anneal!r}")
        self.entropy_anneal = entropy_anneal
        self.dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.group = process_group
        self.rank = dist.get_rank(process_group) if _world(process_group) > 1 else 0
        self.B, self.T, self.A = batch, horizon, n_actions
        self.returns_mode = returns
        # rows per update chunk (gradient accumulation over chunks): 2^21 = a whole 65,536 x 32
        # rollout in one chunk, the reference's single full batch; 2^20-row chunks cost
        # 8.4 vs 7.8 ms per update (twice the per-call partial sums and launches)
        self.chunk = chunk
        self.fused = (self.dev.type == "cuda") if fused is None else fused
        self.amp = amp            # the reference's autocast (fp16 on the GPU); False = fp32 update
        # the fused output layer + loss head (csrc/bg_ppo_fused.hip) while its exactness bound
        # holds (MASK_SHORTCUT_LIMIT; update() falls back to the exact epoch otherwise)
        self.fused_head = True
        # the B lanes as S engines on S streams (bench.py's C3 layout: one shard's policy
        # kernel runs beside another's env step); shard 0 keeps the 1-shard seeds.  4 shards
        # from 65,536 lanes (one per hardware queue: PPO iteration 133 -> 136 M vs 2)
        if shards is None:
            cuda = self.dev.type == "cuda"
            shards = (4 if cuda and batch >= 65536 and batch % 1024 == 0 else
                      2 if cuda and batch >= 32768 and batch % 256 == 0 else 1)
        if batch % shards:
            raise ValueError(f"batch {batch} is not a multiple of shards {shards}")
        self.S = shards
        self.engs = [Engine(batch=batch // shards, max_moves=n_actions,
                            seed=seed * 1_000_003 + self.rank + 7_919 * k, dice="philox", auto_reset=True,
                            device=self.dev) for k in range(shards)]
        self.eng = self.engs[0]
        # rollout steps replayed as HIP graphs (2 steps per graph, one graph per slot pair
        # and shard), captured at the end of the first rollout: the engines' host state is
        # then a 2-step fixed point (bench.py C3).  Equal to the eager rollout
        # (tests/test_gpu_train.py::test_rollout_graphs_match_eager).  With pinned=True each
        # replayed pair's rows go to the host by one copy launch (bgx.hostcopy) on the
        # shard's copy stream, beside the next pair's steps.
        self.graphs = (self.dev.type == "cuda" and horizon % 2 == 0) if graphs is None else graphs
        self._graphs = None
        # the update's fused-head epoch replayed as a HIP graph (round 5): one eager epoch
        # issues ~50 small torch launches between the big kernels, and the GPU idled 1.4 ms
        # per update waiting for the host (profiles/r5/update_trace_plan.txt).  The graph is
        # captured at the second update (the first initialises the Adam and GradScaler
        # state eagerly) over persistent row buffers, and again when its host-side inputs
        # change: the GradScaler scale (a growth or a skipped step) or the entropy
        # coefficient.  Not with a process group (collectives stay eager).
        self.update_graphs = ((self.dev.type == "cuda" and _world(process_group) == 1
                               and not (dist.is_available() and dist.is_initialized()))
                              if update_graphs is None else bool(update_graphs))
        self._ugraph = None            # (key, graph, loss-parts output)
        self._ugraph_captures = 0
        self._ubufs = None             # persistent per-chunk rows in plan order + plans
        self._updates_done = 0
        # fork (Engine.set_fork): an env step's light launch on the engine's side stream.
        # Off by default with graphs: each shard's graph is then one linear chain on its own
        # hardware queue (forked graphs' internal streams share queues with the other
        # shards' and serialise them: rollout 9.2 -> 6.3 ms at 65,536 x 32)
        self.fork = (not self.graphs) if fork is None else bool(fork)
        for e in self.engs:
            e.set_fork(self.fork)
        torch.manual_seed(seed)
        self.net = PolicyNet(hidden_size=hidden, action_size=n_actions).to(self.dev)
        if _world(process_group) > 1:
            for p in self.net.parameters():
                dist.broadcast(p.data, src=0, group=process_group)
        # ppo_agent.py:83 Adam; on the GPU the fused kernel: GradScaler hands it the scale and
        # the inf flag as device tensors, so an optimizer step needs no host sync
        # (the foreach path's found_inf.item() left ~115 us idle per epoch)
        fused_adam = self.dev.type == "cuda"
        self.opt = torch.optim.Adam(self.net.parameters(), lr=LEARNING_RATE, fused=fused_adam)
        self.scaler = GradScaler(device=self.dev.type)
        self.total_episodes = 0
        self.entropy_coef = ENTROPY_COEF_START
        self.step_counter = 0
        self.seed = seed
        T, B = horizon, batch
        kw = dict(device=self.dev)
        self.buf = {"records": torch.empty(T, B, 64, dtype=torch.uint8, **kw),
                    "actions": torch.empty(T, B, dtype=torch.int32, **kw),
                    "logp": torch.empty(T, B, dtype=torch.float32, **kw),
                    "values": torch.empty(T, B, dtype=torch.float32, **kw),
                    "rewards": torch.empty(T, B, dtype=torch.float32, **kw),
                    "dones": torch.empty(T, B, dtype=torch.uint8, **kw)}
        self.pinned = None
        if pinned:                      # the rollout mirrored into pinned host memory
            if (B // self.S) % 16:
                raise ValueError(f"pinned=True copies each shard's lanes in 16-byte chunks: the shard batch "
                                 f"{B // self.S} must be a multiple of 16")
            self.mirror = HostMirror(self.buf)
            self.pinned = self.mirror.host
        self.ep_carry = torch.zeros(B, dtype=torch.float64, **kw)     # train.py:58 episode_rewards
        self.last_episode_stats = None
        for e in self.engs:
            e.reset(want_obs=False)
        # `streams`: the S shard streams to use (a process that already runs shards on
        # streams of its own passes them: HIP maps streams onto its 4 hardware queues in
        # creation order, and a fresh set created after many others may land two shards
        # on one queue -- bench.py's PPO leg after the C3/C4/C2 legs: 113 vs 136 M)
        if streams is not None:
            if len(streams) != self.S:
                raise ValueError(f"streams: {len(streams)} given for {self.S} shards")
            self._streams = list(streams)
        else:
            self._streams = ([torch.cuda.current_stream(self.dev)] +
                             [torch.cuda.Stream(self.dev) for _ in range(self.S - 1)]
                             if self.dev.type == "cuda" else [None])
        # per shard: the stream its host copies run on -- with forked steps a copy stream
        # beside the next steps; with linear shards the shard's own stream (one hardware
        # queue per shard; the other shards' steps run beside the copy)
        self._copy_streams = ([torch.cuda.Stream(self.dev) if self.fork else None for _ in range(self.S)]
                              if pinned else None)

    def _mirror_slots(self, k: int, t0: int, n: int):
        """Shard k's rows of slots [t0, t0 + n) to the pinned host buffers, on the shard's
        copy stream forked from its step stream (joined later by _join_copies)."""
        cs = self._copy_streams[k]
        lo = k * (self.B // self.S)
        if cs is None:                           # linear shards: on the step stream itself
            self.mirror.copy(t0, n, lo, lo + self.B // self.S, stream=torch.cuda.current_stream(self.dev))
            return
        cs.wait_stream(torch.cuda.current_stream(self.dev))
        self.mirror.copy(t0, n, lo, lo + self.B // self.S, stream=cs)

    def _join_copies(self, k: int):
        if self._copy_streams[k] is not None:
            torch.cuda.current_stream(self.dev).wait_stream(self._copy_streams[k])

    def _slot(self, k: int, t: int):
        """Shard k's views of rollout slot t (contiguous row ranges)."""
        n = self.B // self.S
        lo, hi = k * n, (k + 1) * n
        b = self.buf
        return ((b["actions"][t][lo:hi], b["logp"][t][lo:hi], b["values"][t][lo:hi]), b["records"][t][lo:hi],
                (b["rewards"][t][lo:hi], b["dones"][t][lo:hi]))

    def _act_step(self, k: int, t: int, step: int, step_ctr=None):
        out, rec, env_out = self._slot(k, t)
        self.net.act(self.engs[k], seed=self.seed * 7919 + self.rank + 104_729 * k, step=step, step_ctr=step_ctr,
                     out=out, records_out=rec)
        self.engs[k].step(out[0], want_obs=False, want_info=False, out=env_out)

    def _capture(self):
        """One graph per (slot pair, shard): act + step for slots t and t + 1 with the
        noise step read from the shard's device counter (advanced by 2 per replay),
        the engine joined at the end (its side-stream dispatch order).  Thread-local
        capture mode: a communicator's watchdog thread may query events meanwhile.
        A failed capture is terminal (bgx/graphs.py)."""
        self._ctrs = [torch.zeros(1, dtype=torch.int32, device=self.dev) for _ in range(self.S)]
        caps = [torch.cuda.Stream(self.dev) for _ in range(self.S)]
        for k in range(self.S):
            caps[k].wait_stream(self._streams[k])
            with torch.cuda.stream(caps[k]):
                self.engs[k].join()
        torch.cuda.synchronize(self.dev)
        def two_steps(k, t):
            for j in range(2):
                self._act_step(k, t + j, j, self._ctrs[k])
            self.engs[k].join()
            PolicyNet.advance_counter(self._ctrs[k], 2)
        # a failed capture ends the process (bgx/graphs.py: the engines' host state has
        # advanced through steps that never ran)
        graphs = [[capture("trainer", lambda k=k, t=t: two_steps(k, t), caps[k]) for k in range(self.S)]
                  for t in range(0, self.T, 2)]
        torch.cuda.synchronize(self.dev)
        self._graphs = graphs

    def rollout(self, defer_stats: bool = False):
        """T env steps on all B lanes (train.py:46-99 without the Python loops).  Returns
        the episodes finished; with defer_stats the episode statistics stay on the device
        until the next update() reads them with its own final sync (iteration(): no host
        sync, and so no idle GPU, between the rollout and the update) and None is returned."""
        self.net.pack(inplace=True)
        buf = self.buf
        cur = self._streams[0]
        for st in self._streams[1:]:
            st.wait_stream(cur)                  # the packed weights, the previous update
        if self._graphs is not None:
            for k in range(self.S):
                with torch.cuda.stream(self._streams[k]):
                    self._ctrs[k].fill_(self.step_counter)
            for t, row in zip(range(0, self.T, 2), self._graphs):     # the shards' replays side by side
                for k in range(self.S):
                    with torch.cuda.stream(self._streams[k]):
                        row[k].replay()
                        if self.pinned is not None:  # the pair's rows to the host beside the next pair
                            self._mirror_slots(k, t, 2)
            self.step_counter += self.T
            if self.pinned is not None:
                for k in range(self.S):
                    with torch.cuda.stream(self._streams[k]):
                        self._join_copies(k)
        for t in range(self.T if self._graphs is None else 0):
            for k in range(self.S):
                with torch.cuda.stream(self._streams[k]):
                    self._act_step(k, t, self.step_counter)
                    if self.pinned is not None:
                        self._mirror_slots(k, t, 1)
            self.step_counter += 1
        if self.pinned is not None and self._graphs is None:
            for k in range(self.S):
                with torch.cuda.stream(self._streams[k]):
                    self._join_copies(k)
        for st in self._streams[1:]:
            cur.wait_stream(st)
        if cur is not None and cur != torch.cuda.current_stream(self.dev):
            torch.cuda.current_stream(self.dev).wait_stream(cur)   # the statistics and update() run there
        if self.graphs and self._graphs is None:
            self._capture()
        st = episode_stats_records(buf["rewards"], buf["dones"], buf["records"], self.ep_carry)
        if _world(self.group) > 1:
            dist.all_reduce(st, group=self.group)
        if defer_stats:
            if getattr(self, "_pending_stats", None) is not None:   # an earlier deferred rollout, no update since
                self._apply_stats(self._pending_stats)
            self._pending_stats = st
            return None
        return self._apply_stats(st)

    def _apply_stats(self, st):
        self.last_episode_stats = dict(zip(EPISODE_STATS, st.tolist()))
        eps = int(self.last_episode_stats["episodes"])
        self.total_episodes += eps
        return eps

    def load_rollout(self, records, actions, logp, values, rewards, dones):
        """Fill the [T, B] rollout buffers from given data (e.g. a reference
        agent's memory, step-major) instead of running rollout()."""
        src = {"records": records, "actions": actions, "logp": logp, "values": values, "rewards": rewards,
               "dones": dones}
        for k, v in src.items():
            v = torch.as_tensor(v)
            if v.numel() != self.buf[k].numel():
                raise ValueError(f"load_rollout: {k} has {v.numel()} elements, the buffer {self.buf[k].numel()}")
            self.buf[k].copy_(v.reshape(self.buf[k].shape).to(self.buf[k].dtype))

    def update(self):
        """ppo_agent.py:218-366 on the device buffers."""
        buf = self.buf
        manual = self.fused and self.amp and _is_policy_mlp(self.net)
        fused_head = manual and _fused_head_ok(self.net) and self.fused_head
        # the snapshot's host work first: it overlaps the rollout's last kernels instead of
        # idling the GPU between the return computation and the epochs (~0.17 ms)
        snap = self._snapshot() if fused_head else None
        if self.returns_mode == "reference":
            R = reference_returns(buf["rewards"], buf["dones"])
        else:
            R = lane_returns(buf["rewards"], buf["dones"])
        R = global_normalize(R.reshape(-1), self.group)
        adv = R - buf["values"].reshape(-1)
        recs = buf["records"].reshape(-1, 64)
        acts = buf["actions"].reshape(-1)
        old = buf["logp"].reshape(-1)
        N = recs.shape[0]

        if not fused_head:
            parts = self._epochs(recs, acts, old, R, adv, False)
        else:
            if getattr(self, "_guard", None) is None:       # persistent: a captured epoch writes it
                self._guard = torch.zeros((), dtype=torch.bool, device=self.dev)
            guard = self._guard
            guard.zero_()
            # the scaler's state as the previous update verified it (no host sync here, where
            # it would idle the GPU between the return computation and the epochs), else read
            hint = getattr(self, "_scale_next", None)
            self._scale_next = None
            if hint is None:
                hint = self._scale_state()
            parts = self._epochs(recs, acts, old, R, adv, True, guard, scale_hint=hint)
            if hint is not None and self._scale_state() != hint:
                # a non-finite step was skipped (the scale backed off on the device): the
                # later epochs ran at the host's scale; redo the update with get_scale()
                self._restore(snap)
                guard.zero_()
                parts = self._epochs(recs, acts, old, R, adv, True, guard)
            elif hint is not None:
                self._scale_next = dict(hint)      # = the device state after this update
            # the bound check of the update that is kept (after any redo above)
            g = guard.to(torch.int32)
            if _world(self.group) > 1:
                dist.all_reduce(g, op=dist.ReduceOp.MAX, group=self.group)
            if bool(g.item()):               # the masked-action shortcut's bound broke: redo exactly
                self._scale_next = None
                print("[bgx] PPO update: logit bound above the fused head's exact range; update redone on the "
                      "exact epoch, later updates too", flush=True)
                self._restore(snap)
                self.fused_head = False
                parts = self._epochs(recs, acts, old, R, adv, False)
        if getattr(self, "_pending_stats", None) is not None:    # a deferred rollout's statistics
            self._pending_eps = self._apply_stats(self._pending_stats)
            self._pending_stats = None
        self.entropy_coef = entropy_coef_after_update(self.entropy_anneal, self.total_episodes)
        self._updates_done += 1
        p = (parts / NUM_EPOCHS).tolist()
        return {"policy_loss": p[0], "value_loss": p[1], "entropy": p[2], "total_loss": p[3]}

    def _scale_state(self):
        """The GradScaler's (scale, growth tracker) on the host (one sync), or None when
        scaling is off."""
        if not self.scaler.is_enabled():
            return None
        self.scaler.scale(torch.ones((), device=self.dev))     # lazy initialisation
        return {"scale": float(self.scaler._scale.item()), "tracker": int(self.scaler._growth_tracker.item())}

    def _epochs(self, recs, acts, old, R, adv, fused_head: bool, guard=None, scale_hint=None):
        """The NUM_EPOCHS full-batch epochs of one update; returns the summed loss parts
        (device, fp64)."""
        N = recs.shape[0]
        manual = self.fused and self.amp and _is_policy_mlp(self.net)
        # the fused head generates every feature it needs from the records (fc1 forward,
        # gW1); the other paths read features encoded once for the 4 epochs
        feats = [None if fused_head else
                 encode_records(recs[s:min(N, s + self.chunk)], torch.float16 if self.amp else torch.float32,
                                width=FEAT_W if manual else 198)
                 for s in range(0, N, self.chunk)] if self.fused else None
        preps = [{} for _ in range(0, N, self.chunk)]
        sorted_rows = [None for _ in range(0, N, self.chunk)]
        graphed = (fused_head and manual and self.update_graphs and guard is not None and scale_hint is not None
                   and self._updates_done >= 1)
        if graphed:
            return self._epochs_graphed(recs, acts, old, R, adv, guard, scale_hint)
        if fused_head:
            # once per update: each chunk's rows in the order of the fused head's row plan
            # (by the number of action tiles a row needs), gathered so that every kernel
            # of the 4 epochs reads them contiguously
            for i, s in enumerate(range(0, N, self.chunk)):
                e = min(N, s + self.chunk)
                sorted_rows[i], plan, row_plan = plan_rollout(recs[s:e], acts[s:e], old[s:e], R[s:e], adv[s:e],
                                                              self.A)
                preps[i] = {"plan": (None, plan, row_plan)}

        def chunks():
            for i, s in enumerate(range(0, N, self.chunk)):
                e = min(N, s + self.chunk)
                if sorted_rows[i] is not None:
                    rr, aa, oo, RR, dd = sorted_rows[i]
                    yield feats[i], None, aa, oo, RR, dd, rr, preps[i]
                    continue
                if self.fused:      # the loss kernel reads the legal counts from the records
                    f, legal = feats[i], None
                else:
                    f, legal = features_and_masks(recs[s:e], self.A)
                yield f, legal, acts[s:e], old[s:e], R[s:e], adv[s:e], recs[s:e], preps[i]

        parts = torch.zeros(4, dtype=torch.float64, device=self.dev)
        for _ in range(NUM_EPOCHS):
            e = ppo_epoch(self.net, self.opt, self.scaler, chunks(), N, self.entropy_coef, self.group, amp=self.amp,
                          fused=self.fused, sync=False, guard=guard, fused_head=fused_head, scale_hint=scale_hint,
                          parts=parts)
            if e is not parts:                 # the torch epoch returns its own (host) parts
                parts += e.to(parts.device)
        return parts

    def _epochs_graphed(self, recs, acts, old, R, adv, guard, hint):
        """_epochs' fused-head epochs as HIP-graph replays: the rows go into persistent
        plan-order buffers (eager), one epoch is captured per (GradScaler scale, entropy
        coefficient) and replayed NUM_EPOCHS times; the host's copy of the scaler state
        advances per replay as _ppo_epoch_fused advances it."""
        N = recs.shape[0]
        spans = [(s, min(N, s + self.chunk)) for s in range(0, N, self.chunk)]
        if self._ubufs is None or self._ubufs["N"] != N:
            kw = dict(device=self.dev)
            self._ubufs = {"N": N, "chunks": []}
            for s, e in spans:
                m = e - s
                self._ubufs["chunks"].append({
                    "rows": (torch.empty(m, 64, dtype=torch.uint8, **kw), torch.empty(m, dtype=torch.int32, **kw),
                             torch.empty(m, dtype=torch.float32, **kw), torch.empty(m, dtype=torch.float32, **kw),
                             torch.empty(m, dtype=torch.float32, **kw)),
                    "plan": (torch.empty(m, dtype=torch.int32, **kw), torch.empty(33, dtype=torch.int32, **kw),
                             torch.empty(8, dtype=torch.int32, **kw))})
            self._ugraph = None
        for (s, e), c in zip(spans, self._ubufs["chunks"]):
            plan_rollout(recs[s:e], acts[s:e], old[s:e], R[s:e], adv[s:e], self.A, out_rows=c["rows"],
                         out_plan=c["plan"])

        def chunks():
            for c in self._ubufs["chunks"]:
                rr, aa, oo, RR, dd = c["rows"]
                _, plan, row_plan = c["plan"]
                yield None, None, aa, oo, RR, dd, rr, {"plan": (None, plan, row_plan)}

        if getattr(self, "_uparts", None) is None:
            self._uparts = torch.zeros(4, dtype=torch.float64, device=self.dev)
        self._uparts.zero_()                   # the captured epochs add their loss parts to it
        cur = torch.cuda.current_stream(self.dev)
        for _ in range(NUM_EPOCHS):
            key = self._ugraph_key(hint["scale"], N)
            if self._ugraph is None or self._ugraph[0] != key:
                self._ugraph_captures += 1
                self._ugraph = None
                st = torch.cuda.Stream(self.dev)
                st.wait_stream(cur)
                out = {}

                def body():
                    out["e"] = ppo_epoch(self.net, self.opt, self.scaler, chunks(), N, self.entropy_coef, self.group,
                                         amp=self.amp, fused=self.fused, sync=False, guard=guard, fused_head=True,
                                         scale_hint=dict(hint), parts=self._uparts)
                g = capture("ppo_update", body, st)
                cur.wait_stream(st)
                self._ugraph = (key, g, out["e"])
            self._ugraph[1].replay()
            if self.scaler.is_enabled():         # as _ppo_epoch_fused advances its scale_hint
                t = hint["tracker"] + 1
                if t == self.scaler._growth_interval:
                    hint["scale"] = float(np.float32(hint["scale"] * self.scaler._growth_factor))
                    t = 0
                hint["tracker"] = t
        return self._uparts.clone()

    def _snapshot_tensors(self):
        ts = [p for p in self.net.parameters()]
        for p in self.net.parameters():
            ts += [v for _, v in sorted(self.opt.state[p].items()) if torch.is_tensor(v)] if p in self.opt.state else []
        ts += [t for t in (getattr(self.scaler, "_scale", None), getattr(self.scaler, "_growth_tracker", None))
               if torch.is_tensor(t)]
        return ts

    def _snapshot(self):
        """The weights, the Adam state and the GradScaler state (no host sync) as one
        concatenated device copy per dtype, so that an update can be redone.  The tensor
        lists are cached while the same tensors are in place (Adam and the scaler update
        theirs in place), so a snapshot costs one torch.cat per dtype of host time."""
        ts = self._snapshot_tensors()
        sig = tuple(id(t) for t in ts)
        cache = getattr(self, "_snap_cache", None)
        if cache is None or cache[0] != sig:
            groups = {dt: [t.detach().reshape(-1) for t in ts if t.dtype == dt] for dt in {t.dtype for t in ts}}
            keys = {id(p) for p in self.net.parameters() if p in self.opt.state}
            scal = {k: torch.is_tensor(getattr(self.scaler, k, None)) for k in ("_scale", "_growth_tracker")}
            cache = self._snap_cache = (sig, groups, keys, scal)
        _, groups, keys, scal = cache
        flat = {dt: torch.cat(g) for dt, g in groups.items()}
        return flat, set(keys), dict(scal)

    def _restore(self, snap):
        flat, keys, scal = snap
        with torch.no_grad():
            for p in self.net.parameters():
                if id(p) not in keys:                # no Adam state before the update: none after it
                    self.opt.state.pop(p, None)
            for k, had in scal.items():
                if not had:
                    setattr(self.scaler, k, None)    # lazily re-initialised, as before the update
            off = {dt: 0 for dt in flat}
            for t in self._snapshot_tensors():
                n = t.numel()
                t.copy_(flat[t.dtype][off[t.dtype]:off[t.dtype] + n].view_as(t))
                off[t.dtype] += n

    def _ugraph_key(self, scale, N):
        """What the captured update graph bakes in: the GradScaler scale, the entropy
        coefficient and the row count (kernel arguments), Adam's lr / betas / eps (passed by
        value to bgx_adam_step), and the device addresses of every parameter, its Adam state
        and the scaler's tensors (an optimizer or scaler reload replaces them).  Any change
        recaptures."""
        grp = self.opt.param_groups[0]
        ptrs = []
        for p in self.net.parameters():
            ptrs.append(p.data_ptr())
            st = self.opt.state.get(p, {})
            ptrs.extend(st[k].data_ptr() if torch.is_tensor(st.get(k)) else None
                        for k in ("exp_avg", "exp_avg_sq", "step"))
        for k in ("_scale", "_growth_tracker"):
            t = getattr(self.scaler, k, None)
            ptrs.append(t.data_ptr() if torch.is_tensor(t) else None)
        return (scale, float(self.entropy_coef), N, float(grp["lr"]), tuple(float(b) for b in grp["betas"]),
                float(grp["eps"]), id(self.opt), id(self.scaler), tuple(ptrs))

    def iteration(self):
        # rollout and update back to back on the device (the episode statistics are read at
        # the update's final sync); their split is timed with events
        cur = torch.cuda.current_stream(self.dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        t0 = time.perf_counter()
        ev[0].record(cur)
        self.rollout(defer_stats=True)
        ev[1].record(cur)
        m = self.update()
        ev[2].record(cur)
        torch.cuda.synchronize(self.dev)
        t2 = time.perf_counter()
        eps = self._pending_eps
        # both phases on the GPU's clock (ev 0 -> 1 -> 2); the wall time covers the host too
        t_roll = ev[0].elapsed_time(ev[1]) * 1e-3
        t_upd = ev[1].elapsed_time(ev[2]) * 1e-3
        ws = _world(self.group)
        e = self.last_episode_stats
        k = max(e["episodes"], 1.0)
        m.update({"avg_episode_reward": e["episode_reward_sum"] / k, "win_rate": e["wins"] / k,
                  "p1_win_rate": e["p1_wins"] / k, "gammon_rate": e["gammons"] / k,
                  "backgammon_rate": e["backgammons"] / k, "total_episodes": self.total_episodes})
        m.update({"episodes": eps, "env_steps": self.B * self.T * ws, "rollout_s": t_roll, "update_s": t_upd,
                  "env_steps_per_s": self.B * self.T * ws / (t2 - t0), "entropy_coef": self.entropy_coef})
        return m

    def save(self, path: str):
        torch.save(self.net.state_dict(), path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--horizon", type=int, default=64)
    ap.add_argument("--updates", type=int, default=10)
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--metrics", default=None)
    ap.add_argument("--save", default=None)
    ap.add_argument("--returns", default="lane", choices=["lane", "reference"])
    ap.add_argument("--entropy-anneal", default="train", choices=["train", "train_single"])
    args = ap.parse_args()
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if ws > 1:
        backend = os.environ.get("BGX_DIST_BACKEND", "nccl")     # nccl == RCCL over xGMI
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    tr = PPOTrainer(batch=args.batch, horizon=args.horizon, hidden=args.hidden, seed=args.seed,
                    returns=args.returns, entropy_anneal=args.entropy_anneal)
    for u in range(args.updates):
        m = tr.iteration()
        m["update"] = u
        if tr.rank == 0:
            print(json.dumps(m), flush=True)
            if args.metrics:
                with open(args.metrics, "a") as f:
                    f.write(json.dumps(m) + "\n")
    if args.save and tr.rank == 0:
        tr.save(args.save)
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
