"""BackgammonPPOAgent (agent/ppo_agent.py:57-533) with the reference's rollout
memory, returns, PPO clipped loss, autocast + GradScaler + Adam — plus the
multi-GPU exchange the reference never had: one gradient all-reduce per
optimizer step (RCCL over xGMI under torch.distributed "nccl") and an exact
global return normalisation (all-reduce of Σr, Σr², n).

Hyperparameters are agent/config.py:4-22.  Cloud/TensorBoard I/O (S3 writer,
boto3) is out of scope; metrics go to an optional JSONL
file, checkpoints keep the reference state_dict keys (fc1.*, action_head.*,
value_head.*).
"""
from __future__ import annotations

import json
import os
from datetime import datetime
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.optim as optim
from torch.amp import GradScaler, autocast
from torch.distributions import Categorical

from .policy import PolicyNet

# agent/config.py:4-22
NUM_ENVS = 8
NUM_UPDATES = 1_000
T_HORIZON = 512
NUM_EPOCHS = 4
HIDDEN_SIZE = 128
LEARNING_RATE = 1e-3
GAMMA = 0.99
EPS_CLIP = 0.25
VALUE_LOSS_COEF = 0.5
ENTROPY_COEF_START = 0.15
ENTROPY_COEF_END = 0.01
ENTROPY_ANNEAL_EPISODES = 400_000
MAX_TIMESTEPS = 300
NUM_EPISODES = 1_000_000


def _world(group) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def allreduce_mean_(tensors, group=None):
    """Average a list of tensors across ranks in ONE flat bucket (one collective).
    Runs whenever a process group is initialised, also at world size 1 (the
    one-rank RCCL test exercises the collective that way)."""
    if not (dist.is_available() and dist.is_initialized()) or not tensors:
        return
    ws = _world(group)
    flat = torch.cat([t.reshape(-1).float() for t in tensors])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    flat /= ws
    off = 0
    for t in tensors:
        n = t.numel()
        t.copy_(flat[off:off + n].view_as(t).to(t.dtype))
        off += n


def global_normalize(returns: torch.Tensor, group=None) -> torch.Tensor:
    """(R - mean) / (std_unbiased + 1e-5) over the returns of ALL ranks
    (ppo_agent.py:256)."""
    ws = _world(group)
    if ws == 1:
        return (returns - returns.mean()) / (returns.std() + 1e-5)
    # all three partial sums in fp64: var = (S2 - n mean^2) / (n - 1) cancels, and a
    # rank holds millions of returns
    r64 = returns.double()
    s = torch.stack([r64.sum(), (r64 * r64).sum(),
                     torch.tensor(float(returns.numel()), dtype=torch.float64, device=returns.device)])
    dist.all_reduce(s, op=dist.ReduceOp.SUM, group=group)
    n = s[2]
    mean = s[0] / n
    var = (s[1] - n * mean * mean) / (n - 1)
    return (returns - mean.float()) / (var.clamp(min=0).sqrt().float() + 1e-5)


class BackgammonPPOAgent:
    def __init__(self, input_size=198, hidden_size=HIDDEN_SIZE, action_size=10,
                 entropy_coef_start=ENTROPY_COEF_START, entropy_coef_end=ENTROPY_COEF_END,
                 entropy_anneal_episodes=ENTROPY_ANNEAL_EPISODES, log_dir=None, s3_bucket_name=None,
                 s3_model_prefix="models/", s3_log_prefix="logs/", device=None, process_group=None,
                 metrics_path: Optional[str] = None):
        if device is None:
            device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.device = torch.device(device)
        self.action_size = action_size
        self.policy_network = PolicyNet(input_size=input_size, hidden_size=hidden_size,
                                        action_size=action_size).to(self.device)
        self.optimizer = optim.Adam(self.policy_network.parameters(), lr=LEARNING_RATE)
        self.gamma = GAMMA
        self.eps_clip = EPS_CLIP
        self.scaler = GradScaler(device=self.device.type)
        self.entropy_coef_start = entropy_coef_start
        self.entropy_coef_end = entropy_coef_end
        self.entropy_anneal_episodes = entropy_anneal_episodes
        self.entropy_coef = entropy_coef_start
        self.last_policy_loss = self.last_value_loss = self.last_entropy_loss = self.last_total_loss = 0.0
        self.s3_bucket_name = None            # S3 is out of scope (offline); local checkpoints only
        self.s3_model_prefix = s3_model_prefix
        self.LOG_INTERVAL = 1000
        self.total_steps = 0
        self.total_episodes = 0
        self.memory = []
        self.losses = []
        self.win_rates = []
        self.training = True
        self.group = process_group
        self.metrics_path = metrics_path
        if log_dir is None:
            log_dir = os.path.join("runs", f"backgammon_ppo_{datetime.now().strftime('%Y%m%d-%H%M%S')}")
        self.log_dir = log_dir
        # keep every rank on identical weights from the start
        if _world(self.group) > 1:
            for p in self.policy_network.parameters():
                dist.broadcast(p.data, src=0, group=self.group)

    # ------------------------------------------------------- rollout side --
    def select_action(self, observations, action_masks=None):
        """ppo_agent.py:138-191 (torch Categorical sampling, per-sample memory)."""
        if isinstance(observations, np.ndarray):
            observations = torch.from_numpy(observations).float()
        observations = observations.to(self.device)
        if observations.dim() == 1:
            observations = observations.unsqueeze(0)
        if action_masks is not None:
            if isinstance(action_masks, np.ndarray):
                action_masks = torch.from_numpy(action_masks).float()
            action_masks = action_masks.to(self.device)
            if action_masks.dim() == 1:
                action_masks = action_masks.unsqueeze(0)
        else:
            action_masks = torch.ones(observations.size(0), self.action_size, device=self.device)
        logits, state_values = self.policy_network(observations)
        masked_logits = logits + (action_masks + 1e-45).log()
        action_probs = torch.softmax(masked_logits, dim=-1)
        dist_ = Categorical(action_probs)
        if self.training:
            actions = dist_.sample()
            action_log_probs = dist_.log_prob(actions)
            for i in range(observations.size(0)):
                self.memory.append({
                    "observation": observations[i].unsqueeze(0),
                    "action_mask": action_masks[i].unsqueeze(0),
                    "action": actions[i].unsqueeze(0),
                    "action_log_prob": action_log_probs[i].unsqueeze(0),
                    "state_value": state_values[i].unsqueeze(0),
                    "reward": None,
                    "done": None,
                })
            return actions.cpu().numpy()
        actions = torch.argmax(action_probs, dim=-1)
        return actions.cpu().numpy()

    def update_entropy_coef(self):                       # ppo_agent.py:193-204
        progress = min(1.0, self.total_episodes / self.entropy_anneal_episodes)
        self.entropy_coef = self.entropy_coef_start - progress * (self.entropy_coef_start - self.entropy_coef_end)

    def compute_returns(self, rewards, dones):           # ppo_agent.py:206-216
        returns = []
        R = 0
        for reward, done in zip(reversed(rewards.cpu().numpy()), reversed(dones.cpu().numpy())):
            if done:
                R = 0
            R = reward + self.gamma * R
            returns.insert(0, R)
        return returns

    # -------------------------------------------------------- update side --
    def ppo_step(self, observations, action_masks, actions, old_log_probs, returns, advantages):
        """NUM_EPOCHS full-batch PPO epochs (ppo_agent.py:268-351) with the
        gradient all-reduce between backward and the optimizer step."""
        pl, vl, el, tl = [], [], [], []
        params = [p for p in self.policy_network.parameters()]
        for _ in range(NUM_EPOCHS):
            with autocast(device_type=self.device.type):
                logits, new_state_values = self.policy_network(observations)
                masked_logits = logits + (action_masks + 1e-45).log()
                action_probs = torch.softmax(masked_logits, dim=-1)
                dist_ = Categorical(action_probs)
                new_log_probs = dist_.log_prob(actions.squeeze(-1))
                ratios = torch.exp(new_log_probs - old_log_probs.detach().squeeze(-1))
                surr1 = ratios * advantages
                surr2 = torch.clamp(ratios, 1 - self.eps_clip, 1 + self.eps_clip) * advantages
                policy_loss = -torch.min(surr1, surr2).mean()
                value_loss = nn.MSELoss()(new_state_values.squeeze(-1), returns)
                entropy_loss = dist_.entropy().mean()
                loss = policy_loss + VALUE_LOSS_COEF * value_loss - self.entropy_coef * entropy_loss
            self.optimizer.zero_grad()
            self.scaler.scale(loss).backward()
            allreduce_mean_([p.grad for p in params if p.grad is not None], self.group)
            self.scaler.step(self.optimizer)
            self.scaler.update()
            pl.append(policy_loss.item())
            vl.append(value_loss.item())
            el.append(entropy_loss.item())
            tl.append(loss.item())
            self.total_steps += 1
        return pl, vl, el, tl

    def update(self):                                    # ppo_agent.py:218-366
        if not self.memory:
            print("No data to update.")
            return
        m = self.memory
        observations = torch.cat([x["observation"] for x in m], dim=0).to(self.device)
        actions = torch.cat([x["action"] for x in m], dim=0).to(self.device)
        action_log_probs = torch.cat([x["action_log_prob"] for x in m], dim=0).to(self.device)
        state_values = torch.cat([x["state_value"] for x in m], dim=0).to(self.device)
        rewards = torch.tensor([x["reward"] for x in m], device=self.device).float()
        dones = torch.tensor([x["done"] for x in m], device=self.device).float()
        action_masks = torch.cat([x["action_mask"] for x in m], dim=0).to(self.device)
        returns = torch.tensor(self.compute_returns(rewards, dones), device=self.device).float()
        returns = global_normalize(returns, self.group)
        advantages = returns - state_values.detach()
        pl, vl, el, tl = self.ppo_step(observations, action_masks, actions, action_log_probs, returns, advantages)
        self.last_policy_loss = float(np.mean(pl))
        self.last_value_loss = float(np.mean(vl))
        self.last_entropy_loss = float(np.mean(el))
        self.last_total_loss = float(np.mean(tl))
        self.losses.append(float(np.sum(tl)) / NUM_EPOCHS)
        self.memory = []
        self.update_entropy_coef()
        if self.metrics_path:
            with open(self.metrics_path, "a") as f:
                f.write(json.dumps({"policy_loss": self.last_policy_loss, "value_loss": self.last_value_loss,
                                    "entropy": self.last_entropy_loss, "total_loss": self.last_total_loss,
                                    "entropy_coef": self.entropy_coef, "total_steps": self.total_steps}) + "\n")

    def set_training_mode(self, training=True):
        self.training = training
        self.policy_network.train(training)
        print(f"Agent set to {'training' if training else 'evaluation'} mode.")

    # ---------------------------------------------------------- checkpoints --
    def save_model(self, filename=None, to_s3=False):
        """Local torch.save of the state_dict (ppo_agent.py:377-386); S3 is offline."""
        os.makedirs("models", exist_ok=True)
        path = os.path.join("models", filename or "ppo_backgammon.pth")
        torch.save(self.policy_network.state_dict(), path)
        return path

    def load_model(self, filename="ppo_backgammon.pth", from_s3=False, training=True):
        if from_s3:
            raise RuntimeError("S3 loading is unavailable offline (SURVEY.md §8c)")
        sd = torch.load(filename, map_location=self.device, weights_only=True)
        self.policy_network.load_state_dict(sd)
        self.policy_network.train(training)
        self.training = training

    def log_metrics(self, total_episodes, avg_reward, win_rate):
        if self.metrics_path:
            with open(self.metrics_path, "a") as f:
                f.write(json.dumps({"episodes": total_episodes, "avg_reward": float(avg_reward),
                                    "win_rate": float(win_rate)}) + "\n")
