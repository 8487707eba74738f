"""MA-PPO on the device: rollout storage and the PPO update.

Reference: ``MAPPO`` — server/app/core/agents/trainables/mappo.py:37-217 (properties:
``PPOProperties``, ppo.py:20-70; networks: network.py:14-58), driven by TrainingManager.start
(server/app/services/training_manager.py:183-263, update every ``time_steps_per_epoch``).

What is the same: the actor / critic modules and their initialisation order under
``torch.manual_seed(seed)``; Adam optimisers; the discounted return over the buffer in the
reference's storage order (tick-major, house-minor — the reference's ``R`` runs across houses of a
tick; ``returns="per_agent"`` discounts each house over its own ticks instead); ``ppo_update_time``
epochs of ``BatchSampler(SubsetRandomSampler(range(L)), batch_size)`` minibatches drawn from the
global torch CPU generator exactly as the reference draws them; the clipped surrogate on the ratio of
new to stored action probabilities, ``clip_grad_norm_``, and the critic's MSE to the returns.

What is changed, deliberately:
  * ``store_transition`` is O(N) per tick on device tensors (the reference deep-copies the action
    dict per house: O(N^2));
  * the critic input.  The reference builds ``Critic(num_state + num_action - 1)`` but feeds it
    ``state ++ others_actions`` — N-1 extra columns — so it only runs at N = 2 (mappo.py:50-53,
    113-115, 172-174).  Here the extra column is the mean of the other houses' actions, which has
    the declared width and equals the reference's input at N = 2 (tests/test_mappo_gpu.py pins the
    update against the reference MAPPO at N = 2).
Actions are sampled by the fused device actor (mdr_amd.actor.DeviceActor, Philox), not by torch's
Categorical RNG.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from .actor import DeviceActor, make_actor


def _torch():
    import torch

    return torch


@dataclass
class MAPPOConfig:
    """PPOProperties (ppo.py:20-70) defaults."""

    actor_layers: List[int] = field(default_factory=lambda: [100, 100])
    critic_layers: List[int] = field(default_factory=lambda: [100, 100])
    gamma: float = 0.99
    lr_critic: float = 3e-3
    lr_actor: float = 3e-3
    clip_param: float = 0.2
    max_grad_norm: float = 0.5
    ppo_update_time: int = 10
    batch_size: int = 256


def make_critic(num_state: int, layers=(100, 100)):
    """The reference Critic (network.py:36-51): Linear layers with ReLU, one output."""
    torch = _torch()
    nn = torch.nn

    class Critic(nn.Module):
        def __init__(self):
            super().__init__()
            self.layers = [int(x) for x in layers]
            self.fc = nn.ModuleList([nn.Linear(num_state, self.layers[0])])
            self.fc.extend([nn.Linear(self.layers[i], self.layers[i + 1]) for i in range(len(self.layers) - 1)])
            self.fc.append(nn.Linear(self.layers[-1], 1))

        def forward(self, x):
            for i in range(len(self.layers)):
                x = torch.nn.functional.relu(self.fc[i](x))
            return self.fc[len(self.layers)](x)

    return Critic()


def _suffix_affine(r, c):
    """G_i = r_i + c_i * G_{i+1} with G_L = 0, over 1-D float64 tensors, without a host round trip:
    a reverse recurrence inside ~sqrt(L) blocks of ~sqrt(L), the blocks' carries by the same scan one
    level down (G entering block b is itself a suffix recurrence over the blocks), one fix-up pass."""
    torch = _torch()
    L = r.numel()
    if L <= 64:
        g = torch.empty_like(r)
        nxt = r.new_zeros(())
        for j in range(L - 1, -1, -1):
            nxt = r[j] + c[j] * nxt
            g[j] = nxt
        return g
    M = int(np.ceil(np.sqrt(L)))
    B = -(-L // M)
    pad = B * M - L  # (padding after the end: r = c = 0, so G stays 0 there)
    r2 = torch.cat([r, r.new_zeros(pad)]).view(B, M)
    c2 = torch.cat([c, c.new_zeros(pad)]).view(B, M)
    g = torch.empty_like(r2)
    nxt = r.new_zeros(B)
    for j in range(M - 1, -1, -1):  # local returns, each block as if it ended the buffer
        nxt = r2[:, j] + c2[:, j] * nxt
        g[:, j] = nxt
    suf = torch.flip(torch.cumprod(torch.flip(c2, [1]), 1), [1])  # prod_{k >= j} c_k within the block
    # carry[b] = G at the first element of block b + 1 = g[b+1, 0] + suf[b+1, 0] * carry[b+1]
    carry = torch.cat([_suffix_affine(g[1:, 0].contiguous(), suf[1:, 0].contiguous()), r.new_zeros(1)])
    return (g + suf * carry[:, None]).reshape(-1)[:L]


def discounted_returns(reward, done, gamma: float):
    """G_i = r_i + gamma * (0 if done_i else G_{i+1}) over a 1-D device tensor (the reference's
    reversed loop, mappo.py:135-140), as the blocked scan of _suffix_affine: float64, on the
    tensor's device, no host synchronisation."""
    torch = _torch()
    if reward.numel() == 0:
        return reward.double().clone()
    return _suffix_affine(reward.double(), gamma * (1.0 - done.double()))


class DeviceMAPPO:
    """MAPPO with device actor rollouts, device transition storage and the PPO update on the GPU."""

    def __init__(self, env, config: Optional[MAPPOConfig] = None, num_action: int = 2, seed: int = 1,
                 precision: str = "bf16x3", returns: str = "reference", sampler: str = "reference"):
        """``sampler``: the minibatch permutation of each PPO epoch — "reference" (default) draws it
        from the global torch CPU generator exactly as the reference's SubsetRandomSampler does, so
        reference-seeded runs keep the reference's minibatch order and later CPU draws at any size;
        "device" (explicit opt-in) draws it on the GPU (torch.randperm on the device generator: no
        L-element host permutation and copy per epoch at C5's N x T transitions; another order);
        "auto" = "reference" up to 2^20 transitions and "device" beyond.  ``last_sampler`` records
        which one the last update used."""
        torch = _torch()
        if returns not in ("reference", "per_agent"):
            raise ValueError("returns must be 'reference' (the reference's buffer order) or 'per_agent'")
        if sampler not in ("auto", "reference", "device"):
            raise ValueError("sampler must be 'auto', 'reference' or 'device'")
        self.sampler = sampler
        self.last_sampler = None
        self.cfg = config or MAPPOConfig()
        self.env = env
        self.returns = returns
        num_state = env.obs_spec().n_feat
        self.num_state, self.num_action = num_state, num_action
        torch.manual_seed(seed)  # mappo.py:41-42: actor then critic initialised from this stream
        self.actor_net = make_actor(num_state, num_action, self.cfg.actor_layers, seed=None)
        self.critic_net = make_critic(num_state + num_action - 1, self.cfg.critic_layers)
        dev = env.shard.device
        self.actor_net.to(dev)
        self.critic_net.to(dev)
        self.actor_optimizer = torch.optim.Adam(self.actor_net.parameters(), self.cfg.lr_actor)
        self.critic_net_optimizer = torch.optim.Adam(self.critic_net.parameters(), self.cfg.lr_critic)
        self.device_actor = DeviceActor(env, self.actor_net, precision=precision)
        self.buffer = []  # per tick: (state, action, prob, reward, done)
        self.counter = 0
        self.training_step = 0
        self.last_actions = None
        self.last_probs = None

    # ---------------------------------------------------------------- rollout
    def select_actions(self):
        """MAPPO.select_actions for every local house from the env's current state (fused obs +
        actor + sampling, one launch); the actions' ON counts are prepared for the next step."""
        a, p = self.device_actor.select_actions(count_next=True)
        self.last_actions, self.last_probs = a, p
        return a

    def store_transition(self, observations, next_observations, rewards, done: bool) -> None:
        """mappo.py:105-126 for all houses at once: device tensors obs float32 [N, F], rewards float
        [N] (the last select_actions' actions and probabilities).  ``next_observations`` is accepted
        for the reference's signature but not kept: update never reads it (mappo.py:128-217)."""
        self.buffer.append((observations, self.last_actions.clone(), self.last_probs.clone(),
                            rewards.clone(), bool(done)))
        self.counter += observations.shape[0]

    def __len__(self) -> int:
        return sum(b[0].shape[0] for b in self.buffer)

    # ---------------------------------------------------------------- update
    def _returns(self, reward, done_rows, n):
        if self.returns == "reference":
            return discounted_returns(reward.reshape(-1), done_rows.reshape(-1), self.cfg.gamma)
        # each house over its own ticks: the same recurrence along the tick axis, houses in parallel
        torch = _torch()
        T = reward.shape[0]
        g = torch.empty_like(reward, dtype=torch.float64)
        nxt = torch.zeros(n, dtype=torch.float64, device=reward.device)
        for t in range(T - 1, -1, -1):
            nxt = reward[t].double() + self.cfg.gamma * (1.0 - done_rows[t].double()) * nxt
            g[t] = nxt
        return g.reshape(-1)

    def update(self, t=None) -> bool:
        """mappo.py:128-217: returns, then ppo_update_time epochs of minibatch PPO steps.  Returns
        False (and keeps the buffer) while it holds fewer than batch_size transitions."""
        torch = _torch()
        F = torch.nn.functional
        L = len(self)
        if L < self.cfg.batch_size:
            return False
        cfg = self.cfg
        state = torch.cat([b[0] for b in self.buffer]).float()
        act = torch.cat([b[1] for b in self.buffer]).long().view(-1, 1)
        old_prob = torch.cat([b[2] for b in self.buffer]).float().view(-1, 1)
        n = self.buffer[0][0].shape[0]
        acts = torch.stack([b[1] for b in self.buffer]).double()  # [T, N]
        n_glob = self.env.n
        tot = acts.sum(1, keepdim=True)
        if self.env.world > 1:
            self.env._comm.allreduce_sum(self.env.shard, tot)
        others = ((tot - acts) / max(n_glob - 1, 1)).float().reshape(-1, 1)  # mean of the other houses' actions
        reward = torch.stack([b[3] for b in self.buffer])  # [T, N]
        done = torch.tensor([b[4] for b in self.buffer], dtype=torch.float64, device=reward.device)
        done_rows = done[:, None].expand(-1, n)
        Gt = self._returns(reward, done_rows, n).float()
        critic_in = torch.cat([state, others], 1)
        on_device = self.sampler == "device" or (self.sampler == "auto" and L > (1 << 20))
        self.last_sampler = "device" if on_device else "reference"
        for _ in range(cfg.ppo_update_time):
            # SubsetRandomSampler + BatchSampler(drop_last=False): a permutation (the global CPU
            # generator's, or the device generator's — see sampler), cut in order into batch_size chunks
            perm = torch.randperm(L, device=state.device) if on_device else torch.randperm(L).to(state.device)
            for k in range(0, L, cfg.batch_size):
                idx = perm[k:k + cfg.batch_size]
                Gt_index = Gt[idx].view(-1, 1)
                V = self.critic_net(critic_in[idx])
                advantage = (Gt_index - V).detach()
                action_prob = self.actor_net(state[idx]).gather(1, act[idx])
                ratio = action_prob / old_prob[idx]
                clipped_ratio = torch.clamp(ratio, 1 - cfg.clip_param, 1 + cfg.clip_param)
                action_loss = -torch.min(ratio * advantage, clipped_ratio * advantage).mean()
                self.actor_optimizer.zero_grad()
                action_loss.backward()
                torch.nn.utils.clip_grad_norm_(self.actor_net.parameters(), cfg.max_grad_norm)
                self.actor_optimizer.step()
                value_loss = F.mse_loss(Gt_index, V)
                self.critic_net_optimizer.zero_grad()
                value_loss.backward()
                torch.nn.utils.clip_grad_norm_(self.critic_net.parameters(), cfg.max_grad_norm)
                self.critic_net_optimizer.step()
                self.training_step += 1
        del self.buffer[:]
        self.device_actor.load_weights()  # the fused kernel's packed weights follow the update
        return True

    def save(self, path: str, time_step=None) -> None:
        import os

        torch = _torch()
        os.makedirs(path, exist_ok=True)
        name = "actor" + (str(time_step) if time_step else "") + ".pth"
        torch.save(self.actor_net.state_dict(), os.path.join(path, name))
