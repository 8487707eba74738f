"""MA-PPO actor on the device, fused with the observation.

Reference:
  * ``Actor`` — server/app/core/agents/trainables/network.py:14-33: Linear(num_state, l0), ReLU, ...,
    Linear(l_last, num_action), softmax; ``actor_layers`` default [100, 100]
    (server/app/core/agents/trainables/ppo.py:23-26).
  * ``MAPPO.select_actions`` — server/app/core/agents/trainables/mappo.py:83-97: one batch-1 forward
    per agent over ``norm_state_dict`` (server/app/utils/norm.py:178-218), ``Categorical(p).sample()``,
    ``last_probs[i] = p[action]``.

``Actor`` here is the same torch module (same parameter names ``fc.0 / fc.1 / fc.2``, so a reference
``state_dict`` loads unchanged); it is the training-side network.  ``DeviceActor`` binds its
weights to an ``Environment`` shard and runs ``select_actions`` for every house as ONE HIP launch
(``mdr_actor_act``): obs rows built on chip, both hidden layers on MFMA (split-bf16 by default,
~1e-5 of fp32), softmax + sampling in fp32.  ``rollout`` chains actor -> env.step for n ticks in one
hipGraph (``mdr_actor_rollout``).  There is no CPU path: the library raises when it is missing.
"""
from __future__ import annotations

import json
from typing import Optional

import numpy as np

from . import _lib as L


def _torch():
    import torch

    return torch


def make_actor(num_state: int, num_action: int = 2, layers=(100, 100), seed: Optional[int] = 1):
    """The reference Actor (network.py:14-33) as a torch module; ``seed`` reproduces
    ``torch.manual_seed(seed)`` before construction like MAPPO.__init__ (mappo.py:41-42)."""
    torch = _torch()
    nn = torch.nn

    class Actor(nn.Module):
        def __init__(self):
            super().__init__()
            ls = json.loads(layers) if isinstance(layers, str) else list(layers)
            self.layers = [int(x) for x in ls]
            self.fc = nn.ModuleList([nn.Linear(num_state, self.layers[0])])
            self.fc.extend([nn.Linear(self.layers[i], self.layers[i + 1]) for i in range(len(self.layers) - 1)])
            self.fc.append(nn.Linear(self.layers[-1], num_action))

        def forward(self, x):
            for i in range(len(self.layers)):
                x = torch.nn.functional.relu(self.fc[i](x))
            return torch.nn.functional.softmax(self.fc[len(self.layers)](x), dim=1)

    if seed is not None:
        torch.manual_seed(seed)
    return Actor()


class DeviceActor:
    """``MAPPO.select_actions`` for every house of an Environment shard in one launch."""

    def __init__(self, env, actor, precision: str = "bf16x3", fp32_form: str = "f16_split"):
        """precision: "fp32" (the reference Actor's), "bf16x3" or "bf16".  fp32_form: the fused kernel's
        fp32 arithmetic — "f16_split" (fp16 hi/lo operands, 3 MFMAs per term, per-layer power-of-two
        weight scales; ``status()`` counts tiles whose activations left fp16's range) or "bf16_split3"
        (three-way bf16 operands, 6 MFMAs per term, no range limit)."""
        if precision not in L.PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(L.PRECISIONS)}")
        forms = {"f16_split": L.FP32_F16_SPLIT, "bf16_split3": L.FP32_BF16_SPLIT3}
        if fp32_form not in forms:
            raise ValueError(f"fp32_form must be one of {sorted(forms)}")
        env.shard.set_option("actor_fp32_form", forms[fp32_form])
        self.fp32_form = fp32_form
        if not 1 <= len(actor.layers) <= L.ACTOR_MAX_LAYERS:
            raise ValueError(f"1 to {L.ACTOR_MAX_LAYERS} hidden layers (actor_layers)")
        self.env = env
        self.actor = actor
        self.precision = precision
        self.n_in = actor.fc[0].in_features
        self.n_act = actor.fc[-1].out_features
        self.load_weights()

    def load_weights(self):
        """(Re)pack the actor's current fp32 weights (call after every optimiser step)."""
        torch = _torch()
        sh = self.env.shard
        dev = sh.device
        ws = [lin.weight.detach().to(device=dev, dtype=torch.float32).contiguous() for lin in self.actor.fc]
        bs = [lin.bias.detach().to(device=dev, dtype=torch.float32).contiguous() for lin in self.actor.fc]
        hidden = [lin.out_features for lin in self.actor.fc[:-1]]
        net = L.mdr_actor_net(self.n_in, len(hidden), self.n_act, L.PRECISIONS[self.precision])
        for i, h in enumerate(hidden):
            net.hidden[i] = h
        sh.actor_load_net(net, ws, bs)
        torch.cuda.current_stream(dev).synchronize()  # (the copies are read by later launches only)

    def status(self):
        """mdr_actor_status (synchronises): {range_faults, kernel_prec} — see ``Shard.actor_status``."""
        return self.env.shard.actor_status()

    def fused(self) -> bool:
        """True when this actor runs the fused obs + MLP kernel (k_actor) for the env's obs layout:
        two hidden layers <= 128 wide, <= 128 feature slots, weights within the LDS; otherwise the
        layer chain (k_obs -> k_dense per layer -> k_actor_head)."""
        return self.env.shard.actor_fused(self.env.obs_spec())

    def _check_obs(self, spec):
        if spec.n_feat != self.n_in:
            raise ValueError(f"actor expects {self.n_in} obs features, the environment produces {spec.n_feat}")

    def select_actions(self, action=None, prob=None, probs=None, obs_out=None, count_next: bool = True):
        """Actions for the NEXT env.step of every local house (mappo.py:83-97), on device.
        Returns (action u8 [n_local], prob f32 [n_local]).  With ``count_next`` the launch also
        counts the cluster power these actions produce, so ``env.step_tensor(action)`` is one
        launch."""
        torch = _torch()
        env = self.env
        sh = env.shard
        spec, sc, keep = env.bound_obs_spec()
        self._check_obs(spec)
        n = env.n_local
        if action is None:
            action = torch.empty(n, dtype=torch.uint8, device=sh.device)
        if prob is None:
            prob = torch.empty(n, dtype=torch.float32, device=sh.device)
        sh.actor_act(spec, sc, env._tick, action, prob, probs, obs_out, count_next, use_p_dev=env._P_dev_valid)
        if keep:
            torch.cuda.current_stream(sh.device).synchronize()
        env._counts_ready = ("actor", action.data_ptr()) if count_next else 0
        return action, prob

    def rollout(self, n_ticks: int, rewards=None, actions=None, probs=None, use_graph: bool = True):
        """n_ticks of (select_actions -> env.step) in one graph-captured C call (individual_L2;
        sharded: the library's C loop).  The common penalty modes (common_L2, common_max_error,
        mixture: rewards_calculator.py:29-203) need the cluster's penalty sum / max between the
        step and the reward, so they run tick by tick (select_actions -> step_tensor, whose penalty
        reduce — and allreduce when sharded — finishes every tick's rewards).  ``rewards`` float64
        [n_ticks, N] (or [N], overwritten each tick); ``actions`` u8 / ``probs`` f32 [n_ticks, N]
        (or [N]) optional outputs."""
        torch = _torch()
        env = self.env
        sh = env.shard
        if sh.penalty_mode != 0 or (env.world > 1 and not getattr(env._comm, "native", False)):
            return self._rollout_stepwise(n_ticks, rewards, actions, probs)
        sharded = env.world > 1
        spec, _sc, keep = env.bound_obs_spec() if not sharded else (env.obs_spec(), None, [])
        self._check_obs(spec)
        n = env.n_local
        if rewards is None:
            rewards = torch.empty((n_ticks, n), dtype=torch.float64, device=sh.device)
        rs = 0 if rewards.dim() == 1 else n
        as_ = 0 if actions is None or actions.dim() == 1 else n
        ps = 0 if probs is None or probs.dim() == 1 else n
        if not env._P_dev_valid:
            sh.p_dev.fill_(float(env._P_host))
        done = 0
        while done < n_ticks:  # one window unless interpolation ends it early (driver_window)
            solar0 = float(env._solar)
            ticks = env.driver_window(n_ticks - done)
            k = len(ticks)
            # obs before tick t: signal / OD temperature after tick t-1 (= tick t's s_prev,
            # t_od_prev), solar gain of tick t-1's datetime
            osc = np.zeros((k, 4), np.float64)  # mdr_obs_scalars rows (p unused: p_dev)
            osc[:, 1] = ticks.s_prev
            osc[0, 2] = solar0
            osc[1:, 2] = ticks.solar[:-1]
            osc[:, 3] = ticks.t_od_prev
            sl = (lambda x, st: None if x is None else (x[done:done + k] if st else x))
            if sharded:  # C loop: ring halo + actor + count allreduce + step per tick (RCCL)
                sh.actor_rollout_sharded(ticks, osc, spec, sl(actions, as_), as_, sl(probs, ps), ps,
                                         sl(rewards, rs), rs)
            else:
                g = use_graph and (k == n_ticks or not (rs or as_ or ps))
                sh.actor_rollout(ticks, osc, spec, sl(actions, as_), as_, sl(probs, ps), ps, sl(rewards, rs), rs, g)
            env._P_dev_valid = True
            env.finish_grid_step()
            done += k
        if keep:
            torch.cuda.current_stream(sh.device).synchronize()
        env._counts_ready = 0
        env._P_dev_valid = True
        return rewards


    def _rollout_stepwise(self, n_ticks, rewards, actions, probs):
        """Per tick select_actions (sharded: the ring halo, ON counts of the actions) then
        step_tensor (count allreduce, step, and for the common penalty modes the penalty reduce +
        reward finalize) from Python — the same launches and exchanges as the C loop, plus the
        penalty stages the C loops do not have."""
        torch = _torch()
        env = self.env
        sh = env.shard
        n = env.n_local
        if rewards is None:
            rewards = torch.empty((n_ticks, n), dtype=torch.float64, device=sh.device)
        a_tmp = torch.empty(n, dtype=torch.uint8, device=sh.device)
        p_tmp = torch.empty(n, dtype=torch.float32, device=sh.device)
        for t in range(n_ticks):
            a = a_tmp if actions is None else (actions[t] if actions.dim() == 2 else actions)
            p = p_tmp if probs is None else (probs[t] if probs.dim() == 2 else probs)
            self.select_actions(action=a, prob=p, count_next=True)
            env.step_tensor(a, rewards=rewards[t] if rewards.dim() == 2 else rewards)
        return rewards


def reference_probs(actor, obs):
    """Actor.forward in torch fp32 (the reference network on the same obs) — test helper."""
    torch = _torch()
    with torch.no_grad():
        return actor(obs.float())


def to_numpy(x) -> np.ndarray:
    return x.detach().cpu().numpy()
