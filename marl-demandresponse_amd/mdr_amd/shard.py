"""Device shard: the SoA state of a contiguous range of houses + the libmdr_hip context.

``HipShard`` owns the PyTorch-ROCm tensors (the device container) and issues the C-ABI calls on
the current torch stream.  ``Environment`` drives one shard per process; multi-GPU runs add a
collective (``comm``) between phase 1 and phase 2 of every tick.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L

ON_BIT = np.uint32(1 << 31)
LOCK_BIT = np.uint32(1 << 30)
SSO_MASK = np.uint32((1 << 30) - 1)


def decode_hvac(words: np.ndarray):
    w = words.view(np.uint32)
    return (w & ON_BIT) != 0, (w & LOCK_BIT) != 0, (w & SSO_MASK).astype(np.int64)


def encode_hvac(on, lock, sso) -> np.ndarray:
    w = np.minimum(np.asarray(sso, np.int64), int(SSO_MASK)).astype(np.uint32)
    w |= np.where(np.asarray(on, bool), ON_BIT, np.uint32(0))
    w |= np.where(np.asarray(lock, bool), LOCK_BIT, np.uint32(0))
    return w.view(np.int32)


class HipShard:
    """Houses [offset, offset + n) of a cluster of n_global, on one GPU."""

    def __init__(self, props, n: int, offset: int, n_global: int, device, cap_values, seed: int = 0):
        import torch

        from .drivers import reward_normalisers

        self.lib = L.load()
        if not torch.cuda.is_available():
            raise L.MdrLibraryError("no ROCm GPU visible: the HIP step has no CPU fallback")
        self.torch = torch
        self.device = torch.device(device)
        self.n, self.offset, self.n_global = int(n), int(offset), int(n_global)
        hp = props.cluster_prop.house_prop
        hv = hp.hvac_prop
        rp = props.reward_prop
        pp = rp.penalty_props
        cfg = L.mdr_config()
        cfg.abi_version = L.ABI_VERSION
        cfg.device = self.device.index if self.device.index is not None else torch.cuda.current_device()
        cfg.n_local, cfg.global_offset, cfg.n_global = self.n, self.offset, self.n_global
        cfg.dt = props.time_step.seconds
        cfg.lockout_duration = hv.lockout_duration
        cfg.cop, cfg.lcf, cfg.deadband = hv.cop, hv.latent_cooling_fraction, hp.deadband
        cfg.n_cap = len(cap_values)
        cfg.penalty_mode = L.PEN_MODES[pp.mode]
        for i, v in enumerate(cap_values):
            cfg.cap_table[i] = float(v)
        cfg.alpha_temp, cfg.alpha_sig = rp.alpha_temp, rp.alpha_sig
        cfg.norm_temp, cfg.norm_sig = reward_normalisers(rp, hp)
        cfg.alpha_ind_l2, cfg.alpha_common_l2, cfg.alpha_common_max = (
            pp.alpha_ind_l2, pp.alpha_common_l2, pp.alpha_common_max)
        cfg.seed = seed & 0xFFFFFFFFFFFFFFFF
        self.cfg = cfg
        self.penalty_mode = cfg.penalty_mode
        ctx = C.c_void_p()
        L.check(self.lib.mdr_create(C.byref(ctx), C.byref(cfg)), "mdr_create")
        self.ctx = ctx
        f64 = dict(dtype=torch.float64, device=self.device)
        self.t_air = torch.empty(self.n, **f64)
        self.t_mass = torch.empty(self.n, **f64)
        self.hvac = torch.empty(self.n, dtype=torch.int32, device=self.device)
        self.ua = torch.empty(self.n, **f64)
        self.ca = torch.empty(self.n, **f64)
        self.cm = torch.empty(self.n, **f64)
        self.hm = torch.empty(self.n, **f64)
        self.target = torch.empty(self.n, **f64)
        self.cap_idx = torch.empty(self.n, dtype=torch.uint8, device=self.device)
        self.reward = torch.zeros(self.n, **f64)
        self.action = torch.zeros(self.n, dtype=torch.uint8, device=self.device)
        self.p_dev = torch.zeros(1, **f64)
        self._bind()

    # ------------------------------------------------------------------ plumbing
    def _bind(self):
        soa = L.mdr_soa(*(L.ptr(t) for t in (self.t_air, self.t_mass, self.hvac, self.ua, self.ca,
                                             self.cm, self.hm, self.target, self.cap_idx)))
        L.check(self.lib.mdr_bind(self.ctx, C.byref(soa)), "mdr_bind")

    def stream(self):
        return L.stream_handle(self.device)

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.mdr_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ population / state
    def upload(self, pop: dict, cap_idx: np.ndarray, t_air, t_mass, hvac_words):
        t = self.torch
        dev = self.device
        for name in ("ua", "ca", "cm", "hm", "target"):
            getattr(self, name).copy_(t.from_numpy(np.ascontiguousarray(pop[name], np.float64)).to(dev))
        self.cap_idx.copy_(t.from_numpy(np.ascontiguousarray(cap_idx, np.uint8)).to(dev))
        self.t_air.copy_(t.from_numpy(np.ascontiguousarray(t_air, np.float64)).to(dev))
        self.t_mass.copy_(t.from_numpy(np.ascontiguousarray(t_mass, np.float64)).to(dev))
        self.hvac.copy_(t.from_numpy(np.ascontiguousarray(hvac_words, np.int32)).to(dev))
        self.params_changed()

    def set_rollout_window(self, ticks: int):
        """Ticks per temporally blocked rollout launch (0: one launch per tick), mdr_set_rollout_window."""
        L.check(self.lib.mdr_set_rollout_window(self.ctx, int(ticks)), "mdr_set_rollout_window")

    def set_option(self, name: str, value: int):
        """mdr_set_option: an alternative launch form of the same computation (mdr.h MDR_OPT_*:
        step_tpw, fastdiv, window_pipeline, sharded_overlap, greedy_sort, force_halo, halo_overlap,
        actor_generic, window_thermal, halo_in_counts, gq_band, actor_fp32_form)."""
        L.check(self.lib.mdr_set_option(self.ctx, L.OPTIONS[name], int(value)), f"mdr_set_option({name})")

    def params_changed(self):
        L.check(self.lib.mdr_params_changed(self.ctx), "mdr_params_changed")

    def populate(self, hp, cap_values):
        """Synthetic population on device; the capacity of a house is a uniform entry of
        cooling_capacity_list (random.choices, hvac.py:68-70), mapped into ``cap_values``."""
        nz = hp.noise_prop
        spec = L.mdr_pop_spec(hp.target_temp, nz.std_target_temp, nz.factor_thermo_low,
                              nz.factor_thermo_high, hp.Ca, hp.Cm, hp.Hm, hp.init_air_temp,
                              hp.init_mass_temp)
        lst = list(hp.hvac_prop.noise_prop.cooling_capacity_list)
        spec.n_draw = len(lst)
        for k, v in enumerate(lst):
            spec.draw_idx[k] = list(cap_values).index(v)
        L.check(self.lib.mdr_populate(self.ctx, C.byref(spec), self.stream()), "mdr_populate")

    # ------------------------------------------------------------------ tick
    def power_counts(self, action, mode: int, tick: int):
        L.check(self.lib.mdr_power_counts(self.ctx, L.ptr(action), mode, tick, self.stream()),
                "mdr_power_counts")

    def graph_info(self):
        """{rollout_graphs, actor_graphs, rollout_launches, actor_launches, guarded, guarded_nodes}:
        cached graphs, hipGraphLaunch calls, and the captures the memset guard walked (mdr_graph_info)."""
        out = (C.c_int64 * 6)()
        rc = self.lib.mdr_graph_info(self.ctx, out, 6)
        L.check(0 if rc == 6 else rc, "mdr_graph_info")
        return dict(zip(("rollout_graphs", "actor_graphs", "rollout_launches", "actor_launches", "guarded",
                         "guarded_nodes"), list(out)))

    def graph_memset_probe(self):
        """mdr_graph_memset_probe: a memset node captured in this context, its parameters and what
        its replays leave in the count slabs (diagnostic; synchronises and overwrites the slabs)."""
        out = (C.c_int64 * 13)()
        L.check(self.lib.mdr_graph_memset_probe(self.ctx, out, 13, self.stream()), "mdr_graph_memset_probe")
        keys = ("nodes", "memset_nodes", "dst_ok", "value", "element_size", "width", "height", "pitch", "bytes",
                "nonzero_replay1", "nonzero_replay2", "nonzero_replay3", "nonzero_kernel_zero")
        return dict(zip(keys, list(out)))

    def counts_buffer(self):
        p = C.c_void_p()
        n = C.c_int()
        L.check(self.lib.mdr_counts_buffer(self.ctx, C.byref(p), C.byref(n)), "mdr_counts_buffer")
        return p.value, n.value

    def step(self, action, mode: int, tick: L.mdr_tick, lookahead: int = 0, ctrl: int = 0,
             ctrl_out=None, reward=None):
        reward = self.reward if reward is None else reward
        L.check(self.lib.mdr_step(self.ctx, L.ptr(action), mode, C.byref(tick), L.ptr(reward),
                                  lookahead, ctrl, L.ptr(ctrl_out), L.ptr(self.p_dev), self.stream()),
                "mdr_step")
        return reward

    def penalty_partials(self):
        L.check(self.lib.mdr_penalty_partials(self.ctx, self.stream()), "mdr_penalty_partials")
        p = C.c_void_p()
        L.check(self.lib.mdr_penalty_buffer(self.ctx, C.byref(p)), "mdr_penalty_buffer")
        return p.value

    def reward_finalize(self, tick: L.mdr_tick, reward=None):
        reward = self.reward if reward is None else reward
        L.check(self.lib.mdr_reward_finalize(self.ctx, C.byref(tick), L.ptr(reward), self.stream()),
                "mdr_reward_finalize")

    def rollout(self, ticks, action, act_stride, mode, reward, rew_stride, use_graph=True):
        """Many ticks in one C call (``ticks``: a TickWindow), on the caller's current stream; with
        ``use_graph`` the drivers are staged and the launch sequence is captured once (on the
        library's capture stream) and replayed as a hipGraph; without, the windows are launched
        directly with the first window's drivers as kernel arguments."""
        L.check(self.lib.mdr_rollout(self.ctx, len(ticks), ticks.ptr(), L.ptr(action), act_stride, mode,
                                     L.ptr(reward), rew_stride, L.ptr(self.p_dev), int(use_graph), self.stream()),
                "mdr_rollout")

    def rollout_begin(self, n, tick0, action, act_stride, mode):
        """mdr_rollout_begin: the first window's count, launched before the host computes the drivers."""
        L.check(self.lib.mdr_rollout_begin(self.ctx, n, tick0, L.ptr(action), act_stride, mode, self.stream()),
                "mdr_rollout_begin")

    def time_step_kernels(self, ticks, action, act_stride, mode, reward, rew_stride):
        """mdr_time_step_kernels: (summed step-kernel ms, step launches) of one directly launched rollout."""
        ms, nl = C.c_float(), C.c_int()
        L.check(self.lib.mdr_time_step_kernels(self.ctx, len(ticks), ticks.ptr(), L.ptr(action), act_stride, mode,
                                               L.ptr(reward), rew_stride, self.stream(), C.byref(ms), C.byref(nl)),
                "mdr_time_step_kernels")
        return float(ms.value), int(nl.value)

    def launch_stream(self):
        """The torch stream rollout kernels run on (the caller's current stream) — where timing
        events must be recorded."""
        return self.torch.cuda.current_stream(self.device)

    def cluster_stats(self, reward, out):
        """out (device float64 [12]) <- mdr_cluster_stats of the current state (+ reward or None)."""
        L.check(self.lib.mdr_cluster_stats(self.ctx, L.ptr(reward), L.ptr(out), self.stream()), "mdr_cluster_stats")

    def msg_pack(self, spec, out):
        """Message features of every local house into out [n_local, msg_w] (mdr_msg_pack)."""
        L.check(self.lib.mdr_msg_pack(self.ctx, C.byref(spec), L.ptr(out), self.stream()), "mdr_msg_pack")

    def greedy_inputs(self, key, power, lock):
        """This shard's greedy rows: key = -(T - target), P, lockout (mdr_greedy_inputs)."""
        L.check(self.lib.mdr_greedy_inputs(self.ctx, L.ptr(key), L.ptr(power), L.ptr(lock), self.stream()),
                "mdr_greedy_inputs")

    def greedy_select(self, n: int, key, power, lock, budget: float, action):
        """Greedy decisions over n gathered rows (mdr_greedy_select)."""
        L.check(self.lib.mdr_greedy_select(self.ctx, int(n), L.ptr(key), L.ptr(power), L.ptr(lock), float(budget),
                                           L.ptr(action), self.stream()), "mdr_greedy_select")

    def greedy(self, budget: float, action):
        L.check(self.lib.mdr_ctrl_greedy(self.ctx, float(budget), L.ptr(action), self.stream()),
                "mdr_ctrl_greedy")

    def greedy_rollout(self, ticks, action, act_stride, reward, rew_stride):
        """mdr_greedy_rollout: config C3's greedy -> step loop over a TickWindow in one C call."""
        L.check(self.lib.mdr_greedy_rollout(self.ctx, len(ticks), ticks.ptr(), L.ptr(action), act_stride,
                                            L.ptr(reward), rew_stride, L.ptr(self.p_dev), self.stream()),
                "mdr_greedy_rollout")

    # ---- sharded histogram select (mdr_gq_shard_*): the stages between the comm's collectives
    def gq_shard_begin(self) -> dict:
        """This shard's key codes, superbin histogram and key range; returns zero-copy views of the
        buffers the collectives work on: super / bins (int32 views of the uint32 class-count
        histograms: sum-allreduce), range ((min, -max): min-allreduce), window (uint8: all-gather)."""
        from .distributed import device_view

        L.check(self.lib.mdr_gq_shard_begin(self.ctx, self.stream()), "mdr_gq_shard_begin")
        sp, bp, rp, wp = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
        ns, nb, wb = C.c_int64(), C.c_int64(), C.c_int64()
        L.check(self.lib.mdr_gq_shard_buffers(self.ctx, C.byref(sp), C.byref(ns), C.byref(bp), C.byref(nb),
                                              C.byref(rp), C.byref(wp), C.byref(wb)), "mdr_gq_shard_buffers")
        return {"super": device_view(sp.value, ns.value, "<i4", self.device),
                "bins": device_view(bp.value, nb.value, "<i4", self.device),
                "range": device_view(rp.value, 2, "<f8", self.device),
                "window": device_view(wp.value, wb.value, "|u1", self.device)}

    def gq_shard_bins(self, budget: float):
        L.check(self.lib.mdr_gq_shard_bins(self.ctx, float(budget), self.stream()), "mdr_gq_shard_bins")

    def gq_shard_compact(self, budget: float, action):
        L.check(self.lib.mdr_gq_shard_compact(self.ctx, float(budget), L.ptr(action), self.stream()),
                "mdr_gq_shard_compact")

    def gq_shard_select(self, budget: float, gathered, world: int, action):
        L.check(self.lib.mdr_gq_shard_select(self.ctx, float(budget), L.ptr(gathered), int(world), L.ptr(action),
                                             self.stream()), "mdr_gq_shard_select")

    def gq_shard_fallback(self) -> bool:
        """True when this call's window could not decide (synchronises): use the all-gather form."""
        v = C.c_int()
        L.check(self.lib.mdr_gq_shard_fallback(self.ctx, C.byref(v), self.stream()), "mdr_gq_shard_fallback")
        return bool(v.value)

    def greedy_fallbacks(self) -> int:
        """mdr_ctrl_greedy calls whose histogram select fell back to the full sort (mdr_greedy_fallbacks)."""
        v = C.c_uint64()
        L.check(self.lib.mdr_greedy_fallbacks(self.ctx, C.byref(v)), "mdr_greedy_fallbacks")
        return int(v.value)

    def greedy_diag(self) -> dict:
        """Histogram-select diagnostics (mdr_greedy_diag; synchronises)."""
        v = (C.c_uint64 * 4)()
        L.check(self.lib.mdr_greedy_diag(self.ctx, v), "mdr_greedy_diag")
        return {"fallbacks": int(v[0]), "calls": int(v[1]), "window_sum": int(v[2]), "window_last": int(v[3])}

    def greedy_state(self) -> dict:
        """The select's state after its last stage (mdr_greedy_state; synchronises)."""
        v = (C.c_uint64 * 12)()
        L.check(self.lib.mdr_greedy_state(self.ctx, v), "mdr_greedy_state")
        names = ("fallbacks", "calls", "window_sum", "window_last", "sb", "bstar", "bend", "all", "overflow",
                 "more_after", "wcount", "need_fb")
        return {k: C.c_int64(v[i]).value for i, k in enumerate(names)}

    def greedy_band(self) -> dict:
        """The predicted band's record (mdr_greedy_band; synchronises): calls whose bins pass the
        band let k_gq_binsc skip, calls, misses, and the band the next GQ step counts."""
        v = (C.c_uint64 * 4)()
        L.check(self.lib.mdr_greedy_band(self.ctx, v), "mdr_greedy_band")
        return {"skips": int(v[0]), "calls": int(v[1]), "misses": int(v[1]) - int(v[0]), "band_base": int(v[2]),
                "band_width": int(v[3])}

    def greedy_fused_diag(self) -> dict:
        """The fused tick's counters (mdr_greedy_fused_diag; synchronises): decisions, band hits,
        misses (the decision's own pass over the cluster), exact decisions, the last mode and window."""
        v = (C.c_uint64 * 6)()
        L.check(self.lib.mdr_greedy_fused_diag(self.ctx, v), "mdr_greedy_fused_diag")
        return {"calls": int(v[0]), "hits": int(v[1]), "misses": int(v[2]), "exact": int(v[3]),
                "last_mode": int(v[4]), "last_window": int(v[5])}

    def obs(self, spec, scalars, out, use_p_dev=True):
        L.check(self.lib.mdr_obs(self.ctx, C.byref(spec), C.byref(scalars),
                                 L.ptr(self.p_dev) if use_p_dev else 0, L.ptr(out), self.stream()),
                "mdr_obs")

    # ------------------------------------------------------------------ MA-PPO actor (row P)
    def actor_load(self, spec, w1, b1, w2, b2, w3, b3):
        L.check(self.lib.mdr_actor_load(self.ctx, C.byref(spec), *(L.ptr(t) for t in (w1, b1, w2, b2, w3, b3)),
                                        self.stream()), "mdr_actor_load")

    def actor_load_net(self, net, weights, biases):
        """mdr_actor_load_net: any number of hidden layers (weights / biases: device fp32 tensors,
        fc.0 .. fc.L in order)."""
        n = len(weights)
        w = (C.c_void_p * n)(*[L.ptr(t) for t in weights])
        b = (C.c_void_p * n)(*[L.ptr(t) for t in biases])
        L.check(self.lib.mdr_actor_load_net(self.ctx, C.byref(net), w, b, self.stream()), "mdr_actor_load_net")

    def actor_status(self):
        """mdr_actor_status (synchronises; counts since the last call): {range_faults: fused fp16-split
        tiles that met a non-finite logit, kernel_prec: 1 bf16 / 3 bf16x3 / 4 fp16 split / 6 three-way
        bf16, exact: tiles whose values left fp16's range, their logits computed in scalar fp32}."""
        out = (C.c_int64 * 3)()
        L.check(self.lib.mdr_actor_status(self.ctx, out, 3, self.stream()), "mdr_actor_status")
        return {"range_faults": int(out[0]), "kernel_prec": int(out[1]), "exact": int(out[2])}

    def actor_fused(self, spec) -> bool:
        """True when the loaded actor runs the fused k_actor for this obs layout (else the chain)."""
        r = self.lib.mdr_actor_fused(self.ctx, C.byref(spec))
        if r < 0:
            L.check(r, "mdr_actor_fused")
        return r == 1

    def actor_act(self, spec, scalars, tick, action, prob, probs, obs_out, count_next, use_p_dev=True):
        L.check(self.lib.mdr_actor_act(self.ctx, C.byref(spec), C.byref(scalars),
                                       L.ptr(self.p_dev) if use_p_dev else 0, int(tick), L.ptr(action),
                                       L.ptr(prob), L.ptr(probs), L.ptr(obs_out), int(count_next),
                                       self.stream()), "mdr_actor_act")

    def actor_rollout(self, ticks, obs_sc, spec, action, act_stride, prob, prob_stride, reward, rew_stride,
                      use_graph=True):
        """n ticks of actor -> step in one C call (graph-captured, replayed on the current stream).
        ``ticks``: TickWindow; ``obs_sc``: float64 [n, 4] array in the mdr_obs_scalars layout."""
        n = len(ticks)
        obs_sc = np.ascontiguousarray(obs_sc, np.float64)
        assert obs_sc.shape == (n, 4)
        L.check(self.lib.mdr_actor_rollout(self.ctx, n, ticks.ptr(), obs_sc.ctypes.data, C.byref(spec),
                                           L.ptr(action), act_stride, L.ptr(prob), prob_stride, L.ptr(reward),
                                           rew_stride, L.ptr(self.p_dev), int(use_graph), self.stream()),
                "mdr_actor_rollout")

    def actor_rollout_sharded(self, ticks, obs_sc, spec, action, act_stride, prob, prob_stride, reward,
                              rew_stride):
        """n ticks of ring halo -> actor -> count allreduce -> step over the RCCL communicator
        (mdr_actor_rollout_sharded), on the caller's current stream."""
        n = len(ticks)
        obs_sc = np.ascontiguousarray(obs_sc, np.float64)
        assert obs_sc.shape == (n, 4)
        L.check(self.lib.mdr_actor_rollout_sharded(self.ctx, n, ticks.ptr(), obs_sc.ctypes.data, C.byref(spec),
                                                   L.ptr(action), act_stride, L.ptr(prob), prob_stride,
                                                   L.ptr(reward), rew_stride, L.ptr(self.p_dev), self.stream()),
                "mdr_actor_rollout_sharded")

    def interp_load(self, grids, values, cfg):
        """Monte-Carlo table + axes to the device (mdr_interp_load, synchronous)."""
        grid = np.ascontiguousarray(np.concatenate([np.asarray(g, np.float64) for g in grids]))
        vals = np.ascontiguousarray(values, np.float64).reshape(-1)
        spec = L.mdr_interp_spec()
        spec.len[:] = [len(g) for g in grids]
        spec.grid, spec.values = grid.ctypes.data, vals.ctypes.data
        spec.cfg_ua, spec.cfg_cm, spec.cfg_ca, spec.cfg_hm = (float(x) for x in cfg)
        L.check(self.lib.mdr_interp_load(self.ctx, C.byref(spec)), "mdr_interp_load")

    def interp_values(self, ids, od, hour, date, vals):
        L.check(self.lib.mdr_interp_values(self.ctx, L.ptr(ids), int(ids.numel()), float(od), float(hour),
                                           float(date), L.ptr(vals), self.stream()), "mdr_interp_values")

    def interp_sum(self, vals, factor, out):
        L.check(self.lib.mdr_interp_sum(L.ptr(vals), int(vals.numel()), float(factor), L.ptr(out),
                                        self.stream()), "mdr_interp_sum")

    def halo_pack(self, spec, out):
        L.check(self.lib.mdr_halo_pack(self.ctx, C.byref(spec), L.ptr(out), self.stream()), "mdr_halo_pack")

    # ------------------------------------------------------------------ host views
    def host_state(self):
        t = self.torch
        t.cuda.current_stream(self.device).synchronize()
        on, lock, sso = decode_hvac(self.hvac.cpu().numpy())
        return {"T": self.t_air.cpu().numpy(), "Tm": self.t_mass.cpu().numpy(), "on": on, "lock": lock,
                "sso": sso}

    def host_params(self):
        return {k: getattr(self, k).cpu().numpy() for k in ("ua", "ca", "cm", "hm", "target", "cap_idx")}
