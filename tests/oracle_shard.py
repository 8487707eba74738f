"""Test doubles for the multi-process path on CPU (gloo): a shard that computes with the oracle
and a comm over torch.distributed/gloo.  They implement the interface mdr_amd.Environment drives
(HipShard / RcclComm), so the sharding, replicated drivers and per-tick exchanges of the product
orchestration are exercised without a GPU.  Never used by the product path."""
from __future__ import annotations

import numpy as np
import torch

from mdr_amd import _lib as L
from mdr_amd.drivers import reward_normalisers
from mdr_amd.shard import decode_hvac, encode_hvac
from oracle import env_np as O


class OracleShard:
    def __init__(self, props, n, offset, n_global, device, cap_values, seed=0):
        self.props = props
        self.n, self.offset, self.n_global = int(n), int(offset), int(n_global)
        self.device = torch.device("cpu")
        self.cap_values = [float(c) for c in cap_values]
        self.penalty_mode = L.PEN_MODES[props.reward_prop.penalty_props.mode]
        f64 = dict(dtype=torch.float64)
        self.t_air = torch.zeros(self.n, **f64)
        self.t_mass = torch.zeros(self.n, **f64)
        self.hvac = torch.zeros(self.n, dtype=torch.int32)
        for k in ("ua", "ca", "cm", "hm", "target"):
            setattr(self, k, torch.zeros(self.n, **f64))
        self.cap_idx = torch.zeros(self.n, dtype=torch.uint8)
        self.reward = torch.zeros(self.n, **f64)
        self.action = torch.zeros(self.n, dtype=torch.uint8)
        self.p_dev = torch.zeros(1, **f64)
        self.counts = torch.zeros(len(cap_values), dtype=torch.int64)
        self.partial2 = torch.zeros(2, **f64)

    def close(self):
        pass

    def params_changed(self):
        pass

    def upload(self, pop, cap_idx, t_air, t_mass, hvac_words):
        for k in ("ua", "ca", "cm", "hm", "target"):
            getattr(self, k).copy_(torch.from_numpy(np.asarray(pop[k], np.float64)))
        self.cap_idx.copy_(torch.from_numpy(np.asarray(cap_idx, np.uint8)))
        self.t_air.copy_(torch.from_numpy(np.asarray(t_air, np.float64)))
        self.t_mass.copy_(torch.from_numpy(np.asarray(t_mass, np.float64)))
        self.hvac.copy_(torch.from_numpy(np.asarray(hvac_words, np.int32)))

    def _caps(self):
        return np.asarray(self.cap_values)[self.cap_idx.numpy()]

    def _actions(self, action, mode):
        if mode == L.ACT_BUFFER:
            return action.numpy().astype(bool)
        if mode == L.ACT_ALWAYS_ON:
            return np.ones(self.n, bool)
        raise NotImplementedError("oracle shard: buffer / always-on actions only")

    def power_counts(self, action, mode, tick):
        on, lock, sso = decode_hvac(self.hvac.numpy())
        hv = self.props.cluster_prop.house_prop.hvac_prop
        on1, _, _ = O.hvac_step(on, lock, sso, self._actions(action, mode), hv.lockout_duration,
                                self.props.time_step.seconds)
        idx = self.cap_idx.numpy()
        self.counts.copy_(torch.from_numpy(np.bincount(idx[on1], minlength=len(self.cap_values)).astype(np.int64)))

    def step(self, action, mode, tick, lookahead=0, ctrl=0, ctrl_out=None, reward=None):
        p = self.props
        hp = p.cluster_prop.house_prop
        hv = hp.hvac_prop
        on, lock, sso = decode_hvac(self.hvac.numpy())
        on, lock, sso = O.hvac_step(on, lock, sso, self._actions(action, mode), hv.lockout_duration,
                                    p.time_step.seconds)
        caps = self._caps()
        q = O.heat_transfer(on, caps, hv.latent_cooling_fraction)
        T, Tm = O.update_temperature(self.t_air.numpy(), self.t_mass.numpy(), self.ua.numpy(), self.ca.numpy(),
                                     self.cm.numpy(), self.hm.numpy(), q, tick.solar, tick.t_od_prev,
                                     float(p.time_step.seconds))
        self.t_air.copy_(torch.from_numpy(T))
        self.t_mass.copy_(torch.from_numpy(Tm))
        self.hvac.copy_(torch.from_numpy(encode_hvac(on, lock, sso)))
        P = 0.0
        for k, c in enumerate(self.counts.tolist()):
            P += float(c) * (self.cap_values[k] / hv.cop)
        self.p_dev[0] = P
        pen = O.deadband_l2(self.target.numpy(), hp.deadband, T)
        self._pen = pen
        x = (P - tick.s_prev) / self.n_global
        norm_t, norm_s = reward_normalisers(p.reward_prop, hp)
        rp = p.reward_prop
        self._sig = rp.alpha_sig * (x * x) / norm_s
        self._norm_t = norm_t
        r = -(rp.alpha_temp * pen / norm_t + self._sig)
        out = self.reward if reward is None else reward
        out.copy_(torch.from_numpy(r if self.penalty_mode == 0 else pen))
        return out

    def penalty_partials(self):
        s = 0.0
        for v in self._pen:
            s += v / self.n_global
        self.partial2[0] = s
        self.partial2[1] = float(np.max(self._pen, initial=0.0))

    def reward_finalize(self, tick, reward=None):
        pp = self.props.reward_prop.penalty_props
        cl2, cmax = float(self.partial2[0]), float(self.partial2[1])
        pen = self._pen
        if pp.mode == "common_L2":
            tp = np.full_like(pen, cl2)
        elif pp.mode == "common_max_error":
            tp = np.full_like(pen, cmax)
        else:
            tp = (pp.alpha_ind_l2 * pen + pp.alpha_common_l2 * cl2 + pp.alpha_common_max * cmax) / (
                pp.alpha_ind_l2 + pp.alpha_common_l2 + pp.alpha_common_max)
        r = -(self.props.reward_prop.alpha_temp * tp / self._norm_t + self._sig)
        (self.reward if reward is None else reward).copy_(torch.from_numpy(r))

    def interp_load(self, grids, values, cfg):
        from oracle import interp_np as IN

        self._interp = IN.OracleInterp(grids, values, *cfg)

    def interp_values(self, ids, od, hour, date, vals):
        o, caps = self._interp, self._caps()
        out = np.zeros(ids.numel())
        for s, g in enumerate(ids.tolist()):
            j = g - self.offset
            if 0 <= j < self.n:
                x = o.house_point(float(self.ua[j]), float(self.cm[j]), float(self.ca[j]), float(self.hm[j]),
                                  float(self.t_air[j]), float(self.t_mass[j]), float(self.target[j]), od,
                                  float(caps[j]), hour, date)
                out[s] = o.point(x)
        vals.copy_(torch.from_numpy(out))

    def interp_sum(self, vals, factor, out):
        b = 0.0
        for v in vals.tolist():
            b += v
        out[0] = b * factor

    def greedy_inputs(self, key, power, lock):
        _, lk, _ = decode_hvac(self.hvac.numpy().copy())
        key.copy_(-(self.t_air - self.target))
        power.copy_(torch.from_numpy(self._caps() / self.props.cluster_prop.house_prop.hvac_prop.cop))
        lock.copy_(torch.from_numpy(np.asarray(lk, np.uint8)))

    def greedy_select(self, n, key, power, lock, budget, action):
        """O.greedy's rule over the gathered rows (stable order)."""
        k, p, lk = key.numpy(), power.numpy(), lock.numpy().astype(bool)
        act = np.zeros(int(n), np.uint8)
        tot = 0
        for i in np.argsort(k, kind="stable"):
            if p[i] + tot < budget or abs(p[i] + tot - budget) < abs(tot - budget) and not lk[i]:
                tot += p[i]
                act[i] = 1
        action.copy_(torch.from_numpy(act))

    # ---- the sharded histogram select's stages (the protocol of HipShard.gq_shard_*: what is
    # allreduced and gathered between them), restated with NumPy: uniform bins over the previous
    # call's cluster key range, 32 superbins of 32 bins (+ a NaN superbin), class counts
    GQ_SUP, GQ_BPS, GQ_CAP, GQ_AFTER = 32, 32, 4096, 256

    def _gq_bins_of(self, k):
        lo, hi = self._gq_range
        nb = self.GQ_SUP * self.GQ_BPS
        sc = nb / (hi - lo) if hi > lo else 0.0
        with np.errstate(invalid="ignore"):
            b = np.clip(np.floor((k - lo) * sc), 0, nb - 1)
        return np.where(np.isnan(k), nb, b).astype(np.int64)

    def gq_shard_begin(self):
        if not hasattr(self, "_gq_range"):
            self._gq_range = (-4.0, 4.0)
        k = -(self.t_air.numpy() - self.target.numpy())
        self._gq_k, self._gq_b = k, self._gq_bins_of(k)
        cls = self.cap_idx.numpy().astype(np.int64)
        sup = np.zeros((self.GQ_SUP + 1, 4), np.int32)
        np.add.at(sup, (np.minimum(self._gq_b // self.GQ_BPS, self.GQ_SUP), cls), 1)
        fin = k[~np.isnan(k)]
        rng = np.array([fin.min() if fin.size else np.inf, -fin.max() if fin.size else np.inf])
        self._gq = {"super": torch.from_numpy(sup.reshape(-1).copy()), "bins": torch.zeros(2 * self.GQ_BPS * 4, dtype=torch.int32),
                    "range": torch.from_numpy(rng), "window": torch.zeros(1 + 4 * self.GQ_CAP, dtype=torch.float64)}
        return self._gq

    def _gq_p(self):
        hv = self.props.cluster_prop.house_prop.hvac_prop
        return np.asarray(self.cap_values) / hv.cop

    def gq_shard_bins(self, budget):
        sup = self._gq["super"].numpy().reshape(-1, 4).astype(np.int64)
        p = self._gq_p()
        Pc = (sup[:, :len(p)] * p).sum(1)
        cum = np.cumsum(Pc)
        cnt = sup.sum(1)
        hit = np.nonzero((cnt > 0) & ~(cum < budget))[0]
        self._gq_sb = int(hit[0]) if hit.size else self.GQ_SUP + 1
        self._gq_base = float(cum[self._gq_sb - 1]) if 0 < self._gq_sb <= self.GQ_SUP else 0.0
        self._gq_basec = int(cnt[:self._gq_sb].sum())
        self._gq_total = int(cnt.sum())
        lo, mhi = self._gq["range"].tolist()
        self._gq_next = (lo, -mhi) if np.isfinite(lo) else (0.0, 0.0)
        bins = np.zeros((2 * self.GQ_BPS, 4), np.int32)
        if self._gq_sb < self.GQ_SUP:
            rel = self._gq_b - self._gq_sb * self.GQ_BPS
            m = (rel >= 0) & (rel < 2 * self.GQ_BPS) & (self._gq_b < self.GQ_SUP * self.GQ_BPS)
            np.add.at(bins, (rel[m], self.cap_idx.numpy()[m].astype(np.int64)), 1)
        self._gq["bins"].copy_(torch.from_numpy(bins.reshape(-1)))

    def gq_shard_compact(self, budget, action):
        self._gq_range = self._gq_next
        act = np.zeros(self.n, np.uint8)
        sb, n_sup = self._gq_sb, self.GQ_SUP
        whole = sb <= n_sup and self._gq_total <= self.GQ_CAP  # a cluster that fits the window is the window
        self._gq_fb = sb == n_sup and not whole  # a NaN crossing: the all-gather form decides
        win = self._gq["window"].numpy()
        win[0] = 0
        if sb > n_sup:  # everything fits the budget
            act[:] = 1
        elif whole:
            self._gq_wbase, self._gq_more, self._gq_ncand = 0.0, False, self._gq_total
            inw = np.arange(self.n)
            _, lk, _ = decode_hvac(self.hvac.numpy().copy())
            pw = self._gq_p()[self.cap_idx.numpy()]
            win[0] = inw.size
            rows = np.stack([self._gq_k[inw], (inw + self.offset).astype(np.float64), pw[inw],
                             lk[inw].astype(np.float64)], 1)
            win[1:1 + 4 * inw.size] = rows.reshape(-1)
        elif not self._gq_fb:
            bins = self._gq["bins"].numpy().reshape(-1, 4).astype(np.int64)
            p = self._gq_p()
            Pb = (bins[:, :len(p)] * p).sum(1)
            cb = bins.sum(1)
            cum = self._gq_base + np.cumsum(Pb)
            l0 = int(np.nonzero((cb > 0) & ~(cum < budget))[0][0])
            pre = np.cumsum(cb[l0:])
            ok = np.nonzero(pre <= self.GQ_CAP)[0]
            if ok.size == 0:
                self._gq_fb = True
            else:
                enough = ok[pre[ok] >= cb[l0] + self.GQ_AFTER]
                le = int(enough[0]) if enough.size else int(ok[-1])
                bs = sb * self.GQ_BPS + l0
                be = bs + le
                self._gq_wbase = float(cum[l0] - Pb[l0])
                self._gq_more = self._gq_basec + int(cb[:l0].sum()) + int(pre[le]) < self._gq_total
                self._gq_ncand = int(pre[le])
                act[self._gq_b < bs] = 1
                inw = np.nonzero((self._gq_b >= bs) & (self._gq_b <= be))[0]
                _, lk, _ = decode_hvac(self.hvac.numpy().copy())
                pw = self._gq_p()[self.cap_idx.numpy()]
                win[0] = inw.size
                rows = np.stack([self._gq_k[inw], (inw + self.offset).astype(np.float64), pw[inw],
                                 lk[inw].astype(np.float64)], 1)
                win[1:1 + 4 * inw.size] = rows.reshape(-1)
        action.copy_(torch.from_numpy(act))

    def gq_shard_select(self, budget, gathered, world, action):
        if self._gq_fb or self._gq_sb > self.GQ_SUP:
            return
        g = gathered.numpy().reshape(world, -1)
        rows = np.concatenate([g[r, 1:1 + 4 * int(g[r, 0])].reshape(-1, 4) for r in range(world)])
        if rows.shape[0] != self._gq_ncand:
            self._gq_fb = True
            return
        order = np.lexsort((rows[:, 1], rows[:, 0]))  # (key, global house), as the stable sort
        tot, take = self._gq_wbase, np.zeros(rows.shape[0], bool)
        for j in order:  # greedy_myopic_controller.py:93-101 from the P taken before the window
            pj, lk = rows[j, 2], rows[j, 3] != 0
            if pj + tot < budget or (abs(pj + tot - budget) < abs(tot - budget) and not lk):
                take[j], tot = True, tot + pj
        if self._gq_more and not (not tot < budget or 2.0 * (budget - tot) < self._gq_p().min() * (1 - 1e-9)):
            self._gq_fb = True  # the walk could continue past the window
            return
        act = action.numpy()
        for j in np.nonzero(take)[0]:
            li = int(rows[j, 1]) - self.offset
            if 0 <= li < self.n:
                act[li] = 1

    def gq_shard_fallback(self):
        return bool(self._gq_fb)

    def host_state(self):
        on, lock, sso = decode_hvac(self.hvac.numpy().copy())
        return {"T": self.t_air.numpy().copy(), "Tm": self.t_mass.numpy().copy(), "on": on,
                "lock": lock, "sso": sso}

    def host_params(self):
        return {k: getattr(self, k).numpy().copy() for k in ("ua", "ca", "cm", "hm", "target", "cap_idx")}


class GlooComm:
    def __init__(self):
        import torch.distributed as dist

        self.dist = dist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()

    def attach(self, shard):
        pass

    def allreduce_counts(self, shard):
        self.dist.all_reduce(shard.counts)

    def allreduce_penalty(self, shard):
        s = shard.partial2[:1].clone()
        m = shard.partial2[1:].clone()
        self.dist.all_reduce(s)
        self.dist.all_reduce(m, op=self.dist.ReduceOp.MAX)
        shard.partial2[0], shard.partial2[1] = s[0], m[0]

    def allreduce_sum(self, shard, t):
        self.dist.all_reduce(t)

    def allreduce_max(self, shard, t):
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)

    def allreduce_min(self, shard, t):
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)

    def allreduce_count32(self, shard, t):
        self.dist.all_reduce(t)

    def allgather_bytes(self, shard, t):
        parts = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t.contiguous())
        return torch.cat(parts)

    def allgather_cat(self, shard, t, sizes):
        m = max(sizes)
        buf = t if t.numel() == m else torch.cat([t, t.new_zeros(m - t.numel())])
        parts = [torch.empty_like(buf) for _ in range(self.world)]
        self.dist.all_gather(parts, buf.contiguous())
        return torch.cat([p[:s] for p, s in zip(parts, sizes)])

    def allgather_state(self, shard, st, prm, n):
        out_st, out_prm = {}, {}
        for src, dst, keys in ((st, out_st, ("T", "Tm", "on", "lock", "sso")),
                               (prm, out_prm, ("ua", "ca", "cm", "hm", "target", "cap_idx"))):
            for key in keys:
                a = np.asarray(src[key])
                parts = [None] * self.world
                self.dist.all_gather_object(parts, a)
                dst[key] = np.concatenate(parts)
        return out_st, out_prm
