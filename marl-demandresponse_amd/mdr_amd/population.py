"""Reset-time population and communication graph, in the reference's RNG call order.

The reference draws its population from the global ``random`` (MT19937) house by house
(SURVEY Appendix B); reproducing that stream is part of the drop-in contract, so the draw stays
on the host (``draw_reference``).  ``Environment(population="synthetic")`` instead draws the same
noise model on device from Philox (mdr_populate), for benchmark-scale populations.

  draw_reference   server/app/core/environment/cluster/building.py:224-267, hvac.py:66-70
  comm_links       server/app/core/environment/cluster/agent_communication_builder.py:36-203
  sample_excluding random.sample(ids without i, k) as AgentCommunicationBuilder.get_random_sample
"""
from __future__ import annotations

import math
import random as _random

import numpy as np


def _inst(rng):
    return _random._inst if rng is _random else rng


def sample_excluding(rng, n: int, i: int, k: int):
    """``rng.sample([j for j in range(n) if j != i], k)`` without building the list.

    Follows CPython's ``Random.sample`` (pool method for small populations, set method
    otherwise) on the same ``_randbelow`` stream, so the draws and the result are identical.
    """
    m = n - 1
    if not 0 <= k <= m:
        raise ValueError("Sample larger than population or is negative")
    setsize = 21
    if k > 5:
        setsize += 4 ** math.ceil(math.log(k * 3, 4))
    if m <= setsize:
        return rng.sample([j for j in range(n) if j != i], k)
    randbelow = _inst(rng)._randbelow
    selected = set()
    out = []
    for _ in range(k):
        j = randbelow(m)
        while j in selected:
            j = randbelow(m)
        selected.add(j)
        out.append(j if j < i else j + 1)
    return out


def nb_comm(cluster_prop) -> int:
    return int(min(cluster_prop.agents_comm_prop.max_nb_agents_communication, cluster_prop.nb_agents - 1))


def comm_links(cluster_prop, rng=_random):
    """Neighbour ids per house as int32 [N, k]; None for 'random_sample' (drawn per get_obs)."""
    n = cluster_prop.nb_agents
    ac = cluster_prop.agents_comm_prop
    k = nb_comm(cluster_prop)
    mode = ac.mode
    if mode == "neighbours":
        lo, hi = k // 2, (k + 1) // 2
        ids = np.arange(n, dtype=np.int64)[:, None]
        off = np.concatenate([np.arange(-lo, 0), np.arange(1, hi + 1)])
        return ((ids + off[None, :]) % n).astype(np.int32)
    if mode == "closed_groups":
        out = []
        for i in range(n):
            base = i - i % (k + 1)
            if base + k <= n:
                grp = [base + j for j in range(ac.max_nb_agents_communication + 1)]
            else:
                grp = [n - k - 1 + j for j in range(k + 1)]
            grp.remove(i)
            out.append(grp)
        # with nb_comm < max_nb_agents_communication (small clusters) the reference builds ragged
        # groups that may name houses >= N (its get_obs then raises IndexError): keep them as is
        if len({len(g) for g in out}) == 1:
            return np.array(out, np.int32).reshape(n, len(out[0]))
        return out
    if mode == "random_sample":
        return None
    if mode == "random_fixed":
        return np.array([sample_excluding(rng, n, i, k) for i in range(n)], np.int32).reshape(n, k)
    if mode == "neighbours_2D":
        rs, dmax = ac.row_size, ac.max_communication_distance
        if n % rs != 0:
            raise ValueError("Neighbours 2D row_size must be a divisor of nb_agents")
        my = n // rs
        if dmax >= (rs + 1) // 2 or dmax >= (my + 1) // 2:
            raise ValueError(
                f"Neighbours 2D distance_comm ({dmax}) must be strictly smaller than (row_size+1) / 2 "
                f"({(rs + 1) // 2}) and (max_y+1) / 2 ({(my + 1) // 2})")
        pat = [(dx, dy) for dx in range(-dmax, dmax + 1) for dy in range(-dmax, dmax + 1)
               if abs(dx) + abs(dy) <= dmax and (dx or dy)]
        ids = np.arange(n)
        x, y = ids % rs, ids // rs
        cols = [((y + dy) % my) * rs + (x + dx) % rs for dx, dy in pat]
        return np.stack(cols, 1).astype(np.int32)
    raise ValueError(f"unknown agents_comm_prop.mode {mode!r}")


def random_links(cluster_prop, rng=_random):
    """One 'random_sample' draw for every house (Cluster.message, cluster.py:96-99)."""
    n, k = cluster_prop.nb_agents, nb_comm(cluster_prop)
    return np.array([sample_excluding(rng, n, i, k) for i in range(n)], np.int32).reshape(n, k)


def draw_reference(cluster_prop, rng=_random):
    """Building.apply_noise for every house in index order (8 draws per house)."""
    hp = cluster_prop.house_prop
    nz = hp.noise_prop
    n = cluster_prop.nb_agents
    caps = hp.hvac_prop.noise_prop.cooling_capacity_list
    out = {k: np.empty(n) for k in ("ua", "ca", "cm", "hm", "target", "init_air", "init_mass")}
    cap = [None] * n
    gauss, tri, choices = rng.gauss, rng.triangular, rng.choices
    lo, hi = nz.factor_thermo_low, nz.factor_thermo_high
    s_start, s_tgt = nz.std_start_temp, nz.std_target_temp
    ia, im, tt = hp.init_air_temp, hp.init_mass_temp, hp.target_temp
    Ca, Cm, Hm = hp.Ca, hp.Cm, hp.Hm
    ua, ca, cm, hm, tg = out["ua"], out["ca"], out["cm"], out["hm"], out["target"]
    iair, imass = out["init_air"], out["init_mass"]
    for i in range(n):
        iair[i] = ia + abs(gauss(0, s_start))
        imass[i] = im + abs(gauss(0, s_start))
        tg[i] = tt + abs(gauss(0, s_tgt))
        ua[i] = tri(lo, hi, 1)
        cm[i] = Cm * tri(lo, hi, 1)
        ca[i] = Ca * tri(lo, hi, 1)
        hm[i] = Hm * tri(lo, hi, 1)
        cap[i] = choices(caps)[0]
    out["cap"] = cap
    return out


def cap_table(hvac_prop, caps=()):
    """Distinct capacity values (reference list order first) + index of every house's value."""
    table = []
    for v in list(hvac_prop.noise_prop.cooling_capacity_list) + [hvac_prop.cooling_capacity]:
        if v not in table:
            table.append(v)
    idx = np.empty(len(caps), np.uint8)
    pos = {v: i for i, v in enumerate(table)}
    for i, v in enumerate(caps):
        j = pos.get(v)
        if j is None:
            table.append(v)
            j = pos[v] = len(table) - 1
        idx[i] = j
    if len(table) > 64:
        raise ValueError("more than 64 distinct cooling capacities are not supported")
    return table, idx
