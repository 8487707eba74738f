"""Product host-side logic (mdr_amd: config, drivers, population, comm graph) against the
reference goldens — everything per tick that is NOT per house stays on the host and must be
bit-identical to the reference (same expressions, same RNG call order)."""
import copy
import datetime as dt
import json
import math
import random

import numpy as np
import pytest

import golden_util as gu
from mdr_amd import config as C
from mdr_amd import drivers as D
from mdr_amd import population as POP


def test_config_loads_marlconfig_and_validates():
    d = gu.base_env_prop()
    p = C.EnvironmentProperties.from_dict(d)
    assert p.cluster_prop.nb_agents == 1000
    assert p.time_step == dt.timedelta(seconds=4)
    assert p.start_datetime == dt.datetime(2021, 1, 1, 12)
    assert p.cluster_prop.house_prop.hvac_prop.max_consumption == 6000.0
    C.validate(p)
    bad = C.EnvironmentProperties.from_dict(C.override(d, {"power_grid_prop.signal_properties.mode": "nope"}))
    with pytest.raises(ValueError):
        C.validate(bad)
    bad = C.EnvironmentProperties.from_dict(C.override(d, {"cluster_prop.agents_comm_prop.mode": "x"}))
    with pytest.raises(ValueError):
        C.validate(bad)


def test_solar_golden_exact():
    g = gu.load("solar.npz")
    got = [D.solar_gain(gu.from_epoch(e), 7.175, 0.67) for e in g["epoch"]]
    np.testing.assert_array_equal(got, g["gain"])


def test_signal_golden_exact():
    g = gu.load("signal.npz")
    stamps = [gu.from_epoch(e) for e in g["epoch"]]
    for mode in ("flat", "sinusoidals", "regular_steps"):
        for nb in (50, 1000):
            sig = D.Signal(C.SignalProperties(mode=mode), nb)
            np.testing.assert_array_equal([float(sig(4200.0 * nb, t)) for t in stamps], g[f"{mode}_{nb}"])
    sig = D.Signal(C.SignalProperties(mode="sinusoidals", amplitude_ratios=[0.2, 0.05, 0.1],
                                      periods=[300, 900, 3600]), 77)
    np.testing.assert_array_equal([float(sig(77 * 3900.0, t)) for t in stamps], g["sinusoidals_custom_77"])


def test_reward_normalisers():
    rp, hp = C.RewardProperties(), C.BuildingProperties(target_temp=19.0)
    assert D.reward_normalisers(rp, hp) == (1.0, 1875.0 ** 2)


def test_sample_excluding_matches_random_sample():
    for n, k in ((12, 4), (50, 10), (86, 10), (87, 10), (1000, 10), (10_000, 10), (300, 30)):
        for i in (0, 1, n // 2, n - 1):
            r1, r2 = random.Random(n * 7 + i), random.Random(n * 7 + i)
            a = POP.sample_excluding(r1, n, i, k)
            b = r2.sample([j for j in range(n) if j != i], k)
            assert a == b
            assert r1.random() == r2.random()  # same number of draws consumed


def test_comm_links_golden():
    with open(gu.path("comm.json")) as f:
        g = json.load(f)
    for key, val in g.items():
        if key.startswith("random_fixed"):
            continue
        mode, n, kmax = key.rsplit("_", 2)
        n, kmax = int(n), int(kmax)
        cp = C.ClusterPropreties(nb_agents=n, agents_comm_prop=C.AgentsCommunicationProperties(
            mode=mode, max_nb_agents_communication=kmax, row_size=5 if n != 100 else 10,
            max_communication_distance=2 if n != 25 else 1))
        if isinstance(val, str):
            with pytest.raises(ValueError):
                POP.comm_links(cp, random)
        else:
            assert POP.comm_links(cp, random).tolist() == val, key
    cp = C.ClusterPropreties(nb_agents=12, agents_comm_prop=C.AgentsCommunicationProperties(
        mode="random_fixed", max_nb_agents_communication=4))
    assert POP.comm_links(cp, random.Random(99)).tolist() == g["random_fixed_12_4_seed99"]


@pytest.mark.parametrize("seed", [0, 4, 123])
def test_population_rng_order_golden(seed):
    """draw_reference + the reset's surrounding draws consume the stream like the reference."""
    g = gu.load("rng_order.npz")
    p = gu.props_from_overrides({"cluster_prop.nb_agents": 20, "start_datetime_mode": "random",
                                 "power_grid_prop.signal_properties.mode": "flat"})
    rng = random.Random(seed)
    for r in range(3):  # Environment.__init__ + two resets, replayed host-side
        POP.comm_links(p.cluster_prop, rng)
        days, secs = rng.randrange(364), rng.randrange(86400)
        pop = POP.draw_reference(p.cluster_prop, rng)
        date = p.start_datetime + dt.timedelta(days=days, seconds=secs)
        tod = D.od_temp(date, p.temp_prop, rng)
        D.GridSignal(copy.deepcopy(p.power_grid_prop), 20, 20 * 6000.0, rng)
        if r == 0:
            np.testing.assert_array_equal(pop["ua"], g[f"s{seed}_random_r1_Ua"])
    key = f"s{seed}_random_r3"
    for k, gk in (("ua", "Ua"), ("ca", "Ca"), ("cm", "Cm"), ("hm", "Hm"), ("target", "target_temp"),
                  ("init_air", "init_air_temp_noised")):
        np.testing.assert_array_equal(pop[k], g[f"{key}_{gk}"], err_msg=k)
    assert [float(c) for c in pop["cap"]] == list(g[f"{key}_cooling_capacity"])
    assert (date - gu.EPOCH0).total_seconds() == float(g[f"{key}_epoch"])
    assert tod == float(g[f"{key}_Tod"])
    assert rng.random() == float(g[f"{key}_next_random"])


def test_cap_table():
    hv = C.HvacProperties()
    table, idx = POP.cap_table(hv, [12500, 17500, 15000, 17500])
    assert table == [12500, 15000, 17500]
    assert idx.tolist() == [0, 2, 1, 2]
    table, idx = POP.cap_table(hv, [11000])
    assert table[-1] == 11000 and idx.tolist() == [3]


def test_perlin_restatement_statistics():
    """Perlin is parity-unpinned (third-party perlin_noise absent): check the restatement's
    published properties instead — zero at lattice points, bounded, smooth, deterministic."""
    from mdr_amd.perlin import Perlin

    pn = Perlin(1, 5, 5, 300, 0.123)
    xs = np.arange(0, 86400, 37.0)
    v = np.array([pn.calculate_noise(x) for x in xs])
    assert np.all(np.abs(v) < 1.0)
    assert abs(v.mean()) < 0.05 and v.std() > 0.01
    assert pn.calculate_noise(0.0) == 0.0
    assert np.array_equal(v, [Perlin(1, 5, 5, 300, 0.123).calculate_noise(x) for x in xs])
    sig = D.Signal(C.SignalProperties(mode="perlin"), 10, rng=random.Random(1))
    s = [float(sig(42000.0, dt.datetime(2021, 5, 5, 12, 0, k))) for k in range(0, 60, 4)]
    assert min(s) >= 0.0


def test_perlin_published_algorithm():
    """The 1-D lattice noise as perlin_noise publishes it: gradient of lattice point k =
    uniform(-1, 1) of a Mersenne Twister seeded with (k + 1) * seed, contribution fade(1 - |d|) *
    g * d; the pre-1.12 global-RNG side effect reseeds the given generator (parity unpinned)."""
    from mdr_amd.perlin import Perlin, _GradientNoise1D, _fade

    seed = 0.4172
    g = _GradientNoise1D(10, seed)
    for x in (0.0137, 0.5, 2.25, 7.91):
        xs = x * 10
        want = 0
        for k in (math.floor(xs), math.floor(xs + 1)):
            gk = random.Random((k + 1) * seed).uniform(-1, 1)
            want += _fade(1 - abs(xs - k)) * (gk * (xs - k))
        assert g.noise(x) == want
    rng = random.Random(5)
    side = _GradientNoise1D(10, seed, global_rng=rng)
    assert side.noise(0.5) == g.noise(0.5)
    ref = random.Random(7 * seed)  # the last lattice point of xs = 5.0 is k = 6: seed (6 + 1) * seed
    ref.uniform(-1, 1)
    assert rng.random() == ref.random()
    # the octave sum (perlin.py:51-56): last octave divided by 2**n - 1
    pn = Perlin(1, 3, 5, 300, seed)
    x = 1234.5
    n = [pn.noise_list[j].noise(x / 300) for j in range(3)]
    assert pn.calculate_noise(x) == 1 * (0 + n[0] / 1 + n[1] / 2 + n[2] / 7)


def test_perlin_array_equals_oracle():
    """The tabulated (array) perlin noise == the scalar form == the oracle's independent scalar
    restatement, bit for bit: all three evaluate the package's fade with Python float ``**``
    (r03's product form could differ from the package's ``**`` by an ulp)."""
    from mdr_amd.perlin import Perlin
    from oracle.perlin_np import PerlinSignal

    seed = 0.61803
    pn, ora = Perlin(1, 5, 5, 300, seed), PerlinSignal(5, 5, 300, seed)
    xs = np.concatenate([np.arange(0, 86400, 4.0), np.arange(0.5, 3000, 0.37)])
    arr = pn.calculate_noise_array(xs)
    scal = np.array([pn.calculate_noise(float(x)) for x in xs[::7]])
    np.testing.assert_array_equal(arr[::7], scal)
    np.testing.assert_array_equal(scal, [ora.calculate_noise(float(x)) for x in xs[::7]])


def test_actor_init_matches_reference_mappo():
    """make_actor(seed=1) reproduces MAPPO's actor initialisation (mappo.py:41-50) and forward:
    the reference's own weights and probabilities in tests/golden/policy.npz."""
    import torch

    from mdr_amd.actor import make_actor

    d = gu.load("policy.npz")
    for case in ("c1", "wide"):
        a = make_actor(d[f"{case}_fc.0.weight"].shape[1], 2, [100, 100], seed=1)
        for k, v in a.state_dict().items():
            np.testing.assert_array_equal(v.numpy(), d[f"{case}_{k}"], err_msg=k)
        with torch.no_grad():
            p = a(torch.from_numpy(d[f"{case}_obs"])).numpy()
        np.testing.assert_allclose(p, d[f"{case}_probs"], rtol=0, atol=1e-6)
        # select_actions bookkeeping: last_probs[i] = probs[i, action[i]]
        np.testing.assert_allclose(d[f"{case}_sel_prob"],
                                   d[f"{case}_probs"][np.arange(len(p)), d[f"{case}_sel_action"]], atol=1e-6)


def test_device_actor_has_no_cpu_path():
    """DeviceActor needs the HIP library and a GPU: on a CPU box the Environment itself refuses."""
    import pytest as _pt

    from mdr_amd import _lib
    from mdr_amd.environment import Environment

    props = gu.props_from_overrides({"cluster_prop.nb_agents": 4})
    with _pt.raises(_lib.MdrLibraryError):
        Environment(props)
