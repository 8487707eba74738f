"""Server-side consumers on device against the reference services run on the
same trajectory (tests/golden/services.npz, made by tests/golden/make_golden.py gen_services:
reference Metrics + ClientManagerService along a ControllerManager-style deadband-bang-bang loop).

Sums over houses are a fixed blocked device reduction where the reference adds house by house, so
float accumulators agree to rtol 1e-12; integer counts and per-tick scalars (signal, power, OD
temperature, consumption error, RMSE) are exact, and the rounded summary strings are equal."""
import json
import random

import numpy as np
import pytest

import golden_util as gu

pytestmark = pytest.mark.gpu


def test_server_loop_matches_reference_services():
    from mdr_amd.environment import Environment
    from mdr_amd.services import DESCRIPTION_KEYS, ServerLoop

    d = gu.load("services.npz")
    meta = json.loads(bytes(d["meta_json"]).decode())
    N, T = meta["N"], meta["T"]
    props = gu.props_from_overrides({"cluster_prop.nb_agents": N,
                                     "power_grid_prop.signal_properties.mode": meta["signal"]})
    env = Environment(props, rng=random.Random(meta["seed"]))
    env.reset(return_obs=False)
    env.reset(return_obs=False)
    loop = ServerLoop(env, controller="deadband_bangbang", start_stats_from=meta["start_stats_from"], nb_time_steps=T)
    want_desc = json.loads(bytes(d["ui_desc_json"]).decode())
    assert meta["keys"] == DESCRIPTION_KEYS
    for step in range(T):
        loop.run(1)
        m = loop.metrics
        for f in m.FIELDS:
            np.testing.assert_allclose(getattr(m, f), d[f"metrics_{f}"][step], rtol=1e-12, atol=1e-9,
                                       err_msg=f"{f} step {step}")
        desc = [loop.ui.description[step][k] for k in DESCRIPTION_KEYS]
        for k, got, ref in zip(DESCRIPTION_KEYS, desc, want_desc[step]):
            if k in ("Average temperature error",):
                # a difference of two house sums (blocked device order vs the reference's house order):
                # cancellation, so the bound is absolute
                np.testing.assert_allclose(float(got), float(ref), rtol=1e-12, atol=1e-11,
                                           err_msg=f"{k} step {step}")
            else:
                assert got == ref, (k, step, got, ref)
        ui = loop.ui
        got_graph = [ui.temp_diff[-1], ui.temp_err[-1], ui.air_temp[-1], ui.mass_temp[-1], ui.target_temp[-1],
                     ui.outdoor_temp[-1], ui.signal[-1], ui.consumption[-1]]
        np.testing.assert_allclose(got_graph, d["ui_graph"][step], rtol=1e-12, atol=1e-12)
        hl = ui.houses_data[step]
        assert len(hl) == N
        assert list(hl.status_counts()) == list(d["ui_status"][step])
    m.update_rms(T)
    np.testing.assert_allclose([m.rmse_sig_per_ag, m.rmse_temp, m.rms_max_error_temp], d["rms"], rtol=1e-12)


def test_lazy_obs_equals_materialised():
    """get_obs()/step() LazyDicts read back the same values as fully materialised dicts, and
    pandas frames of them (ClientManagerService / GreedyMyopic) are identical."""
    import pandas as pd

    from mdr_amd.environment import Environment

    props = gu.props_from_overrides({"cluster_prop.nb_agents": 300,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    env = Environment(props, rng=random.Random(3))
    obs = env.reset()
    for t in range(5):
        obs2, rew = env.step({i: (i + t) % 3 == 0 for i in range(300)})
        full = {k: obs2[k] for k in range(300)}
        pd.testing.assert_frame_equal(pd.DataFrame(obs2).transpose(), pd.DataFrame(full).transpose())
        assert len(rew) == 300 and all(isinstance(rew[i], float) for i in (0, 299))
    st = env.shard.host_state()
    b = env.cluster.buildings
    assert len(b) == 300 and b[7].indoor_temp == float(st["T"][7]) and b[-1].hvac.turned_on == bool(st["on"][-1])
