"""Helpers to load the golden fixtures (tests/golden, written by tests/golden/make_golden.py)."""
from __future__ import annotations

import datetime as dt
import json
import os
import tempfile

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
EPOCH0 = dt.datetime(1970, 1, 1)


def path(name: str) -> str:
    return os.path.join(GOLDEN, name)


def load(name: str):
    return np.load(path(name), allow_pickle=False)


def base_env_prop() -> dict:
    with open(path("marl_env_prop.json")) as f:
        return json.load(f)


BPP = "power_grid_prop.base_power_props."


def interp_table_path() -> str:
    """The synthetic Monte-Carlo table the interpolation goldens were made with (the reference does
    not ship mergedGridSearchResultFinal.npy): oracle/interp_np.synthetic_table(seed in interp.npz)
    over the reference grid, written once per machine."""
    import numpy as _np

    from oracle.interp_np import synthetic_table

    seed = int(load("interp.npz")["table_seed"])
    out = os.path.join(tempfile.gettempdir(), f"mdr_interp_table_{seed}_{os.getuid()}.npy")
    if not os.path.exists(out):
        with open(path("interp_parameters_dict.json")) as f:
            lens = [len(v) for v in json.load(f).values()]
        tmp = f"{out}.{os.getpid()}.tmp.npy"
        _np.save(tmp, synthetic_table(lens, seed))
        os.replace(tmp, out)
    return out


def localize(overrides: dict) -> dict:
    """Point an interpolation-mode config at this checkout's fixture files."""
    if overrides.get(BPP + "mode") != "interpolation":
        return overrides
    o = dict(overrides)
    o[BPP + "path_datafile"] = interp_table_path()
    o[BPP + "path_parameter_dict"] = path("interp_parameters_dict.json")
    o[BPP + "path_dict_keys"] = path("interp_dict_keys.csv")
    return o


def props_from_overrides(overrides: dict):
    from mdr_amd.config import EnvironmentProperties, override

    return EnvironmentProperties.from_dict(override(base_env_prop(), localize(overrides)))


def traj(name: str):
    d = load(f"traj_{name}.npz")
    meta = json.loads(bytes(d["meta_json"]).decode())
    return d, meta


def from_epoch(x: float) -> dt.datetime:
    return EPOCH0 + dt.timedelta(seconds=float(x))


TRAJ_NAMES = ("c1_sin_dbbc", "c1_flat_random", "fixed_steps_bbc", "n400_random_common",
              "n64_mixture_2d", "n30_maxerr_groups_hvacmsg", "interp_sin_random", "interp_flat_dbbc_nosolar")


def calibrated_actor(n_feat: int, obs_absmax, seed: int = 1, gain: float = 3.0, layers=(100, 100)):
    """The reference Actor (``make_actor``, torch seed ``seed``) with its first layer's columns
    divided by max(1, |feature|max) (``obs_absmax``: float [n_feat]) and the output layer scaled by
    ``gain``: the observation's normalisation folded into the weights, so that at any cluster size
    (the cluster-power feature is ~0.4 N, norm.py:145) the policy stays away from saturation and a
    probability check compares real numbers, not 1.0 with 1.0."""
    import torch

    from mdr_amd.actor import make_actor

    a = make_actor(n_feat, 2, list(layers), seed=seed)
    s = torch.as_tensor(np.maximum(1.0, np.asarray(obs_absmax, np.float64)), dtype=torch.float32)
    with torch.no_grad():
        a.fc[0].weight.div_(s[None, :])
        a.fc[-1].weight.mul_(gain)
        a.fc[-1].bias.mul_(gain)
    return a


def assert_not_saturated(probs, actions=None, lo: float = 0.05, hi: float = 0.95, frac: float = 0.5):
    """At least ``frac`` of the sampled probabilities lie in (lo, hi), and both actions occur."""
    p = np.asarray(probs, np.float64).ravel()
    inside = float(np.mean((p > lo) & (p < hi)))
    assert inside >= frac, f"only {inside:.3f} of the probabilities are in ({lo}, {hi})"
    if actions is not None:
        a = np.asarray(actions).ravel()
        assert a.min() == 0 and a.max() == 1, "both actions must occur"
