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
