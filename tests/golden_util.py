"""Helpers to load the golden fixtures (tests/golden, written by tests/golden/make_golden.py)."""
from __future__ import annotations

import datetime as dt
import json
import os

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


def props_from_overrides(overrides: dict):
    from mdr_amd.config import EnvironmentProperties, override

    return EnvironmentProperties.from_dict(override(base_env_prop(), overrides))


def traj(name: str):
    d = load(f"traj_{name}.npz")
    meta = json.loads(bytes(d["meta_json"]).decode())
    return d, meta


def from_epoch(x: float) -> dt.datetime:
    return EPOCH0 + dt.timedelta(seconds=float(x))


TRAJ_NAMES = ("c1_sin_dbbc", "c1_flat_random", "fixed_steps_bbc", "n400_random_common",
              "n64_mixture_2d", "n30_maxerr_groups_hvacmsg")
