"""Configuration schema for the vectorised environment step.

Mirrors the reference's pydantic property tree (field names, defaults and meaning), so a
``MARLconfig.json`` ``env_prop`` subtree loads unchanged and the reference's own
``EnvironmentProperties`` object can be passed to :class:`mdr_amd.Environment` instead (only
attribute access is used):

* ``server/app/core/environment/environment_properties.py:13-372`` (house / hvac / noise / reward /
  state / message / cluster / environment models);
* ``server/app/core/environment/power_grid/power_grid_properties.py:6-70`` (signal / base power /
  grid);
* ``server/app/core/environment/cluster/cluster_properties.py:4-48`` (temperature / comm).

Unlike the reference (which fails late with ``AttributeError`` from ``getattr(self, mode)``),
mode strings are validated up front by :func:`validate`.
"""
from __future__ import annotations

import copy
import datetime as _dt
import json
from typing import List, Literal

from pydantic import BaseModel, Field

# ---------------------------------------------------------------- house / hvac (env_properties:13-207)


class HvacNoiseProperties(BaseModel):
    std_latent_cooling_fraction: float = 0.05
    factor_COP_low: float = 0.95
    factor_COP_high: float = 1.05
    factor_cooling_capacity_low: float = 0.9
    factor_cooling_capacity_high: float = 1.1
    lockout_noise: int = 0
    cooling_capacity_list: List[int] = [12500, 15000, 17500]


class HvacProperties(BaseModel):
    cop: float = Field(default=2.5, gt=0)
    cooling_capacity: float = Field(default=15000.0, gt=0)
    latent_cooling_fraction: float = Field(default=0.35, gt=0, lt=1)
    lockout_duration: int = 40
    noise_prop: HvacNoiseProperties = HvacNoiseProperties()

    @property
    def max_consumption(self) -> float:
        # environment_properties.py:92-98 — a property of the (possibly noised) capacity
        return self.cooling_capacity / self.cop


class BuildingNoiseProperties(BaseModel):
    std_start_temp: float = 3.0
    std_target_temp: float = 1.0
    factor_thermo_low: float = 0.9
    factor_thermo_high: float = 1.1


class BuildingProperties(BaseModel):
    Ua: float = 2.18e02
    Ca: float = 9.08e05
    Hm: float = 2.84e03
    Cm: float = 3.45e06
    target_temp: float = 20.0
    deadband: float = 0.0
    init_air_temp: float = 20.0
    init_mass_temp: float = 20.0
    solar_gain: bool = True
    window_area: float = 7.175
    shading_coeff: float = 0.67
    noise_prop: BuildingNoiseProperties = BuildingNoiseProperties()
    hvac_prop: HvacProperties = HvacProperties()


# ---------------------------------------------------------------- reward / state (env_properties:210-310)

PENALTY_MODES = ("common_L2", "individual_L2", "common_max_error", "mixture")


class PenaltyProperties(BaseModel):
    mode: Literal["common_L2", "individual_L2", "common_max_error", "mixture"] = "individual_L2"
    alpha_ind_l2: float = 1.0
    alpha_common_l2: float = 1.0
    alpha_common_max: float = 0.0


class RewardProperties(BaseModel):
    alpha_temp: float = 1.0
    alpha_sig: float = 1.0
    norm_reg_sig: int = 7500
    penalty_props: PenaltyProperties = PenaltyProperties()
    sig_penalty_mode: Literal["common_L2"] = "common_L2"


class StateProperties(BaseModel):
    hour: bool = False
    day: bool = False
    solar_gain: bool = False
    thermal: bool = False
    hvac: bool = False


class MessageProperties(BaseModel):
    thermal: bool = False
    hvac: bool = False


# ---------------------------------------------------------------- cluster_properties.py:4-48

COMM_MODES = ("neighbours", "closed_groups", "random_sample", "random_fixed", "neighbours_2D")


class TemperatureProperties(BaseModel):
    day_temp: float = 26.0
    night_temp: float = 20.0
    temp_std: float = 1.0
    random_phase_offset: bool = False
    phase: float = 0.0


class AgentsCommunicationProperties(BaseModel):
    mode: str = "neighbours"
    row_size: int = 5
    max_communication_distance: int = 2
    max_nb_agents_communication: int = 10


class ClusterPropreties(BaseModel):  # (sic) — the reference's class name
    nb_agents: int = 1000
    nb_agents_comm: int = 10
    agents_comm_prop: AgentsCommunicationProperties = AgentsCommunicationProperties()
    message_prop: MessageProperties = MessageProperties()
    house_prop: BuildingProperties = BuildingProperties()


ClusterProperties = ClusterPropreties

# ---------------------------------------------------------------- power_grid_properties.py:6-70

SIGNAL_MODES = ("flat", "sinusoidals", "regular_steps", "perlin")
BASE_POWER_MODES = ("constant", "interpolation")


class SignalProperties(BaseModel):
    mode: str = "perlin"
    amplitude_ratios: List[float] = [0.1, 0.3]
    amplitude_per_hvac: int = 6000
    nb_octaves: int = 5
    octaves_step: int = 5
    period: int = 300
    periods: List[int] = [400, 1200]


class BasePowerProperties(BaseModel):
    mode: str = "constant"
    avg_power_per_hvac: int = 4200
    init_signal_per_hvac: int = 910
    path_datafile: str = "./monteCarlo/mergedGridSearchResultFinal.npy"
    path_parameter_dict: str = "./monteCarlo/interp_parameters_dict.json"
    path_dict_keys: str = "./monteCarlo/interp_dict_keys.csv"
    interp_update_period: int = 300
    interp_nb_agents: int = 100


class PowerGridProperties(BaseModel):
    artificial_signal_ratio_range: int = 1
    base_power_props: BasePowerProperties = BasePowerProperties()
    signal_properties: SignalProperties = SignalProperties()
    artificial_ratio: float = 1.0


# ---------------------------------------------------------------- environment_properties.py:339-372


class EnvironmentProperties(BaseModel):
    start_datetime: _dt.datetime = _dt.datetime(2021, 1, 1, 0, 0, 0)
    start_datetime_mode: Literal["fixed", "random"] = "random"
    time_step: _dt.timedelta = _dt.timedelta(0, 4)
    temp_prop: TemperatureProperties = TemperatureProperties()
    state_prop: StateProperties = StateProperties()
    reward_prop: RewardProperties = RewardProperties()
    cluster_prop: ClusterPropreties = ClusterPropreties()
    power_grid_prop: PowerGridProperties = PowerGridProperties()

    @classmethod
    def from_dict(cls, d: dict) -> "EnvironmentProperties":
        return cls.model_validate(copy.deepcopy(d))

    @classmethod
    def from_json(cls, path: str, key: str = "env_prop") -> "EnvironmentProperties":
        """Load a MARLconfig-style JSON file (``server/app/core/config/MARLconfig.json``)."""
        with open(path) as f:
            d = json.load(f)
        return cls.from_dict(d[key] if key in d else d)


def override(d: dict, dotted: dict) -> dict:
    """Return a copy of a nested config dict with ``{"a.b.c": v}`` overrides applied."""
    d = copy.deepcopy(d)
    for path, val in dotted.items():
        cur = d
        keys = path.split(".")
        for k in keys[:-1]:
            cur = cur.setdefault(k, {})
        cur[keys[-1]] = val
    return d


def validate(p) -> None:
    """Validate mode strings and comm geometry up front (raises ValueError)."""
    cp = p.cluster_prop
    if cp.agents_comm_prop.mode not in COMM_MODES:
        raise ValueError(f"unknown agents_comm_prop.mode {cp.agents_comm_prop.mode!r}")
    sm = p.power_grid_prop.signal_properties
    if sm.mode not in SIGNAL_MODES:
        raise ValueError(f"unknown signal_properties.mode {sm.mode!r}")
    if sm.mode == "sinusoidals" and len(sm.periods) != len(sm.amplitude_ratios):
        raise ValueError("signal_properties: periods and amplitude_ratios must have the same length")
    if p.power_grid_prop.base_power_props.mode not in BASE_POWER_MODES:
        raise ValueError(f"unknown base_power_props.mode {p.power_grid_prop.base_power_props.mode!r}")
    if p.reward_prop.penalty_props.mode not in PENALTY_MODES:
        raise ValueError(f"unknown penalty_props.mode {p.reward_prop.penalty_props.mode!r}")
    if p.reward_prop.sig_penalty_mode != "common_L2":
        raise ValueError(f"Unknown signal penalty mode: {p.reward_prop.sig_penalty_mode}")
    if cp.nb_agents < 1:
        raise ValueError("nb_agents must be >= 1")
