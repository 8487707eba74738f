"""ctypes binding of the C ABI in include/mdr.h (libmdr_hip.so, built in-tree for gfx950).

There is no fallback: if the library is missing or fails to load, ``load()`` raises
:class:`MdrLibraryError`.  The product path never computes the step on the CPU.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MDR_LIB", os.path.join(HERE, "libmdr_hip.so"))

ABI_VERSION = 5
MAX_CAP = 64

# enums (mdr.h)
ACT_BUFFER, ACT_RANDOM, ACT_ALWAYS_ON, ACT_BANGBANG, ACT_DEADBAND_BANGBANG = 0, 1, 2, 16, 17
CTRL_NONE, CTRL_BANGBANG, CTRL_DEADBAND_BANGBANG, CTRL_GREEDY_KEYS = 0, 1, 2, 3
COMM_RING, COMM_TABLE = 0, 1
PEN_MODES = {"individual_L2": 0, "common_L2": 1, "common_max_error": 2, "mixture": 3}
ERRORS = {-1: "MDR_EARG", -2: "MDR_EHIP", -3: "MDR_ERCCL", -4: "MDR_ENOMEM", -5: "MDR_ESTATE"}
# mdr_set_option (mdr.h): alternative launch forms of the same computation
OPTIONS = {"step_tpw": 1, "fastdiv": 2, "window_pipeline": 3, "sharded_overlap": 4, "greedy_sort": 5, "halo_overlap": 9, "actor_generic": 10,
           "force_halo": 6, "window_thermal": 7, "halo_in_counts": 12,
           "gq_band": 13, "actor_fp32_form": 14, "gq_fused": 15, "gq_adaptive": 16}
THERMAL_EXACT, THERMAL_AFFINE = 0, 1
FP32_F16_SPLIT, FP32_BF16_SPLIT3 = 0, 1  # MDR_OPT_ACTOR_FP32_FORM


class MdrLibraryError(RuntimeError):
    """libmdr_hip.so is missing or unusable (no CPU fallback exists)."""


class MdrError(RuntimeError):
    pass


class mdr_config(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32), ("device", C.c_int32),
        ("n_local", C.c_int64), ("global_offset", C.c_int64), ("n_global", C.c_int64),
        ("dt", C.c_int32), ("lockout_duration", C.c_int32),
        ("cop", C.c_double), ("lcf", C.c_double), ("deadband", C.c_double),
        ("n_cap", C.c_int32), ("penalty_mode", C.c_int32),
        ("cap_table", C.c_double * MAX_CAP),
        ("alpha_temp", C.c_double), ("alpha_sig", C.c_double),
        ("norm_temp", C.c_double), ("norm_sig", C.c_double),
        ("alpha_ind_l2", C.c_double), ("alpha_common_l2", C.c_double), ("alpha_common_max", C.c_double),
        ("seed", C.c_uint64),
    ]


class mdr_soa(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in
                ("t_air", "t_mass", "hvac", "ua", "ca", "cm", "hm", "target", "cap_idx")]


class mdr_tick(C.Structure):
    _fields_ = [("t_od_prev", C.c_double), ("solar", C.c_double), ("s_prev", C.c_double),
                ("tick", C.c_uint64)]


class mdr_pop_spec(C.Structure):
    _fields_ = [(k, C.c_double) for k in
                ("target_temp", "std_target", "thermo_lo", "thermo_hi", "ca", "cm", "hm",
                 "init_air", "init_mass")] + [("n_draw", C.c_int32), ("draw_idx", C.c_uint8 * MAX_CAP)]


class mdr_obs_spec(C.Structure):
    _fields_ = [
        ("n_feat", C.c_int32), ("hvac_state", C.c_int32), ("solar_state", C.c_int32),
        ("thermal_state", C.c_int32), ("msg_thermal", C.c_int32), ("msg_hvac", C.c_int32),
        ("n_comm", C.c_int32), ("comm_mode", C.c_int32),
        ("comm_table", C.c_void_p), ("halo_msg", C.c_void_p),
        ("norm_reg_sig", C.c_double), ("cfg_ua", C.c_double), ("cfg_ca", C.c_double),
        ("cfg_cm", C.c_double), ("cfg_hm", C.c_double), ("cfg_cap", C.c_double), ("msg_all", C.c_void_p),
    ]


class mdr_obs_scalars(C.Structure):
    _fields_ = [("p", C.c_double), ("s", C.c_double), ("solar", C.c_double), ("t_od", C.c_double)]


class mdr_actor_spec(C.Structure):
    _fields_ = [("n_in", C.c_int32), ("h1", C.c_int32), ("h2", C.c_int32), ("n_act", C.c_int32),
                ("precision", C.c_int32)]


ACTOR_MAX_LAYERS = 8


class mdr_actor_net(C.Structure):
    _fields_ = [("n_in", C.c_int32), ("n_hidden", C.c_int32), ("n_act", C.c_int32), ("precision", C.c_int32),
                ("hidden", C.c_int32 * ACTOR_MAX_LAYERS)]


INTERP_AXES = 10


class mdr_interp_spec(C.Structure):
    _fields_ = [("len", C.c_int32 * INTERP_AXES), ("grid", C.c_void_p), ("values", C.c_void_p),
                ("cfg_ua", C.c_double), ("cfg_cm", C.c_double), ("cfg_ca", C.c_double), ("cfg_hm", C.c_double)]


PREC_BF16, PREC_BF16X3, PREC_FP32 = 1, 3, 6
PRECISIONS = {"bf16": PREC_BF16, "bf16x3": PREC_BF16X3, "fp32": PREC_FP32}

# the structs mdr_abi_sizes reports, in its order
ABI_STRUCTS = (mdr_config, mdr_soa, mdr_tick, mdr_pop_spec, mdr_obs_spec, mdr_obs_scalars, mdr_actor_spec,
               mdr_interp_spec, mdr_actor_net)

P, VP, I, I64, U64, D = C.POINTER, C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_double

# mdr_comm_host callbacks (include/mdr.h mdr_host_allreduce_fn / mdr_host_sendrecv_fn)
HOST_ALLREDUCE_FN = C.CFUNCTYPE(I, VP, VP, I64, I)
HOST_SENDRECV_FN = C.CFUNCTYPE(I, VP, VP, I64, I, VP, I64, I, I)

# name -> (restype, argtypes); every symbol declared in include/mdr.h
SIGNATURES = {
    "mdr_abi_version": (I, []),
    "mdr_abi_sizes": (I, [P(I64), I]),
    "mdr_last_error": (C.c_char_p, []),
    "mdr_graph_info": (I, [VP, P(I64), I]),
    "mdr_graph_memset_probe": (I, [VP, P(I64), I, VP]),
    "mdr_actor_status": (I, [VP, P(I64), I, VP]),
    "mdr_greedy_fused_diag": (I, [VP, P(U64)]),
    "mdr_greedy_fused_stamps": (I, [VP, I, P(U64)]),
    "mdr_create": (I, [P(VP), P(mdr_config)]),
    "mdr_destroy": (I, [VP]),
    "mdr_bind": (I, [VP, P(mdr_soa)]),
    "mdr_params_changed": (I, [VP]),
    "mdr_set_rollout_window": (I, [VP, I]),
    "mdr_set_option": (I, [VP, I, I64]),
    "mdr_window_onb_bytes": (C.c_size_t, [I64, I]),
    "mdr_window_geometry_check": (I, [I64, C.c_size_t, C.c_size_t]),
    "mdr_time_step_kernels": (I, [VP, I, VP, VP, I64, I, VP, I64, VP, P(C.c_float), P(I)]),
    "mdr_rollout_begin": (I, [VP, I, U64, VP, I64, I, VP]),
    "mdr_populate": (I, [VP, P(mdr_pop_spec), VP]),
    "mdr_power_counts": (I, [VP, VP, I, U64, VP]),
    "mdr_counts_buffer": (I, [VP, P(VP), P(I)]),
    "mdr_step": (I, [VP, VP, I, P(mdr_tick), VP, I, I, VP, VP, VP]),
    "mdr_penalty_partials": (I, [VP, VP]),
    "mdr_penalty_buffer": (I, [VP, P(VP)]),
    "mdr_reward_finalize": (I, [VP, P(mdr_tick), VP, VP]),
    "mdr_rollout": (I, [VP, I, VP, VP, I64, I, VP, I64, VP, I, VP]),  # ticks: const mdr_tick*
    "mdr_msg_width": (I, [P(mdr_obs_spec)]),
    "mdr_obs": (I, [VP, P(mdr_obs_spec), P(mdr_obs_scalars), VP, VP, VP]),
    "mdr_halo_pack": (I, [VP, P(mdr_obs_spec), VP, VP]),
    "mdr_msg_pack": (I, [VP, P(mdr_obs_spec), VP, VP]),
    "mdr_ctrl_greedy": (I, [VP, D, VP, VP]),
    "mdr_greedy_fallbacks": (I, [VP, VP]),
    "mdr_greedy_diag": (I, [VP, VP]),
    "mdr_greedy_state": (I, [VP, VP]),
    "mdr_greedy_band": (I, [VP, VP]),
    "mdr_greedy_rollout": (I, [VP, I, VP, VP, I64, VP, I64, VP, VP]),
    "mdr_build_id": (C.c_char_p, []),
    "mdr_greedy_inputs": (I, [VP, VP, VP, VP, VP]),
    "mdr_greedy_select": (I, [VP, I64, VP, VP, VP, D, VP, VP]),
    "mdr_gq_shard_begin": (I, [VP, VP]),
    "mdr_gq_shard_buffers": (I, [VP, VP, VP, VP, VP, VP, VP, VP]),
    "mdr_gq_shard_bins": (I, [VP, D, VP]),
    "mdr_gq_shard_compact": (I, [VP, D, VP, VP]),
    "mdr_gq_shard_select": (I, [VP, D, VP, I, VP, VP]),
    "mdr_gq_shard_fallback": (I, [VP, VP, VP]),
    "mdr_cluster_stats": (I, [VP, VP, VP, VP]),
    "mdr_actor_load": (I, [VP, P(mdr_actor_spec), VP, VP, VP, VP, VP, VP, VP]),
    "mdr_actor_load_net": (I, [VP, P(mdr_actor_net), VP, VP, VP]),
    "mdr_actor_fused": (I, [VP, P(mdr_obs_spec)]),
    "mdr_actor_act": (I, [VP, P(mdr_obs_spec), P(mdr_obs_scalars), VP, U64, VP, VP, VP, VP, I, VP]),
    "mdr_actor_rollout": (I, [VP, I, VP, VP, P(mdr_obs_spec), VP, I64, VP, I64,
                              VP, I64, VP, I, VP]),
    "mdr_actor_rollout_sharded": (I, [VP, I, VP, VP, P(mdr_obs_spec), VP, I64, VP, I64, VP, I64, VP, VP]),
    "mdr_actor_profile": (I, [VP, P(mdr_obs_spec), P(mdr_obs_scalars), VP, P(D), VP]),
    "mdr_interp_load": (I, [VP, P(mdr_interp_spec)]),
    "mdr_interp_values": (I, [VP, VP, I, D, D, D, VP, VP]),
    "mdr_interp_sum": (I, [VP, I, D, VP, VP]),
    "mdr_rccl_unique_id": (I, [VP]),
    "mdr_rccl_init": (I, [VP, VP, I, I]),
    "mdr_rccl_allreduce": (I, [VP, VP, I64, I, VP]),
    "mdr_rccl_allgather": (I, [VP, VP, VP, I64, VP]),
    "mdr_comm_host": (I, [VP, I, I, VP, VP, VP]),
    "mdr_rollout_sharded": (I, [VP, I, VP, VP, I64, I, VP, I64, VP, VP]),
    "mdr_rollout_sharded_mode": (I, [VP, P(I), P(I)]),
    "mdr_probe_stream": (I, [VP, VP, VP]),
    "mdr_div_check": (I, [VP, VP, I64, VP, VP]),
    "mdr_event_record": (I, [VP, I, VP]),
    "mdr_event_elapsed_ms": (I, [VP, I, I, P(C.c_float)]),
}

_lock = threading.Lock()
_lib = None


_fn_addrs = {}


def fn_addr(name: str) -> int:
    """Address of a library entry point (for the host-driver extension's fused rollout call)."""
    a = _fn_addrs.get(name)
    if a is None:
        a = _fn_addrs[name] = C.cast(getattr(load(), name), C.c_void_p).value
    return a


def build_id(lib=None) -> str | None:
    """The source hash the loaded library was built from (mdr_build_id)."""
    lib = lib if lib is not None else _lib
    s = lib.mdr_build_id().decode()
    return s.split(":", 1)[1] if s.startswith("MDR_SRC_HASH:") else None


def source_hash() -> str | None:
    """build_ext.src_hash() of the sources in this tree (None when they are not next to the
    package, e.g. an installed copy)."""
    import importlib.util

    be = os.path.join(os.path.dirname(HERE), "build_ext.py")
    if not os.path.exists(be):
        return None
    spec = importlib.util.spec_from_file_location("_mdr_build_ext", be)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    if not all(os.path.exists(p) for p in m.SRC + m.HDR):
        return None
    return m.src_hash()


def _build_ext():
    import importlib.util

    be = os.path.join(os.path.dirname(HERE), "build_ext.py")
    if not os.path.exists(be):
        return None
    spec = importlib.util.spec_from_file_location("_mdr_build_ext", be)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def check_host_ext(mod) -> None:
    """Refuse a _mdr_host extension that was not built from csrc/mdr_host.c as it is in this tree
    (its stamped build_id() against build_ext.host_src_hash(); skipped when the source is absent)."""
    m = _build_ext()
    if m is None or not os.path.exists(m.HOST_SRC):
        return
    want = m.host_src_hash()
    have = mod.build_id().split(":", 1)[1]
    if have != want:
        raise MdrLibraryError(f"_mdr_host was built from other sources (extension {have}, tree {want}): "
                              "rebuild it with __graft_entry__.build()")


def load(path: str = LIB_PATH):
    """Load libmdr_hip.so (after torch, so one HIP runtime serves both) and bind SIGNATURES."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  (torch's libamdhip64 / librccl must be the process's copies)

        if not os.path.exists(path):
            raise MdrLibraryError(
                f"{path} not found: build it with `python marl-demandresponse_amd/build_ext.py` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        try:
            lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
        except OSError as e:
            raise MdrLibraryError(f"cannot load {path}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.mdr_abi_version() != ABI_VERSION:
            raise MdrLibraryError("libmdr_hip.so ABI version mismatch; rebuild it")
        want_id = source_hash()
        have_id = build_id(lib)
        if want_id is not None and have_id != want_id:
            raise MdrLibraryError(f"{path} was built from other sources (library {have_id}, tree {want_id}): "
                                  "rebuild it with __graft_entry__.build()")
        sizes = (C.c_int64 * len(ABI_STRUCTS))()
        lib.mdr_abi_sizes(sizes, len(ABI_STRUCTS))
        want = [C.sizeof(t) for t in ABI_STRUCTS]
        if list(sizes) != want:
            raise MdrLibraryError(f"ABI struct sizes differ: library {list(sizes)} vs binding {want}")
        _lib = lib
        return lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = _lib.mdr_last_error().decode() if _lib is not None else ""
        raise MdrError(f"{what or 'mdr call'} failed: {ERRORS.get(rc, rc)}: {msg}")


def ptr(t) -> int:
    """Raw device pointer of a torch tensor (None -> NULL)."""
    return 0 if t is None else t.data_ptr()


def stream_handle(device) -> int:
    """The caller's current HIP stream on `device` (raw handle; no torch Stream object is built)."""
    import torch

    idx = getattr(device, "index", None)
    if idx is None:
        return torch.cuda.current_stream(device).cuda_stream
    return torch._C._cuda_getCurrentRawStream(idx)
