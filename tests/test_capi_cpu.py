"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/mdr.h declares,
and the ctypes struct layouts match the C structs (no GPU calls)."""
import os
import re

import pytest

import golden_util as gu  # noqa: F401  (sys.path set by conftest)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    with open(os.path.join(ROOT, "include", "mdr.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"^(?:int|size_t|const char\*)\s+(mdr_\w+)\s*\(", src, re.M)))


def test_header_symbols_exported():
    from mdr_amd import _lib

    lib = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)


def test_abi_struct_sizes_and_version():
    import ctypes as C

    from mdr_amd import _lib

    lib = _lib.load()
    assert lib.mdr_abi_version() == _lib.ABI_VERSION
    sizes = (C.c_int64 * 9)()
    assert lib.mdr_abi_sizes(sizes, 9) == 9
    assert list(sizes) == [C.sizeof(t) for t in (_lib.mdr_config, _lib.mdr_soa, _lib.mdr_tick,
                                                 _lib.mdr_pop_spec, _lib.mdr_obs_spec, _lib.mdr_obs_scalars,
                                                 _lib.mdr_actor_spec, _lib.mdr_interp_spec, _lib.mdr_actor_net)]
    assert _lib.ABI_STRUCTS[-1] is _lib.mdr_actor_net


def test_argument_errors_without_gpu():
    """Argument validation happens before any HIP call: these return MDR_EARG on a CPU box."""
    import ctypes as C

    from mdr_amd import _lib

    lib = _lib.load()
    assert lib.mdr_create(None, None) == -1
    cfg = _lib.mdr_config()
    cfg.abi_version = 999
    ctx = C.c_void_p()
    assert lib.mdr_create(C.byref(ctx), C.byref(cfg)) == -1
    assert b"ABI" in lib.mdr_last_error()
    cfg.abi_version = _lib.ABI_VERSION
    cfg.n_local, cfg.n_global = 10, 5
    assert lib.mdr_create(C.byref(ctx), C.byref(cfg)) == -1
    assert lib.mdr_step(None, None, 0, None, None, 0, 0, None, None, None) == -1
    assert lib.mdr_rccl_allreduce(None, None, 1, 0, None) == -1
    spec = _lib.mdr_obs_spec()
    spec.msg_thermal, spec.msg_hvac = 1, 1
    assert lib.mdr_msg_width(C.byref(spec)) == 11
    assert lib.mdr_interp_load(None, None) == -1
    assert lib.mdr_interp_values(None, None, 1, 0.0, 0.0, 0.0, None, None) == -1
    assert lib.mdr_interp_sum(None, -1, 1.0, None, None) == -1


def test_window_geometry_guard():
    """The host-side check every k_count_window / k_step_window launch makes (the
    r04j overrun of the ON-mask rows by a ragged 16-wave count block): buffers sized by mdr_create
    pass at every shard size, and a buffer one byte short of what the launch geometry touches, or
    an end-word buffer shorter than the shard, is refused with MDR_EARG before anything launches."""
    from mdr_amd import _lib

    lib = _lib.load()
    hpt, kmax = 2, 32  # kWinHpt, kWindowMax (mdr_kernels.h)
    for n in (1, 63, 64, 128, 129, 2049, 65536, 131071, 1 << 20, (1 << 20) + 7):
        tiles = (n + 64 * hpt - 1) // (64 * hpt)
        need = max(lib.mdr_window_onb_bytes(n, w) for w in (4, 16))
        assert need >= tiles * hpt * kmax * 8  # every real tile's rows
        assert lib.mdr_window_onb_bytes(n, 16) == (tiles + 15) // 16 * 16 * hpt * kmax * 8
        # the allocation of mdr_create (mdr_capi.hip: whole count blocks + one row)
        alloc = ((tiles + 16) // 16 * 16 * hpt + 1) * kmax * 8
        assert lib.mdr_window_geometry_check(n, alloc, (n + 1) * 4) == 0, lib.mdr_last_error()
        assert lib.mdr_window_geometry_check(n, need, n * 4) == 0
        assert lib.mdr_window_geometry_check(n, need - 1, n * 4) == -1
        assert b"ON-mask" in lib.mdr_last_error()
        assert lib.mdr_window_geometry_check(n, need, n * 4 - 1) == -1
    assert lib.mdr_window_geometry_check(0, 1 << 20, 1 << 20) == -1


def test_environment_fails_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from mdr_amd import _lib
    from mdr_amd.config import EnvironmentProperties
    from mdr_amd.environment import Environment

    p = EnvironmentProperties()
    p.cluster_prop.nb_agents = 10
    p.power_grid_prop.signal_properties.mode = "flat"
    with pytest.raises(_lib.MdrLibraryError):
        Environment(p)
