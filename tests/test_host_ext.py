"""The rollout host-driver extension (csrc/mdr_host.c, ``mdr_amd._mdr_host``), host code only:

* ``rollout1``'s status contract: a failing mdr_rollout is raised, never read as
  "the window crossed midnight" (which would re-issue the same ticks); a begin failure is raised;
  a window that crosses midnight reports "not called" and the caller launches it.  The library
  entry points are replaced by ctypes callbacks, so no GPU is needed.
* the extension refuses to load when built from other sources (hash stamp, as libmdr_hip.so);
* an AddressSanitizer + UBSan build of the same source runs the driver parity checks of
  tests/test_driver_window.py and the rollout1 cases in a subprocess (ASan host build).
"""
import ctypes as C
import datetime as dt
import os
import random
import subprocess
import sys

import numpy as np
import pytest

import golden_util as gu
from oracle_shard import OracleShard

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "marl-demandresponse_amd")

BEGIN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_uint64, C.c_void_p, C.c_int64, C.c_int, C.c_void_p)
ROLL = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p,
                   C.c_int64, C.c_void_p, C.c_int, C.c_void_p)
ROLL_SHARDED = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_void_p,
                           C.c_int64, C.c_void_p, C.c_void_p)


def _env(start):
    from mdr_amd.environment import Environment

    props = gu.props_from_overrides({"cluster_prop.nb_agents": 10,
                                     "power_grid_prop.signal_properties.mode": "sinusoidals"})
    props.start_datetime = start
    props.start_datetime_mode = "fixed"
    return Environment(props, rng=random.Random(3), _shard_factory=OracleShard)


def _launch(rc_begin, rc_roll, calls, sharded=False):
    def begin(ctx, n, tick0, action, stride, mode, stream):
        calls.append(("begin", n, tick0, mode))
        return rc_begin

    def roll(ctx, n, ticks, action, stride, mode, reward, rew_stride, p_out, use_graph, stream):
        rows = np.ctypeslib.as_array(C.cast(ticks, C.POINTER(C.c_double)), shape=(n, 4)).copy()
        calls.append(("rollout", n, int(rows[0, 3:].view(np.uint64)[0]), mode))
        return rc_roll

    def roll_sharded(ctx, n, ticks, action, stride, mode, reward, rew_stride, p_out, stream):
        rows = np.ctypeslib.as_array(C.cast(ticks, C.POINTER(C.c_double)), shape=(n, 4)).copy()
        calls.append(("rollout_sharded", n, int(rows[0, 3:].view(np.uint64)[0]), mode))
        return rc_roll

    cb = (BEGIN(begin), ROLL_SHARDED(roll_sharded) if sharded else ROLL(roll))
    addr = [C.cast(f, C.c_void_p).value for f in cb]
    return cb, (addr[0], addr[1], 0x1000, 0, 0x2000, 10, 0x3000, 1, 1 if sharded else 0)


def rollout1_cases():
    """The three status paths of Environment._driver_window_vec(n, launch) (importable by the ASan
    subprocess)."""
    from mdr_amd import _lib as L

    noon = dt.datetime(2021, 7, 4, 12, 0)
    # 1. mdr_rollout fails: raised, with the library status
    calls = []
    cb, launch = _launch(0, -2, calls)  # MDR_EHIP
    env = _env(noon)
    with pytest.raises(L.MdrError):
        env._driver_window_vec(20, launch)
    assert [c[0] for c in calls] == ["begin", "rollout"]
    # 2. mdr_rollout_begin fails: raised before any rollout
    calls = []
    cb, launch = _launch(-5, 0, calls)
    with pytest.raises(L.MdrError):
        _env(noon)._driver_window_vec(20, launch)
    assert [c[0] for c in calls] == ["begin"]
    # 3. success, and a window across midnight: not launched by rollout1 (the caller launches)
    calls = []
    cb, launch = _launch(0, 0, calls)
    w, launched = _env(noon)._driver_window_vec(20, launch)
    assert launched and len(w) == 20 and calls[-1] == ("rollout", 20, 0, 1)
    calls = []
    cb, launch = _launch(0, 0, calls)
    w, launched = _env(dt.datetime(2021, 7, 4, 23, 59, 30))._driver_window_vec(20, launch)
    assert not launched and len(w) == 20 and [c[0] for c in calls] == ["begin"]
    # 4. a sharded context (a communicator attached in the library): mdr_rollout_sharded's signature
    calls = []
    cb, launch = _launch(0, 0, calls, sharded=True)
    w, launched = _env(noon)._driver_window_vec(20, launch)
    assert launched and len(w) == 20 and calls[-1] == ("rollout_sharded", 20, 0, 1)
    calls = []
    cb, launch = _launch(0, -2, calls, sharded=True)
    with pytest.raises(L.MdrError):
        _env(noon)._driver_window_vec(20, launch)
    assert [c[0] for c in calls] == ["begin", "rollout_sharded"]
    del cb


def test_rollout1_status_contract():
    from mdr_amd import environment

    if environment._host is None:
        pytest.skip("_mdr_host not built")
    rollout1_cases()


def test_host_ext_hash_stamp():
    """The extension carries the hash of the source it was built from, equal to this tree's."""
    import build_ext

    from mdr_amd import environment

    assert environment._host is not None
    assert environment._host.build_id() == "MDR_HOST_SRC_HASH:" + build_ext.host_src_hash()
    assert build_ext.host_hash() == build_ext.host_src_hash()


def _asan_body(so_path):
    """Runs inside the sanitized subprocess: the sanitized build as mdr_amd._mdr_host, then the
    driver parity checks and the rollout1 cases."""
    import importlib.machinery
    import importlib.util

    loader = importlib.machinery.ExtensionFileLoader("mdr_amd._mdr_host", so_path)
    spec = importlib.util.spec_from_file_location("mdr_amd._mdr_host", so_path, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    import mdr_amd

    sys.modules["mdr_amd._mdr_host"] = mod
    mdr_amd._mdr_host = mod
    from mdr_amd import environment

    assert environment._host is mod
    import test_driver_window as tdw

    for case in tdw.CASES:
        tdw._check(*case)
    tdw.test_native_drivers_module_rng_and_short_windows()
    rollout1_cases()
    print("ASAN_BODY_OK", flush=True)


def test_host_ext_under_asan(tmp_path):
    """csrc/mdr_host.c built with -fsanitize=address,undefined runs the driver-window parity
    cases and the rollout1 status cases clean (any report aborts the subprocess)."""
    if os.environ.get("LD_PRELOAD"):
        pytest.skip("a preload is already set in this environment")
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(asan) or not os.path.exists(asan):
        pytest.skip("no libasan runtime")
    import build_ext

    import sysconfig

    so = str(tmp_path / ("_mdr_host_asan" + sysconfig.get_config_var("EXT_SUFFIX")))
    build_ext.build_host(sanitize=True, out=so)
    env = dict(os.environ, LD_PRELOAD=asan, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", PYTHONPATH=os.pathsep.join([HERE, PKG, ROOT]))
    code = f"import test_host_ext as t; t._asan_body({so!r})"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600,
                       cwd=HERE)
    assert r.returncode == 0 and "ASAN_BODY_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-6000:]
    assert "runtime error" not in r.stderr, r.stderr[-6000:]
