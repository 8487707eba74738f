"""Build libmdr_hip.so in-tree for gfx950 (hipcc, no JIT cache) and the host-driver extension
mdr_amd/_mdr_host (gcc, CPython C API): ``python build_ext.py``.

Flags that matter for parity: ``-ffp-contract=off`` (no a*b+c fusion: the reference evaluates every
operation with its own rounding) and no fast-math (correctly rounded fp64 division / sqrt).
"""
from __future__ import annotations

import hashlib
import os
import re
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = [os.path.join(HERE, "csrc", f) for f in ("mdr_kernels.hip", "mdr_actor.hip", "mdr_interp.hip", "mdr_capi.hip")]
HDR = [os.path.join(HERE, "csrc", f) for f in ("mdr_kernels.h", "mdr_device.h", "mdr_obs_dev.h", "mdr_actor.h", "mdr_interp.h")] + [
    os.path.join(ROOT, "include", "mdr.h")]
OUT = os.path.join(HERE, "mdr_amd", "libmdr_hip.so")
ARCH = os.environ.get("MDR_OFFLOAD_ARCH", "gfx950")

FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
         f"--offload-arch={ARCH}", "-Wno-unused-value", "-Wno-unused-result",
         "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(HERE, "csrc")]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def src_hash() -> str:
    """sha256 (16 hex digits) of the library's sources, headers and build flags: stamped into the
    library at build time (mdr_build_id) and checked by mdr_amd._lib.load, so a library that was
    not built from the sources next to it is refused."""
    h = hashlib.sha256(" ".join(f for f in FLAGS if not f.startswith("-I")).encode())  # (no paths: the tree moves)
    for p in SRC + HDR:
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def lib_hash(path: str = OUT) -> str | None:
    """The source hash stamped into a built library (None if absent or unstamped)."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        m = re.search(rb"MDR_SRC_HASH:([0-9a-f]{16})", f.read())
    return m.group(1).decode() if m else None


def up_to_date() -> bool:
    return lib_hash(OUT) == src_hash()


HOST_SRC = os.path.join(HERE, "csrc", "mdr_host.c")


def host_out() -> str:
    import sysconfig

    return os.path.join(HERE, "mdr_amd", "_mdr_host" + sysconfig.get_config_var("EXT_SUFFIX"))


HOST_FLAGS = ["-O2", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math", "-Wall"]


def host_src_hash() -> str:
    """sha256 (16 hex digits) of csrc/mdr_host.c and its build flags: stamped into _mdr_host
    (build_id()) and checked when mdr_amd.environment imports it, so a stale extension is refused."""
    h = hashlib.sha256(" ".join(HOST_FLAGS).encode())
    with open(HOST_SRC, "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def host_hash(path: str | None = None) -> str | None:
    """The source hash stamped into a built _mdr_host (None if absent or unstamped)."""
    path = path or host_out()
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        m = re.search(rb"MDR_HOST_SRC_HASH:([0-9a-f]{16})", f.read())
    return m.group(1).decode() if m else None


def build_host(force: bool = False, verbose: bool = False, sanitize: bool = False, out: str | None = None) -> str:
    """The rollout host drivers (csrc/mdr_host.c) as a CPython extension next to the package
    (``sanitize``: an AddressSanitizer + UBSan build for the host tests, written to ``out``)."""
    import sysconfig

    out = out or host_out()
    if not force and not sanitize and host_hash(out) == host_src_hash():
        return out
    cc = os.environ.get("CC", "gcc")
    san = ["-g", "-O1", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=all"] \
        if sanitize else []
    cmd = [cc] + HOST_FLAGS + san + [f"-DMDR_HOST_SRC_HASH=\"{host_src_hash()}\"",
                                     "-I" + sysconfig.get_paths()["include"], HOST_SRC, "-o", out + ".tmp", "-lm"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"{cc} failed ({r.returncode})")
    os.replace(out + ".tmp", out)
    return out


def build(force: bool = False, verbose: bool = False, out: str = OUT, defines=()) -> str:
    """Build the library (``defines``: extra -D flags for A/B variants built next to it, e.g.
    ``out=mdr_amd/libmdr_w4.so, defines=["MDR_WIN_WAVES=4"]``, loaded with MDR_LIB=...)."""
    if not force and out == OUT and up_to_date():
        return out
    import tempfile

    tmp = out + ".tmp"
    # one hipcc per translation unit, in parallel (each carries its own device code), then one link
    cflags = [f for f in FLAGS if f != "-shared"] + ["-D" + d for d in defines] + [f"-DMDR_SRC_HASH=\"{src_hash()}\""]
    with tempfile.TemporaryDirectory(prefix="mdr_build_") as td:
        objs, procs = [], []
        for src in SRC:
            obj = os.path.join(td, os.path.basename(src) + ".o")
            cmd = [hipcc()] + cflags + ["-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd), flush=True)
            objs.append(obj)
            procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
        failed = []
        for src, pr in zip(SRC, procs):
            log = pr.communicate()[0]
            if pr.returncode != 0:
                failed.append(os.path.basename(src))
                sys.stderr.write(log)
        if failed:
            raise RuntimeError(f"hipcc failed: {failed}")
        cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}"] + objs + [
            "-o", tmp, "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise RuntimeError(f"hipcc link failed ({r.returncode})")
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    # python build_ext.py [--force] [--variant NAME DEFINE ...]  (variant -> mdr_amd/libmdr_NAME.so)
    if "--variant" in sys.argv:
        i = sys.argv.index("--variant")
        name, defs = sys.argv[i + 1], sys.argv[i + 2:]
        print(build(force=True, verbose=True, out=os.path.join(HERE, "mdr_amd", f"libmdr_{name}.so"), defines=defs))
    else:
        print(build(force="--force" in sys.argv, verbose=True))
        print(build_host(force="--force" in sys.argv, verbose=True))
