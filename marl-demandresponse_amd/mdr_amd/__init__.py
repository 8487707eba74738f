"""mdr_amd — MI355X-native vectorised environment step of marl-demandresponse.

The product path is HIP (libmdr_hip.so, C ABI in include/mdr.h) driven from this Python layer
with PyTorch-ROCm tensors as the device container.  ``import mdr_amd`` does not touch the GPU;
constructing an ``Environment`` loads the library and fails loudly if it (or a GPU) is missing.
"""
from . import config
from .config import EnvironmentProperties

__all__ = ["Environment", "EnvironmentProperties", "config", "load_library"]


def load_library():
    from ._lib import load

    return load()


def __getattr__(name):
    if name == "Environment":
        from .environment import Environment

        return Environment
    raise AttributeError(name)
