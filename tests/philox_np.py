"""NumPy restatement of the device random controller (csrc/mdr_device.h philox4x32_10 /
philox_words / bit_of) — test infrastructure: lets the oracle replay exactly the actions the
fused HIP kernels draw (MDR_ACT_RANDOM), so the benched kernel's action source is checked against
the oracle, not only HIP-against-HIP.

Philox4x32-10 is Salmon et al., "Parallel random numbers: as easy as 1, 2, 3" (SC'11); the
known-answer vectors of its reference implementation (Random123 kat_vectors) pin this restatement
(tests/test_philox_cpu.py).
"""
from __future__ import annotations

import numpy as np

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10; every argument is an array (or scalar) of 32-bit values."""
    c0, c1, c2, c3, k0, k1 = (np.asarray(x, np.uint64) & _MASK for x in (c0, c1, c2, c3, k0, k1))
    for _ in range(10):
        p0 = _M0 * c0
        p1 = _M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + _W0) & _MASK
        k1 = (k1 + _W1) & _MASK
    return c0, c1, c2, c3


def philox_words(seed: int, grp, tick):
    """philox_words (mdr_device.h): counter (grp lo, grp hi, tick lo, tick hi ^ 0x5A17), key = seed."""
    grp = np.asarray(grp, np.uint64)
    tick = np.asarray(tick, np.uint64)
    s = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
    r = philox4x32_10(grp & _MASK, grp >> np.uint64(32), tick & _MASK,
                      (tick >> np.uint64(32)) ^ np.uint64(0x5A17), s & _MASK, s >> np.uint64(32))
    return r[0], r[1]


def random_actions(seed: int, gids, tick: int) -> np.ndarray:
    """MDR_ACT_RANDOM action of global houses `gids` at tick `tick`: bit (gid & 63) of the first
    64 bits of Philox4x32-10(seed; gid >> 6, tick)."""
    gids = np.asarray(gids, np.uint64)
    lo, hi = philox_words(seed, gids >> np.uint64(6), np.full(gids.shape, tick, np.uint64))
    b = gids & np.uint64(63)
    word = np.where(b < 32, lo, hi)
    sh = np.where(b < 32, b, b - np.uint64(32))
    return ((word >> sh) & np.uint64(1)).astype(bool)
