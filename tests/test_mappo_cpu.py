"""The blocked parallel scan of the MAPPO returns (mdr_amd.mappo.discounted_returns) equals the
reference's reversed Python loop (mappo.py:135-140), on the golden buffer and on long random ones."""
import numpy as np
import torch

import golden_util as gu
from mdr_amd.mappo import discounted_returns


def _loop(r, d, g):
    R, out = 0.0, np.empty(len(r))
    for i in reversed(range(len(r))):
        if d[i]:
            R = 0.0
        R = r[i] + g * R
        out[i] = R
    return out


def test_returns_golden_buffer():
    z = gu.load("mappo.npz")
    r = z["rewards"].reshape(-1)  # buffer order: tick-major, house-minor
    d = np.repeat(z["done"], 2)
    got = discounted_returns(torch.from_numpy(r), torch.from_numpy(d), 0.99).numpy()
    np.testing.assert_allclose(got, z["Gt"], rtol=1e-12, atol=1e-12)


def test_returns_long_random():
    rs = np.random.RandomState(0)
    for L in (1, 2, 17, 65, 1000, 12345, 300001):  # (300,001: three levels of block carries)
        r = rs.normal(size=L)
        d = rs.rand(L) < 0.01
        got = discounted_returns(torch.from_numpy(r), torch.from_numpy(d), 0.97).numpy()
        np.testing.assert_allclose(got, _loop(r, d, 0.97), rtol=1e-10, atol=1e-10)
