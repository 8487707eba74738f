"""Scalar restatement of the reference's perlin regulation signal — TEST INFRASTRUCTURE ONLY.

PARITY UNPINNED: the reference (server/app/core/environment/power_grid/perlin.py:17-56,
signal_calculator.py:24-31,100-115) sums octaves of the third-party ``perlin_noise`` package
(``perlin_noise==1.*``, server/requirements.txt:11), which is absent here and has no reference
fixture.  This is the package's published 1-D algorithm (PerlinNoise.noise with its fade, hasher
and per-lattice-point seeded ``random.uniform(-1, 1)`` gradient), written independently of
``mdr_amd/perlin.py`` and in the package's own operation forms (``t ** 5``, Python float pow);
the product evaluates the same expressions, so the two agree bit for bit
(tests/test_host_logic.py::test_perlin_array_equals_oracle).
Used by the oracle (oracle/env_np.py) when ``signal_properties.mode == "perlin"``.
"""
from __future__ import annotations

import math
import random


class PerlinNoise1D:
    def __init__(self, octaves: float, seed: float):
        self.octaves = octaves
        self.seed = seed
        self._g = {}

    def _gradient(self, k: int) -> float:
        # rand_vec: random.seed(hasher(coors) * seed); uniform(-1, 1) (1-D);  hasher = max(1, |k| + 1)
        if k not in self._g:
            self._g[k] = random.Random(max(1, int(abs(k) + 1)) * self.seed).uniform(-1, 1)
        return self._g[k]

    def noise(self, x: float) -> float:
        xs = x * self.octaves
        total = 0
        for k in (math.floor(xs), math.floor(xs + 1)):
            d = xs - k
            w = 1 - abs(d)
            total += (6 * w ** 5 - 15 * w ** 4 + 10 * w ** 3) * (self._gradient(k) * d)
        return total


class PerlinSignal:
    """perlin.py:17-56 (Perlin.calculate_noise) with amplitude 1, as SignalCalculator builds it."""

    def __init__(self, nb_octaves: int, octaves_step: float, period: float, seed: float):
        self.period = period
        self.noises = [PerlinNoise1D(2 ** i * octaves_step, seed) for i in range(nb_octaves)]

    def calculate_noise(self, x: float) -> float:
        n = len(self.noises)
        noise = 0
        for j in range(n - 1):
            noise += self.noises[j].noise(x / self.period) / (2 ** j)
        noise += self.noises[-1].noise(x / self.period) / (2 ** n - 1)
        return 1 * noise
