"""Perlin regulation-signal noise — PARITY UNPINNED.

The reference (server/app/core/environment/power_grid/perlin.py:17-56) sums octaves of the
third-party ``perlin_noise`` package (pinned ``perlin_noise==1.*``, server/requirements.txt:11),
which is absent from this image and cannot be fetched; no reference test or fixture pins its
values.  This module restates the package's published algorithm — 1-D gradient noise: the input
is scaled by the octave count, the two surrounding integer lattice points each carry a unit
gradient drawn from an RNG seeded by (lattice point, seed), and their contributions
``fade(1 - |d|) * g * d`` (fade = 6t^5 - 15t^4 + 10t^3) are summed — with a PRIVATE RNG (the
package reseeds the global ``random``; we do not), so values are statistically equivalent but not
bit-identical.  The octave combination follows the reference exactly, including its last-octave
divisor ``2**n - 1`` (perlin.py:55).
"""
from __future__ import annotations

import math
import random


def _fade(t: float) -> float:
    return 6 * t ** 5 - 15 * t ** 4 + 10 * t ** 3


class _GradientNoise1D:
    def __init__(self, octaves: float, seed):
        if octaves <= 0:
            raise ValueError("octaves expected to be positive number")
        self.octaves = octaves
        self.seed = seed
        self.cache = {}

    def _grad(self, k: int) -> float:
        g = self.cache.get(k)
        if g is None:
            r = random.Random(hash((k, self.seed)))
            g = 1.0 if r.random() * 2 - 1 >= 0 else -1.0  # a normalised 1-D vector is +-1
            self.cache[k] = g
        return g

    def noise(self, x: float) -> float:
        x = x * self.octaves
        k0 = math.floor(x)
        total = 0.0
        for k in (k0, k0 + 1):
            d = x - k
            total += _fade(1 - abs(d)) * self._grad(k) * d
        return total


class Perlin:
    """Octave sum of the reference's Perlin helper (perlin.py:5-56)."""

    def __init__(self, amplitude, nb_octaves, octaves_step, period, seed):
        self.amplitude = amplitude
        self.nb_octaves = nb_octaves
        self.octaves_step = octaves_step
        self.period = period
        self.seed = seed
        self.noise_list = [_GradientNoise1D(2 ** i * octaves_step, seed) for i in range(nb_octaves)]

    def calculate_noise(self, x) -> float:
        noise = 0
        for j in range(self.nb_octaves - 1):
            noise += self.noise_list[j].noise(x / self.period) / (2 ** j)
        noise += self.noise_list[-1].noise(x / self.period) / (2 ** self.nb_octaves - 1)
        return self.amplitude * noise
