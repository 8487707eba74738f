"""Perlin regulation-signal noise — PARITY UNPINNED.

The reference (server/app/core/environment/power_grid/perlin.py:17-56) sums octaves of the
third-party ``perlin_noise`` package (pinned ``perlin_noise==1.*``, server/requirements.txt:11),
which is absent from this image and cannot be fetched; no reference test or fixture pins its
values.  This module restates the package's published 1-D algorithm (PerlinNoise.noise,
rand_vec.RandVec, tools.sample_vector / hasher / fade) as we know it:

* the coordinate is scaled by the octave count: xs = x * octaves;
* the two lattice points floor(xs), floor(xs + 1) each carry a gradient drawn as
  ``uniform(-1, 1)`` from a Mersenne Twister seeded with ``hasher([k]) * seed`` — hasher([k]) =
  max(1, int(|k| + 1)) and ``seed`` is the float ``random.random()`` SignalCalculator passes
  (signal_calculator.py:24-31), so ``random.seed`` hashes the float;
* a lattice point contributes ``fade(1 - |xs - k|) * g * (xs - k)`` with fade(t) = 6 * t ** 5 -
  15 * t ** 4 + 10 * t ** 3, the package's expression with Python float ``**`` (libm pow); the
  vectorised form evaluates that same scalar expression once per distinct t, so both forms equal
  the package's operations bit for bit; the contributions are summed with Python's ``sum`` (from
  int 0), in the order of ``itertools.product``.

The package draws the gradient by reseeding the GLOBAL ``random`` module; releases from 1.12 save
and restore the global state around it, earlier ones leave it reseeded (the reference's later
``random.gauss`` OD-temperature draws would then follow the last lattice seed).  ``global_rng``
selects that behaviour: None (default) = the restoring releases (no side effect), or a module /
``random.Random`` whose state is left reseeded as the older releases leave ``random``.  The octave
combination follows the reference exactly, including its last-octave divisor ``2**n - 1``
(perlin.py:55).
"""
from __future__ import annotations

import math
import random

import numpy as np


def _fade(t: float) -> float:
    # tools.fade: the package rejects t outside [-0.1, 1.1]; 1 - |d| with |d| <= 1 never is
    return 6 * t ** 5 - 15 * t ** 4 + 10 * t ** 3


_fade_py = np.frompyfunc(_fade, 1, 1)


def _fade_array(t: np.ndarray) -> np.ndarray:
    """_fade of every element through the scalar expression (Python float ``**``, not NumPy's
    power, whose rounding may differ by an ulp), once per distinct value."""
    u, inv = np.unique(t, return_inverse=True)
    return _fade_py(u).astype(np.float64)[inv.reshape(t.shape)]


def _hasher(k: int) -> int:
    return max(1, int(abs(k) + 1))


class _GradientNoise1D:
    """PerlinNoise(octaves, seed) restricted to scalar coordinates."""

    def __init__(self, octaves: float, seed, global_rng=None):
        if octaves <= 0:
            raise ValueError("octaves expected to be positive number")
        if seed is not None and not isinstance(seed, int) and seed <= 0:
            raise ValueError("seed expected to be positive integer number")
        self.octaves = octaves
        self.seed = seed if seed else random.randint(1, 10 ** 5)
        self.global_rng = global_rng
        self._r = random.Random()
        self.cache = {}

    def _grad(self, k: int) -> float:
        if self.global_rng is not None:  # pre-1.12 releases: the caller's generator is left reseeded
            self.global_rng.seed(_hasher(k) * self.seed)
            return self.global_rng.uniform(-1, 1)
        g = self.cache.get(k)
        if g is None:
            self._r.seed(_hasher(k) * self.seed)
            g = self._r.uniform(-1, 1)
            self.cache[k] = g
        return g

    def noise(self, x: float) -> float:
        xs = x * self.octaves
        total = 0
        for k in (math.floor(xs), math.floor(xs + 1)):
            d = xs - k
            total += _fade(1 - abs(d)) * (self._grad(k) * d)  # weight_to * dot(vec, dists)
        return total

    def noise_array(self, x: np.ndarray) -> np.ndarray:
        """``noise`` of every element of a float64 array, bit for bit (the gradients of the lattice
        points it touches are drawn once each, in increasing k; no global-RNG side effect)."""
        if self.global_rng is not None:
            raise ValueError("the pre-1.12 global-RNG side effect has no array form")
        xs = x * self.octaves
        total = np.zeros_like(xs)
        for k in (np.floor(xs), np.floor(xs + 1)):
            ks = np.unique(k)
            g = np.array([self._grad(int(v)) for v in ks], np.float64)[np.searchsorted(ks, k)]
            d = xs - k
            total = total + _fade_array(1 - np.abs(d)) * (g * d)
        return total


class Perlin:
    """Octave sum of the reference's Perlin helper (perlin.py:5-56)."""

    def __init__(self, amplitude, nb_octaves, octaves_step, period, seed, global_rng=None):
        self.amplitude = amplitude
        self.nb_octaves = nb_octaves
        self.octaves_step = octaves_step
        self.period = period
        self.seed = seed
        self.noise_list = [_GradientNoise1D(2 ** i * octaves_step, seed, global_rng) for i in range(nb_octaves)]

    def calculate_noise(self, x) -> float:
        noise = 0
        for j in range(self.nb_octaves - 1):
            noise += self.noise_list[j].noise(x / self.period) / (2 ** j)
        noise += self.noise_list[-1].noise(x / self.period) / (2 ** self.nb_octaves - 1)
        return self.amplitude * noise

    def calculate_noise_array(self, x: np.ndarray) -> np.ndarray:
        """``calculate_noise`` of every element of a float64 array, bit for bit."""
        xp = np.asarray(x, np.float64) / self.period
        noise = np.zeros_like(xp)
        for j in range(self.nb_octaves - 1):
            noise = noise + self.noise_list[j].noise_array(xp) / (2 ** j)
        noise = noise + self.noise_list[-1].noise_array(xp) / (2 ** self.nb_octaves - 1)
        return self.amplitude * noise
