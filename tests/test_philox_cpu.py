"""The NumPy restatement of the device random controller (tests/philox_np.py) reproduces the
published Philox4x32-10 known-answer vectors (Random123 kat_vectors), and its bit layout matches
mdr_device.h (one 64-bit word per 64-house group and tick)."""
import numpy as np

import philox_np as P

KAT = [  # (counter x4, key x2) -> output x4
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_philox_known_answers():
    for ctr, key, want in KAT:
        got = P.philox4x32_10(*ctr, *key)
        assert [int(x) for x in got] == list(want)


def test_random_action_bit_layout():
    seed, tick = 1234, 7
    gids = np.arange(0, 256, dtype=np.uint64)
    a = P.random_actions(seed, gids, tick)
    for g in range(4):
        lo, hi = P.philox_words(seed, np.uint64(g), np.uint64(tick))
        word = int(lo) | (int(hi) << 32)
        bits = np.array([(word >> b) & 1 for b in range(64)], bool)
        np.testing.assert_array_equal(a[64 * g:64 * (g + 1)], bits)
    # a shard offset does not change a house's action (keyed by global id)
    np.testing.assert_array_equal(P.random_actions(seed, gids[100:], tick), a[100:])


def test_random_actions_are_fair():
    a = P.random_actions(99, np.arange(1 << 18, dtype=np.uint64), 3)
    assert abs(a.mean() - 0.5) < 4 * 0.5 / np.sqrt(a.size)
