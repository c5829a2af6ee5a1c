"""Pin the oracle's Philox4x32-10 to the Random123 known-answer vectors."""
import numpy as np

from oracle import philox as rng

KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_philox_kat():
    for c, k, want in KAT:
        got = rng.philox4x32_10(*c, *k)
        assert tuple(int(x) for x in got) == want


def test_uniform_range_and_exactness():
    w = rng.draw_u32(123, np.arange(10000), 7, rng.RNG_RESET_POS)
    u = rng.u32_to_unit_f32(w[0])
    assert u.dtype == np.float32 and u.min() >= 0 and u.max() < 1
    x = rng.uniform_f32(w[1], -1.5, 1.5)
    assert x.min() >= -1.5 and x.max() < 1.5
    # mean of 10k uniforms within 4 sigma
    assert abs(float(u.mean()) - 0.5) < 4 * (1 / 12 / 10000) ** 0.5


def test_counter_independence():
    a = rng.draw_u32(5, np.arange(8), 0, rng.RNG_TARGET)[0]
    b = rng.draw_u32(5, np.arange(8), 1, rng.RNG_TARGET)[0]
    c = rng.draw_u32(6, np.arange(8), 0, rng.RNG_TARGET)[0]
    assert not np.array_equal(a, b) and not np.array_equal(a, c)
