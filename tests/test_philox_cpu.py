"""The numpy Philox restatement (oracle/philox.py) against the published
Philox4x32-10 known-answer vectors (Random123 kat_vectors, Salmon et al. SC'11),
so the GPU noise tests check against a pinned generator."""
import numpy as np

from oracle.philox import normal4, philox4x32_10

KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_philox4x32_10_known_answers():
    for ctr, key, want in KAT:
        got = philox4x32_10(*[np.uint64(x) for x in ctr], key[0] | (key[1] << 32))
        assert tuple(int(x) for x in got) == want


def test_normal4_vectorised_and_moments():
    z = normal4(1234, 0x4F4D414E, np.zeros(1, np.uint64), np.arange(50_000, dtype=np.uint64))
    assert z.shape == (50_000, 4)
    one = normal4(1234, 0x4F4D414E, np.uint64(0), np.uint64(777))
    assert np.array_equal(one, z[777])
    assert abs(z.mean()) < 0.01 and abs(z.var() - 1.0) < 0.01


def test_fill_c_restatement_matches_numpy():
    """oracle/philox_fill.c (the fast restatement of the device fill used for large
    well-posedness inputs) agrees bit for bit with the numpy restatement."""
    import numpy as np

    import oracle.philox as ph
    lib = ph._fill_lib()
    assert lib is not None, "gcc could not build oracle/_philox_fill.so"
    a = ph.fill_clients(9, 1003, 3, 0.0, 0.05, 0.25, 0.5, 777, col_off=5)
    b = ph.fill_normal(1003, 0.0, 0.01, 99, off=7)
    saved, ph._FILL_LIB = ph._FILL_LIB, False
    try:
        a2 = ph.fill_clients(9, 1003, 3, 0.0, 0.05, 0.25, 0.5, 777, col_off=5)
        b2 = ph.fill_normal(1003, 0.0, 0.01, 99, off=7)
    finally:
        ph._FILL_LIB = saved
    assert np.array_equal(a, a2) and np.array_equal(b, b2)
