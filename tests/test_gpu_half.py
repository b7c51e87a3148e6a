"""The half-size scalar search on the device (through the C-ABI diagnostic
fd_ed25519_hip_diag_half_scalars) against the host build of the same
header (tests/half_harness.cpp) and against Python integers: identical
(ok, c, d) for random and edge k.  The device estimates reciprocals with
v_rcp_f64; the exact remainder corrections must make that invisible."""
import random

import numpy as np
import pytest

from test_half import BITS, DBITS_EXT, L, N8L, half, run  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu


def words(k):
    return [(k >> (32 * i)) & 0xffffffff for i in range(8)]


@pytest.mark.parametrize("mode,dbits", [("extended", DBITS_EXT), ("strict", BITS)])
def test_device_matches_host(half, mode, dbits):
    from firedancer_amd import ed25519
    rng = random.Random(21)
    ks = [rng.randrange(L) for _ in range(6000)]
    ks += [0, 1, 2, 3, L - 1, L - 2, (L - 1) // 2, 2**BITS - 1, 2**BITS, 2**BITS + 1, 2**200, 2**252 - 1, 8]
    ks += [pow(2, e, L) for e in range(0, 253, 3)]
    ks += [((N8L * num) // den + delta) % L for den in (3, 7, 11, 1001) for num in (1, 2)
           for delta in (-1, 0, 1, 2**60)]
    e = ed25519.Engine(0, max_chunk=1 << 12, half=mode)
    try:
        out = e.diag_half_scalars(np.array([words(k) for k in ks], dtype=np.uint32))
    finally:
        e.close()
    found = 0
    for i, k in enumerate(ks):
        ok, c, d = run(half, k, dbits)
        o = out[i]
        cv = sum(int(o[2 + w]) << (32 * w) for w in range(5))
        dv = sum(int(o[7 + w]) << (32 * w) for w in range(5))
        dv = -dv if o[1] else dv
        assert int(o[0]) == ok, (hex(k), int(o[0]), ok)
        if ok:
            found += 1
            assert (cv, dv) == (c, d), hex(k)
            assert (cv - dv * k) % N8L == 0 and dv % 2 and 0 <= cv < 2**BITS and abs(dv) < 2**dbits
    assert found > 0.97 * len(ks)   # the near-rational k are built to fail more often
