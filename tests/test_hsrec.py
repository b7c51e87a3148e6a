"""The drop-in's host-side scalars (host/fd_ed25519_hip_hsrec.cc): for the
fixtures' signatures -- random, adversarial S, mixed-order, and k without
a strict half-size pair -- the 32-word record equals what prep16's hash
blocks write: k = SHA-512(R||A||M) mod L, S < L, a pair c = d k (mod 8L)
with d odd, c < 2^131, |d| < 2^dbits, and s' = d S mod L split at 2^144,
checked here with Python integers.  CPU only (the library's host code)."""
import ctypes
import hashlib
import time

import numpy as np
import pytest

L = 2**252 + 27742317777372353535851937790883648493


@pytest.fixture(scope="module")
def hsrec():
    from firedancer_amd import ed25519
    f = ed25519.library().fd_ed25519_hip_private_hsrec
    f.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_ulong, ctypes.c_int, ctypes.c_void_p]
    f.restype = ctypes.c_int
    return f


def _words(rec, a, n):
    return sum(int(rec[a + i]) << (32 * i) for i in range(n))


def _check(f, msg, sig, pub, dbits):
    rec = np.zeros(32, np.uint32)
    ok = f(sig, pub, msg, len(msg), dbits, rec.ctypes.data)
    k = int.from_bytes(hashlib.sha512(sig[:32] + pub + msg).digest(), "little") % L
    S = int.from_bytes(sig[32:], "little")
    if not ok:
        return "no-pair", k
    assert _words(rec, 0, 8) == k
    assert rec[27] == (1 if S < L else 0)
    c, dm, dneg = _words(rec, 8, 5), _words(rec, 13, 5), int(rec[28]) & 1
    assert rec[28] in (0, 1) and not rec[29:].any()
    d = -dm if dneg else dm
    if S < L:
        assert (c - d * k) % (8 * L) == 0 and dm % 2 == 1
        assert c < 2**131 and dm < 2**dbits
    sp = (d * S) % L
    lo, hi = _words(rec, 18, 5), _words(rec, 23, 4)
    assert lo == sp % 2**144 and hi == sp >> 144
    return "ok", k


@pytest.mark.parametrize("fixture", ["adversarial", "mixed_order", "halfsize", "longd", "vectors"])
@pytest.mark.parametrize("dbits", [151, 131])
def test_records_match_the_device_definition(hsrec, request, fixture, dbits):
    from conftest import case
    d = request.getfixturevalue(fixture)
    n = len(d["msg_sz"])
    idx = range(n) if n <= 1500 else range(0, n, 7)
    outcomes = {"ok": 0, "no-pair": 0}
    for i in idx:
        m, s, p = case(d, i)
        o, _ = _check(hsrec, m, s, p, dbits)
        outcomes[o] += 1
    assert outcomes["ok"] > 0 or (fixture in ("longd", "halfsize") and dbits == 131)   # |d| >= 2^131 by design
    if fixture in ("adversarial", "mixed_order", "vectors") and dbits == 151:
        assert outcomes["no-pair"] == 0


def test_record_costs_a_few_microseconds(hsrec, adversarial):
    from conftest import case
    rec = np.zeros(32, np.uint32)
    cases = [case(adversarial, i) for i in range(200)]
    t = time.perf_counter()
    for m, s, p in cases:
        hsrec(s, p, m, len(m), 151, rec.ctypes.data)
    per = (time.perf_counter() - t) / len(cases)
    assert per < 50e-6, per   # ~5 us here; the bound only catches a pathology
