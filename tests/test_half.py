"""The half-size scalar search of the verify kernel (csrc/fd25519_half.h),
compiled for the host from the same header, checked against Python integers:
c == d k (mod 8L), d odd, 0 <= c < 2^131, |d| < 2^dbits whenever it reports
success, for the strict bound (dbits = 131) and the extended one the kernel
uses by default (dbits = 151: a few more windows for ~0.16% of k), and the
fallback rate to the full-length form stays small.  The identity behind it (E == 0 <=> [d]E == 0
for odd d in a cyclic group of order 8L) is argued in the header; the GPU
parity tests pin the kernel that uses it against the oracle.  CPU only."""
import ctypes
import os
import random
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = 2**252 + 27742317777372353535851937790883648493
N8L = 8 * L
BITS = 131
DBITS_EXT = 151


@pytest.fixture(scope="module")
def half(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("half") / "half.so")
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17",
                           "-I", os.path.join(REPO, "firedancer_amd", "csrc"),
                           os.path.join(REPO, "tests", "half_harness.cpp"), "-o", out])
    lib = ctypes.CDLL(out)
    lib.half_scalars.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int]
    lib.half_scalars.restype = ctypes.c_int
    return lib


def run(lib, k, dbits=BITS):
    kb = (ctypes.c_uint32 * 8)(*[(k >> (32 * i)) & 0xffffffff for i in range(8)])
    c = (ctypes.c_uint32 * 5)()
    d = (ctypes.c_uint32 * 5)()
    neg = ctypes.c_int()
    ok = lib.half_scalars(ctypes.addressof(kb), ctypes.addressof(c), ctypes.addressof(d), ctypes.addressof(neg),
                          dbits)
    cv = sum(int(c[i]) << (32 * i) for i in range(5))
    dv = sum(int(d[i]) << (32 * i) for i in range(5))
    return ok, cv, (-dv if neg.value else dv)


def check(lib, k, dbits=BITS):
    ok, c, d = run(lib, k, dbits)
    if ok:
        assert (c - d * k) % N8L == 0, hex(k)
        assert d % 2 != 0, hex(k)
        assert 0 <= c < 2**BITS and abs(d) < 2**dbits, hex(k)
    return ok


def test_random_k(half):
    rng = random.Random(1)
    n = 20000
    ks = [rng.randrange(L) for _ in range(n)]
    fails = sum(not check(half, k) for k in ks)
    assert 0 < fails < 0.004 * n, fails   # ~0.16% expected: those need |d| >= 2^131
    fails_ext = sum(not check(half, k, DBITS_EXT) for k in ks)
    assert fails_ext == 0, fails_ext      # ~1e-6 expected at 151 bits


def test_extended_pairs_are_the_strict_ones(half):
    """The extended bound changes nothing for k that have a strict pair
    (same c, d), and gives the rest a pair with |d| just above 2^131."""
    rng = random.Random(5)
    longer = 0
    for _ in range(6000):
        k = rng.randrange(L)
        ok, c, d = run(half, k)
        ok2, c2, d2 = run(half, k, DBITS_EXT)
        assert ok2, hex(k)
        if ok:
            assert (c, d) == (c2, d2), hex(k)
        else:
            longer += 1
            assert 2**BITS <= abs(d2) < 2**DBITS_EXT and 0 <= c2 < 2**BITS, hex(k)
            assert (c2 - d2 * k) % N8L == 0 and d2 % 2, hex(k)
    assert longer > 0


def test_edge_k(half):
    ks = [0, 1, 2, 3, L - 1, L - 2, (L - 1) // 2, 2**BITS - 1, 2**BITS, 2**BITS + 1, 2**131, 2**200, 2**252 - 1,
          2**252, 8, 2**125 + 1]
    ks += [pow(2, e, L) for e in range(0, 253, 7)]
    for k in ks:
        for dbits in (BITS, DBITS_EXT):
            ok = check(half, k, dbits)
            if k < 2**BITS:
                assert ok, hex(k)   # (c, d) = (k, 1)


def test_small_quotient_neighbourhood(half):
    """k near rationals with small denominators (large partial quotients):
    the search must either succeed correctly or report failure."""
    for den in (3, 5, 7, 9, 11, 13, 1001):
        for num in range(1, 4):
            base = (N8L * num) // den
            for delta in (-2**60, -1, 0, 1, 2**60):
                k = (base + delta) % L
                check(half, k)
                check(half, k, DBITS_EXT)


def test_matches_exact_euclid(half):
    """Same answer as a plain-integer restatement of the selection rule
    (first remainder below 2^131; (r_i, t_i) if t_i odd, else
    (r_{i-1} - m r_i, t_{i-1} - m t_i) with the least m), at both bounds."""
    def ref(k, dbits):
        r0, t0, r1, t1 = N8L, 0, k, 1
        while r1 >= 2**BITS:
            q = r0 // r1
            r0, t0, r1, t1 = r1, t1, r0 - q * r1, t0 - q * t1
        if t1 % 2:
            c, d = r1, t1
        else:
            m = -(-(r0 - 2**BITS + 1) // r1) if r0 >= 2**BITS else 0
            c, d = r0 - m * r1, t0 - m * t1
        ok = d % 2 != 0 and 0 <= c < 2**BITS and abs(d) < 2**dbits
        return ok, c, d
    rng = random.Random(3)
    for dbits in (BITS, DBITS_EXT):
        agree = 0
        for _ in range(3000):
            k = rng.randrange(L)
            ok, c, d = run(half, k, dbits)
            rok, rc, rd = ref(k, dbits)
            if ok and rok:
                agree += (c, d) == (rc, rd)
        assert agree > 2900, (dbits, agree)


def test_fixture_k_have_no_half_pair(half):
    """tests/golden/halfsize.npz (gen_halfsize.py) holds signatures whose k
    has no strict half-size pair (the full-length form under
    FLAG_HALF_STRICT; the extended-window form by default): check that
    property on the fixture."""
    import hashlib
    import numpy as np
    from conftest import load_golden
    d = load_golden("halfsize")
    for i in range(len(d["msg_sz"])):
        off, sz = int(d["msg_off"][i]), int(d["msg_sz"][i])
        m = bytes(d["msgs"][off:off + sz])
        k = int.from_bytes(hashlib.sha512(d["sigs"][i][:32].tobytes() + d["pubs"][i].tobytes() + m).digest(),
                           "little") % L
        ok, _, _ = run(half, k)
        assert not ok, (i, str(d["tags"][i]))
        ok, _, dd = run(half, k, DBITS_EXT)
        assert ok and abs(dd) >= 2**BITS, (i, str(d["tags"][i]))
    assert len(set(d["codes_avx512"].tolist())) == 4 and np.any(d["codes_avx512"] == 0)


def test_fixture_k_need_long_d(half):
    """tests/golden/longd.npz (gen_longd.py): k whose pair needs
    2^139 <= |d| < 2^151, i.e. 36..38 dsm windows as tagged."""
    import hashlib
    from conftest import load_golden
    d = load_golden("longd")
    for i in range(len(d["msg_sz"])):
        off, sz = int(d["msg_off"][i]), int(d["msg_sz"][i])
        m = bytes(d["msgs"][off:off + sz])
        k = int.from_bytes(hashlib.sha512(d["sigs"][i][:32].tobytes() + d["pubs"][i].tobytes() + m).digest(),
                           "little") % L
        tag = str(d["tags"][i])
        w = int(tag.split("_")[1][1:])
        ok, c, dd = run(half, k, DBITS_EXT)
        assert ok and (c - dd * k) % N8L == 0 and 0 <= c < 2**BITS, tag
        assert (abs(dd).bit_length() + 4) // 4 == w, (tag, abs(dd).bit_length())
        assert not run(half, k, 139)[0], tag


@pytest.mark.parametrize("form", [0, 1, 2, 3])
def test_inner_step_forms_agree(half, tmp_path, form):
    """The Lehmer inner step's earlier forms (FD_HALF_INNER 0-3: the
    double-precision division, one branch per step, the single-precision
    estimate with an exactness test, the estimate bounded below 2^20 with
    the operand checks in the branch) give the same (ok, c, d) as the
    default (4: that with two steps per branch, falling back to the last
    step that passed) -- the remainder sequence is unique, only where a
    round ends may differ."""
    out = str(tmp_path / ("half%d.so" % form))
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-DFD_HALF_INNER=%d" % form,
                           "-I", os.path.join(REPO, "firedancer_amd", "csrc"),
                           os.path.join(REPO, "tests", "half_harness.cpp"), "-o", out])
    other = ctypes.CDLL(out)
    other.half_scalars.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int]
    other.half_scalars.restype = ctypes.c_int
    rng = random.Random(17 + form)
    ks = [rng.randrange(L) for _ in range(20000)] + [0, 1, L - 1, 2**BITS, 2**252 - 1]
    for k in ks:
        for dbits in (BITS, DBITS_EXT):
            assert run(half, k, dbits) == run(other, k, dbits), (hex(k), dbits)
