"""The host-side point decompression (host/fd_ed25519_hip_hsdec.cc) that
launches of a few signatures use instead of prep16's decode blocks: for
every public key and R of the fixtures plus the edge encodings (y = 0, 1,
p - 1, every non-canonical y >= p, the order-8 points' y with either sign,
random bytes with no root), the flags equal the reference's decompression
rules (restated here with Python integers: fd_ed25519_point_frombytes and
fd_ed25519_affine_is_small_order, src/ballet/ed25519/fd_curve25519.h), x's
ten limbs hold (sign-adjusted) x mod p in the device's tight centered form,
and y's are the encoding's bits as fe_frombytes splits them.  CPU only."""
import ctypes
import time

import numpy as np
import pytest

P = 2**255 - 19
D = (-121665 * pow(121666, P - 2, P)) % P
SQRTM1 = pow(2, (P - 1) // 4, P)
OFF = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]
# the order-8 points' y (fd25519_dsm.h ge_decode)
Y0 = int.from_bytes(bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05"), "little")
Y1 = int.from_bytes(bytes.fromhex("c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a"), "little")


@pytest.fixture(scope="module")
def hsdec():
    from firedancer_amd import ed25519
    f = ed25519.library().fd_ed25519_hip_private_hsdec
    f.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p]
    f.restype = ctypes.c_uint
    return f


def expected(enc, avx):
    raw = int.from_bytes(enc, "little")
    sign = raw >> 255
    yr = raw & (2**255 - 1)
    y = yr % P
    u, v = (y * y - 1) % P, (D * y * y + 1) % P
    x = u * pow(v, 3, P) * pow(u * pow(v, 7, P), (P - 5) // 8, P) % P
    vxx = v * x * x % P
    root, iroot = vxx == u, vxx == (-u) % P
    if not root:
        x = x * SQRTM1 % P
    x0 = x == 0
    fail = not (root or iroot) or (avx and x0 and sign == 1)
    if (x & 1) != sign:
        x = (P - x) % P
    small = x0 or y == 0 or y == Y0 or y == Y1
    return (1 if fail else 0) | (2 if small else 0), x, yr


def check(f, enc, avx):
    pt = np.zeros(20, np.int32)
    flags = f(enc, 1 if avx else 0, pt.ctypes.data)
    want, x, yr = expected(enc, avx)
    assert flags == want, (enc.hex(), avx, flags, want)
    ylimbs = [(yr >> o) & ((1 << (26 if i % 2 == 0 else 25)) - 1) for i, o in enumerate(OFF)]
    assert [int(v) for v in pt[10:]] == ylimbs
    if not want & 1:   # a failed decode's x is never used (precheck's code)
        val = sum(int(pt[i]) << OFF[i] for i in range(10))
        assert val % P == x, enc.hex()
        for i in range(10):   # tight: what fe_carry leaves, limb 1 / 5 one carry more
            assert abs(int(pt[i])) <= (1 << (25 if i % 2 == 0 else 24)) + (1 << 6), (i, int(pt[i]))
    return want


def edge_encodings():
    out = []
    for yv in [0, 1, 2, P - 1, P - 2, Y0, Y1, P - Y0, P - Y1] + [P + i for i in range(19)] + [2**255 - 1]:
        for s in (0, 1):
            out.append((yv | (s << 255)).to_bytes(32, "little"))
    rng = np.random.default_rng(5)
    out += [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(200)]
    return out


@pytest.mark.parametrize("avx", [True, False])
def test_edge_encodings(hsdec, avx):
    seen = set()
    for e in edge_encodings():
        seen.add(check(hsdec, e, avx))
    assert seen >= {0, 1, 2}   # accepted, no root, small order all reached


@pytest.mark.parametrize("fixture", ["adversarial", "mixed_order", "vectors"])
def test_fixture_points(hsdec, request, fixture):
    from conftest import case
    d = request.getfixturevalue(fixture)
    n = len(d["msg_sz"])
    idx = range(n) if n <= 1500 else range(0, n, 7)
    for i in idx:
        _, s, p = case(d, i)
        for avx in (True, False):
            check(hsdec, p, avx)
            check(hsdec, s[:32], avx)


def test_decompression_costs_a_few_microseconds(hsdec, adversarial):
    from conftest import case
    pts = [case(adversarial, i)[2] for i in range(200)]
    out = np.zeros(20, np.int32)
    t = time.perf_counter()
    for p in pts:
        hsdec(p, 1, out.ctypes.data)
    per = (time.perf_counter() - t) / len(pts)
    print(f"host decompression {per * 1e6:.1f} us")
    assert per < 50e-6, per   # a few us; the bound only catches a pathology


def _edwards_add(P1, P2):
    (x1, y1), (x2, y2) = P1, P2
    t = D * x1 * x2 * y1 * y2 % P
    x3 = (x1 * y2 + y1 * x2) * pow(1 + t, P - 2, P) % P
    y3 = (y1 * y2 + x1 * x2) * pow(1 - t, P - 2, P) % P   # a = -1
    return x3, y3


def _limbs_value(limbs):
    return sum(int(limbs[i]) << OFF[i] for i in range(10)) % P


@pytest.fixture(scope="module")
def hsdec3():
    from firedancer_amd import ed25519
    f = ed25519.library().fd_ed25519_hip_private_hsdec3_n
    f.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                  ctypes.c_int, ctypes.c_void_p]
    f.restype = None
    return f


@pytest.mark.parametrize("waves", [4, 8])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 8])
def test_doubled_points_for_the_split_forms(hsdec3, adversarial, mixed_order, n, waves):
    """dsm16s's A_i = [2^(G i)]A and R_i = [2^(G i)]R from the host
    (interleaved doubling chains, extended coordinates, no inversion; G =
    66 for four waves, 33 for eight): every decodable point of the
    fixtures, in groups of n, against Python's affine doubling; the plain
    limbs stay the single-point function's."""
    from conftest import case
    nx, step = (1, 66) if waves == 4 else (3, 33)
    encs = []
    for d in (adversarial, mixed_order):
        for i in range(0, 200):
            _, s, p = case(d, i)
            encs += [p, s[:32]]
    for g in range(0, 48, n):
        grp = encs[g:g + n]
        bufs = [ctypes.create_string_buffer(e, 32) for e in grp]
        arr = (ctypes.c_void_p * len(grp))(*[ctypes.addressof(b) for b in bufs])
        pt = np.zeros((len(grp), 20), np.int32)
        px = np.zeros((len(grp), nx, 40), np.int32)
        fl = np.zeros(len(grp), np.uint8)
        hsdec3(ctypes.addressof(arr), len(grp), 1, pt.ctypes.data, px.ctypes.data, nx, step, fl.ctypes.data)
        for e, a, bx, f in zip(grp, pt, px, fl):
            want, x, yr = expected(e, True)
            assert f == want
            if want & 1:
                continue
            assert _limbs_value(a[:10]) == x and _limbs_value(a[10:]) == yr % P
            Q = (x, yr % P)
            for m in range(nx):
                for _ in range(step):
                    Q = _edwards_add(Q, Q)
                X, Y, Z, T = (_limbs_value(bx[m][10 * c:10 * c + 10]) for c in range(4))
                zi = pow(Z, P - 2, P)
                assert (X * zi % P, Y * zi % P) == Q, (e.hex(), m)   # extended: x = X/Z, y = Y/Z
                assert T * Z % P == X * Y % P
                assert all(abs(int(v)) <= (1 << 25) + 64 for v in bx[m])   # tight (fe_carry's)


@pytest.mark.parametrize("waves", [4, 8])
def test_split_scalars(adversarial, halfsize, waves):
    """hssplit: the record's c and |d| split every 66 (four waves) or 33
    (eight) bits, the last part the rest, and s' in 72- or 32-bit chunks,
    every part summing back exactly (long |d| included: halfsize.npz)."""
    from conftest import case
    from firedancer_amd import ed25519
    lib = ed25519.library()
    rec_f = lib.fd_ed25519_hip_private_hsrec
    rec_f.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_ulong, ctypes.c_int, ctypes.c_void_p]
    q_f = lib.fd_ed25519_hip_private_hssplit
    q_f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_ulong, ctypes.c_ulong]
    q_f.restype = None
    cap = 7
    H, G, KW, CB = (2, 66, 3, 72) if waves == 4 else (4, 33, 2, 32)
    BW = (CB + 31) // 32
    seen_long = False
    for d in (adversarial, halfsize):
        for i in range(min(200, len(d["msg_sz"]))):
            m, s, p = case(d, i)
            rec = np.zeros(32, np.uint32)
            if not rec_f(s, p, m, len(m), 151, rec.ctypes.data):
                continue
            hq = np.zeros((24, cap), np.uint32)
            j = i % cap
            q_f(rec.ctypes.data, waves, hq.ctypes.data, cap, j)
            w = lambda a, k: sum(int(rec[a + t]) << (32 * t) for t in range(k))
            c, dm = w(8, 5), w(13, 5)
            seen_long |= dm >= 2**131
            sp = w(18, 5) % 2**144 + (w(23, 4) << 144)
            part = [sum(int(hq[KW * q + t, j]) << (32 * t) for t in range(KW)) for q in range(waves)]
            chunk = [sum(int(hq[waves * KW + BW * q + t, j]) << (32 * t) for t in range(BW)) for q in range(waves)]
            for side, v in ((0, c), (1, dm)):
                ps = part[side * H:(side + 1) * H]
                assert all(x < 2**G for x in ps[:-1])
                assert sum(x << (G * k) for k, x in enumerate(ps)) == v
            assert all(x < 2**CB for x in chunk)
            assert sum(x << (CB * q) for q, x in enumerate(chunk)) == sp
    assert seen_long
