"""CPU model of the lane-split field and group arithmetic
(firedancer_amd/csrc/fd25519_r16.h, fd_ed25519_dsm16_kernel): every limb
operation restated on Python integers in the device's order, with the
header's bounds asserted at every step -- the 32-bit lanes never wrap, the
64-bit column sums never overflow, every multiplication input stays below
2^19, every subtraction's 4p / 8p offset is above what it subtracts -- and
the results checked against exact arithmetic: products mod p, and the
dsm16 window loop's group element against [c](-A) + [s]B computed by
plain affine Edwards arithmetic.  Worst cases (all limbs at their bound)
are run alongside random ones."""
import random

import pytest

P = 2**255 - 19
D = (-121665 * pow(121666, P - 2, P)) % P
D2 = 2 * D % P
M32, M64 = 2**32, 2**64
B_IN = 2**19            # mul / sq input bound
TIGHT = 2**16 + 64      # mul / sq output bound
P4 = [2**17 - 76] + [2**17 - 2] * 15
P8 = [2**18 - 152] + [2**18 - 4] * 15
assert sum(l << (16 * c) for c, l in enumerate(P4)) == 4 * P
assert sum(l << (16 * c) for c, l in enumerate(P8)) == 8 * P


def val(x):
    return sum(l << (16 * c) for c, l in enumerate(x)) % P


def limbs(v):
    v %= P
    return [(v >> (16 * c)) & 0xffff for c in range(16)]


def ror(x, t):
    """row_ror:t -- lane c gets lane (c - t) mod 16"""
    return [x[(c - t) % 16] for c in range(16)]


def m(t):
    return [38 if c < t else 1 for c in range(16)]


def r16_mul(f, g):
    assert all(0 <= v < B_IN for v in f + g), (max(f), max(g))
    acc = [0] * 16
    for t in range(16):
        rt = ror(f, t)
        for c in range(16):
            assert rt[c] < 2**24                 # v_mul_u32_u24: 24-bit inputs ...
            r = rt[c] * m(t)[c]
            assert r < M32                       # ... and the product's low 32 bits are all of it
            acc[c] += g[t] * r
    assert all(a < M64 for a in acc)
    # round 1: 32-bit lo + (hi rotated) * m1, the product formed in 64 bits, the sum kept in 32
    lo = [a & 0xffff for a in acc]
    hi = [a >> 16 for a in acc]
    assert all(h < M32 for h in hi)
    hr = ror(hi, 1)
    l = [lo[c] + hr[c] * m(1)[c] for c in range(16)]
    assert all(v < M32 for v in l), max(l)
    for _ in range(2):   # rounds 2, 3: 24-bit multiplies
        lo = [v & 0xffff for v in l]
        hi = ror([v >> 16 for v in l], 1)
        assert all(h < 2**24 for h in hi)
        l = [lo[c] + hi[c] * m(1)[c] for c in range(16)]
        assert all(v < M32 for v in l)
    assert all(v < TIGHT for v in l), max(l)
    return l


def sub(x, y, off):
    assert all(o >= v for o, v in zip(off, y)), "offset below the subtrahend: a lane would wrap"
    return [a + o - b for a, o, b in zip(x, off, y)]


def add(x, y):
    return [a + b for a, b in zip(x, y)]


def neg(x, off):
    """off - x (4p or 8p minus x, limb by limb)"""
    assert all(o >= v for o, v in zip(off, x)), "offset below the negated value: a lane would wrap"
    return [o - v for o, v in zip(off, x)]


# ---- points: 4 rows, row q = coordinate q, as fd25519_ge4.h / fd25519_r16.h

def rp(pt, src):
    return [pt[s] for s in src]


def to_qc(p, d2):
    v = rp(p, (1, 0, 3, 2))
    t = r16_mul(v[2], d2)
    return [sub(v[0], p[0], P4), add(v[1], p[1]), t, add(v[3], v[3])]


def cneg(pt, rows, negate, off):
    return [neg(x, off) if (q in rows and negate) else x for q, x in enumerate(pt)]


def ext(pt):
    """(X, Y, Z, T) p3 -> affine (x, y)"""
    X, Y, Z, T = (val(c) for c in pt)
    zi = pow(Z, P - 2, P)
    assert X * Y % P == T * Z % P
    return X * zi % P, Y * zi % P


def edwards_add(a, b):
    (x1, y1), (x2, y2) = a, b
    t = D * x1 * x2 * y1 * y2 % P
    return ((x1 * y2 + x2 * y1) * pow(1 + t, P - 2, P) % P, (y1 * y2 + x1 * x2) * pow(1 - t, P - 2, P) % P)


def edwards_mul(k, pt):
    r, q = (0, 1), pt
    while k:
        if k & 1:
            r = edwards_add(r, q)
        q = edwards_add(q, q)
        k >>= 1
    return r


BY = 4 * pow(5, P - 2, P) % P


def recover_x(y, sign):
    u, v = (y * y - 1) % P, (D * y * y + 1) % P
    x = u * pow(v, 3, P) * pow(u * pow(v, 7, P), (P - 5) // 8, P) % P
    if (v * x * x - u) % P:
        x = x * pow(2, (P - 1) // 4, P) % P
    return P - x if (x & 1) != sign else x


BASE = (recover_x(BY, 0), BY)


def table(x, y, negate, d2):
    xs = neg(x, P4) if negate else x
    xy = r16_mul(xs, y)
    one, zero, two = limbs(1), [0] * 16, limbs(2)
    p0 = [xs, y, one, xy]
    tab = [[one, one, zero, two]]
    c1 = to_qc(p0, d2)
    tab.append(c1)
    cur = p0
    for _ in range(2, 9):
        cur = add2(cur, c1, False, True)
        tab.append(to_qc(cur, d2))
    return tab


def test_mul_exact_and_bounded():
    rng = random.Random(5)
    worst = [B_IN - 1] * 16
    for f, g in [(worst, worst), ([TIGHT - 1] * 16, worst)] + \
                [([rng.randrange(B_IN) for _ in range(16)], [rng.randrange(B_IN) for _ in range(16)]) for _ in range(300)]:
        assert val(r16_mul(f, g)) == val(f) * val(g) % P


# ---- the device's row moves (fd25519_r16.h): gfx950's permlane swaps as
# measured by tools/ubench/permlane_probe.hip, composed with per-row selects

def swap16(x):
    """v_permlane16_swap_b32 with both operands x -> (e, o)"""
    return [x[0], x[0], x[2], x[2]], [x[1], x[1], x[3], x[3]]


def swap32(x):
    """v_permlane32_swap_b32 with both operands x -> (l, h)"""
    return [x[0], x[1], x[0], x[1]], [x[2], x[3], x[2], x[3]]


def bsel(rows, a, b):
    return [a[q] if q in rows else b[q] for q in range(4)]


def test_row_moves_compose_the_quad_permutations():
    x = ["x0", "x1", "x2", "x3"]
    # r16_xor1
    e, o = swap16(x)
    assert bsel((1, 3), e, o) == rp(x, (1, 0, 3, 2))
    # ge16_dbl2's operands from a p3: f row 3 <- X, g row 3 <- Y
    assert bsel((3,), swap32(swap16(x)[0])[0], x) == ["x0", "x1", "x2", "x0"]
    assert bsel((3,), swap32(x)[0], x) == ["x0", "x1", "x2", "x1"]


# ---- prep16's decompression (fd25519_r16.h decode16, a row per point)

def digits(x):
    """r16_digits: the canonical digits from limbs < 2^19, in the device's steps"""
    assert all(0 <= v < B_IN for v in x)
    l, acc = list(x), 0
    for c in range(16):
        acc += l[c]
        l[c], acc = acc & 0xffff, acc >> 16
    for _ in range(2):
        acc = acc * 38 + 19 * (l[15] >> 15)
        l[15] &= 0x7fff
        for c in range(16):
            acc += l[c]
            l[c], acc = acc & 0xffff, acc >> 16
    assert acc == 0
    v = sum(d << (16 * c) for c, d in enumerate(l))
    assert v < 2**255 + 2**6, "the folds leave less than 2^255 + 2^6"
    t, a = [], 19
    for c in range(16):
        a += l[c]
        t.append(a & 0xffff)
        a >>= 16
    if t[15] >> 15:
        t[15] &= 0x7fff
        l = t
    assert sum(d << (16 * c) for c, d in enumerate(l)) == v % P
    return l


SQRTM1 = pow(2, (P - 1) // 4, P)
Y0 = 0x05fc536d880238b13933c6d305acdfd5f098eff289f4c345b027b2c28f95e826
Y1 = 0x7a03ac9277fdc74ec6cc392cfa53202a0f67100d760b3cba4fd84d3d706a17c7


def decode16(enc, avx_rule):
    """decode16's steps on the model's limbs -> (x with its sign applied, fail, small)"""
    y = [(enc >> (16 * c)) & 0xffff for c in range(16)]
    y[15] &= 0x7fff
    sign = enc >> 255
    one = limbs(1)
    u = r16_mul(y, y)
    v = add(r16_mul(u, limbs(D)), one)
    u = sub(u, one, P4)
    v3 = r16_mul(r16_mul(v, v), v)
    x = r16_mul(r16_mul(r16_mul(v3, v3), v), u)
    # the addition chain's value (r16_pow22523 is r16_mul / r16_sq, modelled above)
    x = limbs(pow(val(x), 2**252 - 3, P))
    x = r16_mul(r16_mul(x, v3), u)
    vxx = r16_mul(r16_mul(x, x), v)
    root = not any(digits(sub(vxx, u, P8)))
    iroot = not any(digits(add(vxx, u)))
    xi = r16_mul(x, limbs(SQRTM1))
    xd = digits(x if root else xi)
    x0 = not any(xd)
    xv = sum(d << (16 * c) for c, d in enumerate(xd))
    fail = not (root or iroot) or (avx_rule and x0 and sign == 1)
    xv = (P - xv) % P if (xd[0] & 1) != sign else xv
    yc = sum(d << (16 * c) for c, d in enumerate(digits(y)))
    small = x0 or yc in (0, Y0, Y1)
    return xv, fail, small


def decode_ref(enc, avx_rule):
    """ge_decode's rules (fd25519_dsm.h; fd_ed25519_point_frombytes_2x and
    fd_ed25519_affine_is_small_order) on Python integers"""
    y, sign = enc & (2**255 - 1), enc >> 255
    u, v = (y * y - 1) % P, (D * y * y + 1) % P
    x = u * pow(v, 3, P) * pow(u * pow(v, 7, P), (P - 5) // 8, P) % P
    vxx = v * x * x % P
    root, iroot = vxx == u, vxx == (P - u) % P
    if not root:
        x = x * SQRTM1 % P
    x0 = x == 0
    fail = not (root or iroot) or (avx_rule and x0 and sign == 1)
    if (x & 1) != sign:
        x = (P - x) % P
    return x, fail, x0 or y % P in (0, Y0, Y1)


def test_decode16_matches_ge_decode():
    rng = random.Random(16)
    encs = []
    for _ in range(40):   # points of the group, both signs of x
        x, y = edwards_mul(rng.randrange(1, 2**252), BASE)
        encs.append(y | ((x & 1) << 255))
        encs.append(y | (((x & 1) ^ 1) << 255))
    encs += [rng.randrange(2**256) for _ in range(40)]          # mostly no root
    specials = [0, 1, P - 1, P, P + 1, 2**255 - 1, Y0, Y1, P - Y0 % P, 2**255 - 20, 2**255 - 19]
    encs += specials + [s | (1 << 255) for s in specials]
    for enc in encs:
        for avx_rule in (True, False):
            xv, fail, small = decode16(enc, avx_rule)
            want = decode_ref(enc, avx_rule)
            if want[1]:
                assert fail, hex(enc)          # x is not used when the point fails
                assert small == want[2], hex(enc)
            else:
                assert (xv, fail, small) == want, hex(enc)


# ---- the broadcast-routed group operations (ge16_dbl2 / ge16_add2), with
# the permlane swaps modelled as the probe measured them

def bcast4(x):
    """r16_bcast4: swap16, then swap32 of both halves -> every row of x in every row"""
    e, o = swap16(x)
    (al, ah), (bl, bh) = swap32(e), swap32(o)
    return al, bl, ah, bh


def bsel_rows(rows, a, b):
    return [a[q] if q in rows else b[q] for q in range(4)]


def dbl2(p, lx, want_t):
    f = p if lx else bsel_rows((3,), swap32(swap16(p)[0])[0], p)
    g = bsel_rows((3,), swap32(p)[0], p)
    s = [r16_mul(f[q], g[q]) for q in range(4)]
    assert [b[0] for b in bcast4([0, 1, 2, 3])] == [0, 1, 2, 3]   # which row each broadcast holds
    nh = add(s[0], s[1])
    gg = sub(s[1], s[0], P4)
    e = add(s[3], s[3])
    nf = sub(add(s[2], s[2]), gg, P8)
    a = [e, gg, nf, e]
    b = [nf, nh, gg, nh if want_t else nf]
    assert all(v < B_IN for x in a + b for v in x)
    return [r16_mul(a[q], b[q]) for q in range(4)]


def add2(p, qc, neg, want_t):
    v = rp(p, (1, 0, 3, 2))
    o = [sub(v[0], p[0], P4), add(v[1], p[1]), v[2], v[3]]
    q = [r16_mul(o[i], qc[i]) for i in range(4)]
    r0 = sub(q[0], q[1], P4) if neg else sub(q[1], q[0], P4)
    r1, r2, r3 = add(q[1], q[0]), add(q[3], q[2]), sub(q[3], q[2], P4)
    a = [r0, r1, r2, r0]
    b = [r3, r2, r3, r1 if want_t else r3]
    assert all(x < B_IN for y in a + b for x in y)
    return [r16_mul(a[i], b[i]) for i in range(4)]


def proj(pt):
    """(X, Y, Z, .) -> affine (x, y)"""
    X, Y, Z = (val(c) for c in pt[:3])
    zi = pow(Z, P - 2, P)
    return X * zi % P, Y * zi % P


def test_broadcast_rows():
    x = [["x0"], ["x1"], ["x2"], ["x3"]]
    b = bcast4(x)
    assert [list(r) for r in b] == [[["x0"]] * 4, [["x1"]] * 4, [["x2"]] * 4, [["x3"]] * 4]


def test_dbl2_add2_group_law_and_bounds():
    rng = random.Random(21)
    d2 = limbs(D2)
    for _ in range(6):
        x, y = edwards_mul(rng.randrange(1, 2**64), BASE)
        p3 = [limbs(x), limbs(y), limbs(1), limbs(x * y)]
        q = edwards_mul(rng.randrange(1, 2**64), BASE)
        qc = to_qc([limbs(q[0]), limbs(q[1]), limbs(1), limbs(q[0] * q[1])], d2)
        two = edwards_add((x, y), (x, y))
        r = dbl2(p3, False, True)
        assert ext(r) == two                                     # T consistent: a p3
        l = dbl2(p3, False, False)
        assert proj(l) == two and val(l[3]) == val(l[0])         # (X, Y, Z, X)
        assert ext(dbl2(l, True, True)) == edwards_add(two, two)
        assert ext(add2(p3, qc, False, True)) == edwards_add((x, y), q)
        pn = cneg(p3, (0, 3), True, P4)
        assert ext(add2(pn, qc, True, True)) == edwards_add((x, y), ((P - q[0]) % P, q[1]))
        # limbs at the top of their ranges
        hi = [[TIGHT - 1] * 16 for _ in range(4)]
        dbl2(hi, False, True), dbl2(hi, True, False), add2(hi, qc, False, True)
        add2(cneg(hi, (0, 3), True, P4), qc, True, True)


@pytest.mark.parametrize("seed", [3, 4])
def test_window_loop2_matches_scalar_multiplication(seed):
    """dsm16's loop as the kernel now runs it: per window four doublings
    (p3 in, (X, Y, Z, X) between them, T again before the addition), the
    digit's table addition with the negation folded into it, the base
    addition every 6th window -- against [c](-A) + [s]B"""
    rng = random.Random(seed)
    d2 = limbs(D2)
    A = edwards_mul(rng.randrange(1, 2**250), BASE)
    c = rng.randrange(2**130)
    s = rng.randrange(2**144)
    tab = table(limbs(A[0]), limbs(A[1]), True, d2)
    digs, carry = [], 0
    for i in range(33):
        e = ((c >> (4 * i)) & 15) + carry
        carry = (e + 8) >> 4
        digs.append(e - 16 * carry)
    sdigs = [(s >> (24 * i)) & (2**24 - 1) for i in range(6)]
    pt = [limbs(0), limbs(1), limbs(1), limbs(0)]
    for it in range(32, -1, -1):
        e = digs[it]
        if it != 32:
            pt = dbl2(pt, False, False)
            pt = dbl2(pt, True, False)
            pt = dbl2(pt, True, False)
            pt = dbl2(pt, True, True)
        pt = cneg(pt, (0, 3), e < 0, P4)
        pt = add2(pt, tab[abs(e)], e < 0, True)
        if it % 6 == 0:
            b = edwards_mul(sdigs[it // 6], BASE)
            ypx, ymx, xy2d = (b[1] + b[0]) % P, (b[1] - b[0]) % P, 2 * D * b[0] * b[1] % P
            pt = add2(pt, [limbs(ymx), limbs(ypx), limbs(xy2d), limbs(2)], False, True)
    negA = ((P - A[0]) % P, A[1])
    assert ext(pt) == edwards_add(edwards_mul(c, negA), edwards_mul(s, BASE))
