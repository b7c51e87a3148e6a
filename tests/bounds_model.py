"""Interval model of the GPU field and group arithmetic -- test
infrastructure, not product code.

The kernels keep field elements in ten 32-bit limbs (radix 2^25.5) and
never check a bound at run time: every operand of every 32x32->64
multiply-add must fit in int32, every 64-bit column accumulator (every
partial sum) in int64, every 32-bit limb sum in int32.  The argument for
that is written in the headers (firedancer_amd/csrc/fd25519_fe.h,
fd25519_ge.h); this module re-derives it mechanically: each operation is
restated over integer intervals, in the order the device code performs it
(the same operand choices, the same carry chains, the same joins), and
every intermediate is checked against the machine type it lives in.

The group-level functions mirror fd25519_ge.h and the dsm loop of
fd_ed25519_kernels.hip (dsm_half_one / dsm_full_one / table_build), and
the exponentiation chain mirrors fe_pow22523.  Feeding the loop its own
outputs until the intervals stop growing shows the bounds hold for every
iteration, whatever the inputs (tests/test_bounds.py).
"""

W = [26 if k % 2 == 0 else 25 for k in range(10)]
BIAS = [1 << (w - 1) for w in W]
I32 = (-(1 << 31), (1 << 31) - 1)
I64 = (-(1 << 63), (1 << 63) - 1)


class Overflow(AssertionError):
    pass


def _chk(iv, rng, what):
    if iv[0] < rng[0] or iv[1] > rng[1]:
        raise Overflow(f"{what}: [{iv[0]}, {iv[1]}] outside [{rng[0]}, {rng[1]}]")
    return iv


def c32(iv, what="32-bit value"):
    return _chk(iv, I32, what)


def c64(iv, what="64-bit accumulator"):
    return _chk(iv, I64, what)


def add(a, b):
    return (a[0] + b[0], a[1] + b[1])


def neg(a):
    return (-a[1], -a[0])


def mul(a, b):
    p = (a[0] * b[0], a[0] * b[1], a[1] * b[0], a[1] * b[1])
    return (min(p), max(p))


def scale(a, c):
    return mul(a, (c, c))


def shr(a, s):
    return (a[0] >> s, a[1] >> s)   # arithmetic (floor) shift, as on the device


def mask(a, w):
    m = 1 << w
    if a[1] - a[0] >= m:
        return (0, m - 1)
    lo, hi = a[0] % m, a[1] % m
    return (lo, hi) if lo <= hi else (0, m - 1)


def hull(a, b):
    return (min(a[0], b[0]), max(a[1], b[1]))


def point(v):
    return (v, v)


# ---- field elements: lists of 10 intervals ------------------------------

def fe_const(vals):
    return [point(v) for v in vals]


def fe_hull(f, g):
    return [hull(a, b) for a, b in zip(f, g)]


def fe_add(f, g):
    return [c32(add(a, b), "fe_add limb") for a, b in zip(f, g)]


def fe_sub(f, g):
    return [c32(add(a, neg(b)), "fe_sub limb") for a, b in zip(f, g)]


def fe_neg(f):
    return [c32(neg(a), "fe_neg limb") for a in f]


def fe_cneg(f):
    """either f or -f (a run-time sign): the hull of both"""
    return fe_hull(f, fe_neg(f))


def frombytes():
    return [(0, (1 << w) - 1) for w in W]


def centered_tight():
    return [(-(1 << (w - 1)), (1 << (w - 1)) - 1) for w in W]


FE_P_LIMBS = [(1 << 26) - 19] + [(1 << W[k]) - 1 for k in range(1, 10)]


def _mul_terms(f, g, g19, k):
    """fe_mul19's terms of column k in the device's order (i outer)"""
    out = []
    for i in range(10):
        j = (k - i) % 10
        x = scale(f[i], 2) if (i & 1 and j & 1) else f[i]
        y = g19[j] if i + j >= 10 else g[j]
        out.append((c32(x, "mul operand x"), c32(y, "mul operand y (19-side)")))
    return out


def _sq_terms(f, k, s):
    out = []
    for i in range(10):
        for j in range(i, 10):
            if (i + j) % 10 != k:
                continue
            m = (2 if (i & 1 and j & 1) else 1) * (19 if i + j >= 10 else 1)
            x = scale(f[i], s) if i == j else scale(f[i], 2 * s)
            y = scale(f[j], m)
            out.append((c32(x, "sq operand x"), c32(y, "sq operand y")))
    return out


def fe_19(g):
    return [point(0)] + [c32(scale(g[j], 19), "19 g") for j in range(1, 10)]


def _accumulate(start, terms):
    acc = start
    for x, y in terms:
        acc = c64(add(acc, mul(x, y)))
    return acc


def fe_carry_wide(a):
    """fd25519_fe.h fe_carry_wide: pre-biased columns -> centered limbs"""
    a = list(a)
    h = [None] * 10
    m26, m25 = 26, 25

    def step(src, dst, w):
        c = shr(a[src], w)
        a[dst] = c64(add(a[dst], c))
        return c

    step(0, 1, 26); a[0] = mask(a[0], m26)
    step(4, 5, 26); a[4] = mask(a[4], m26)
    step(1, 2, 25); h[1] = c32(add(mask(a[1], m25), point(-(1 << 24))))
    step(5, 6, 25); h[5] = c32(add(mask(a[5], m25), point(-(1 << 24))))
    step(2, 3, 26); h[2] = c32(add(mask(a[2], m26), point(-(1 << 25))))
    step(6, 7, 26); h[6] = c32(add(mask(a[6], m26), point(-(1 << 25))))
    step(3, 4, 25); h[3] = c32(add(mask(a[3], m25), point(-(1 << 24))))
    step(7, 8, 25); h[7] = c32(add(mask(a[7], m25), point(-(1 << 24))))
    c = shr(a[4], 26); h[5] = c32(add(h[5], c32(c, "carry 4->5"))); h[4] = c32(add(mask(a[4], m26), point(-(1 << 25))))
    step(8, 9, 26); h[8] = c32(add(mask(a[8], m26), point(-(1 << 25))))
    c = shr(a[9], 25); a[0] = c64(add(a[0], scale(c, 19))); h[9] = c32(add(mask(a[9], m25), point(-(1 << 24))))
    c = shr(a[0], 26); h[1] = c32(add(h[1], c32(c, "carry 0->1"))); h[0] = c32(add(mask(a[0], m26), point(-(1 << 25))))
    return h


def fe_mul19(f, g, g19):
    a = [_accumulate(point(BIAS[k]), _mul_terms(f, g, g19, k)) for k in range(10)]
    return fe_carry_wide(a)


def fe_mul(f, g):
    return fe_mul19(f, g, fe_19(g))


def fe_sqs(f, s=1):
    a = [_accumulate(point(BIAS[k]), _sq_terms(f, k, s)) for k in range(10)]
    return fe_carry_wide(a)


def fe_carry(f):
    return fe_carry_wide([c64(add(f[i], point(BIAS[i]))) for i in range(10)])


def _join_u(u, c4, c9):
    """fd25519_fe.h fe_join_u"""
    t = c64(add(c4, u[5]))
    u[5] = mask(t, 25)
    u[6] = c32(add(u[6], c32(shr(t, 25), "join: carry into limb 6")))
    t = c64(add(scale(c9, 19), u[0]))
    u[0] = mask(t, 26)
    u[1] = c32(add(u[1], c32(shr(t, 26), "join: carry into limb 1")))
    return u


def _chains_u(terms_of):
    u = [None] * 10
    cA = cB = point(0)
    for s in range(5):
        for half in (0, 1):
            k = s + 5 * half
            acc = _accumulate(cB if half else cA, terms_of(k))
            u[k] = mask(acc, W[k])
            c = shr(acc, W[k])
            if half:
                cB = c
            else:
                cA = c
    return _join_u(u, cA, cB)


def fe_mul19_u(f, g, g19):
    return _chains_u(lambda k: _mul_terms(f, g, g19, k))


def fe_mul_u(f, g):
    return fe_mul19_u(f, g, fe_19(g))


def fe_sqs_u(f, s=1):
    return _chains_u(lambda k: _sq_terms(f, k, s))


def fe_pow22523(z):
    """fd25519_fe.h fe_pow22523 (unsigned forms); returns the output and
    checks every step, the chain's inputs being its own outputs"""
    def sqn(f, n):
        h = fe_sqs_u(f)
        # a squaring of an unsigned output maps into the same interval: a
        # fixed point after one extra step
        for _ in range(min(n - 1, 2)):
            h = fe_hull(h, fe_sqs_u(h))
        return h
    t0 = fe_sqs_u(z)
    t1 = sqn(t0, 2)
    t1 = fe_mul_u(z, t1)
    t0 = fe_mul_u(t0, t1)
    t0 = fe_sqs_u(t0)
    t0 = fe_mul_u(t1, t0)
    t1 = sqn(t0, 5)
    t0 = fe_mul_u(t1, t0)
    t1 = sqn(t0, 10)
    t1 = fe_mul_u(t1, t0)
    t2 = sqn(t1, 20)
    t1 = fe_mul_u(t2, t1)
    t1 = sqn(t1, 10)
    t0 = fe_mul_u(t1, t0)
    t1 = sqn(t0, 50)
    t1 = fe_mul_u(t1, t0)
    t2 = sqn(t1, 100)
    t1 = fe_mul_u(t2, t1)
    t1 = sqn(t1, 50)
    t0 = fe_mul_u(t1, t0)
    t0 = sqn(t0, 2)
    return fe_mul_u(t0, z)


# ---- group operations (fd25519_ge.h) -------------------------------------
# points: dicts of coordinate -> field-element interval

def ge_hull(p, q):
    return {k: fe_hull(p[k], q[k]) for k in p}


def p1p1_to_p2(p):
    x19, z19 = fe_19(p["X"]), fe_19(p["Z"])
    return {"X": fe_mul19_u(p["T"], p["X"], x19),
            "Y": fe_mul19_u(p["Y"], p["Z"], z19),
            "Z": fe_mul19_u(p["T"], p["Z"], z19)}


def p1p1_to_p3(p, uxyt, uz):
    x19, z19 = fe_19(p["X"]), fe_19(p["Z"])
    mu = fe_mul19_u if uxyt else fe_mul19
    r = {"X": mu(p["T"], p["X"], x19), "T": mu(p["Y"], p["X"], x19), "Y": mu(p["Y"], p["Z"], z19)}
    r["Z"] = (fe_mul19_u if uz else fe_mul19)(p["T"], p["Z"], z19)
    return r


def p2_dbl(p):
    xx = fe_sqs(p["X"])
    a = fe_sub(p["X"], p["Y"])
    yy = fe_sqs_u(p["Y"])
    b = fe_sqs_u(p["Z"], 2)
    aa = fe_sqs_u(a)
    rY = fe_add(yy, xx)
    rZ = fe_sub(yy, xx)
    return {"Y": rY, "Z": rZ, "X": fe_sub(rY, aa), "T": fe_sub(b, rZ)}


def p3_to_cached(p, uxy):
    d2 = centered_tight()   # FE_D2: a centered constant
    if uxy:
        ypx = [c32(add(add(p["Y"][i], p["X"][i]), point(-FE_P_LIMBS[i]))) for i in range(10)]
    else:
        ypx = fe_add(p["Y"], p["X"])
    return {"YplusX": ypx, "YminusX": fe_sub(p["Y"], p["X"]), "Z2": fe_add(p["Z"], p["Z"]),
            "T2d": fe_mul_u(p["T"], d2)}


def cached_cneg(c):
    """the run-time digit sign: Y+X / Y-X swapped, 2dT negated"""
    sw = fe_hull(c["YplusX"], c["YminusX"])
    return {"YplusX": sw, "YminusX": sw, "Z2": c["Z2"], "T2d": fe_cneg(c["T2d"])}


def ge_add(p, q, nt):
    a = fe_mul_u(fe_add(p["Y"], p["X"]), q["YplusX"])
    b = fe_mul_u(fe_sub(p["Y"], p["X"]), q["YminusX"])
    zz2 = fe_mul_u(p["Z"], q["Z2"])
    c = (fe_mul_u if nt else fe_mul)(q["T2d"], p["T"])
    r = {"X": fe_sub(a, b), "Y": fe_add(a, b)}
    if nt:
        r["Z"], r["T"] = fe_sub(zz2, c), fe_add(zz2, c)
    else:
        r["Z"], r["T"] = fe_add(zz2, c), fe_sub(zz2, c)
    return r


def ge_madd(p, q):
    a = fe_mul_u(fe_add(p["Y"], p["X"]), q["yplusx"])
    b = fe_mul_u(fe_sub(p["Y"], p["X"]), q["yminusx"])
    c = fe_mul(q["xy2d"], p["T"])
    t0 = fe_add(p["Z"], p["Z"])
    return {"X": fe_sub(a, b), "Y": fe_add(a, b), "Z": fe_add(t0, c), "T": fe_sub(t0, c)}


def precomp_cneg(b):
    sw = fe_hull(b["yplusx"], b["yminusx"])
    return {"yplusx": sw, "yminusx": sw, "xy2d": fe_cneg(b["xy2d"])}


def identity_p3():
    return {"X": fe_const([0] * 10), "Y": fe_const([1] + [0] * 9), "Z": fe_const([1] + [0] * 9),
            "T": fe_const([0] * 10)}


def decoded_x():
    """decode's x: a centered product (fe_mul), either sign"""
    ctr = fe_mul(centered_tight(), centered_tight())
    return fe_cneg(ctr)


def table_entries(nt):
    """table_build<NT>: the hull of the 9 entries of [0..8](+-P), P = (x, y)
    affine from decode, after the digit sign (cneg) at load"""
    x, y = decoded_x(), frombytes()
    x = fe_cneg(x)                          # negate flag
    P0 = {"X": x, "Y": y, "Z": fe_const([1] + [0] * 9), "T": fe_mul(x, y)}
    ident = {"YplusX": fe_const([1] + [0] * 9), "YminusX": fe_const([1] + [0] * 9),
             "Z2": fe_const([2] + [0] * 9), "T2d": fe_const([0] * 10)}
    c1 = p3_to_cached(P0, False)
    pre = {"yplusx": c1["YplusX"], "yminusx": c1["YminusX"], "xy2d": c1["T2d"]}

    def stored(c):
        return dict(c, T2d=fe_neg(c["T2d"])) if nt else c
    tab = ge_hull_c(ident, stored(c1))
    cur = P0
    for _ in range(2, 9):
        s = ge_madd(cur, pre)
        cur = p1p1_to_p3(s, True, False)
        tab = ge_hull_c(tab, stored(p3_to_cached(cur, True)))
    return cached_cneg(tab)


def ge_hull_c(a, b):
    return {k: fe_hull(a[k], b[k]) for k in a}


def base_entry():
    """wide base table entries: (y+x, y-x) carried, 2dxy a centered product;
    either digit sign"""
    ctr = fe_carry(fe_add(centered_tight(), centered_tight()))
    return precomp_cneg({"yplusx": ctr, "yminusx": ctr,
                         "xy2d": fe_mul(centered_tight(), centered_tight())})


def dsm_half_loop(max_iter=6):
    """dsm_half_one's loop body, fed its own outputs until the intervals stop
    growing; returns the fixed point of Q (the p2 carried between
    iterations) and P"""
    tabA, tabR, bt = table_entries(True), table_entries(True), base_entry()
    P = identity_p3()
    Q = None
    for it in range(max_iter):
        if Q is not None:
            Rt = p2_dbl(Q)
            for _ in range(3):
                Rt = p2_dbl(p1p1_to_p2(Rt))
            P = p1p1_to_p3(Rt, True, True)
        Rt = ge_add(P, tabA, True)
        P = p1p1_to_p3(Rt, True, True)
        Rt = ge_add(P, tabR, True)
        # with and without the base additions (windows 30, 25, .., 0)
        P2 = p1p1_to_p3(Rt, True, False)
        Rb = ge_madd(P2, bt)
        Rb = ge_madd(p1p1_to_p3(Rb, True, False), bt)
        Rt = {k: fe_hull(Rt[k], Rb[k]) for k in Rt}
        Qn = p1p1_to_p2(Rt)
        if Q is not None and Qn == Q:
            return Q, it
        Q = Qn if Q is None else {k: fe_hull(Q[k], Qn[k]) for k in Q}
    return Q, max_iter


def dsm_full_loop(max_iter=6):
    """dsm_full_one's loop: table_build<false>, general additions followed by
    the p2 / uxyt conversions"""
    tabA, bt = table_entries(False), base_entry()
    P = identity_p3()
    Q = None
    for it in range(max_iter):
        if Q is not None:
            Rt = p2_dbl(Q)
            for _ in range(3):
                Rt = p2_dbl(p1p1_to_p2(Rt))
            P = p1p1_to_p3(Rt, True, True)
        Rt = ge_add(P, tabA, False)
        Rb = ge_madd(p1p1_to_p3(Rt, True, False), bt)
        Rt = {k: fe_hull(Rt[k], Rb[k]) for k in Rt}
        Qn = p1p1_to_p2(Rt)
        if Q is not None and Qn == Q:
            return Q, it
        Q = Qn if Q is None else {k: fe_hull(Q[k], Qn[k]) for k in Q}
    return Q, max_iter
