#!/usr/bin/env python3
"""Generate tests/golden/mixed_order.npz (run in the build container): public
keys A and nonces R that carry a torsion component, so they pass the
reference's decode and small-order checks and their verdict depends on how
that component cancels in the cofactorless equation.

Why this class matters: `fd_ed25519_affine_is_small_order`
(src/ballet/ed25519/fd_curve25519.h:81-111) rejects only the eight *pure*
small-order points, so A = [a]B + T_A and R = [r]B + T_R with T_A, T_R in the
8-torsion decode fine.  The reference's equation (fd_ed25519_user.c:215-224)
is cofactorless: it computes R' = [S]B - [k]A = [r]B - [k]T_A and accepts iff
R' == R, i.e. iff T_R == -[k mod ord(T_A)] T_A, where k = SHA-512(R||A||M)
mod L.  The engine's half-size equation is right on such points only because
its (c, d) pair satisfies c = d*k mod 8L with d odd, so this
set is the at-scale check of that claim.

Construction (plain Python big-int Edwards arithmetic; test infrastructure):
  * T8 = the order-8 point c7176a70...ac037a (fd_curve25519.h:84-92 list),
    T_A = [jA]T8, T_R = [jR]T8 with jA, jR in 0..7 (orders 1, 2, 4, 8);
  * a = clamp(SHA-512(privA)[0:32]), [a]B = the reference's
    fd_ed25519_public_from_private(privA) (likewise r and [r]B from a second
    seed), A = [a]B + T_A, R = [r]B + T_R;
  * S = r + k a mod L (so [S]B - [k]A = [r]B - [k]T_A exactly);
  * messages re-drawn until k mod 8 puts the case in its class.
Classes (tags): TA_cancel (T_R = 0, [k]T_A = 0: accepted), TA_noncancel,
TR_only (T_A = 0: always rejected), TATR_cancel (T_R = -[k]T_A != 0:
accepted), TATR_noncancel, TATR_plus (T_R = +[k]T_A != -[k]T_A: a sign slip
would accept it), and TATR_cancel_* (a cancelling case then made invalid:
S + L, a flipped message bit, A or R negated by its sign bit).  A
batch_single_msg set (txns of 1..12 such signatures over one message each)
goes with it.

Expected codes come from the reference compiled from its sources
(oracle/_ref/libfdref_{avx512,portable}.so), as in gen_golden.py.  Messages
are a case counter repeated to the drawn size, so the fixture compresses.
"""
import hashlib
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import L, P, Soa, enc_le, load_ref  # noqa: E402

D = (-121665 * pow(121666, P - 2, P)) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)
IDENT = (0, 1)
T8_ENC = "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a"
B_ENC = "5866666666666666666666666666666666666666666666666666666666666666"


def add(p, q):
    (x1, y1), (x2, y2) = p, q
    t = D * x1 * x2 * y1 * y2 % P
    x3 = (x1 * y2 + y1 * x2) * pow(1 + t, P - 2, P) % P
    y3 = (y1 * y2 + x1 * x2) * pow(1 - t, P - 2, P) % P
    return x3, y3


def neg(p):
    return (-p[0]) % P, p[1]


def mul(k, p):
    acc = IDENT
    while k:
        if k & 1:
            acc = add(acc, p)
        p = add(p, p)
        k >>= 1
    return acc


def decode(b):
    v = int.from_bytes(b, "little")
    y, sign = v & (2**255 - 1), v >> 255
    assert y < P
    u, w = (y * y - 1) % P, (D * y * y + 1) % P
    x = u * pow(w, 3, P) * pow(u * pow(w, 7, P), (P - 5) // 8, P) % P
    if w * x * x % P != u:
        x = x * SQRT_M1 % P
    assert w * x * x % P == u, "not on the curve"
    if (x & 1) != sign:
        x = (-x) % P
    assert not (x == 0 and sign), "x = 0 with the sign bit"
    return x, y


def encode(p):
    x, y = p
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


def clamp(h32):
    a = bytearray(h32)
    a[0] &= 248
    a[31] &= 127
    a[31] |= 64
    return int.from_bytes(a, "little")


class Gen:
    def __init__(self, libs, seed):
        self.ref = libs["avx512"]
        self.rng = random.Random(seed)
        self.T8 = decode(bytes.fromhex(T8_ENC))
        self.T = [mul(j, self.T8) for j in range(8)]
        assert self.T[0] == IDENT and mul(8, self.T8) == IDENT and self.T[4] != IDENT
        assert len({encode(t) for t in self.T}) == 8
        self.B = decode(bytes.fromhex(B_ENC))
        self.ctr = 0

    def scalar_point(self):
        """(s, [s]B) with [s]B from the reference's own keygen."""
        import ctypes
        priv = bytes(self.rng.getrandbits(8) for _ in range(32))
        pub = ctypes.create_string_buffer(32)
        self.ref.fdref_public_from_private(pub, priv)
        return clamp(hashlib.sha512(priv).digest()[:32]), decode(pub.raw)

    def msg(self):
        self.ctr += 1
        sz = self.rng.choice([0, 1, 31, 32, 64, 111, 112, 128, 200, 239, 240, 1232]) if self.rng.random() < 0.2 \
            else self.rng.randrange(1, 400)
        head = b"mixed-order %010d|" % self.ctr
        return (head * (sz // len(head) + 1))[:sz]

    def case(self, jA, jR, want, m=None):
        """A, R carrying [jA]T8, [jR]T8; draw messages (or, with m fixed,
        nonces) until want(k mod 8) holds.  Returns (msg, sig, pub, k)."""
        a, aB = self.scalar_point()
        A = add(aB, self.T[jA])
        Aenc = encode(A)
        while True:
            r, rB = self.scalar_point()
            Renc = encode(add(rB, self.T[jR]))
            for _ in range(64 if m is None else 1):
                mm = self.msg() if m is None else m
                k = int.from_bytes(hashlib.sha512(Renc + Aenc + mm).digest(), "little") % L
                if want(k):
                    S = (r + k * a) % L
                    return mm, Renc + enc_le(S), Aenc, k


def cancels(jA, jR, k):
    return (jR + k * jA) % 8 == 0


def build_single(g, n):
    soa = Soa()
    rng = g.rng
    quota = [("TA_cancel", 0.15), ("TA_noncancel", 0.15), ("TR_only", 0.12), ("TATR_cancel", 0.22),
             ("TATR_noncancel", 0.14), ("TATR_plus", 0.10), ("TATR_cancel_S_plus_L", 0.03),
             ("TATR_cancel_msg_flip", 0.03), ("TATR_cancel_A_negated", 0.03), ("TATR_cancel_R_negated", 0.03)]
    tags = []
    for name, frac in quota:
        tags += [name] * int(round(frac * n))
    tags = (tags + ["TATR_cancel"] * n)[:n]
    rng.shuffle(tags)
    for tag in tags:
        jA = rng.randrange(1, 8)
        if tag == "TA_cancel":
            m, s, p, _ = g.case(jA, 0, lambda k: cancels(jA, 0, k))
        elif tag == "TA_noncancel":
            m, s, p, _ = g.case(jA, 0, lambda k: not cancels(jA, 0, k))
        elif tag == "TR_only":
            m, s, p, _ = g.case(0, rng.randrange(1, 8), lambda k: True)
        elif tag == "TATR_noncancel":
            jR = rng.randrange(1, 8)
            m, s, p, _ = g.case(jA, jR, lambda k: not cancels(jA, jR, k))
        elif tag == "TATR_plus":
            # T_R = +[k]T_A != -[k]T_A needs T_R of order > 2, reachable as k*jA
            jA = rng.choice([1, 2, 3, 5, 6, 7])
            jR = rng.choice(sorted({(k * jA) % 8 for k in range(8)} - {0, 4}))
            m, s, p, _ = g.case(jA, jR, lambda k: (jR - k * jA) % 8 == 0 and not cancels(jA, jR, k))
        else:
            # a cancelling pair: jR must be reachable as -k*jA mod 8
            reach = sorted({(-k * jA) % 8 for k in range(8)} - {0})
            jR = rng.choice(reach)
            m, s, p, _ = g.case(jA, jR, lambda k: cancels(jA, jR, k))
            if tag == "TATR_cancel_S_plus_L":
                s = s[:32] + enc_le(int.from_bytes(s[32:], "little") + L)
            elif tag == "TATR_cancel_msg_flip":
                m = bytes(m[:-1]) + bytes([m[-1] ^ 1]) if m else b"\x01"
            elif tag == "TATR_cancel_A_negated":
                p = p[:31] + bytes([p[31] ^ 0x80])
            elif tag == "TATR_cancel_R_negated":
                s = s[:31] + bytes([s[31] ^ 0x80]) + s[32:]
        soa.add(m, s, p, tag)
    return soa


def build_batch(g, libs, n_txn):
    """batch_single_msg transactions of 1..12 mixed-order signatures over one
    message: all cancelling (accepted), or one / two members that do not."""
    rng = g.rng
    msgs = bytearray()
    txn_msg_off, txn_msg_sz, txn_first, txn_cnt, tags = [], [], [], [], []
    sigs, pubs = bytearray(), bytearray()
    exp = {"avx512": [], "portable": []}
    for t in range(n_txn):
        n = rng.randrange(1, 13)
        m = g.msg()
        bad = set() if t % 3 == 0 else set(rng.sample(range(n), min(n, 1 + (t % 3 == 2))))
        sl, pl = [], []
        for j in range(n):
            jA = rng.randrange(0, 8)
            reach = sorted({(-k * jA) % 8 for k in range(8)})
            if j in bad:
                jR = rng.randrange(1, 8) if jA == 0 else rng.randrange(0, 8)
                _, s, p, _ = g.case(jA, jR, lambda k: not cancels(jA, jR, k), m=m)
            else:
                jR = rng.choice(reach)
                _, s, p, _ = g.case(jA, jR, lambda k: cancels(jA, jR, k), m=m)
            sl.append(s)
            pl.append(p)
        txn_msg_off.append(len(msgs)); txn_msg_sz.append(len(m)); msgs.extend(m)
        txn_first.append(len(sigs) // 64); txn_cnt.append(n)
        tags.append("all_cancel" if not bad else f"noncancel_at_{sorted(bad)}")
        for s, p in zip(sl, pl):
            sigs.extend(s); pubs.extend(p)
        for fl in ("avx512", "portable"):
            exp[fl].append(libs[fl].fdref_verify_batch_single_msg(m, len(m), b"".join(sl), b"".join(pl), n))
    return dict(b_msgs=np.frombuffer(bytes(msgs) or b"\0", dtype=np.uint8),
                b_txn_msg_off=np.array(txn_msg_off, dtype=np.uint64),
                b_txn_msg_sz=np.array(txn_msg_sz, dtype=np.uint32),
                b_txn_first=np.array(txn_first, dtype=np.uint32), b_txn_cnt=np.array(txn_cnt, dtype=np.uint32),
                b_sigs=np.frombuffer(bytes(sigs), dtype=np.uint8).reshape(-1, 64),
                b_pubs=np.frombuffer(bytes(pubs), dtype=np.uint8).reshape(-1, 32),
                b_tags=np.array(tags), b_codes_avx512=np.array(exp["avx512"], dtype=np.int8),
                b_codes_portable=np.array(exp["portable"], dtype=np.int8))


def main(n=10240, n_txn=600):
    libs = load_ref()
    g = Gen(libs, 0x70851)
    # the reference's keygen is the scalar multiplication used throughout: pin it
    for _ in range(3):
        s, sB = g.scalar_point()
        assert mul(s, g.B) == sB
    soa = build_single(g, n)
    out = soa.arrays(libs)
    out.update(build_batch(g, libs, n_txn))
    tags, codes = out["tags"], out["codes_avx512"]
    acc = int((codes == 0).sum())
    for t in sorted(set(tags.tolist())):
        sel = tags == t
        want_ok = t in ("TA_cancel", "TATR_cancel")
        assert ((codes[sel] == 0) == want_ok).all(), (t, np.unique(codes[sel], return_counts=True))
    assert acc >= 1000, acc
    np.savez_compressed(os.path.join(HERE, "mixed_order.npz"), **out)
    print("single", n, "accepted", acc, "codes", dict(zip(*[x.tolist() for x in np.unique(codes, return_counts=True)])),
          "| txns", n_txn, "accepted", int((out["b_codes_avx512"] == 0).sum()),
          "| avx512 != portable", int((out["codes_avx512"] != out["codes_portable"]).sum()))


if __name__ == "__main__":
    main()
