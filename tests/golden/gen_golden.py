#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run in the build container).

Inputs are the reference's own test data, read as data (never copied as source):
  * src/ballet/ed25519/test_ed25519_wycheproof.c   (133 vectors, accept/reject)
  * src/ballet/ed25519/test_ed25519_cctv.c         (914 vectors, accept/reject)
  * src/ballet/ed25519/test_ed25519_signature_malleability_should_{fail,pass}.bin
  * the sign KAT of src/ballet/ed25519/test_ed25519.c:821-825
  * the point-validate encodings of src/ballet/ed25519/test_ed25519.c:610-651
plus an adversarial set drawn from a seeded PRNG (every invalid class named in
SURVEY.md §8(d) C2) and a batch_single_msg set.

Expected error codes come from the reference itself, compiled from its
sources by `make -C oracle ref` (oracle/_ref/libfdref_{avx512,portable}.so):
"codes_avx512" is the production (AVX-512 IFMA backend) code, "codes_portable"
the fiat-crypto backend code.  The reference tests pin accept/reject only;
these codes pin the exact int returned.

Outputs (all plain data, loadable with numpy.load(allow_pickle=False) / json):
  vectors.npz        wycheproof + cctv + malleability + point-encoding cases
  adversarial.npz    seeded adversarial single-signature set
  batch.npz          seeded batch_single_msg set (txn-grouped)
  sign_kat.json      keygen/sign known answers
"""
import ctypes
import json
import os
import random
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SRC = os.environ.get("FD_REF_SRC", "/root/reference/src")

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493


def load_ref():
    libs = {}
    for flavour in ("avx512", "portable"):
        path = os.path.join(REPO, "oracle", "_ref", f"libfdref_{flavour}.so")
        if not os.path.exists(path):
            sys.exit(f"missing {path}: run `make -C oracle ref` first")
        lib = ctypes.CDLL(path)
        lib.fdref_verify.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p]
        lib.fdref_verify.restype = ctypes.c_int
        lib.fdref_verify_batch_single_msg.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p,
                                                      ctypes.c_char_p, ctypes.c_uint]
        lib.fdref_verify_batch_single_msg.restype = ctypes.c_int
        lib.fdref_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p]
        lib.fdref_public_from_private.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        libs[flavour] = lib
    return libs


def c_bytes(lit):
    """Decode the body of a C string literal made of \\xNN escapes and plain chars."""
    out = bytearray()
    i = 0
    while i < len(lit):
        if lit[i] == "\\" and lit[i + 1] == "x":
            out.append(int(lit[i + 2:i + 4], 16))
            i += 4
        elif lit[i] == "\\":
            esc = {"n": 10, "t": 9, "\\": 92, '"': 34, "0": 0}[lit[i + 1]]
            out.append(esc)
            i += 2
        else:
            out.append(ord(lit[i]))
            i += 1
    return bytes(out)


ENTRY = re.compile(
    r'\{\s*\.tc_id\s*=\s*(\d+),\s*\.comment\s*=\s*"([^"]*)",\s*\.msg\s*=\s*\(uchar const \*\)"([^"]*)",'
    r'\s*\.msg_sz\s*=\s*(\d+)UL,\s*\.sig\s*=\s*"([^"]*)",\s*\.pub\s*=\s*"([^"]*)",\s*\.ok\s*=\s*(\d)\s*\}')


def parse_vectors(path, suite):
    text = open(path).read()
    cases = []
    for m in ENTRY.finditer(text):
        tc, comment, msg, msg_sz, sig, pub, ok = m.groups()
        msg_b = c_bytes(msg)
        assert len(msg_b) == int(msg_sz), (suite, tc)
        cases.append(dict(suite=suite, tc_id=int(tc), comment=comment, msg=msg_b, sig=c_bytes(sig),
                          pub=c_bytes(pub), ok=int(ok)))
    return cases


def enc_le(x):
    return x.to_bytes(32, "little")


class Soa:
    """Accumulates single-signature cases into SoA arrays."""

    def __init__(self):
        self.msgs = bytearray()
        self.off, self.sz, self.sigs, self.pubs, self.tags = [], [], bytearray(), bytearray(), []

    def add(self, msg, sig, pub, tag):
        assert len(sig) == 64 and len(pub) == 32
        self.off.append(len(self.msgs))
        self.sz.append(len(msg))
        self.msgs += msg
        self.sigs += sig
        self.pubs += pub
        self.tags.append(tag)

    def codes(self, lib):
        out = []
        for i in range(len(self.off)):
            m = bytes(self.msgs[self.off[i]:self.off[i] + self.sz[i]])
            out.append(lib.fdref_verify(m, len(m), bytes(self.sigs[64 * i:64 * i + 64]),
                                        bytes(self.pubs[32 * i:32 * i + 32])))
        return np.array(out, dtype=np.int8)

    def arrays(self, libs):
        return dict(msgs=np.frombuffer(bytes(self.msgs), dtype=np.uint8),
                    msg_off=np.array(self.off, dtype=np.uint64), msg_sz=np.array(self.sz, dtype=np.uint32),
                    sigs=np.frombuffer(bytes(self.sigs), dtype=np.uint8).reshape(-1, 64),
                    pubs=np.frombuffer(bytes(self.pubs), dtype=np.uint8).reshape(-1, 32),
                    tags=np.array(self.tags), codes_avx512=self.codes(libs["avx512"]),
                    codes_portable=self.codes(libs["portable"]))


def keypair(lib, rng):
    priv = bytes(rng.getrandbits(8) for _ in range(32))
    pub = ctypes.create_string_buffer(32)
    lib.fdref_public_from_private(pub, priv)
    return priv, pub.raw


def sign(lib, msg, pub, priv):
    sig = ctypes.create_string_buffer(64)
    lib.fdref_sign(sig, msg, len(msg), pub, priv)
    return sig.raw


# Low-order point encodings (fd_curve25519.h:84-92) plus non-canonical ones.
SMALL_ORDER = [
    "0100000000000000000000000000000000000000000000000000000000000000",
    "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "0000000000000000000000000000000000000000000000000000000000000000",
    "0000000000000000000000000000000000000000000000000000000000000080",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc85",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac03fa",
    # non-canonical / sign-bit variants (SURVEY.md §8(c) probe list)
    "0100000000000000000000000000000000000000000000000000000000000080",
    "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff",
    "eeffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "eeffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff",
    "edffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "edffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff",
]
# test_ed25519.c:610-651 point-validate encodings (positive then negative)
POINT_VALIDATE = [
    "0000000000000000000000000000000000000000000000000000000000000000",
    "0100000000000000000000000000000000000000000000000000000000000000",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac03fa",
    "0100000000000000000000000000000000000000000000000000000000000080",
    "eeffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff",
    "edffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff",
    "0300000000000000000000000000000000000000000000000000000000000000",
    "f0ffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "0200000000000000000000000000000000000000000000000000000000000000",
    "b898e00f6f6df758b3f9a05cbf73b15fd392a008a9a417d471c178c1b28c7447",
]


def noncanon_y_encodings():
    """y in [p, 2^255): y' = y - p in [0,18], both sign bits."""
    out = []
    for yv in range(P, 2**255):
        for sgn in (0, 1):
            b = bytearray(enc_le(yv))
            b[31] |= sgn << 7
            out.append(bytes(b))
    return out


def build_vectors(libs):
    soa = Soa()
    ed = os.path.join(REF_SRC, "ballet", "ed25519")
    ok_flags = []
    for suite, fname in (("wycheproof", "test_ed25519_wycheproof.c"), ("cctv", "test_ed25519_cctv.c")):
        for c in parse_vectors(os.path.join(ed, fname), suite):
            soa.add(c["msg"], c["sig"], c["pub"], f'{suite}:{c["tc_id"]}')
            ok_flags.append(c["ok"])
    for name, ok in (("should_fail", 0), ("should_pass", 1)):
        raw = open(os.path.join(ed, f"test_ed25519_signature_malleability_{name}.bin"), "rb").read()
        assert len(raw) % 96 == 0
        for i in range(len(raw) // 96):
            rec = raw[96 * i:96 * i + 96]
            soa.add(b"Zcash", rec[:64], rec[64:], f"malleability_{name}:{i}")
            ok_flags.append(ok)
    # point encodings used as A and as R of an otherwise valid signature
    rng = random.Random(0xED25519)
    lib = libs["avx512"]
    priv, pub = keypair(lib, rng)
    msg = b"point-encoding"
    good = sign(lib, msg, pub, priv)
    encs = POINT_VALIDATE + SMALL_ORDER + [e.hex() for e in noncanon_y_encodings()]
    for e in dict.fromkeys(encs):
        eb = bytes.fromhex(e)
        soa.add(msg, good, eb, f"point_as_A:{e}")
        ok_flags.append(-1)
        soa.add(msg, eb + good[32:], pub, f"point_as_R:{e}")
        ok_flags.append(-1)
        soa.add(msg, eb + good[32:], eb, f"point_as_AR:{e}")
        ok_flags.append(-1)
    arr = soa.arrays(libs)
    arr["ok"] = np.array(ok_flags, dtype=np.int8)
    return arr


def mutate_bit(b, rng):
    b = bytearray(b)
    i = rng.randrange(len(b))
    b[i] ^= 1 << rng.randrange(8)
    return bytes(b)


def undecodable(rng):
    """A random 32-byte string whose y has no x (u/v non-square)."""
    while True:
        e = bytes(rng.getrandbits(8) for _ in range(32))
        y = int.from_bytes(e, "little") & (2**255 - 1)
        y %= P
        u = (y * y - 1) % P
        d = (-121665 * pow(121666, P - 2, P)) % P
        v = (d * y * y + 1) % P
        r = u * pow(v, P - 2, P) % P
        if r and pow(r, (P - 1) // 2, P) != 1:
            return e


def build_adversarial(libs, n_valid=600):
    rng = random.Random(20250117)
    lib = libs["avx512"]
    soa = Soa()
    keys = [keypair(lib, rng) for _ in range(64)]
    sizes = [0, 1, 5, 63, 64, 65, 111, 112, 127, 128, 129, 200, 239, 240, 241, 1000, 1231, 1232]

    def rand_msg():
        sz = rng.choice(sizes) if rng.random() < 0.3 else rng.randrange(64, 1233)
        return bytes(rng.getrandbits(8) for _ in range(sz))

    for i in range(n_valid):
        priv, pub = keys[i % len(keys)]
        m = rand_msg()
        soa.add(m, sign(lib, m, pub, priv), pub, "valid")
    classes = []
    for i in range(400):
        priv, pub = keys[i % len(keys)]
        m = rand_msg()
        s = sign(lib, m, pub, priv)
        S = int.from_bytes(s[32:], "little")
        kind = i % 20
        if kind == 0:   # S + L (non-canonical S)
            soa.add(m, s[:32] + enc_le(S + L), pub, "S_plus_L")
        elif kind == 1:  # S with a high bit set
            soa.add(m, s[:32] + enc_le(S | (1 << (253 + rng.randrange(3)))), pub, "S_highbit")
        elif kind == 2:  # S = L, L-1, L+1, 2^256-1
            v = rng.choice([L - 1, L, L + 1, 2**256 - 1, 0])
            soa.add(m, s[:32] + enc_le(v), pub, f"S_edge")
        elif kind == 3:  # small-order A
            soa.add(m, s, bytes.fromhex(rng.choice(SMALL_ORDER)), "A_small_order")
        elif kind == 4:  # small-order R
            soa.add(m, bytes.fromhex(rng.choice(SMALL_ORDER)) + s[32:], pub, "R_small_order")
        elif kind == 5:  # undecodable A
            soa.add(m, s, undecodable(rng), "A_undecodable")
        elif kind == 6:  # undecodable R
            soa.add(m, undecodable(rng) + s[32:], pub, "R_undecodable")
        elif kind == 7:  # non-canonical y as A
            soa.add(m, s, rng.choice(noncanon_y_encodings()), "A_noncanonical")
        elif kind == 8:  # non-canonical y as R
            soa.add(m, rng.choice(noncanon_y_encodings()) + s[32:], pub, "R_noncanonical")
        elif kind == 9:  # corrupted message
            m2 = mutate_bit(m, rng) if m else b"\x00"
            soa.add(m2, s, pub, "msg_corrupt")
        elif kind == 10:  # corrupted R
            soa.add(m, mutate_bit(s[:32], rng) + s[32:], pub, "R_bitflip")
        elif kind == 11:  # corrupted S (stays < L mostly)
            soa.add(m, s[:32] + mutate_bit(s[32:62], rng) + s[62:], pub, "S_bitflip")
        elif kind == 12:  # corrupted pubkey
            soa.add(m, s, mutate_bit(pub, rng), "A_bitflip")
        elif kind == 13:  # wrong key
            soa.add(m, s, keys[(i + 1) % len(keys)][1], "A_wrong_key")
        elif kind == 14:  # A sign bit flipped (negated A)
            p2 = bytearray(pub); p2[31] ^= 0x80
            soa.add(m, s, bytes(p2), "A_negated")
        elif kind == 15:  # R sign bit flipped
            s2 = bytearray(s); s2[31] ^= 0x80
            soa.add(m, bytes(s2), pub, "R_negated")
        elif kind == 16:  # both undecodable
            soa.add(m, undecodable(rng) + s[32:], undecodable(rng), "AR_undecodable")
        elif kind == 17:  # A undecodable, R small order
            soa.add(m, bytes.fromhex(rng.choice(SMALL_ORDER)) + s[32:], undecodable(rng), "A_undec_R_small")
        elif kind == 18:  # A small order, R undecodable
            soa.add(m, undecodable(rng) + s[32:], bytes.fromhex(rng.choice(SMALL_ORDER)), "A_small_R_undec")
        else:            # random garbage
            soa.add(m, bytes(rng.getrandbits(8) for _ in range(64)),
                    bytes(rng.getrandbits(8) for _ in range(32)), "random")
    return soa.arrays(libs)


def build_batch(libs):
    """batch_single_msg txns (C3): n in {1,2,4,8,12,16} + priority cases + n=0/17."""
    rng = random.Random(1232)
    lib = libs["avx512"]
    keys = [keypair(lib, rng) for _ in range(32)]
    msgs = bytearray()
    txn_msg_off, txn_msg_sz, txn_first, txn_cnt, tags = [], [], [], [], []
    sigs, pubs = bytearray(), bytearray()
    exp = {"avx512": [], "portable": []}
    nsig = 0

    def add_txn(m, sl, pl, tag, cnt=None):
        nonlocal nsig
        cnt = len(sl) if cnt is None else cnt
        txn_msg_off.append(len(msgs)); txn_msg_sz.append(len(m)); msgs.extend(m)
        txn_first.append(nsig); txn_cnt.append(cnt); tags.append(tag)
        for s, p in zip(sl, pl):
            sigs.extend(s); pubs.extend(p); nsig += 1
        for fl in ("avx512", "portable"):
            exp[fl].append(libs[fl].fdref_verify_batch_single_msg(m, len(m), b"".join(sl) or b"\0" * 64,
                                                                  b"".join(pl) or b"\0" * 32, cnt))

    bad_sig_fns = [
        ("S_plus_L", lambda s, p, m: (s[:32] + enc_le(int.from_bytes(s[32:], "little") + L), p)),
        ("A_small", lambda s, p, m: (s, bytes.fromhex(SMALL_ORDER[rng.randrange(len(SMALL_ORDER))]))),
        ("R_small", lambda s, p, m: (bytes.fromhex(SMALL_ORDER[rng.randrange(len(SMALL_ORDER))]) + s[32:], p)),
        ("A_undec", lambda s, p, m: (s, undecodable(rng))),
        ("R_undec", lambda s, p, m: (undecodable(rng) + s[32:], p)),
        ("eq_fail", lambda s, p, m: (s[:32] + mutate_bit(s[32:62], rng) + s[62:], p)),
    ]
    for t in range(240):
        n = [1, 2, 4, 8, 12, 16][t % 6]
        sz = rng.randrange(64, 1233) if t % 3 else rng.randrange(150, 260)
        m = bytes(rng.getrandbits(8) for _ in range(sz))
        ks = [keys[rng.randrange(len(keys))] for _ in range(n)]
        sl = [sign(lib, m, pub, priv) for priv, pub in ks]
        pl = [pub for _, pub in ks]
        kind = t % 5
        tag = "valid"
        if kind >= 2:
            # one or two corrupted sigs; with two, an eq failure at an earlier
            # index and a phase-1 error at a later one exercises the priority rule
            j = rng.randrange(n)
            name, fn = bad_sig_fns[rng.randrange(len(bad_sig_fns))]
            sl[j], pl[j] = fn(sl[j], pl[j], m)
            tag = name
            if kind == 4 and n >= 2:
                j0 = rng.randrange(n - 1)
                j1 = rng.randrange(j0 + 1, n)
                sl[j0], pl[j0] = bad_sig_fns[5][1](sl[j0], pl[j0], m)
                name1, fn1 = bad_sig_fns[rng.randrange(5)]
                sl[j1], pl[j1] = fn1(sl[j1], pl[j1], m)
                tag = f"eq_fail_then_{name1}"
        add_txn(m, sl, pl, tag)
    # invalid batch sizes: the reference returns ERR_SIG without reading inputs
    add_txn(b"x", [], [], "n0", cnt=0)
    priv, pub = keys[0]
    m = b"seventeen"
    add_txn(m, [sign(lib, m, pub, priv)] * 17, [pub] * 17, "n17")
    return dict(msgs=np.frombuffer(bytes(msgs), dtype=np.uint8),
                txn_msg_off=np.array(txn_msg_off, dtype=np.uint64),
                txn_msg_sz=np.array(txn_msg_sz, dtype=np.uint32),
                txn_first=np.array(txn_first, dtype=np.uint32), txn_cnt=np.array(txn_cnt, dtype=np.uint32),
                sigs=np.frombuffer(bytes(sigs), dtype=np.uint8).reshape(-1, 64),
                pubs=np.frombuffer(bytes(pubs), dtype=np.uint8).reshape(-1, 32),
                tags=np.array(tags), codes_avx512=np.array(exp["avx512"], dtype=np.int8),
                codes_portable=np.array(exp["portable"], dtype=np.int8))


def build_sign_kat(libs):
    lib = libs["avx512"]
    kats = [{  # test_ed25519.c:821-825
        "priv": "57835dc6a20e4efd70e90882dbd832b577dbc469960284e0ee718fb526d2ec84",
        "msg": "",
        "sig": "d65759870ce42b34fd955871f0371ce1c9a976edbe98417b84541bb4c68b65a0"
               "673799895c61d530624ffbf92c047d47d4eb4cd1bac2ecee1365faebb53a6303",
    }]
    rng = random.Random(42)
    for i in range(24):
        priv = bytes(rng.getrandbits(8) for _ in range(32))
        msg = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 400)))
        pub = ctypes.create_string_buffer(32)
        lib.fdref_public_from_private(pub, priv)
        kats.append({"priv": priv.hex(), "msg": msg.hex(), "pub": pub.raw.hex(),
                     "sig": sign(lib, msg, pub.raw, priv).hex()})
    for k in kats[:1]:
        pub = ctypes.create_string_buffer(32)
        lib.fdref_public_from_private(pub, bytes.fromhex(k["priv"]))
        k["pub"] = pub.raw.hex()
        assert sign(lib, b"", pub.raw, bytes.fromhex(k["priv"])).hex() == k["sig"], "reference sign KAT failed"
    return kats


def main():
    libs = load_ref()
    vec = build_vectors(libs)
    # the reference's own accept/reject expectations must hold for both backends
    ok = vec["ok"]
    for fl in ("avx512", "portable"):
        got = (vec[f"codes_{fl}"] == 0).astype(np.int8)
        sel = ok >= 0
        assert np.array_equal(got[sel], ok[sel]), f"reference {fl} disagrees with its own vectors"
    np.savez_compressed(os.path.join(HERE, "vectors.npz"), **vec)
    np.savez_compressed(os.path.join(HERE, "adversarial.npz"), **build_adversarial(libs))
    np.savez_compressed(os.path.join(HERE, "batch.npz"), **build_batch(libs))
    with open(os.path.join(HERE, "sign_kat.json"), "w") as f:
        json.dump(build_sign_kat(libs), f, indent=1)
    print("vectors", len(vec["ok"]), "diverging codes",
          int((vec["codes_avx512"] != vec["codes_portable"]).sum()))


if __name__ == "__main__":
    main()
