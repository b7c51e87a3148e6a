#!/usr/bin/env python3
"""Generate tests/golden/halfsize.npz (run in the build container): signatures
whose k = SHA-512(R||A||M) mod L has no half-size pair (fd25519_half.h), so
the verify kernel takes its full-length form for them, in every outcome
class: valid, equation failure, S >= L, small-order A / R, undecodable R.

Selection uses the product's own search compiled for the host
(tests/half_harness.cpp); signing and the expected codes come from the
reference itself compiled from its sources (oracle/_ref, see gen_golden.py).
Plain data out (numpy.load(allow_pickle=False))."""
import ctypes
import hashlib
import os
import random
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gen_golden import L, SMALL_ORDER, Soa, keypair, load_ref, sign, undecodable  # noqa: E402


def half_lib():
    out = os.path.join(tempfile.mkdtemp(), "half.so")
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-I",
                           os.path.join(REPO, "firedancer_amd", "csrc"),
                           os.path.join(REPO, "tests", "half_harness.cpp"), "-o", out])
    lib = ctypes.CDLL(out)
    lib.half_scalars.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int]
    lib.half_scalars.restype = ctypes.c_int
    return lib


def has_half(lib, r, a, m, dbits=131):
    """a pair with |d| < 2^dbits (131: the strict half-size form)"""
    k = int.from_bytes(hashlib.sha512(r + a + m).digest(), "little") % L
    kb = (ctypes.c_uint32 * 8)(*[(k >> (32 * i)) & 0xffffffff for i in range(8)])
    c, d, neg = (ctypes.c_uint32 * 5)(), (ctypes.c_uint32 * 5)(), ctypes.c_int()
    return lib.half_scalars(ctypes.addressof(kb), ctypes.addressof(c), ctypes.addressof(d), ctypes.addressof(neg),
                            dbits)


def main():
    libs = load_ref()
    ref = libs["avx512"]
    half = half_lib()
    rng = random.Random(0x4a1f)
    soa = Soa()

    def rand_msg():
        return bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 300)))

    # valid signatures with a full-length k, and their S-perturbed twins
    # (same k, equation fails), and S + L (rejected before the equation)
    n_valid = 0
    while n_valid < 48:
        priv, pub = keypair(ref, rng)
        for _ in range(64):
            m = rand_msg()
            sig = sign(ref, m, pub, priv)
            if has_half(half, sig[:32], pub, m):
                continue
            soa.add(m, sig, pub, "full_valid")
            s = int.from_bytes(sig[32:], "little")
            soa.add(m, sig[:32] + ((s + 1 + rng.randrange(1000)) % L).to_bytes(32, "little"), pub, "full_bad_s")
            if s + L < 2**256:
                soa.add(m, sig[:32] + (s + L).to_bytes(32, "little"), pub, "full_s_plus_l")
            n_valid += 1
            break

    # small-order A, small-order R, undecodable R with a full-length k
    def search(tag, make, count):
        got = 0
        while got < count:
            m, sig, pub = make()
            if not has_half(half, sig[:32], pub, m):
                soa.add(m, sig, pub, tag)
                got += 1

    def small_a():
        priv, _ = keypair(ref, rng)
        pub = bytes.fromhex(rng.choice(SMALL_ORDER))
        m = rand_msg()
        return m, sign(ref, m, pub, priv), pub

    def small_r():
        priv, pub = keypair(ref, rng)
        m = rand_msg()
        sig = sign(ref, m, pub, priv)
        return m, bytes.fromhex(rng.choice(SMALL_ORDER)) + sig[32:], pub

    def bad_r():
        priv, pub = keypair(ref, rng)
        m = rand_msg()
        sig = sign(ref, m, pub, priv)
        return m, undecodable(rng) + sig[32:], pub

    search("full_small_a", small_a, 16)
    search("full_small_r", small_r, 16)
    search("full_bad_r", bad_r, 16)

    arr = soa.arrays(libs)
    np.savez_compressed(os.path.join(HERE, "halfsize.npz"), **arr)
    print({t: int((arr["tags"] == t).sum()) for t in sorted(set(arr["tags"].tolist()))},
          "codes", sorted(set(arr["codes_avx512"].tolist())))


if __name__ == "__main__":
    main()
