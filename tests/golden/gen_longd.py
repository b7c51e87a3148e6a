#!/usr/bin/env python3
"""Generate tests/golden/longd.npz (run in the build container): signatures
whose k = SHA-512(R||A||M) mod L gets its half-size pair only with a long d
(2^139 <= |d| < 2^151), so the dsm kernels run 36..38 windows for the wave
holding them (fd25519_half.h, the extended form).  Such k are rare (~1e-5
to ~1e-7 of random k), so they are found by hashing many messages under one
fixed nonce point R = [r]B: S = r + k a mod L is then a valid signature
(ed25519 verification does not care how r was chosen).  Each valid
signature comes with an S-perturbed twin (same k, equation fails).

Selection uses the product's own search compiled for the host
(tests/half_harness.cpp); A, R and the expected codes come from the
reference itself compiled from its sources (oracle/_ref, see gen_golden.py).
Plain data out (numpy.load(allow_pickle=False))."""
import hashlib
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import L, Soa, keypair, load_ref  # noqa: E402
from gen_halfsize import has_half, half_lib  # noqa: E402


def clamp_scalar(priv):
    h = bytearray(hashlib.sha512(priv).digest()[:32])
    h[0] &= 248
    h[31] &= 127
    h[31] |= 64
    return int.from_bytes(h, "little")


def main():
    libs = load_ref()
    ref = libs["avx512"]
    half = half_lib()
    rng = random.Random(0x10D6)
    soa = Soa()
    priv, pub = keypair(ref, rng)
    a = clamp_scalar(priv)
    rpriv, rpt = keypair(ref, rng)      # R = [r]B with r the clamped scalar of rpriv
    r = clamp_scalar(rpriv)
    want = {36: 2, 37: 2, 38: 1}        # windows: bits(|d|) in [4W-4, 4W-1]
    got = {w: 0 for w in want}
    prefix = bytes(rng.getrandbits(8) for _ in range(40))
    trials, budget = 0, 60_000_000
    while trials < budget and any(got[w] < want[w] for w in want):
        trials += 1
        m = prefix + trials.to_bytes(8, "little")
        if has_half(half, rpt, pub, m, 139):
            continue
        w = next((w for w in (36, 37, 38) if has_half(half, rpt, pub, m, 4 * w - 1)), None)
        if w is None or got[w] >= want[w]:
            continue
        k = int.from_bytes(hashlib.sha512(rpt + pub + m).digest(), "little") % L
        s = (r + k * a) % L
        soa.add(m, rpt + s.to_bytes(32, "little"), pub, f"longd_w{w}_valid")
        soa.add(m, rpt + ((s + 1) % L).to_bytes(32, "little"), pub, f"longd_w{w}_bad_s")
        got[w] += 1
        print(f"trial {trials}: W={w}", flush=True)
    arr = soa.arrays(libs)
    np.savez_compressed(os.path.join(HERE, "longd.npz"), **arr)
    print(trials, "trials;", {t: int((arr["tags"] == t).sum()) for t in sorted(set(arr["tags"].tolist()))},
          "codes", sorted(set(arr["codes_avx512"].tolist())))


if __name__ == "__main__":
    main()
