"""The integer re-check of every half-size pair (fd_ed25519_kernels.hip
half_pair_ok: c == d k mod 8L, d odd, bounds) is what keeps the verdicts
exact, not the floating-point-assisted Euclid that finds the pair
(VERDICT r1, weak #1).  The fault-injection build
(libfd_ed25519_hip_faultinj.so, -DFD_ED25519_HALF_FAULT=1) flips a bit of c
for 1/8 of the signatures and a bit of |d| for another 1/8 after the
search: the check must reject exactly those pairs (the device diagnostic
reports ok = 0 for ~1/4 of random k, and every pair it still reports
satisfies the invariant), and every verdict must stay bit-identical to the
reference's codes, because the rejected items take the full-length form.
Run in a child process, since the library is chosen at import."""
import os
import random
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO, oracle_many
from test_gpu_parity import _random_set
from test_half import L, N8L

pytestmark = pytest.mark.gpu

FAULT_LIB = os.path.join(REPO, "firedancer_amd", "_lib", "libfd_ed25519_hip_faultinj.so")


def _words(k):
    return [(k >> (32 * i)) & 0xffffffff for i in range(8)]


def test_half_check_under_fault_injection(tmp_path, oracle, vectors, adversarial, halfsize, longd):
    if not os.path.exists(FAULT_LIB):
        pytest.fail(f"{FAULT_LIB} not built (make -C firedancer_amd/csrc)")
    rnd = _random_set(oracle, 3000, seed=31)
    sets = {"vectors": vectors, "adversarial": adversarial, "halfsize": halfsize, "longd": longd, "random": rnd}
    want = {nm: {"avx512": d["codes_avx512"], "portable": d["codes_portable"]}
            for nm, d in sets.items() if nm != "random"}
    want["random"] = {"avx512": oracle_many(oracle, rnd, 0), "portable": oracle_many(oracle, rnd, 1)}
    blob = {}
    for nm, d in sets.items():
        for f in ("msgs", "msg_off", "msg_sz", "sigs", "pubs"):
            blob[f"{nm}/{f}"] = np.ascontiguousarray(d[f])
    rng = random.Random(5)
    ks = [rng.randrange(L) for _ in range(4000)]
    blob["k_words"] = np.array([_words(k) for k in ks], np.uint32)
    src, dst = str(tmp_path / "in.npz"), str(tmp_path / "out.npz")
    np.savez(src, **blob)
    env = dict(os.environ, FD_ED25519_HIP_LIB=FAULT_LIB)
    r = subprocess.run([sys.executable, "-u", os.path.join(REPO, "tests", "faultinj_child.py"), src, dst], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    got = dict(np.load(dst, allow_pickle=False))

    # the check rejects the injected pairs: ~1/4 of random k
    diag = got["diag"]
    ok = diag[:, 0] == 1
    frac_rejected = 1.0 - ok.mean()
    assert 0.18 < frac_rejected < 0.32, frac_rejected
    for i in np.nonzero(ok)[0][:1500]:
        o = diag[i]
        c = sum(int(o[2 + w]) << (32 * w) for w in range(5))
        d = sum(int(o[7 + w]) << (32 * w) for w in range(5))
        d = -d if o[1] else d
        assert (c - d * ks[i]) % N8L == 0 and d % 2 and 0 <= c < 2**131 and abs(d) < 2**151, hex(ks[i])

    # ... and every verdict is still the reference's
    for key, codes in got.items():
        if key == "diag":
            continue
        nm, dsm, flavour = key.split("/")
        w = want[nm][flavour]
        bad = np.nonzero(codes != w)[0]
        assert len(bad) == 0, (key, [(int(i), int(codes[i]), int(w[i])) for i in bad[:8]])
