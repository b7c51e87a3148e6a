"""C3: multi-signer transactions through
fd_ed25519_verify_batch_single_msg semantics on the GPU -- n in {1,2,4,8,12}
signers over one ~200-byte message, with the priority cases: a later
signature's phase-1 error (bad S, small-order or undecodable key or R) must
win over signature 0's equation failure.  Per-transaction codes are compared
with the reference's own batch_single_msg (oracle/_ref), and per-signature
codes with its fd_ed25519_verify."""
import ctypes
import random

import numpy as np
import pytest

from txn_util import Signer, ref_lib

pytestmark = pytest.mark.gpu

L = 2**252 + 27742317777372353535851937790883648493
UNDECODABLE = bytes([2]) + bytes(31)     # y = 2: no square root
SMALL_ORDER = bytes(32)                  # y = 0: order 4
IDENTITY = bytes([1]) + bytes(31)        # order 1


def _bump_s(sig, k):
    s = int.from_bytes(sig[32:], "little") + k
    return sig[:32] + (s % 2**256).to_bytes(32, "little")


def _phase1(rng, sig, pub):
    kind = rng.randrange(5)
    if kind == 0:
        return _bump_s(sig, L), pub          # S >= L
    if kind == 1:
        return sig, SMALL_ORDER              # small-order A
    if kind == 2:
        return sig, UNDECODABLE              # undecodable A
    if kind == 3:
        return IDENTITY + sig[32:], pub      # small-order R
    return UNDECODABLE + sig[32:], pub       # undecodable R


def make_txns(oracle, seed, ntxn):
    rng = random.Random(seed)
    signer = Signer(oracle, seed)
    msgs, t_off, t_sz, first, cnt, sigs, pubs = bytearray(), [], [], [], [], [], []
    for t in range(ntxn):
        n = rng.choice([1, 2, 4, 8, 12])
        m = bytes(rng.getrandbits(8) for _ in range(200 + rng.randrange(-8, 9)))
        keys = [signer.key() for _ in range(n)]
        ss = [signer.sign(m, priv, pub) for priv, pub in keys]
        ps = [pub for _, pub in keys]
        cls = rng.random()
        if cls < 0.15 and n > 1:   # priority: sig j>0 phase-1 error, sig 0 equation failure
            j = rng.randrange(1, n)
            ss[j], ps[j] = _phase1(rng, ss[j], ps[j])
            ss[0] = _bump_s(ss[0], 1)
        elif cls < 0.25:           # one phase-1 error anywhere
            j = rng.randrange(n)
            ss[j], ps[j] = _phase1(rng, ss[j], ps[j])
        elif cls < 0.35:           # one equation failure
            ss[rng.randrange(n)] = _bump_s(ss[rng.randrange(n)], 1) if n == 1 else _bump_s(ss[0], 3)
        elif cls < 0.40 and n > 2:  # two different phase-1 errors: the first in signature order wins
            a, b = sorted(rng.sample(range(n), 2))
            ss[a], ps[a] = _phase1(rng, ss[a], ps[a])
            ss[b], ps[b] = _phase1(rng, ss[b], ps[b])
        t_off.append(len(msgs)); t_sz.append(len(m)); msgs += m
        first.append(len(sigs)); cnt.append(n)
        sigs += ss; pubs += ps
    return (np.frombuffer(bytes(msgs), np.uint8), np.array(t_off, np.uint64), np.array(t_sz, np.uint32),
            np.array(first, np.uint32), np.array(cnt, np.uint32), np.frombuffer(b"".join(sigs), np.uint8),
            np.frombuffer(b"".join(pubs), np.uint8))


@pytest.mark.parametrize("codes", ["avx512", "portable"])
def test_c3_batch_single_msg_priority(oracle, codes):
    from firedancer_amd import ed25519
    ref = ref_lib(codes)
    if ref is None:
        pytest.skip(f"oracle/_ref {codes} build not available on this host")
    ref.fdref_verify_batch_single_msg.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p,
                                                  ctypes.c_uint]
    ref.fdref_verify.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p]
    msgs, t_off, t_sz, first, cnt, sigs, pubs = make_txns(oracle, 33, 1500)
    eng = ed25519.Engine(0, max_chunk=1 << 12, codes=codes)
    got_txn, got_sig = eng.verify_txns_host(msgs, t_off, t_sz, first, cnt, sigs, pubs, want_sig_codes=True)
    eng.close()
    want_txn = np.zeros(len(cnt), np.int8)
    want_sig = np.zeros(int(cnt.sum()), np.int8)
    for t in range(len(cnt)):
        m = bytes(msgs[t_off[t]:t_off[t] + t_sz[t]])
        f, n = int(first[t]), int(cnt[t])
        ss, ps = bytes(sigs[64 * f:64 * (f + n)]), bytes(pubs[32 * f:32 * (f + n)])
        want_txn[t] = ref.fdref_verify_batch_single_msg(m, len(m), ss, ps, n)
        for j in range(n):
            want_sig[f + j] = ref.fdref_verify(m, len(m), ss[64 * j:64 * j + 64], ps[32 * j:32 * j + 32])
    bad = np.nonzero(got_txn != want_txn)[0]
    assert len(bad) == 0, [(int(t), int(cnt[t]), int(got_txn[t]), int(want_txn[t])) for t in bad[:10]]
    assert np.array_equal(got_sig[:len(want_sig)], want_sig)
    # every code class occurs
    assert {0, -1, -2, -3} <= set(np.unique(want_txn).tolist())
    if codes == "avx512":
        # the same transactions through the drop-in, one synchronous
        # fd_ed25519_verify_batch_single_msg call each (the drop-in engines
        # keep the AVX-512 backend's codes unless FD_ED25519_HIP_CODES says
        # otherwise at their creation)
        got_drop = np.array([ed25519.verify_batch_single_msg(bytes(msgs[t_off[t]:t_off[t] + t_sz[t]]),
                                                              bytes(sigs[64 * first[t]:64 * (first[t] + cnt[t])]),
                                                              bytes(pubs[32 * first[t]:32 * (first[t] + cnt[t])]))
                             for t in range(len(cnt))], np.int8)
        bad = np.nonzero(got_drop != want_txn)[0]
        assert len(bad) == 0, [(int(t), int(cnt[t]), int(got_drop[t]), int(want_txn[t])) for t in bad[:10]]
