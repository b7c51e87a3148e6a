"""Pins the CPU restatement (oracle/) against the reference's own vectors and
against codes produced by the reference compiled from its sources
(tests/golden/gen_golden.py).  CPU only."""
import hashlib
import json
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN, case, oracle_many

L = 2**252 + 27742317777372353535851937790883648493


def test_sha512_matches_fips(oracle):
    import ctypes
    rng = random.Random(7)
    for sz in list(range(0, 300)) + [1232, 1296, 4096]:
        m = bytes(rng.getrandbits(8) for _ in range(sz))
        out = ctypes.create_string_buffer(64)
        oracle.oracle_sha512(out, m, sz)
        assert out.raw == hashlib.sha512(m).digest(), sz


def test_scalar_reduce(oracle):
    import ctypes
    rng = random.Random(8)
    vals = [0, 1, L - 1, L, L + 1, 2**512 - 1, 2**252, 2**253 - 1]
    vals += [rng.getrandbits(512) for _ in range(500)]
    for v in vals:
        out = ctypes.create_string_buffer(32)
        oracle.oracle_scalar_reduce(out, v.to_bytes(64, "little"))
        assert int.from_bytes(out.raw, "little") == v % L


@pytest.mark.parametrize("codes,key", [(0, "codes_avx512"), (1, "codes_portable")])
def test_vectors_codes(oracle, vectors, codes, key):
    got = oracle_many(oracle, vectors, codes)
    want = vectors[key]
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(str(vectors["tags"][i]), int(got[i]), int(want[i])) for i in bad[:10]]


def test_vectors_accept_reject(oracle, vectors):
    """The reference's own expectations (wycheproof/cctv/malleability ok flags)."""
    got = oracle_many(oracle, vectors, 0)
    sel = vectors["ok"] >= 0
    assert np.array_equal((got[sel] == 0).astype(np.int8), vectors["ok"][sel])
    assert int(sel.sum()) == 133 + 914 + 196 + 200


@pytest.mark.parametrize("codes,key", [(0, "codes_avx512"), (1, "codes_portable")])
def test_adversarial_codes(oracle, adversarial, codes, key):
    got = oracle_many(oracle, adversarial, codes)
    want = adversarial[key]
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(str(adversarial["tags"][i]), int(got[i]), int(want[i])) for i in bad[:10]]


@pytest.mark.parametrize("codes,key", [(0, "codes_avx512"), (1, "codes_portable")])
def test_batch_single_msg_codes(oracle, batch, codes, key):
    for t in range(len(batch["txn_cnt"])):
        off, sz = int(batch["txn_msg_off"][t]), int(batch["txn_msg_sz"][t])
        f, n = int(batch["txn_first"][t]), int(batch["txn_cnt"][t])
        m = bytes(batch["msgs"][off:off + sz])
        nn = min(n, len(batch["sigs"]) - f)
        sigs = batch["sigs"][f:f + nn].tobytes() or b"\0" * 64
        pubs = batch["pubs"][f:f + nn].tobytes() or b"\0" * 32
        got = oracle.oracle_ed25519_verify_batch_single_msg(m, sz, sigs, pubs, n, codes)
        assert got == int(batch[key][t]), (t, str(batch["tags"][t]), got, int(batch[key][t]))


def test_sign_kat(oracle):
    import ctypes
    for k in json.load(open(os.path.join(GOLDEN, "sign_kat.json"))):
        priv, msg = bytes.fromhex(k["priv"]), bytes.fromhex(k["msg"])
        pub = ctypes.create_string_buffer(32)
        oracle.oracle_ed25519_public_from_private(pub, priv)
        assert pub.raw.hex() == k["pub"]
        sig = ctypes.create_string_buffer(64)
        oracle.oracle_ed25519_sign(sig, msg, len(msg), pub.raw, priv)
        assert sig.raw.hex() == k["sig"]
        assert oracle.oracle_ed25519_verify(msg, len(msg), sig.raw, pub.raw, 0) == 0


def test_strerror(oracle):
    assert oracle.oracle_ed25519_strerror(0) == b"success"
    assert oracle.oracle_ed25519_strerror(-1) == b"bad signature"
    assert oracle.oracle_ed25519_strerror(-2) == b"bad public key"
    assert oracle.oracle_ed25519_strerror(-3) == b"bad message"
    assert oracle.oracle_ed25519_strerror(7) == b"unknown"


def test_empty_message_null(oracle):
    """msg==NULL with sz==0 is fine (src/ballet/ed25519/fd_ed25519.h:78-80)."""
    d = json.load(open(os.path.join(GOLDEN, "sign_kat.json")))[0]
    assert oracle.oracle_ed25519_verify(None, 0, bytes.fromhex(d["sig"]), bytes.fromhex(d["pub"]), 0) == 0


@pytest.mark.parametrize("codes,key", [(0, "codes_avx512"), (1, "codes_portable")])
def test_halfsize_fallback_codes(oracle, halfsize, codes, key):
    """Signatures whose k has no half-size pair (gen_halfsize.py)."""
    got = oracle_many(oracle, halfsize, codes)
    bad = np.nonzero(got != halfsize[key])[0]
    assert len(bad) == 0, [(str(halfsize["tags"][i]), int(got[i]), int(halfsize[key][i])) for i in bad[:10]]


@pytest.mark.parametrize("codes,key", [(0, "codes_avx512"), (1, "codes_portable")])
def test_mixed_order_codes(oracle, mixed_order, codes, key):
    """A and R carrying an 8-torsion component (gen_mixed.py): accepted only
    when it cancels in the cofactorless equation; 10,240 signatures."""
    d = mixed_order
    got = oracle_many(oracle, d, codes)
    bad = np.nonzero(got != d[key])[0]
    assert len(bad) == 0, [(str(d["tags"][i]), int(got[i]), int(d[key][i])) for i in bad[:10]]
    assert int((d[key] == 0).sum()) >= 1000 and len(got) >= 10000


@pytest.mark.parametrize("codes,key", [(0, "b_codes_avx512"), (1, "b_codes_portable")])
def test_mixed_order_batch_codes(oracle, mixed_order, codes, key):
    d = mixed_order
    for t in range(len(d["b_txn_cnt"])):
        off, sz = int(d["b_txn_msg_off"][t]), int(d["b_txn_msg_sz"][t])
        f, n = int(d["b_txn_first"][t]), int(d["b_txn_cnt"][t])
        got = oracle.oracle_ed25519_verify_batch_single_msg(bytes(d["b_msgs"][off:off + sz]), sz,
                                                            d["b_sigs"][f:f + n].tobytes(),
                                                            d["b_pubs"][f:f + n].tobytes(), n, codes)
        assert got == int(d[key][t]), (t, str(d["b_tags"][t]), got, int(d[key][t]))
