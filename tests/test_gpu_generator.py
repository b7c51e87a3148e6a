"""The device-side batch signer and workload generator (bench.py's data) vs
the oracle and the host definition in firedancer_amd/workload.py."""
import ctypes
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, oracle_many

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fd():
    from firedancer_amd import ed25519
    return ed25519


@pytest.fixture(scope="module")
def eng(fd):
    e = fd.Engine(0, max_chunk=1 << 14)
    yield e
    e.close()


def _download(wl):
    n = wl.n
    sizes = wl.sizes.astype(np.uint64)
    off = np.zeros(n, np.uint64)
    np.cumsum(sizes[:-1], out=off[1:])
    return dict(msgs=wl.msgs.download(np.uint8, max(wl.msg_bytes, 1)), msg_off=off, msg_sz=wl.sizes,
                sigs=wl.sigs.download(np.uint8, 64 * n).reshape(n, 64),
                pubs=wl.pubs.download(np.uint8, 32 * n).reshape(n, 32),
                expect=wl.expect.download(np.int8, n), cls=wl.cls.download(np.uint8, n))


def test_sign_dev_matches_sign_kat(fd, eng):
    kats = json.load(open(os.path.join(GOLDEN, "sign_kat.json")))
    n = len(kats)
    msgs = b"".join(bytes.fromhex(k["msg"]) for k in kats)
    sz = np.array([len(k["msg"]) // 2 for k in kats], np.uint32)
    off = np.zeros(n, np.uint64)
    np.cumsum(sz[:-1].astype(np.uint64), out=off[1:])
    privs = np.frombuffer(b"".join(bytes.fromhex(k["priv"]) for k in kats), np.uint8)
    d_m = eng.alloc(len(msgs) + 16).upload(np.frombuffer(msgs, np.uint8))
    d_off, d_sz, d_pr = eng.alloc(8 * n).upload(off), eng.alloc(4 * n).upload(sz), eng.alloc(32 * n).upload(privs)
    d_sig, d_pub = eng.alloc(64 * n), eng.alloc(32 * n)
    eng.sign_dev(n, d_m.ptr, d_off.ptr, d_sz.ptr, d_pr.ptr, d_sig.ptr, d_pub.ptr)
    eng.sync()
    sigs = d_sig.download(np.uint8, 64 * n).reshape(n, 64)
    pubs = d_pub.download(np.uint8, 32 * n).reshape(n, 32)
    for i, k in enumerate(kats):
        assert pubs[i].tobytes().hex() == k["pub"], i
        assert sigs[i].tobytes().hex() == k["sig"], i


def test_generator_matches_host_definition_and_oracle(fd, eng, oracle):
    from firedancer_amd import workload
    seed, base, n = 1234, 5000, 1024
    wl = fd.DeviceWorkload(eng, n, 64, 1232, 0, seed=seed, index_base=base)
    d = _download(wl)
    assert np.array_equal(d["msg_sz"], workload.msg_sizes(seed, base, n, 64, 1232))
    assert np.array_equal(d["msgs"][:wl.msg_bytes], workload.msg_buffer(seed, wl.msg_bytes))
    privs = workload.private_keys(seed, base, n)
    for i in range(0, n, 17):
        pub = ctypes.create_string_buffer(32)
        oracle.oracle_ed25519_public_from_private(pub, privs[i].tobytes())
        assert pub.raw == d["pubs"][i].tobytes(), i
        m = d["msgs"][int(d["msg_off"][i]):int(d["msg_off"][i]) + int(d["msg_sz"][i])].tobytes()
        sig = ctypes.create_string_buffer(64)
        oracle.oracle_ed25519_sign(sig, m, len(m), pub.raw, privs[i].tobytes())
        assert sig.raw == d["sigs"][i].tobytes(), i
    assert (d["expect"] == 0).all()
    wl.free()


def test_corruption_labels_are_reference_codes(fd, eng, oracle):
    """Every injected class carries the code the reference returns (checked
    with the oracle on the very bytes the GPU produced)."""
    from firedancer_amd import workload
    seed, n = 99, 2048
    wl = fd.DeviceWorkload(eng, n, 64, 1232, 250000, seed=seed, index_base=0)
    d = _download(wl)
    cls, _ = workload.corruption(seed, 0, n, 250000)
    assert np.array_equal(cls, d["cls"])
    assert set(np.unique(cls).tolist()) == set(range(8))
    want = oracle_many(oracle, d, 0)
    bad = np.nonzero(want != d["expect"])[0]
    assert len(bad) == 0, [(int(d["cls"][i]), int(want[i]), int(d["expect"][i])) for i in bad[:10]]
    wl.verify()
    eng.sync()
    assert np.array_equal(wl.out.download(np.int8, n), want)
    wl.free()
