"""The drop-ins take any msg_sz, as the reference does
(src/ballet/ed25519/fd_ed25519.h:96-101, `ulong msg_sz`): messages the
device path's 32-bit sizes cannot carry (4 GiB and more) are hashed on the
host with the library's own SHA-512 and verified on the GPU from their
digests (fd_ed25519_hip_verify_digests_dev).

  - with the test hook lowering the limit to 1 byte (every message but the
    empty one takes the host-hash path), the fixture vectors and random
    batches give the reference's codes, through both drop-ins, mixed in one
    combined launch with device-hashed requests;
  - a real message of 4 GiB + 1000 bytes (a sparse anonymous mapping),
    signed by the oracle: valid verifies, and a flipped byte past the 4 GiB
    mark fails with ERR_MSG, as the reference's own fd_ed25519_verify
    (oracle/_ref) says for the same bytes -- nothing is truncated."""
import ctypes
import mmap
import os
import random

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ed():
    from firedancer_amd import ed25519
    lib = ed25519.library()
    lib.fd_ed25519_hip_dropin_set_host_hash_min.argtypes = [ctypes.c_ulong]
    yield ed25519, lib
    lib.fd_ed25519_hip_dropin_set_host_hash_min(0)


def test_host_hashed_dropins_match_the_reference_codes(ed, vectors, oracle):
    ed25519, lib = ed
    lib.fd_ed25519_hip_dropin_set_host_hash_min(1)
    try:
        msgs, sigs, pubs = vectors["msgs"], vectors["sigs"].reshape(-1, 64), vectors["pubs"].reshape(-1, 32)
        off, sz, codes = vectors["msg_off"], vectors["msg_sz"], vectors["codes_avx512"]
        got = [ed25519.verify(bytes(msgs[int(off[i]):int(off[i]) + int(sz[i])]), bytes(sigs[i]), bytes(pubs[i]))
               for i in range(len(sz))]
        assert np.array_equal(np.array(got, np.int8), codes)
        # batch_single_msg: n signers over one message, one of them bad at random
        rng = random.Random(99)
        for t in range(60):
            n = rng.randint(1, 12)
            m = bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 200, 1232, 5000])))
            privs = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(n)]
            ps, ss = [], []
            for pr in privs:
                pk = ctypes.create_string_buffer(32)
                oracle.oracle_ed25519_public_from_private(pk, pr)
                sg = ctypes.create_string_buffer(64)
                oracle.oracle_ed25519_sign(sg, m, len(m), pk.raw, pr)
                ps.append(pk.raw)
                ss.append(bytearray(sg.raw))
            if t % 3 == 1:
                ss[rng.randrange(n)][rng.randrange(64)] ^= 1 << rng.randrange(8)
            want = oracle.oracle_ed25519_verify_batch_single_msg(m, len(m), b"".join(map(bytes, ss)), b"".join(ps), n, 0)
            assert ed25519.verify_batch_single_msg(m, b"".join(map(bytes, ss)), b"".join(ps)) == want, t
    finally:
        lib.fd_ed25519_hip_dropin_set_host_hash_min(0)


def test_message_past_4gib_is_verified_whole(ed, oracle):
    """4 GiB + 1000 bytes: the drop-in accepts the signature, rejects it
    with ERR_MSG once a byte past the 4 GiB mark changes, and agrees with
    the reference's fd_ed25519_verify (compiled from its sources) on both.
    The test hook's limit is set above 4 GiB first: it is
    clamped, and a size the device's 32-bit lengths would truncate is
    hashed on the host whatever the limit says."""
    ed25519, lib = ed
    lib.fd_ed25519_hip_dropin_set_host_hash_min(1 << 40)
    ref_path = os.path.join(REPO, "oracle", "_ref", "libfdref_avx512.so")
    sz = (1 << 32) + 1000
    m = mmap.mmap(-1, sz, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    try:
        m[0:16] = b"firedancer-amd!!"
        m[sz - 16:sz] = b"tail past 4 GiB!"
        base = ctypes.addressof(ctypes.c_char.from_buffer(m))
        priv = bytes(range(32))
        pub, sig = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
        oracle.oracle_ed25519_public_from_private(pub, priv)
        sign = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle_ed25519.so")).oracle_ed25519_sign   # own handle
        sign.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_char_p]
        sign(sig, base, sz, pub.raw, priv)
        v = lib.fd_ed25519_verify
        v.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]
        v.restype = ctypes.c_int
        ref = None
        if os.path.exists(ref_path):
            ref = ctypes.CDLL(ref_path).fd_ed25519_verify
            ref.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]
            ref.restype = ctypes.c_int
        sha = ctypes.create_string_buffer(512)
        sha_p = (ctypes.addressof(sha) + 127) & ~127
        got_ok = v(base, sz, sig.raw, pub.raw, None)
        want_ok = ref(base, sz, sig.raw, pub.raw, sha_p) if ref else 0
        m[sz - 3] ^= 0x01                     # a byte past the 4 GiB mark
        got_bad = v(base, sz, sig.raw, pub.raw, None)
        want_bad = ref(base, sz, sig.raw, pub.raw, sha_p) if ref else -3
        bv = lib.fd_ed25519_verify_batch_single_msg
        bv.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p,
                       ctypes.c_ubyte]
        bv.restype = ctypes.c_int
        got_batch = bv(base, sz, sig.raw * 2, pub.raw * 2, None, 2)
    finally:
        m.close()
    assert (got_ok, got_bad) == (want_ok, want_bad) == (0, -3)
    assert got_batch == -3


@pytest.mark.parametrize("sz", [65536 - 400, 65536 - 160, 65536 - 159, 1 << 20, 8 << 20],
                         ids=["below-direct-limit", "at-direct-limit", "past-direct-limit", "1MiB", "8MiB"])
def test_device_hashed_large_message_dropin(ed, oracle, sz):
    """MB-scale messages stay on the device hash (below the 4 GiB host-hash
    limit): a launch whose staged block is at most 64 KiB reads it in place
    over the link (the direct path), a larger one is pulled into HBM first
    (ADVICE r5).  The sizes straddle that limit (a one-signature block is
    160 bytes of offsets, sizes, signature and key, then the message);
    valid verifies, a flipped last byte gives ERR_MSG."""
    ed25519, lib = ed
    lib.fd_ed25519_hip_dropin_set_host_hash_min(0)
    rng = np.random.default_rng(sz)
    m = bytearray(rng.integers(0, 256, sz, dtype=np.uint8).tobytes())
    priv = bytes(rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
    pub, sig = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    oracle.oracle_ed25519_public_from_private(pub, priv)
    oracle.oracle_ed25519_sign(sig, bytes(m), sz, pub.raw, priv)
    assert ed25519.verify(bytes(m), sig.raw, pub.raw) == 0
    m[-1] ^= 1
    assert ed25519.verify(bytes(m), sig.raw, pub.raw) == -3
    assert oracle.oracle_ed25519_verify(bytes(m), sz, sig.raw, pub.raw, 0) == -3
