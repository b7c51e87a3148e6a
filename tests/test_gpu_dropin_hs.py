"""The drop-in's host-scalar launches (fd_ed25519_hip_dropin_set_host_scalars,
host/fd_ed25519_hip_hsrec.cc): a direct launch of a few signatures takes
k, S < L and the half-size pair from the calling thread while the GPU
decompresses A and R, and dsm16 reads them from the page-locked block; the
fewest-signature launches (fd_ed25519_hip_dropin_set_host_decode,
host/fd_ed25519_hip_hsdec.cc) decompress A and R on the calling thread too
and launch the group equation alone, reading the points in place -- over
eight or four waves on A and R doubled by the host every 33 or 66 bits
(dsm16s, fd_ed25519_hip_dropin_set_split_waves) or in dsm16's two.  Every
fixture class -- the reference's vectors, the adversarial set,
mixed-order points, k needing long |d| -- through fd_ed25519_verify with
each mode on (the default) and off, code by code against the reference's
own codes (tests/golden/, oracle/_ref)."""
import ctypes
import threading

import numpy as np
import pytest

from conftest import case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ed():
    from firedancer_amd import ed25519
    lib = ed25519.library()
    lib.fd_ed25519_hip_dropin_set_host_scalars.argtypes = [ctypes.c_ulong]
    lib.fd_ed25519_hip_dropin_set_host_decode.argtypes = [ctypes.c_ulong]
    lib.fd_ed25519_hip_dropin_set_split_waves.argtypes = [ctypes.c_int]
    yield ed25519, lib
    lib.fd_ed25519_hip_dropin_set_host_scalars(4)
    lib.fd_ed25519_hip_dropin_set_host_decode(2)
    lib.fd_ed25519_hip_dropin_set_split_waves(4)


def _run(ed25519, d, idx):
    return np.array([ed25519.verify(*case(d, i)) for i in idx], np.int8)


@pytest.mark.parametrize("mode", [(4, 2, 8), (4, 2, 4), (4, 2, 2), (4, 0, 8), (0, 0, 8)],
                         ids=["host-decode-eight-waves", "host-decode-four-waves", "host-decode-two-waves",
                              "host-scalars", "device"])
@pytest.mark.parametrize("fixture", ["vectors", "adversarial", "mixed_order", "halfsize", "longd"])
def test_dropin_codes_every_host_path(ed, request, mode, fixture):
    ed25519, lib = ed
    lib.fd_ed25519_hip_dropin_set_host_scalars(mode[0])
    lib.fd_ed25519_hip_dropin_set_host_decode(mode[1])
    lib.fd_ed25519_hip_dropin_set_split_waves(mode[2])
    d = request.getfixturevalue(fixture)
    n = len(d["msg_sz"])
    idx = list(range(0, n, 3 if n > 3000 else 1))
    got = _run(ed25519, d, idx)
    want = d["codes_avx512"][idx]
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(str(d["tags"][idx[i]]), int(got[i]), int(want[i])) for i in bad[:10]]


@pytest.mark.parametrize("callers,hd,waves", [(2, 2, 8), (4, 4, 8), (4, 4, 4), (4, 0, 8)])
def test_dropin_host_scalars_concurrent_callers(ed, adversarial, mixed_order, callers, hd, waves):
    """Threads calling at once: their requests may combine into launches of
    two to four signatures (still host-scalar launches; with the host
    decompressions up to hd of them) -- codes exact."""
    ed25519, lib = ed
    lib.fd_ed25519_hip_dropin_set_host_scalars(4)
    lib.fd_ed25519_hip_dropin_set_host_decode(hd)
    lib.fd_ed25519_hip_dropin_set_split_waves(waves)
    for d in (adversarial, mixed_order):
        n = min(len(d["msg_sz"]), 2000)
        out = np.zeros(n, np.int8)

        def work(par):
            for i in range(par, n, callers):
                out[i] = ed25519.verify(*case(d, i))
        ths = [threading.Thread(target=work, args=(p,)) for p in range(callers)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert np.array_equal(out, d["codes_avx512"][:n])
    lib.fd_ed25519_hip_dropin_set_host_decode(2)
    lib.fd_ed25519_hip_dropin_set_split_waves(4)


def test_dropin_host_scalars_fallback_to_the_device_path(ed, halfsize, adversarial):
    """A signature whose k has no pair within the host search's bound sends
    its launch down the device path from its digest (the messages are not
    staged in host-scalar launches).  With the host bound lowered to 131
    bits (test hook) every halfsize.npz signature takes that fallback, whose
    device search runs at 151 bits; the codes stay the reference's, and the
    adversarial set (pairs within 131 bits for most) is unaffected."""
    ed25519, lib = ed
    lib.fd_ed25519_hip_dropin_set_host_scalars.argtypes = [ctypes.c_ulong]
    lib.fd_ed25519_hip_dropin_set_host_scalars_dbits.argtypes = [ctypes.c_int]
    lib.fd_ed25519_hip_dropin_set_host_scalars(4)
    lib.fd_ed25519_hip_dropin_set_host_scalars_dbits(131)
    try:
        for d in (halfsize, adversarial):
            idx = list(range(len(d["msg_sz"])))
            got = _run(ed25519, d, idx)
            bad = np.nonzero(got != d["codes_avx512"])[0]
            assert len(bad) == 0, [(str(d["tags"][i]), int(got[i]), int(d["codes_avx512"][i])) for i in bad[:10]]
    finally:
        lib.fd_ed25519_hip_dropin_set_host_scalars_dbits(0)


@pytest.mark.parametrize("mode", [(4, 2, 4), (4, 4, 4), (4, 2, 2), (4, 0, 4), (0, 0, 4)],
                         ids=["hs-decode2-four-waves", "hs-decode4-four-waves", "hs-decode2-two-waves", "host-scalars",
                              "device"])
def test_dropin_batch_single_msg_every_host_path(ed, batch, mixed_order, mode):
    """fd_ed25519_verify_batch_single_msg: a transaction of at most 4
    signatures over one message takes the host-scalar launch too (its
    signatures' records from the calling thread, the decompressions as well
    for at most hd of them), its codes combined on the host by the batch
    rule -- every transaction of the batch fixture and the mixed-order set,
    code for code against the reference's, in every mode."""
    ed25519, lib = ed
    lib.fd_ed25519_hip_dropin_set_host_scalars(mode[0])
    lib.fd_ed25519_hip_dropin_set_host_decode(mode[1])
    lib.fd_ed25519_hip_dropin_set_split_waves(mode[2])
    try:
        n_small = 0
        for d, pre in ((batch, ""), (mixed_order, "b_")):
            for t in range(len(d[pre + "txn_cnt"])):
                c = int(d[pre + "txn_cnt"][t])
                if c < 1 or c > 16:
                    continue
                o, z, f = int(d[pre + "txn_msg_off"][t]), int(d[pre + "txn_msg_sz"][t]), int(d[pre + "txn_first"][t])
                got = ed25519.verify_batch_single_msg(bytes(d[pre + "msgs"][o:o + z]), d[pre + "sigs"][f:f + c].tobytes(),
                                                      d[pre + "pubs"][f:f + c].tobytes(), c)
                assert got == int(d[pre + "codes_avx512"][t]), (pre, t, c, got)
                n_small += c <= 4
        assert n_small > 100
    finally:
        lib.fd_ed25519_hip_dropin_set_host_scalars(4)
        lib.fd_ed25519_hip_dropin_set_host_decode(2)
        lib.fd_ed25519_hip_dropin_set_split_waves(4)
