"""Mixed-order A and R at scale: public keys and nonces that
carry an 8-torsion component pass the reference's decode and small-order
checks (src/ballet/ed25519/fd_curve25519.h:81-111), and the cofactorless
equation (src/ballet/ed25519/fd_ed25519_user.c:215-224) accepts them only
when T_R = -[k]T_A.  The engine's half-size equation relies on its (c, d)
pair satisfying c = d k mod 8L with d odd; these 10,240 signatures (3,789
accepted because the torsion cancels) and 600 batch_single_msg transactions
(tests/golden/gen_mixed.py, codes from the reference compiled from its
sources) check that claim in every launch form, in both code flavours, under
FLAG_HALF_STRICT, and through the drop-ins.  Bit-exact codes."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FORMS = ["r16", "oct", "quad", "wide", "r16-compact", "wide-compact"]


@pytest.fixture(scope="module")
def fd():
    from firedancer_amd import ed25519
    return ed25519


def _check(got, want, tags):
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (len(bad), [(str(tags[i]), int(got[i]), int(want[i])) for i in bad[:12]])


def _engine(fd, form, **kw):
    dsm, _, compact = form.partition("-")
    return fd.Engine(0, max_chunk=1 << 14, dsm=dsm, compact=bool(compact), **kw)


@pytest.mark.parametrize("half", ["extended", "strict"])
@pytest.mark.parametrize("form", FORMS)
def test_mixed_order_every_form(fd, mixed_order, form, half):
    d = mixed_order
    e = _engine(fd, form, half=half)
    try:
        got = e.verify_host(d["msgs"], d["msg_off"], d["msg_sz"], d["sigs"], d["pubs"])
    finally:
        e.close()
    _check(got, d["codes_avx512"], d["tags"])
    assert int((got == 0).sum()) == 3789


@pytest.mark.parametrize("form", ["r16", "wide"])
def test_mixed_order_portable_codes(fd, mixed_order, form):
    d = mixed_order
    e = _engine(fd, form, codes="portable")
    try:
        got = e.verify_host(d["msgs"], d["msg_off"], d["msg_sz"], d["sigs"], d["pubs"])
    finally:
        e.close()
    _check(got, d["codes_portable"], d["tags"])


def test_mixed_order_auto_form_scattered(fd, mixed_order, adversarial):
    """The automatic form choice on one large call with the mixed-order cases
    scattered among the adversarial set (the throughput path's waves mix
    them with ordinary lanes)."""
    parts = [mixed_order, adversarial, adversarial]
    rng = np.random.default_rng(6)
    msgs, off, sz, sigs, pubs, want = [], [], [], [], [], []
    base = 0
    for p in parts:
        msgs.append(p["msgs"])
        off.append(p["msg_off"].astype(np.uint64) + np.uint64(base))
        base += len(p["msgs"])
        sz.append(p["msg_sz"]); sigs.append(p["sigs"]); pubs.append(p["pubs"]); want.append(p["codes_avx512"])
    order = rng.permutation(sum(len(p["msg_sz"]) for p in parts))
    msgs = np.concatenate(msgs)
    off, sz = np.concatenate(off)[order], np.concatenate(sz)[order]
    sigs, pubs, want = np.concatenate(sigs)[order], np.concatenate(pubs)[order], np.concatenate(want)[order]
    e = fd.Engine(0)
    try:
        _check(e.verify_host(msgs, off, sz, sigs, pubs), want, order)
    finally:
        e.close()


@pytest.mark.parametrize("form", ["r16", "wide"])
def test_mixed_order_txns(fd, mixed_order, form):
    d = mixed_order
    e = _engine(fd, form)
    try:
        out, _ = e.verify_txns_host(d["b_msgs"], d["b_txn_msg_off"], d["b_txn_msg_sz"], d["b_txn_first"],
                                    d["b_txn_cnt"], d["b_sigs"], d["b_pubs"])
    finally:
        e.close()
    _check(out, d["b_codes_avx512"], d["b_tags"])


def test_mixed_order_dropin(fd, mixed_order):
    """fd_ed25519_verify, one synchronous call per signature (the direct
    launch of the drop-in engine), every 4th case; then every transaction
    through fd_ed25519_verify_batch_single_msg."""
    d = mixed_order
    for i in range(0, len(d["msg_sz"]), 4):
        o, n = int(d["msg_off"][i]), int(d["msg_sz"][i])
        got = fd.verify(bytes(d["msgs"][o:o + n]), d["sigs"][i].tobytes(), d["pubs"][i].tobytes())
        assert got == int(d["codes_avx512"][i]), (i, str(d["tags"][i]), got)
    for t in range(len(d["b_txn_cnt"])):
        o, n = int(d["b_txn_msg_off"][t]), int(d["b_txn_msg_sz"][t])
        f, c = int(d["b_txn_first"][t]), int(d["b_txn_cnt"][t])
        got = fd.verify_batch_single_msg(bytes(d["b_msgs"][o:o + n]), d["b_sigs"][f:f + c].tobytes(),
                                         d["b_pubs"][f:f + c].tobytes(), c)
        assert got == int(d["b_codes_avx512"][t]), (t, str(d["b_tags"][t]), got)
