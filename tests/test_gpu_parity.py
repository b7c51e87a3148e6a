"""Parity of the MI355X engine (through the C-ABI library) with the reference:
golden fixtures produced by the reference itself (tests/golden/), and the
oracle restatement on seeded random / adversarial inputs.  Bit-exact codes."""
import ctypes
import random

import numpy as np
import pytest

from conftest import oracle_many

pytestmark = pytest.mark.gpu

L = 2**252 + 27742317777372353535851937790883648493


@pytest.fixture(scope="module")
def fd():
    from firedancer_amd import ed25519
    return ed25519


# Every engine test runs with each dsm form: two quads of lanes per
# signature (chunks of up to FD_ED25519_HIP_OCT_MAX_DEFAULT signatures), a
# quad (up to FD_ED25519_HIP_QUAD_MAX_DEFAULT) and one lane per signature;
# each with the wide radix-2^24 base tables and with the compact radix-2^16
# ones (FD_ED25519_HIP_FLAG_COMPACT_TABLES, the drop-ins' engines).
@pytest.fixture(scope="module", params=["r16", "oct", "quad", "wide", "r16-compact", "oct-compact", "quad-compact",
                                        "wide-compact"])
def eng(fd, request):
    form, _, compact = request.param.partition("-")
    e = fd.Engine(0, max_chunk=1 << 16, dsm=form, compact=bool(compact))
    yield e
    e.close()


@pytest.fixture(scope="module", params=["r16", "oct", "quad", "wide"])
def eng_portable(fd, request):
    e = fd.Engine(0, max_chunk=1 << 14, codes="portable", dsm=request.param)
    yield e
    e.close()


def _check(got, want, tags=None):
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [((str(tags[i]) if tags is not None else i), int(got[i]), int(want[i])) for i in bad[:12]]


def _run(e, d):
    return e.verify_host(d["msgs"], d["msg_off"], d["msg_sz"], d["sigs"], d["pubs"])


def test_engine_info(eng):
    info = eng.info()
    assert info["arch"].startswith("gfx950")
    assert info["cu_cnt"] > 0 and info["dsm_grid"] > 0


def test_reference_vectors(eng, vectors):
    _check(_run(eng, vectors), vectors["codes_avx512"], vectors["tags"])


def test_reference_vectors_accept_reject(eng, vectors):
    got = _run(eng, vectors)
    sel = vectors["ok"] >= 0
    assert np.array_equal((got[sel] == 0).astype(np.int8), vectors["ok"][sel])


def test_reference_vectors_portable_codes(eng_portable, vectors):
    _check(_run(eng_portable, vectors), vectors["codes_portable"], vectors["tags"])


def test_adversarial(eng, adversarial):
    _check(_run(eng, adversarial), adversarial["codes_avx512"], adversarial["tags"])


def test_adversarial_portable_codes(eng_portable, adversarial):
    _check(_run(eng_portable, adversarial), adversarial["codes_portable"], adversarial["tags"])


def test_batch_single_msg_txns(eng, batch):
    out, _ = eng.verify_txns_host(batch["msgs"], batch["txn_msg_off"], batch["txn_msg_sz"], batch["txn_first"],
                                  batch["txn_cnt"], batch["sigs"], batch["pubs"])
    _check(out, batch["codes_avx512"], batch["tags"])


def test_batch_single_msg_txns_portable(eng_portable, batch):
    out, _ = eng_portable.verify_txns_host(batch["msgs"], batch["txn_msg_off"], batch["txn_msg_sz"],
                                           batch["txn_first"], batch["txn_cnt"], batch["sigs"], batch["pubs"])
    _check(out, batch["codes_portable"], batch["tags"])


def _random_set(oracle, n, seed, sizes=None, mutate=True):
    rng = random.Random(seed)
    msgs = bytearray()
    off, sz, sigs, pubs = [], [], bytearray(), bytearray()
    keys = []
    for _ in range(32):
        priv = bytes(rng.getrandbits(8) for _ in range(32))
        pub = ctypes.create_string_buffer(32)
        oracle.oracle_ed25519_public_from_private(pub, priv)
        keys.append((priv, pub.raw))
    for i in range(n):
        priv, pub = keys[i % len(keys)]
        m = bytes(rng.getrandbits(8) for _ in range(sizes(i, rng) if sizes else rng.randrange(0, 1233)))
        s = ctypes.create_string_buffer(64)
        oracle.oracle_ed25519_sign(s, m, len(m), pub, priv)
        sig, pk = bytearray(s.raw), bytearray(pub)
        if mutate:
            r = rng.random()
            if r < 0.05:
                sig[rng.randrange(64)] ^= 1 << rng.randrange(8)
            elif r < 0.08:
                pk[rng.randrange(32)] ^= 1 << rng.randrange(8)
            elif r < 0.10 and m:
                mm = bytearray(m); mm[rng.randrange(len(m))] ^= 1; m = bytes(mm)
        # misalign message starts on purpose
        msgs += bytes(rng.randrange(0, 4))
        off.append(len(msgs)); sz.append(len(m)); msgs += m
        sigs += sig; pubs += pk
    return dict(msgs=np.frombuffer(bytes(msgs) or b"\0", dtype=np.uint8), msg_off=np.array(off, np.uint64),
                msg_sz=np.array(sz, np.uint32), sigs=np.frombuffer(bytes(sigs), np.uint8).reshape(-1, 64),
                pubs=np.frombuffer(bytes(pubs), np.uint8).reshape(-1, 32))


def test_random_vs_oracle(eng, oracle):
    d = _random_set(oracle, 3000, seed=11)
    want = oracle_many(oracle, d, 0)
    assert (want == 0).sum() > 2500
    _check(_run(eng, d), want)


def test_every_message_size_vs_oracle(eng, oracle):
    """All sizes 0..400 (every SHA-512 block boundary and padding split) and
    the Solana MTU."""
    d = _random_set(oracle, 402, seed=12, sizes=lambda i, rng: i if i <= 400 else 1232, mutate=False)
    want = oracle_many(oracle, d, 0)
    assert (want == 0).all()
    _check(_run(eng, d), want)


def test_long_messages_vs_oracle(eng, oracle):
    """Messages past the Solana MTU (the drop-in takes any size): 1233 B ..
    70 KB, the 2^16 boundary, and 1 MiB -- one lane hashes a whole message,
    all of these in the sort's open-ended last bucket."""
    big = [1233, 4096, 65535, 65536, 65537, 70000, 1 << 20]
    d = _random_set(oracle, 64, seed=15, mutate=False,
                    sizes=lambda i, rng: big[i] if i < len(big) else rng.randrange(1233, 70001))
    sigs = d["sigs"].copy()
    sigs[1::3, 5] ^= 1   # a third of them invalid (R corrupted)
    d["sigs"] = sigs
    want = oracle_many(oracle, d, 0)
    assert (want == 0).sum() > 30 and (want != 0).sum() > 15
    _check(_run(eng, d), want)


def test_scalar_edges(eng, eng_portable, oracle):
    """S around L and all-ones; S+kL for small k; both code flavours."""
    d = _random_set(oracle, 64, seed=13, mutate=False)
    sigs = d["sigs"].copy()
    for i in range(64):
        S = int.from_bytes(sigs[i, 32:].tobytes(), "little")
        choice = [S, S + L, L - 1, L, L + 1, 2**256 - 1, 0, 2**253, S + 2 * L, 2**255 + S][i % 10]
        sigs[i, 32:] = np.frombuffer((choice % 2**256).to_bytes(32, "little"), np.uint8)
    d["sigs"] = sigs
    _check(_run(eng, d), oracle_many(oracle, d, 0))
    _check(_run(eng_portable, d), oracle_many(oracle, d, 1))


def test_chunking(fd, oracle):
    """A batch larger than max_chunk goes through several kernel sequences."""
    e = fd.Engine(0, max_chunk=700)
    d = _random_set(oracle, 2500, seed=14)
    _check(_run(e, d), oracle_many(oracle, d, 0))
    e.close()


def test_dsm_form_by_size(fd, oracle):
    """The automatic choice by chunk size (thresholds lowered with
    fd_ed25519_hip_engine_set_forms / _set_r16_max so the test stays small):
    a batch of two chunks (1000 wide, 600 quad), one of 600 (quad), one of
    300 (oct), one of 100 (r16) and a batch of 1100 (1000 wide + 100 r16),
    against the oracle."""
    e = fd.Engine(0, max_chunk=1000, forms=(600, 300), r16_max=100)
    for n, seed in ((1600, 15), (600, 16), (300, 17), (100, 18), (1100, 21)):
        d = _random_set(oracle, n, seed=seed)
        _check(_run(e, d), oracle_many(oracle, d, 0))
    e.close()


@pytest.mark.parametrize("overlap,pipeline", [(False, False), (True, False), (False, True), (True, True)],
                         ids=["sequential", "overlap", "pipelined", "overlap-pipelined"])
def test_launch_options_large_chunks(fd, oracle, overlap, pipeline):
    """The engine's launch sequences for one-lane-per-signature chunks (the
    small-chunk threshold lowered so the batches stay small): phases in
    sequence on one stream or decode on a side stream beside hash + scalar,
    with the chunks of one call on one set of work arrays or alternating
    between two (each set used twice, the last chunk a short one) -- each
    against the oracle; then a second call on the same engine, which must
    order after the first's lane-1 work."""
    e = fd.Engine(0, max_chunk=1000, overlap=overlap, pipeline=pipeline, forms=(300, 100))
    for n, seed in ((3700, 19), (2400, 20)):
        d = _random_set(oracle, n, seed=seed)
        _check(_run(e, d), oracle_many(oracle, d, 0))
    e.close()


def test_empty_batch(eng):
    out = eng.verify_host(np.zeros(0, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32),
                          np.zeros((0, 64), np.uint8), np.zeros((0, 32), np.uint8))
    assert out.shape == (0,)


def test_dropin_single(fd, vectors):
    """fd_ed25519_verify drop-in on the default engine."""
    for i in range(0, len(vectors["msg_sz"]), 37):
        off, sz = int(vectors["msg_off"][i]), int(vectors["msg_sz"][i])
        m = bytes(vectors["msgs"][off:off + sz])
        got = fd.verify(m, vectors["sigs"][i].tobytes(), vectors["pubs"][i].tobytes())
        assert got == int(vectors["codes_avx512"][i]), str(vectors["tags"][i])


def test_dropin_batch_single_msg(fd, batch):
    for t in range(0, len(batch["txn_cnt"]), 7):
        off, sz = int(batch["txn_msg_off"][t]), int(batch["txn_msg_sz"][t])
        f, n = int(batch["txn_first"][t]), int(batch["txn_cnt"][t])
        m = bytes(batch["msgs"][off:off + sz])
        got = fd.verify_batch_single_msg(m, batch["sigs"][f:f + n].tobytes(), batch["pubs"][f:f + n].tobytes(), n)
        assert got == int(batch["codes_avx512"][t]), (t, str(batch["tags"][t]))


def test_strerror(fd):
    assert fd.strerror(0) == "success" and fd.strerror(-3) == "bad message" and fd.strerror(5) == "unknown"


@pytest.fixture(scope="module", params=["r16", "oct", "quad", "wide"])
def eng_strict(fd, request):
    e = fd.Engine(0, max_chunk=1 << 14, half="strict", dsm=request.param)
    yield e
    e.close()


def test_halfsize_fallback(eng, halfsize):
    """k with no strict half-size pair (|d| >= 2^131): by default the
    extended-window form (W > 33 for the waves holding them)."""
    _check(_run(eng, halfsize), halfsize["codes_avx512"], halfsize["tags"])


def test_halfsize_fallback_strict(eng_strict, halfsize):
    """The same signatures under FLAG_HALF_STRICT: the dsm kernel's
    full-length items (waves of their own)."""
    _check(_run(eng_strict, halfsize), halfsize["codes_avx512"], halfsize["tags"])


def test_long_d_windows(eng, longd):
    """k whose half-size pair needs |d| up to 2^151: waves of 36..38 windows."""
    _check(_run(eng, longd), longd["codes_avx512"], longd["tags"])


def test_long_d_strict(eng_strict, longd):
    """The same under FLAG_HALF_STRICT: the full-length form."""
    _check(_run(eng_strict, longd), longd["codes_avx512"], longd["tags"])


def test_long_d_mixed_into_waves(eng, longd, adversarial):
    """One long-d signature in each wave of an otherwise ordinary chunk: the
    other lanes run the longer window count with zero top digits."""
    parts_m, off, sz, sigs, pubs, want = [], [], [], [], [], []
    base = 0
    for i in range(len(longd["msg_sz"])):
        for d, j in ((longd, i), (adversarial, None)):
            if j is None:
                sel = np.arange(63 * i, 63 * i + 63) % len(d["msg_sz"])
            else:
                sel = np.array([j])
            for t in sel:
                o, n = int(d["msg_off"][t]), int(d["msg_sz"][t])
                parts_m.append(d["msgs"][o:o + n])
                off.append(base); sz.append(n); base += n
                sigs.append(d["sigs"][t]); pubs.append(d["pubs"][t]); want.append(d["codes_avx512"][t])
    msgs = np.concatenate(parts_m) if base else np.zeros(1, np.uint8)
    got = eng.verify_host(msgs, np.array(off, np.uint64), np.array(sz, np.uint32), np.stack(sigs), np.stack(pubs))
    _check(got, np.array(want, np.int8))


def test_halfsize_fallback_portable(eng_portable, halfsize):
    _check(_run(eng_portable, halfsize), halfsize["codes_portable"], halfsize["tags"])


def test_halfsize_fallback_portable_strict(fd, halfsize):
    e = fd.Engine(0, max_chunk=1 << 12, codes="portable", half="strict")
    try:
        _check(_run(e, halfsize), halfsize["codes_portable"], halfsize["tags"])
    finally:
        e.close()


@pytest.mark.parametrize("mode", ["extended", "strict"])
def test_halfsize_fallback_scattered(fd, eng, eng_strict, halfsize, adversarial, mode):
    """Those signatures scattered through a larger chunk: extended-window
    lanes mixed into ordinary waves, or (strict) full-length items handed
    out first by the dsm work counter, the rest after them."""
    e = eng if mode == "extended" else eng_strict
    rng = np.random.default_rng(11)
    reps = 24
    parts = [halfsize] * reps + [adversarial] * 4
    order = rng.permutation(sum(len(p["msg_sz"]) for p in parts))
    msgs, off, sz, sigs, pubs, want = [], [], [], [], [], []
    base = 0
    for p in parts:
        msgs.append(p["msgs"])
        off.append(p["msg_off"].astype(np.uint64) + np.uint64(base))
        base += len(p["msgs"])
        sz.append(p["msg_sz"]); sigs.append(p["sigs"]); pubs.append(p["pubs"]); want.append(p["codes_avx512"])
    msgs = np.concatenate(msgs)
    off, sz = np.concatenate(off)[order], np.concatenate(sz)[order]
    sigs, pubs, want = np.concatenate(sigs)[order], np.concatenate(pubs)[order], np.concatenate(want)[order]
    got = e.verify_host(msgs, off, sz, sigs, pubs)
    _check(got, want)


def test_engines_share_base_tables(fd, adversarial):
    """The 2 x 2 GiB base tables are shared by the engines of a device and
    freed with the last one: engines created and destroyed in overlapping
    order all verify correctly, including after a full release."""
    want = adversarial["codes_avx512"]
    a = fd.Engine(0, max_chunk=1 << 12)
    b = fd.Engine(0, max_chunk=1 << 12)
    _check(_run(a, adversarial), want)
    a.close()
    _check(_run(b, adversarial), want)
    c = fd.Engine(0, max_chunk=1 << 12)
    b.close()
    _check(_run(c, adversarial), want)
    c.close()
    d = fd.Engine(0, max_chunk=1 << 12)   # the module's engines may still hold them; either way correct
    _check(_run(d, adversarial), want)
    d.close()


@pytest.mark.parametrize("compact", [False, True], ids=["wide", "compact"])
def test_base_tables_are_exact(fd, oracle, compact):
    """The half-size form's 2 x 2^24-entry base tables (and the full-length
    form's 2^15 + 1): on the device every
    entry e+1 equals entry e + entry 1 (entry 0 the identity), and entries
    1, 2, the run boundaries of the generator (runs of 32), the middle and
    the last, plus random ones, equal the oracle's [e 2^shift]B -- anchors
    that, with the chain, pin every entry; 2dxy checked too."""
    eng = fd.Engine(0, max_chunk=1 << 12, compact=compact)
    assert eng.check_base_tables() == (0, 0, 0)
    bits = 16 if compact else 24
    P = 2**255 - 19
    L = 2**252 + 27742317777372353535851937790883648493
    d = (-121665 * pow(121666, P - 2, P)) % P
    off = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]

    def val(limbs):
        return sum(int(l) << o for l, o in zip(limbs, off)) % P

    rng = np.random.default_rng(7)
    top = 1 << bits
    idx = [1, 2, 3, 31, 32, 33, 63, 64, top >> 1, top - 33, top - 32, top - 2, top - 1]
    idx += [int(x) for x in rng.integers(1, top, 8)]
    for which, shift in ((0, 0), (1, fd.BASE_TABLE_SHIFT)):
        for e in idx:
            ent = eng.base_entry(which, e)
            ypx, ymx, xy2d = val(ent[0:10]), val(ent[10:20]), val(ent[20:30])
            inv2 = (P + 1) // 2
            y, x = (ypx + ymx) * inv2 % P, (ypx - ymx) * inv2 % P
            assert xy2d == 2 * d * x * y % P, (which, e)
            want = ctypes.create_string_buffer(32)
            oracle.oracle_base_mul_encode(want, ((e << shift) % L).to_bytes(32, "little"))
            assert (y | ((x & 1) << 255)).to_bytes(32, "little") == want.raw, (which, e)
    eng.close()
