"""CPU tests of the verify-tile host layer (include/fd_ed25519_hip_tile.h):
the fd_txn_parse restatement against the reference's parser (compiled from
its sources into oracle/_ref) on the reference's own fixtures
(tests/golden/txn/, copied from src/ballet/txn/fixtures/) and on mutated /
synthesized payloads, and the tcache against the reference's FD_TCACHE_*
macros through the sequential verify-tile replay."""
import glob
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN
from txn_util import (message, mutate, random_txn, ref_after_frag, ref_lib, ref_parse, ref_parse_raw, ref_vtile,
                      tile_workload, txn, Signer)


@pytest.fixture(scope="module")
def tile():
    from firedancer_amd import tile as t
    return t


@pytest.fixture(scope="module")
def ref():
    lib = ref_lib()
    if lib is None:
        pytest.skip("oracle/_ref not built")
    return lib


def fixtures():
    return [open(p, "rb").read() for p in sorted(glob.glob(os.path.join(GOLDEN, "txn", "*.bin")))]


def _same(tile, ref, p):
    mine = tile.txn_parse(p)
    want, _ = ref_parse(ref, p)
    if want is None:
        assert mine is None, p.hex()
    else:
        assert mine is not None, p.hex()
        assert tuple(mine.values()) == want, (mine, want)


def test_reference_fixtures(tile, ref):
    fx = fixtures()
    assert len(fx) == 6
    for p in fx:
        _same(tile, ref, p)
    # the reference test's expectations (src/ballet/txn/test_txn_parse.c): 1-4, 6 parse, 5 does not
    ok = [tile.txn_parse(p) is not None for p in fx]
    assert ok == [True, True, True, True, False, True]
    t1 = tile.txn_parse(fx[0])
    assert t1["transaction_version"] == 0xFF and fx[0][t1["recent_blockhash_off"]] == 155


def test_mutated_fixtures(tile, ref):
    rng = random.Random(7)
    for p in fixtures():
        for _ in range(1500):
            q = p
            for _ in range(rng.randrange(1, 4)):
                q = mutate(rng, q)
            _same(tile, ref, q)


def test_synthesized(tile, ref, oracle):
    rng = random.Random(11)
    signer = Signer(oracle, 11)
    for _ in range(300):
        p = random_txn(signer, rng, rng.choice([1, 2, 5, 12, 17]), v0=rng.random() < 0.5, msg_pad=rng.randrange(400))
        _same(tile, ref, p)
        for _ in range(10):
            _same(tile, ref, mutate(rng, p))


def test_edge_encodings(tile, ref):
    accts = [bytes([i]) * 32 for i in range(3)]
    sig = b"\x01" * 64
    good = txn([sig], message(1, accts, ro_unsigned=1, instrs=[(2, [0, 1], b"x")]))
    _same(tile, ref, good)
    assert tile.txn_parse(good) is not None
    cases = [
        good + b"\0",                                                  # trailing byte
        txn([sig], message(1, accts, instrs=[(0, [0], b"")])),         # program id = fee payer
        txn([sig], message(1, accts, instrs=[(3, [0], b"")])),         # program id out of range
        txn([sig], message(1, accts, instrs=[(2, [5], b"")])),         # account index out of range
        txn([sig], message(1, accts[:1], instrs=[])),                  # one account, no instruction: valid
        txn([sig], message(1, accts, ro_signed=1, instrs=[])),         # fee payer read-only
        txn([sig], message(2, accts, instrs=[])),                      # header count != signature count
        txn([sig], message(1, accts, version=1)),                      # unknown version
        txn([sig], message(1, accts, version=0, luts=[(b"\0" * 32, [], [])])),  # empty lookup table
        txn([sig], message(1, accts, version=0, luts=[(b"\0" * 32, [0], [])], instrs=[(2, [3], b"")])),
        b"\x00", b"", b"\x80\x01",
        bytes([0x81, 0x00]) + sig,                                     # non-minimal compact-u16 count
        good[:-1],
    ]
    for p in cases:
        _same(tile, ref, p)
    big = txn([sig], message(1, accts, instrs=[(2, [0], b"\0" * 1200)]))
    assert len(big) > 1232
    _same(tile, ref, big)


def _same_full(tile, ref, p):
    """fd_txn_t byte for byte (instr[], address table lookups, padding) and
    the frag after_frag publishes (payload, pad, fd_txn_t, payload_sz)."""
    assert tile.txn_parse_full(p) == ref_parse_raw(ref, p), p.hex()
    assert tile.txn_frag(p) == ref_after_frag(ref, p), p.hex()


def test_full_txn_and_frag_on_fixtures_and_mutations(tile, ref):
    rng = random.Random(17)
    n_ok = 0
    for p in fixtures():
        _same_full(tile, ref, p)
        for _ in range(1500):
            q = p
            for _ in range(rng.randrange(1, 4)):
                q = mutate(rng, q)
            _same_full(tile, ref, q)
            n_ok += tile.txn_parse_full(q) is not None
    assert n_ok > 500


def test_full_txn_and_frag_synthesized(tile, ref, oracle):
    """Legacy and v0, 1..9 instructions, 0..4 lookup tables (fd_txn_t from
    20 to ~150 bytes), odd and even payload sizes (the pad byte)."""
    rng = random.Random(19)
    signer = Signer(oracle, 19)
    sizes = set()
    for _ in range(400):
        v0 = rng.random() < 0.5
        p = random_txn(signer, rng, rng.choice([1, 2, 5, 12]), v0=v0, msg_pad=rng.randrange(300),
                       instr_n=rng.randrange(1, 10), lut_n=rng.randrange(0, 5))
        _same_full(tile, ref, p)
        t = tile.txn_parse_full(p)
        if t is not None:
            sizes.add((len(t), len(p) & 1))
        for _ in range(5):
            _same_full(tile, ref, mutate(rng, p))
    assert len({s for s, _ in sizes}) > 10 and {o for _, o in sizes} == {0, 1}


class PyTCache:
    """Straight restatement of FD_TCACHE_QUERY / INSERT for the model check."""

    def __init__(self, depth, map_cnt):
        self.depth, self.m = depth, map_cnt
        self.ring = [0] * depth
        self.map = [0] * map_cnt
        self.oldest = 0

    def _probe(self, tag):
        i = tag & (self.m - 1)
        while True:
            t = self.map[i]
            if t == tag:
                return True, i
            if t == 0:
                return False, i
            i = (i + 1) & (self.m - 1)

    def query(self, tag):
        return self._probe(tag)[0]

    def _remove(self, tag):
        if tag == 0:
            return
        found, slot = self._probe(tag)
        if not found:
            return
        while True:
            self.map[slot] = 0
            hole = slot
            while True:
                slot = (slot + 1) & (self.m - 1)
                t = self.map[slot]
                if t == 0:
                    return
                start = t & (self.m - 1)
                if not (((hole < start) and (start <= slot)) or ((hole > slot) and ((hole < start) or (start <= slot)))):
                    break
            self.map[hole] = self.map[slot]

    def insert(self, tag):
        found, i = self._probe(tag)
        if found:
            return True
        self.map[i] = tag
        ev = self.ring[self.oldest]
        self.ring[self.oldest] = tag
        self.oldest = (self.oldest + 1) % self.depth
        self._remove(ev)
        return False


@pytest.mark.parametrize("depth,map_cnt", [(16, 64), (4, 8), (1, 4), (30, 32)])
def test_tcache_model(tile, depth, map_cnt):
    rng = random.Random(depth * 1000 + map_cnt)
    a, b = tile.TCache(depth, map_cnt), PyTCache(depth, map_cnt)
    pool = [rng.getrandbits(64) or 1 for _ in range(3 * depth)]
    # colliding tags (same low bits) exercise probing and backward-shift deletion
    pool += [(rng.getrandbits(58) << 6) | 5 for _ in range(depth)] + [0]
    for _ in range(20000):
        tag = rng.choice(pool)
        if rng.random() < 0.5:
            assert a.query(tag) == b.query(tag)
        else:
            assert a.insert(tag) == b.insert(tag)


def test_tcache_geometry(tile):
    with pytest.raises(ValueError):
        tile.TCache(16, 48)
    with pytest.raises(ValueError):
        tile.TCache(16, 16)


def test_reference_vtile_replay_semantics(ref, oracle):
    """The reference harness's sequential tile on a small crafted stream."""
    rng = random.Random(3)
    signer = Signer(oracle, 3)
    a = random_txn(signer, rng, 1)
    bad = random_txn(signer, rng, 2, bad_sig=True)
    junk = b"\x05\x00"
    v, tags = ref_vtile(ref, [a, a, bad, junk, a])
    assert v.tolist() == [0, -2, -1, -3, -2]
    assert int(tags[0]) == int.from_bytes(a[1:9], "little")


def test_workload_classes(ref, oracle):
    ps = tile_workload(oracle, 5, 400)
    v, _ = ref_vtile(ref, ps)
    counts = {int(k): int((v == k).sum()) for k in (0, -1, -2, -3)}
    assert all(c > 0 for c in counts.values()), counts
