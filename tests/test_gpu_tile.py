"""GPU parity of the verify-tile layer (include/fd_ed25519_hip_tile.h): the
batched tile's verdict stream against the reference tile replayed
sequentially on the same frags (oracle/_ref: fd_txn_parse + FD_TCACHE_* +
fd_ed25519_verify_batch_single_msg), the latency mode through the ring,
the pipe, and the multi-device pool."""
import random

import numpy as np
import pytest

from txn_util import Signer, random_txn, ref_lib, ref_vtile, ref_vtile_frags, tile_workload

pytestmark = pytest.mark.gpu


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


@pytest.fixture(scope="module")
def frags(oracle):
    return tile_workload(oracle, 2024, 3000)


@pytest.mark.parametrize("gpu_parse", [False, True])
@pytest.mark.parametrize("batch_sigs,slot_cnt", [(64, 3), (1000, 2), (16, 1), (4096, 4), (1, 2)])  # 1: raised to 16
def test_vtile_matches_reference_tile(tile, ref, frags, batch_sigs, slot_cnt, gpu_parse):
    """Verdicts, dedup tags and the published frags (payload, pad, fd_txn_t,
    payload_sz: after_frag, src/app/fdctl/run/tiles/fd_verify.c:102-133)
    against the reference tile replayed sequentially."""
    want, want_tags, want_frags = ref_vtile_frags(ref, frags)
    vt = tile.VerifyTile(0, slot_cnt=slot_cnt, batch_sigs=batch_sigs, gpu_parse=gpu_parse)
    got, tags, got_frags = vt.run(frags, frags=True)
    vt.close()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(int(i), int(got[i]), int(want[i])) for i in bad[:10]]
    ok = want != -3
    assert np.array_equal(tags[ok], want_tags[ok])
    bad = [i for i in range(len(frags)) if got_frags[i] != want_frags[i]]
    assert not bad, (bad[:5], [(got_frags[i] or b"")[-40:].hex() for i in bad[:2]],
                     [(want_frags[i] or b"")[-40:].hex() for i in bad[:2]])
    assert sum(f is not None for f in want_frags) > len(frags) // 2
    # some published fd_txn_t exceed the device parser's 64-byte trailer slot
    assert any(f is not None and len(f) - 2 - ((len(fr) + 1) & ~1) > 64 for f, fr in zip(want_frags, frags))


@pytest.fixture(scope="module")
def frags_30k(oracle, ref):
    frags = tile_workload(oracle, 5150, 30000)
    return frags, ref_vtile_frags(ref, frags)


@pytest.mark.parametrize("gpu_parse", [False, True])
def test_vtile_at_scale_in_the_c5_shape(tile, frags_30k, gpu_parse):
    """30,000 frags (about 90,000 signatures: bad signatures, duplicates
    near and across tcache evictions, unparseable and 17+-signer payloads)
    through the C5 shape -- 256-signature batches, 8 slots, so every batch
    takes the r16 form -- against the reference tile replayed on the same
    frags: verdicts, dedup tags and published frags."""
    frags, (want, want_tags, want_frags) = frags_30k
    vt = tile.VerifyTile(0, slot_cnt=8, batch_sigs=256, gpu_parse=gpu_parse)
    got, tags, got_frags = vt.run(frags, frags=True)
    vt.close()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(int(i), int(got[i]), int(want[i])) for i in bad[:10]]
    ok = want != -3
    assert np.array_equal(tags[ok], want_tags[ok])
    bad = [i for i in range(len(frags)) if got_frags[i] != want_frags[i]]
    assert not bad, bad[:5]
    assert (want == 0).sum() > len(frags) // 2 and (want != 0).sum() > len(frags) // 20


def test_vtile_dedup_across_batches(tile, ref, oracle):
    """Duplicates of a transaction in an earlier batch and in the same batch,
    and copies that come back after the tcache (depth 16) evicted them."""
    rng = random.Random(1)
    signer = Signer(oracle, 1)
    base = [random_txn(signer, rng, 1) for _ in range(40)]
    seq = base[:5] + [base[0]] + base[5:21] + [base[4]] + base[21:38] + [base[20], base[21], base[30], base[38],
                                                                         base[38]]
    want, _ = ref_vtile(ref, seq)
    vt = tile.VerifyTile(0, slot_cnt=2, batch_sigs=4)
    got, _ = vt.run(seq)
    vt.close()
    assert got.tolist() == want.tolist()
    assert want.tolist()[5] == -2 and want.tolist()[-3:] == [-2, 0, -2]  # dups of base[0], base[30], base[38]
    assert want.tolist()[22] == 0                                         # base[4] came back after eviction


@pytest.mark.parametrize("gpu_parse", [False, True])
def test_latency_run(tile, ref, frags, gpu_parse):
    frags = [p for p in frags if len(p) <= tile.TXN_MTU]  # a dcache frag is at most the TPU MTU
    want, _ = ref_vtile(ref, frags)
    lat, got, res = tile.latency_run(frags, offered_txn_per_s=20000.0, batch_sigs=256, slot_cnt=3, ring_depth=1024,
                                     gpu_parse=gpu_parse)
    assert res["ring_overruns"] == 0
    assert np.array_equal(got, want)
    assert (lat > 0).all() and res["batches"] > 1
    assert res["achieved_txn_per_s"] > 0.5 * 20000.0


def test_latency_run_unpaced(tile, ref, frags):
    frags = [p for p in frags if len(p) <= tile.TXN_MTU]
    want, _ = ref_vtile(ref, frags)
    lat, got, res = tile.latency_run(frags, offered_txn_per_s=0.0, batch_sigs=512, slot_cnt=4, ring_depth=256)
    assert res["ring_overruns"] == 0
    assert np.array_equal(got, want)


def _pool_set(oracle, n, seed):
    rng = random.Random(seed)
    signer = Signer(oracle, seed)
    msgs, off, sz, sigs, pubs = bytearray(), [], [], bytearray(), bytearray()
    for i in range(n):
        priv, pub = signer.key() if i % 50 == 0 else signer.keys[-1]
        m = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 300)))
        s = bytearray(signer.sign(m, priv, pub))
        if i % 9 == 4:
            s[rng.randrange(64)] ^= 1
        off.append(len(msgs)); sz.append(len(m)); msgs += m; sigs += s; pubs += pub
    return (np.frombuffer(bytes(msgs), np.uint8).copy(), np.array(off, np.uint64), np.array(sz, np.uint32),
            np.frombuffer(bytes(sigs), np.uint8).copy(), np.frombuffer(bytes(pubs), np.uint8).copy())


@pytest.mark.parametrize("mode", ["staged", "direct", "scattered"])
def test_pool_vs_oracle(tile, oracle, mode):
    """The multi-device pool (round-robin batches, one feeder thread per
    entry; device 0 repeated on a one-GPU box) against the oracle: staged
    from pageable arrays, DMA'd in place from registered ones, and with the
    messages scattered in reverse order (their span too wide to DMA as one
    range: packed)."""
    from conftest import oracle_many
    msgs, off, sz, sigs, pubs = _pool_set(oracle, 3000, 9)
    if mode == "scattered":
        # messages stored back to front, with 4 KB gaps: each batch's span
        # is many times its bytes
        order = np.arange(len(sz))[::-1]
        parts, noff, pos = [], np.zeros(len(sz), np.uint64), 0
        for i in order:
            parts.append(np.zeros(4096, np.uint8))
            pos += 4096
            parts.append(msgs[off[i]:off[i] + sz[i]])
            noff[i] = pos
            pos += int(sz[i])
        msgs, off = np.concatenate(parts), noff
    want = oracle_many(oracle, dict(msgs=msgs, msg_off=off, msg_sz=sz, sigs=sigs.reshape(-1, 64),
                                    pubs=pubs.reshape(-1, 32)), 0)
    assert (want != 0).sum() > 0
    out = np.zeros(len(sz), np.int8)
    for devices, batch in [([0], 1000), ([0, 0], 256), ([0, 0, 0], 7)]:
        out[:] = 99
        if mode == "staged":
            got, sec, st = tile.pool_verify(devices, msgs, off, sz, sigs, pubs, batch_sigs=batch, slot_cnt=2,
                                            out=out, stats=True)
            assert st["direct_batches"] == 0 and st["staged_batches"] > 0
        else:
            with tile.HostRegistration(msgs, off, sz, sigs, pubs, out):
                got, sec, st = tile.pool_verify(devices, msgs, off, sz, sigs, pubs, batch_sigs=batch, slot_cnt=3,
                                                out=out, stats=True)
            if mode == "direct":
                assert st["staged_batches"] == 0 and st["direct_batches"] == -(-len(sz) // batch)
            elif batch >= 256:   # a 7-signature batch's span is small enough to DMA as it is
                assert st["staged_batches"] > 0
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, (mode, devices, [(int(i), int(got[i]), int(want[i])) for i in bad[:8]])
        assert sec > 0


def test_h2d_bandwidth_probe(tile):
    gbps = tile.h2d_gbps(0, 64 << 20, 4)
    assert gbps > 1.0


def test_txn_payload_generator(tile, ref):
    """bench.py's C5 transactions: GPU-signed, parseable, all valid, and the
    reference tile agrees."""
    from firedancer_amd import ed25519, workload
    eng = ed25519.Engine(0, max_chunk=1 << 12)
    for signers in (1, 3):
        pay, size = workload.txn_payloads(eng, 300, 5, msg_sz=200 + 64 * signers, signers=signers)
        payloads = [bytes(p) for p in pay]
        t = tile.txn_parse(payloads[0])
        assert t is not None and t["signature_cnt"] == signers
        assert size - t["message_off"] == 200 + 64 * signers
        want, _ = ref_vtile(ref, payloads)
        assert (want == 0).all()
        vt = tile.VerifyTile(0, slot_cnt=2, batch_sigs=128)
        got, _ = vt.run(payloads)
        vt.close()
        assert (got == 0).all()
    eng.close()


def test_device_parse_on_mutated_fixtures(tile, ref):
    """fd_txn_parse on the device (GPU-parse tile) against the reference's
    parser: the reference's 6 fixtures and 9000 mutations of them, plus the
    whole verdict (parse, dedup, verify) against the reference tile."""
    import glob
    import os
    from conftest import GOLDEN
    from txn_util import mutate, ref_parse
    fx = [open(p, "rb").read() for p in sorted(glob.glob(os.path.join(GOLDEN, "txn", "*.bin")))]
    rng = random.Random(7)
    corpus = list(fx)
    for p in fx:
        for _ in range(1500):
            q = p
            for _ in range(rng.randrange(1, 4)):
                q = mutate(rng, q)
            corpus.append(q)
    want, _ = ref_vtile(ref, corpus)
    vt = tile.VerifyTile(0, slot_cnt=3, batch_sigs=512, gpu_parse=True)
    got, _ = vt.run(corpus)
    vt.close()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(int(i), int(got[i]), int(want[i])) for i in bad[:10]]
    parsed = np.array([ref_parse(ref, p)[0] is not None for p in corpus])
    assert np.array_equal(got != tile.TXN_PARSE_FAILED, parsed)
    assert 500 < parsed.sum() < len(corpus) - 500


@pytest.mark.parametrize("gpu_parse", [False, True])
@pytest.mark.parametrize("load", ["frags", "frags_30k"])
def test_sandboxed_tile_with_gpu_service(tile, ref, request, tmp_path, gpu_parse, load):
    """the verify tile in seccomp strict mode (the
    standalone producer: memory operations, write and _exit only) and the
    GPU in a separate service process, connected by two shared-memory
    links.  The verdict stream equals the reference tile's -- on the 3000
    fixture frags and on the 30,000-frag workload."""
    import subprocess
    import sys
    import uuid
    frags = request.getfixturevalue(load)
    if load == "frags_30k":
        frags = frags[0]
    frags = [p for p in frags if len(p) <= tile.TXN_MTU]
    want, _, want_frags = ref_vtile_frags(ref, frags)
    path = str(tmp_path / "payloads.bin")
    tile.write_payload_file(path, frags)
    tag = uuid.uuid4().hex[:12]
    txl = tile.ShLink(f"/fdg_tx_{tag}", 256, create=True)
    vdl = tile.ShLink(f"/fdg_vd_{tag}", 256, create=True)
    repo = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); from firedancer_amd import tile; "
            "a = tile.ShLink(%r); b = tile.ShLink(%r); "
            "print(tile.vservice_run(a, b, batch_sigs=256, slot_cnt=3, gpu_parse=%r))"
            % (repo, txl.name, vdl.name, gpu_parse))
    svc = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    prod = subprocess.Popen([tile.PRODUCER_BIN, txl.name, vdl.name, path], stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE)
    try:
        out, perr = prod.communicate(timeout=90)
        sout, serr = svc.communicate(timeout=30)
    finally:
        for p in (prod, svc):
            if p.poll() is None:
                p.kill()
        txl.close()
        vdl.close()
    if prod.returncode == 3:
        pytest.skip(f"seccomp strict mode unavailable: {perr.decode()}")
    assert svc.returncode == 0, serr.decode()
    assert prod.returncode == 0, perr.decode()
    got = np.frombuffer(out[:len(frags)], np.int8)
    bad = np.nonzero(got != want)[0]
    assert len(got) == len(want) and len(bad) == 0, [(int(i), int(got[i]), int(want[i])) for i in bad[:10]]
    assert b"'txn_cnt': %d" % len(frags) in sout
    # the frags the sandboxed tile receives for its SUCCESS transactions are
    # the reference tile's published frags
    assert tile.parse_producer_frags(out[len(frags):]) == [f for f in want_frags if f is not None]


def test_pipe_stages_in_place_and_rejects_out_of_range(tile, adversarial):
    """The raw pipe API (fd_ed25519_hip_pipe_*): a batch staged in a slot's
    pinned arrays verifies to the reference's codes, several batches in
    flight; a message or transaction range outside what was staged is
    refused on the host (ERR_INVAL, nothing enqueued) -- the kernels would
    read out of bounds -- and the pipe keeps working after it."""
    d = adversarial
    want = d["codes_avx512"]
    n = len(want)
    cap = 512
    p = tile.Pipe(0, slot_cnt=2, sig_cap=cap, msg_cap=cap * 1300, txn_cap=cap)

    def stage(slot, i0, i1):
        a = tile.Pipe.arrays(slot)
        pos = 0
        for k, i in enumerate(range(i0, i1)):
            o, z = int(d["msg_off"][i]), int(d["msg_sz"][i])
            a["msgs"][pos:pos + z] = d["msgs"][o:o + z]
            a["msg_off"][k], a["msg_sz"][k] = pos, z
            a["sigs"][64 * k:64 * k + 64] = d["sigs"][i]
            a["pubs"][32 * k:32 * k + 32] = d["pubs"][i]
            pos += z
        return a, pos

    got = np.zeros(n, np.int8)
    spans, inflight = [(i, min(i + cap, n)) for i in range(0, n, cap)], []
    for i0, i1 in spans:
        s = p.acquire()
        while s is None:
            done = p.poll(True)
            j0, j1 = done.contents.user, done.contents.user + done.contents.sig_cnt
            got[j0:j1] = tile.Pipe.arrays(done)["sig_out"][:j1 - j0]
            p.release(done)
            s = p.acquire()
        a, pos = stage(s, i0, i1)
        s.contents.user = i0
        assert p.submit(s, i1 - i0, pos) == 0
    while True:
        done = p.poll(True)
        if done is None:
            break
        j0, j1 = done.contents.user, done.contents.user + done.contents.sig_cnt
        got[j0:j1] = tile.Pipe.arrays(done)["sig_out"][:j1 - j0]
        p.release(done)
    assert np.array_equal(got, want)

    # out-of-range stagings are refused before any device work
    s = p.acquire()
    a, pos = stage(s, 0, 8)
    a["msg_off"][3] = pos                      # message starts at the end, size > 0
    assert p.submit(s, 8, pos) != 0
    a["msg_off"][3], a["msg_sz"][3] = 0, pos + 1   # runs one byte past the staged bytes
    assert p.submit(s, 8, pos) != 0
    a, pos = stage(s, 0, 8)
    a["txn_first"][0], a["txn_sig_cnt"][0] = 6, 3  # signatures 6..8 of 8 staged
    assert p.submit(s, 8, pos, txn_cnt=1) != 0
    a["txn_first"][0], a["txn_sig_cnt"][0] = 5, 3
    assert p.submit(s, 8, pos, txn_cnt=1) == 0
    done = p.poll(True)
    assert np.array_equal(tile.Pipe.arrays(done)["sig_out"][:8], want[:8])
    p.release(done)
    s = p.acquire()
    a = tile.Pipe.arrays(s)
    a["msgs"][:64] = 1
    a["msg_off"][0], a["msg_sz"][0] = 10, 100      # raw mode: payload past the 64 bytes staged
    assert p.submit_txns(s, 1, 64) != 0
    p.close()


@pytest.mark.parametrize("hs,hd,waves", [(4, 2, 2), (4, 4, 2), (4, 4, 4), (4, 4, 8), (4, 0, 2), (0, 0, 2)],
                         ids=["host-decode2", "host-decode4", "host-decode4-four-waves", "host-decode4-eight-waves",
                              "host-scalars", "device-path"])
def test_pipe_tiny_batches_every_path(tile, adversarial, mixed_order, batch, hs, hd, waves):
    """Batches of one to four signatures (a tile at a low load), through the
    host-scalar path (prep16's decode blocks + dsm16 reading the staged
    block in place, transaction codes combined on the host), with the
    decompressions on the submitting thread too for batches of at most hd
    signatures (the group equation alone, reading the points in place: over
    dsm16s's four or eight waves or dsm16's two), and through the device path: single signatures of the adversarial and mixed-order sets,
    and the batch_single_msg transactions of one to four signatures (the
    priority rule included), against the reference's codes."""
    tile.pipe_set_host_scalars(hs)
    tile.pipe_set_host_decode(hd)
    tile.pipe_set_split_waves(waves)
    try:
        p = tile.Pipe(0, slot_cnt=3, sig_cap=256, msg_cap=256 * 1300, txn_cap=256)
        jobs = []   # (msgs [(bytes)], sigs, pubs, txn?, want)
        for d in (adversarial, mixed_order):
            n = len(d["msg_sz"])
            for i in range(0, n, 5):
                o, z = int(d["msg_off"][i]), int(d["msg_sz"][i])
                k = min(1 + (i // 5) % 4, n - i)   # 1..4 signatures a batch
                idx = list(range(i, i + k))
                jobs.append(([bytes(d["msgs"][int(d["msg_off"][j]):int(d["msg_off"][j]) + int(d["msg_sz"][j])])
                              for j in idx], [d["sigs"][j] for j in idx], [d["pubs"][j] for j in idx], False,
                             [int(d["codes_avx512"][j]) for j in idx]))
        for b, pre in ((batch, ""), (mixed_order, "b_")):
            for t in range(len(b[pre + "txn_cnt"])):
                c = int(b[pre + "txn_cnt"][t])
                if c < 1 or c > 4:
                    continue
                o, z, f = int(b[pre + "txn_msg_off"][t]), int(b[pre + "txn_msg_sz"][t]), int(b[pre + "txn_first"][t])
                m = bytes(b[pre + "msgs"][o:o + z])
                jobs.append(([m] * c, [b[pre + "sigs"][f + j] for j in range(c)],
                             [b[pre + "pubs"][f + j] for j in range(c)], True, [int(b[pre + "codes_avx512"][t])]))
        assert sum(j[3] for j in jobs) > 40

        results = {}

        def drain(wait):
            done = p.poll(wait)
            if done is None:
                return False
            k = done.contents.user
            a = tile.Pipe.arrays(done)
            results[k] = (list(a["txn_out"][:1]) if jobs[k][3] else list(a["sig_out"][:done.contents.sig_cnt]))
            p.release(done)
            return True

        for k, (msgs, sigs, pubs, txn, want) in enumerate(jobs):
            s = p.acquire()
            while s is None:
                drain(True)
                s = p.acquire()
            a = tile.Pipe.arrays(s)
            pos = 0
            for q, (m, sg, pk) in enumerate(zip(msgs, sigs, pubs)):
                if txn and q:   # one shared message
                    a["msg_off"][q], a["msg_sz"][q] = a["msg_off"][0], len(m)
                else:
                    a["msgs"][pos:pos + len(m)] = np.frombuffer(m, np.uint8)
                    a["msg_off"][q], a["msg_sz"][q] = pos, len(m)
                    pos += len(m)
                a["sigs"][64 * q:64 * q + 64] = sg
                a["pubs"][32 * q:32 * q + 32] = pk
            if txn:
                a["txn_first"][0], a["txn_sig_cnt"][0] = 0, len(sigs)
            s.contents.user = k
            assert p.submit(s, len(sigs), pos, txn_cnt=1 if txn else 0) == 0
        while drain(True):
            pass
        p.close()
        bad = [(k, results.get(k), j[4]) for k, j in enumerate(jobs) if [int(x) for x in results.get(k, [])] != j[4]]
        assert not bad, bad[:10]
    finally:
        tile.pipe_set_host_scalars(4)
        tile.pipe_set_host_decode(4)
        tile.pipe_set_split_waves(2)
