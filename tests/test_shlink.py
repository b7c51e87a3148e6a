"""The shared-memory link between a sandboxed verify tile and the GPU
process (fd_ed25519_hip_shlink).  CPU only: the
producer is the standalone tool (firedancer_amd/_lib/fd_shlink_producer)
running under seccomp strict mode, the service side is played by this
process with a stand-in verdict function; the GPU service itself is
tested in test_gpu_tile.py."""
import os
import random
import subprocess
import time
import uuid

import numpy as np
import pytest

from firedancer_amd import tile


def fake_verdict(payload):
    return (len(payload) % 7) - 3


def serve_fake(txl, vdl, proc, deadline_s=60.0):
    """Consume txn frags, answer each with fake_verdict, until EOS."""
    t0 = time.time()
    pending = []
    eos = False
    n = 0
    while True:
        while pending:
            sig, v = pending[0]
            if not vdl.publish(bytes([v & 0xff]), sig):
                break
            pending.pop(0)
        if eos and not pending:
            while not vdl.publish(b"", 0, tile.SHLINK_CTL_EOS):
                pass
            return n
        f = txl.consume()
        if f is None:
            if proc.poll() is not None and proc.returncode != 0:
                raise AssertionError(f"producer exited with {proc.returncode}")
            if time.time() - t0 > deadline_s:
                raise AssertionError("timeout")
            continue
        payload, sig, ctl = f
        if ctl & tile.SHLINK_CTL_EOS:
            eos = True
            continue
        assert sig == n
        pending.append((sig, fake_verdict(payload)))
        n += 1


@pytest.mark.parametrize("sandbox", [True, False])
@pytest.mark.parametrize("n,depth", [(1, 4), (3000, 64), (500, 1024)])
def test_sandboxed_producer_round_trip(tmp_path, sandbox, n, depth):
    rng = random.Random(n * 7 + depth)
    payloads = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 63, 64, 65, 200, 1232])))
                for _ in range(n)]
    path = str(tmp_path / "payloads.bin")
    tile.write_payload_file(path, payloads)
    tag = uuid.uuid4().hex[:12]
    txl = tile.ShLink(f"/fdt_tx_{tag}", depth, create=True)
    vdl = tile.ShLink(f"/fdt_vd_{tag}", depth, create=True)
    args = [tile.PRODUCER_BIN, txl.name, vdl.name, path] + ([] if sandbox else ["--no-sandbox"])
    proc = subprocess.Popen(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    try:
        served = serve_fake(txl, vdl, proc)
        out, err = proc.communicate(timeout=60)
    finally:
        if proc.poll() is None:
            proc.kill()
        txl.close()
        vdl.close()
    if proc.returncode == 3:
        pytest.skip(f"seccomp strict mode unavailable: {err.decode()}")
    assert proc.returncode == 0, err.decode()
    assert served == n
    got = np.frombuffer(out, np.int8)
    want = np.array([fake_verdict(p) for p in payloads], np.int8)
    assert np.array_equal(got, want)


def test_link_credits_and_overrun_free():
    """The producer never runs more than depth frags ahead of the consumer."""
    name = f"/fdt_cr_{uuid.uuid4().hex[:12]}"
    a = tile.ShLink(name, 16, create=True)
    b = tile.ShLink(name)
    try:
        sent = 0
        while a.publish(b"p%d" % sent, sent):
            sent += 1
        assert sent == 16
        for i in range(5):
            assert b.consume()[1] == i
        for _ in range(5):
            assert a.publish(b"p%d" % sent, sent)
            sent += 1
        assert not a.publish(b"x", 0)
        got = []
        while True:
            f = b.consume()
            if f is None:
                break
            got.append(f[1])
        assert got == list(range(5, sent))
    finally:
        b.close()
        a.close()


def test_join_missing_fails():
    with pytest.raises(Exception):
        tile.ShLink(f"/fdt_missing_{uuid.uuid4().hex[:12]}")
    assert os.path.exists(tile.PRODUCER_BIN)
