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


# the sanitizer run (tests/test_sanitizers.py): the sanitizer runtime needs
# system calls that seccomp strict mode forbids, so the producer runs
# unsandboxed there (its code and checks are the same)
NO_SANDBOX = ["--no-sandbox"] if os.environ.get("FD_TEST_SANITIZE") else []


def fake_verdict(payload):
    return (len(payload) % 7) - 3


def fake_trailer(payload):
    """A SUCCESS verdict frag carries the published frag's trailer (the
    fd_txn_t, then the u16 payload_sz): here a stand-in of some length."""
    return b"\x5a" * (len(payload) % 13) + len(payload).to_bytes(2, "little")


def assembled(payload):
    """what the tile publishes: payload, the alignment pad (0), the trailer
    (fd_ed25519_hip_frag_assemble)"""
    return payload + b"\0" * (len(payload) % 2) + fake_trailer(payload)


def serve_fake(txl, vdl, proc, deadline_s=60.0, stop_after=None, fail_after=None):
    """Consume txn frags, answer each with fake_verdict, until EOS; tick the
    heartbeat of the verdict link as the GPU service does.  stop_after:
    go silent (no heartbeat, no verdicts) after that many verdicts, as a
    killed service would; fail_after: mark both links failed instead."""
    t0 = time.time()
    pending = []
    eos = False
    n = 0
    sent = 0
    beat = 0
    while True:
        if stop_after is not None and sent >= stop_after:
            return n
        if fail_after is not None and sent >= fail_after:
            txl.fail(-1000 - 700)
            vdl.fail(-1000 - 700)
            return n
        beat += 1
        vdl.heartbeat(beat)
        while pending:
            sig, v, fr = pending[0]
            if not vdl.publish(bytes([v & 0xff]) + fr, sig):
                break
            pending.pop(0)
            sent += 1
            if stop_after is not None and sent >= stop_after:
                break
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
        v = fake_verdict(payload)
        pending.append((sig, v, fake_trailer(payload) if v == 0 else b""))
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
    if NO_SANDBOX and sandbox:
        args += NO_SANDBOX
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
    got = np.frombuffer(out[:n], np.int8)
    want = np.array([fake_verdict(p) for p in payloads], np.int8)
    assert np.array_equal(got, want)
    assert tile.parse_producer_frags(out[n:]) == [assembled(p) for p in payloads if fake_verdict(p) == 0]


@pytest.mark.parametrize("how", ["killed", "failed"])
def test_producer_stops_when_service_dies(tmp_path, how):
    """Liveness across the sandbox split: the stand-in service stops
    mid-stream -- silent (no heartbeat, no verdicts: a killed or hung
    process) or marking both links failed (its failure policy) -- while the
    producer is under seccomp strict mode; the producer notices with the
    time-stamp counter alone and exits with status 4 within its bound
    instead of waiting on credits forever."""
    rng = random.Random(5)
    n = 4000
    payloads = [bytes(rng.getrandbits(8) for _ in range(rng.choice([1, 64, 200]))) for _ in range(n)]
    path = str(tmp_path / "payloads.bin")
    tile.write_payload_file(path, payloads)
    tag = uuid.uuid4().hex[:12]
    txl = tile.ShLink(f"/fdt_tx_{tag}", 64, create=True)
    vdl = tile.ShLink(f"/fdt_vd_{tag}", 64, create=True)
    # the staleness bound well above a loaded host's pauses (the fake
    # service is Python, and under the sanitizer suites a pause of a few
    # hundred ms would let "stale" win over the explicit failure mark)
    proc = subprocess.Popen([tile.PRODUCER_BIN, txl.name, vdl.name, path, "--stale-ms", "1500", *NO_SANDBOX],
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    try:
        if how == "killed":
            serve_fake(txl, vdl, proc, stop_after=500)
        else:
            serve_fake(txl, vdl, proc, fail_after=500)
        t0 = time.time()
        out, err = proc.communicate(timeout=30)
        dt = time.time() - t0
    finally:
        if proc.poll() is None:
            proc.kill()
        txl.close()
        vdl.close()
    if proc.returncode == 3:
        pytest.skip(f"seccomp strict mode unavailable: {err.decode()}")
    assert proc.returncode == 4, (proc.returncode, err.decode())
    assert (b"stale" if how == "killed" else b"marked a link failed") in err
    assert dt < 8.0


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


def test_credits_come_back_in_groups_and_when_the_link_runs_empty():
    """Lazy credit exchange (fd_fctl's refill, src/tango/fctl/fd_fctl.h):
    the consumer publishes its count every depth/16 frags and whenever it
    finds the link empty; the producer never runs more than depth ahead of
    the count it last saw, so a credit can arrive late but never early."""
    name = f"/fdt_lz_{uuid.uuid4().hex[:12]}"
    depth = 64                                   # credits come back 4 at a time
    a = tile.ShLink(name, depth, create=True)
    b = tile.ShLink(name)
    try:
        sent = 0
        while a.publish(b"q", sent):
            sent += 1
        assert sent == depth
        for i in range(3):                        # fewer than depth/16: no credit returned yet
            assert b.consume()[1] == i
        assert not a.publish(b"x", 0)
        assert b.consume()[1] == 3                # the 4th frag: 4 credits come back
        for _ in range(4):
            assert a.publish(b"q", sent)
            sent += 1
        assert not a.publish(b"x", 0)
        got = []
        while (f := b.consume()) is not None:     # drained: the empty poll returns the rest
            got.append(f[1])
        assert got == list(range(4, sent))
        for _ in range(depth):                    # the whole window is free again
            assert a.publish(b"q", sent)
            sent += 1
        assert not a.publish(b"x", 0)
    finally:
        b.close()
        a.close()


def test_join_missing_fails():
    with pytest.raises(Exception):
        tile.ShLink(f"/fdt_missing_{uuid.uuid4().hex[:12]}")
    assert os.path.exists(tile.PRODUCER_BIN)


# shared layout (host/fd_ed25519_hip_shlink.c): a 128-byte header
# (magic, depth, chunk_cnt, mtu, pad, consumed, pad) then 32-byte mcache
# lines (seq, sig, chunk u32, sz u16, ctl u16, tsorig, tspub)
_HDR, _LINE = 128, 32


def _shm(name):
    return open("/dev/shm" + name, "r+b", buffering=0)


def _poke(f, off, fmt, *vals):
    import struct
    f.seek(off)
    f.write(struct.pack(fmt, *vals))


def test_hostile_header_is_ignored_after_join():
    """A compromised peer rewrites depth / chunk_cnt / mtu in the shared
    header after both sides joined: both sides keep the geometry they
    validated at join, so publish and consume stay inside the mapping and
    the MTU-sized buffer (the service must not trust the tile)."""
    name = f"/fdt_hh_{uuid.uuid4().hex[:12]}"
    a = tile.ShLink(name, 8, create=True)
    b = tile.ShLink(name)
    try:
        with _shm(name) as f:
            _poke(f, 8, "<QQQ", 1 << 40, 1 << 40, 65535)
        # a frag above the MTU is refused by the producer's local MTU
        with pytest.raises(Exception):
            a.publish(b"\0" * (tile.SHLINK_MTU + 1), 0)
        for i in range(8):
            assert a.publish(bytes([i]) * 100, i)
        assert not a.publish(b"x", 99)   # credits still counted against depth 8
        for i in range(8):
            assert b.consume() == (bytes([i]) * 100, i, 0)
    finally:
        b.close()
        a.close()


@pytest.mark.parametrize("field", ["chunk", "sz"])
def test_hostile_frag_is_refused(field):
    """A published line whose chunk points past the dcache or whose size is
    above the MTU: consume refuses it (-1, an overrun for the caller)
    instead of copying out of bounds (the reference tile's own check,
    src/app/fdctl/run/tiles/fd_verify.c:67)."""
    name = f"/fdt_hf_{uuid.uuid4().hex[:12]}"
    a = tile.ShLink(name, 8, create=True)
    b = tile.ShLink(name)
    try:
        assert a.publish(b"hello", 7)
        with _shm(name) as f:
            line = _HDR + 0 * _LINE
            if field == "chunk":
                _poke(f, line + 16, "<I", 0xFFFFFFF0)
            else:
                _poke(f, line + 20, "<H", 65535)
        with pytest.raises(Exception):
            b.consume()
    finally:
        b.close()
        a.close()


def test_join_rejects_bad_geometry():
    """A header whose geometry differs from what create makes (MTU, depth
    not a power of two) is refused at join."""
    for off, fmt, val in ((24, "<Q", 65535), (8, "<Q", 6)):
        name = f"/fdt_bg_{uuid.uuid4().hex[:12]}"
        a = tile.ShLink(name, 8, create=True)
        try:
            with _shm(name) as f:
                _poke(f, off, fmt, val)
            with pytest.raises(Exception):
                tile.ShLink(name)
        finally:
            a.close()


# ---- versioning, restarts, the consumer's heartbeat watch (ABI 5) ----

SHLINK_HDR_PROTO_OFF = 48     # shlink_hdr_t: magic, depth, chunk_cnt, mtu, heartbeat, status, proto, creator
SHLINK_HDR_CREATOR_OFF = 56


def _hdr_word(name, off, value=None):
    import mmap
    import struct
    with open("/dev/shm" + name, "r+b") as f:
        m = mmap.mmap(f.fileno(), 64)
        old = struct.unpack_from("<Q", m, off)[0]
        if value is not None:
            struct.pack_into("<Q", m, off, value)
        m.close()
    return old


def test_link_records_protocol_and_creator_and_join_refuses_another_protocol():
    """create writes FD_ED25519_HIP_SHLINK_PROTO and its pid into the
    header; a link of another protocol (a tile or service of another
    revision) is refused at join with EPROTO instead of exchanging frags."""
    name = f"/fdt_pr_{uuid.uuid4().hex[:12]}"
    link = tile.ShLink(name, 64, create=True)
    try:
        assert _hdr_word(name, SHLINK_HDR_PROTO_OFF) == tile.SHLINK_PROTO
        assert _hdr_word(name, SHLINK_HDR_CREATOR_OFF) == os.getpid()
        peer = tile.ShLink(name)
        peer.close()
        _hdr_word(name, SHLINK_HDR_PROTO_OFF, tile.SHLINK_PROTO - 1)   # the verdict protocol of ABI 4
        with pytest.raises(tile.HipError, match="EPROTO"):
            tile.ShLink(name)
    finally:
        link.close()


def test_create_reclaims_a_killed_creators_link_but_not_a_live_ones():
    """A service killed with SIGKILL leaves its links in /dev/shm: the next
    create of the same name reclaims them (its creator has exited); while
    the creator lives, create still refuses (EEXIST)."""
    import signal
    import sys
    name = f"/fdt_rc_{uuid.uuid4().hex[:12]}"
    code = ("import sys, time; sys.path.insert(0, %r); from firedancer_amd import tile; "
            "l = tile.ShLink(%r, 64, create=True); print('up', flush=True); time.sleep(60)"
            % (os.path.dirname(os.path.dirname(os.path.abspath(tile.__file__))), name))
    p = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True)
    try:
        assert p.stdout.readline().strip() == "up"
        assert _hdr_word(name, SHLINK_HDR_CREATOR_OFF) == p.pid
        with pytest.raises(tile.HipError, match="EEXIST"):
            tile.ShLink(name, 64, create=True)          # its creator lives
        p.send_signal(signal.SIGKILL)
        p.wait(timeout=30)
        assert os.path.exists("/dev/shm" + name)        # left behind
        link = tile.ShLink(name, 128, create=True)      # reclaimed, made anew
        assert link.depth == 128 and _hdr_word(name, SHLINK_HDR_CREATOR_OFF) == os.getpid()
        link.close()
        assert not os.path.exists("/dev/shm" + name)
    finally:
        if p.poll() is None:
            p.kill()
        if os.path.exists("/dev/shm" + name):
            os.unlink("/dev/shm" + name)


def test_heartbeat_watch():
    """fd_ed25519_hip_shlink_watch: 1 until the producer first ticks, 0
    while the heartbeat changes, -1 once it has been unchanged for longer
    than the bound, 0 again when it moves; a bound <= 0 is never stale."""
    name = f"/fdt_hb_{uuid.uuid4().hex[:12]}"
    link = tile.ShLink(name, 64, create=True)
    try:
        w, ms = tile.ShLinkWatch(), 1000000
        assert w.check(link, 0, 100 * ms) == 1
        assert w.check(link, 10_000 * ms, 100 * ms) == 1       # never ticked: not stale, however long
        link.heartbeat(1)
        assert w.check(link, 10_001 * ms, 100 * ms) == 0
        assert w.check(link, 10_100 * ms, 100 * ms) == 0       # at the bound
        assert w.check(link, 10_102 * ms, 100 * ms) == -1      # past it
        assert w.check(link, 10_102 * ms, -1) == 0             # no bound
        link.heartbeat(2)
        assert w.check(link, 10_103 * ms, 100 * ms) == 0
        assert w.check(link, 10_150 * ms, 100 * ms) == 0
    finally:
        link.close()


def test_a_live_creators_link_is_not_reclaimed_whatever_its_pid_says():
    """a pid is not meaningful across PID namespaces.  The
    creator's claim is an exclusive flock held on the link's object for the
    link's lifetime: a creator whose recorded pid names no process here (as
    a live service in another PID namespace would look) still keeps its
    link, and create refuses with EEXIST; once the creator closes it the
    name is free."""
    name = f"/fdt_ns_{uuid.uuid4().hex[:12]}"
    link = tile.ShLink(name, 64, create=True)
    try:
        _hdr_word(name, SHLINK_HDR_CREATOR_OFF, (1 << 31) - 7)   # no such process in this namespace
        with pytest.raises(tile.HipError, match="EEXIST"):
            tile.ShLink(name, 64, create=True)
        peer = tile.ShLink(name)   # the link itself still works for its peers
        peer.close()
    finally:
        link.close()
    assert not os.path.exists("/dev/shm" + name)
    again = tile.ShLink(name, 64, create=True)
    again.close()


def test_protocol5_link_reclaimed_only_when_its_creator_is_gone():
    """A protocol-5 creator held no flock on its link, so a free lock on such
    a link does not mean its creator exited: create reclaims it only when
    the recorded creator pid no longer exists."""
    import struct
    name = f"/fdt_p5_{uuid.uuid4().hex[:12]}"
    path = "/dev/shm" + name
    hdr = bytearray(4096)
    struct.pack_into("<QQQQ", hdr, 0, 0xfd25519517a4c0df, 64, 128, 1232)
    struct.pack_into("<QQ", hdr, SHLINK_HDR_PROTO_OFF, 5, os.getpid())   # a live creator, no lock held
    with open(path, "wb") as f:
        f.write(hdr)
    try:
        with pytest.raises(tile.HipError, match="EEXIST"):
            tile.ShLink(name, 64, create=True)
        assert os.path.exists(path)
        _hdr_word(name, SHLINK_HDR_CREATOR_OFF, (1 << 31) - 7)   # no such process in this namespace
        link = tile.ShLink(name, 64, create=True)
        assert _hdr_word(name, SHLINK_HDR_PROTO_OFF) == tile.SHLINK_PROTO == 6
        link.close()
    finally:
        if os.path.exists(path):
            os.unlink(path)
