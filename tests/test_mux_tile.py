"""The accelerated verify tile (integration/fd_verify_hip.c) inside the
reference's own tile runtime, next to the reference's fd_tile_verify on the
same stream (§8(f) row 1).

oracle/_ref/mux/mux_harness starts a tile the way fd_topo_run_tile does
(privileged_init, the tile's own seccomp filter, unprivileged_init, then
the reference's fd_mux_tile run loop, src/disco/mux/fd_mux.c), with a
producer on the quic -> verify link and a reliable consumer on the verify ->
dedup link; both tiles' published frags (sig, size, bytes, order) must
agree.  CPU only: the GPU verify service is played by oracle/_ref/mux/
ref_vservice, the reference's own after_frag + fd_txn_verify behind the
same links and protocol (the real service is tested the same way in
test_gpu_mux_tile.py).  Also the failure policy across the split: a service
that dies, marks its links failed, or breaks the protocol ends the tile
within its bound instead of leaving it blocked."""
import json
import os
import struct
import subprocess
import time
import uuid

import pytest

from firedancer_amd import tile
from txn_util import tile_workload

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the sanitizer run (tests/test_sanitizers.py) points this at oracle/_ref/mux-san
MUX = os.environ.get("FD_TEST_MUX_DIR") or os.path.join(REPO, "oracle", "_ref", "mux")
HARNESS = os.path.join(MUX, "mux_harness")
STANDIN = os.path.join(MUX, "ref_vservice")

pytestmark = pytest.mark.skipif(not (os.path.exists(HARNESS) and os.path.exists(STANDIN)),
                                reason="oracle/_ref/mux not built (make -C oracle ref-mux)")

MTU = 1232


# the sanitizer run: the sanitizer runtime needs system calls the verify
# tile's seccomp policy forbids, so the tile runs unsandboxed there
SANITIZE = bool(os.environ.get("FD_TEST_SANITIZE"))


def run_harness(kind, payloads, out, app="harness", rr=(1, 0), depth=4096, timeout=120, extra=()):
    args = [HARNESS, kind, payloads, out, "--app", app, *(["--rr-cnt", str(rr[0]), "--rr-idx", str(rr[1])] if rr else []),
            "--depth", str(depth), "--timeout", str(timeout), "--log-path", "", *extra,
            *(["--no-sandbox"] if SANITIZE else [])]
    return subprocess.Popen(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)


def parse_out(path):
    b = open(path, "rb").read()
    out, i = [], 0
    while i < len(b):
        sig, sz = struct.unpack_from("<QI", b, i)
        out.append((sig, b[i + 12:i + 12 + sz]))
        i += 12 + sz
    return out


def assert_same_frags(ref, hip):
    """Same frags, sigs and order.  The one byte allowed to differ is the
    alignment pad between an odd-sized payload and its fd_txn_t: the
    reference tile never writes it (fd_verify.c:102-113), so it holds
    whatever the out dcache held there before; the accelerated tile writes
    0."""
    assert len(ref) == len(hip)
    for k, ((s1, a), (s2, b)) in enumerate(zip(ref, hip)):
        assert s1 == s2, (k, hex(s1), hex(s2))
        assert len(a) == len(b), (k, len(a), len(b))
        psz = struct.unpack_from("<H", a, len(a) - 2)[0]
        diff = [j for j in range(len(a)) if a[j] != b[j]]
        assert diff == [] or (diff == [psz] and psz % 2 == 1), (k, diff[:8])
        if psz % 2:
            assert b[psz] == 0


def start_standin(app, tiles, *extra):
    svc = subprocess.Popen([STANDIN, "--prefix", f"/fd_vhip_{app}_", "--tiles", str(tiles), "--log-path", "", *extra],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    line = svc.stdout.readline()
    assert line.startswith("ready"), (line, svc.stderr.read() if svc.poll() is not None else "")
    return svc


def cleanup(app):
    for f in os.listdir("/dev/shm"):
        if f.startswith(f"fd_vhip_{app}_"):
            try:
                os.unlink(os.path.join("/dev/shm", f))
            except OSError:
                pass


@pytest.fixture(scope="module")
def stream(oracle, tmp_path_factory):
    frags = [p for p in tile_workload(oracle, 11, 2600) if len(p) <= MTU]
    path = str(tmp_path_factory.mktemp("mux") / "payloads.bin")
    tile.write_payload_file(path, frags)
    return path, frags


@pytest.fixture(scope="module")
def reference_runs(stream, tmp_path_factory):
    """The reference's fd_tile_verify under the same runtime, per round-robin
    position (sandboxed under its own policy)."""
    path, _ = stream
    d = tmp_path_factory.mktemp("muxref")
    runs = {}
    for rr in ((1, 0), (3, 0), (3, 1), (3, 2)):
        out = str(d / f"ref_{rr[0]}_{rr[1]}.bin")
        p = run_harness("verify", path, out, rr=rr)
        so, se = p.communicate(timeout=180)
        assert p.returncode == 0, se[-2000:]
        runs[rr] = (json.loads(so.strip().splitlines()[-1]), parse_out(out))
    return runs


@pytest.mark.parametrize("depth,hold", [(16384, 1), (64, 1), (64, 300)], ids=["deep", "tight-credits", "batched"])
def test_mux_tile_matches_reference_tile(stream, reference_runs, tmp_path, depth, hold):
    """One accelerated tile under fd_mux_tile against fd_tile_verify: the
    same published frags, byte for byte and in order (dedup, bad signatures,
    parse failures, 17+ signers included).  tight-credits: the txn link has
    64 lines, so during_frag waits for room; batched: the service holds its
    verdicts until 300 are pending, as GPU batches do."""
    path, frags = stream
    app = uuid.uuid4().hex[:10]
    svc = start_standin(app, 1, "--depth", str(depth), "--hold", str(hold))
    try:
        out = str(tmp_path / "hip.bin")
        p = run_harness("verify_hip", path, out, app=app)
        so, se = p.communicate(timeout=180)
        assert p.returncode == 0, se[-2000:]
        assert svc.wait(timeout=30) == 0, svc.stderr.read()[-2000:]
    finally:
        if svc.poll() is None:
            svc.kill()
        cleanup(app)
    res = json.loads(so.strip().splitlines()[-1])
    ref_res, ref = reference_runs[(1, 0)]
    assert res["frags"] == ref_res["frags"] == len(frags)
    assert res["sandbox"] == (0 if SANITIZE else 1)
    assert_same_frags(ref, parse_out(out))
    assert len(ref) > len(frags) // 2


def test_three_tiles_round_robin_one_service(stream, reference_runs, tmp_path):
    """Three accelerated verify tiles (seq % 3, fd_verify.c:46) served by one
    service process over three link pairs, run concurrently; each publishes
    what the reference tile at its round-robin position publishes."""
    path, _ = stream
    app = uuid.uuid4().hex[:10]
    svc = start_standin(app, 3)
    try:
        procs = [(k, run_harness("verify_hip", path, str(tmp_path / f"hip{k}.bin"), app=app, rr=(3, k)))
                 for k in range(3)]
        for k, p in procs:
            so, se = p.communicate(timeout=180)
            assert p.returncode == 0, (k, se[-2000:])
        assert svc.wait(timeout=30) == 0, svc.stderr.read()[-2000:]
    finally:
        if svc.poll() is None:
            svc.kill()
        cleanup(app)
    total = 0
    for k in range(3):
        ref = reference_runs[(3, k)][1]
        assert_same_frags(ref, parse_out(str(tmp_path / f"hip{k}.bin")))
        total += len(ref)
    # the three positions partition the stream: together they publish what
    # one tile would, up to dedup (each tile has its own tcache, as in the reference)
    assert total >= len(reference_runs[(1, 0)][1])


def _normalized(frags):
    """(sig, bytes) with the alignment pad byte zeroed (assert_same_frags),
    sorted: the published set, whatever order the links were read in"""
    out = []
    for sig, b in frags:
        psz = struct.unpack_from("<H", b, len(b) - 2)[0]
        if psz % 2:
            b = b[:psz] + b"\0" + b[psz + 1:]
        out.append((sig, bytes(b)))
    return sorted(out)


@pytest.mark.parametrize("kind", ["verify", "verify_hip"])
def test_shared_quic_link_k_tiles_in_one_topology(stream, reference_runs, tmp_path, kind):
    """fdctl's topology: one quic -> verify link that three
    verify tiles read, each keeping seq % 3 == its kind id (fd_verify.c:
    36-47) and publishing to its own verify -> dedup link, one consumer
    reading all three -- five spinning threads, not three harnesses.  The
    reference tile and the accelerated one (stand-in service, three link
    pairs) publish together exactly what the three single-position
    reference runs publish."""
    path, frags = stream
    app = uuid.uuid4().hex[:10]
    svc = start_standin(app, 3) if kind == "verify_hip" else None
    try:
        out = str(tmp_path / "k3.bin")
        p = run_harness(kind, path, out, app=app, rr=None, extra=("--tiles", "3"))
        so, se = p.communicate(timeout=180)
        assert p.returncode == 0, se[-2000:]
        if svc is not None:
            assert svc.wait(timeout=30) == 0, svc.stderr.read()[-2000:]
    finally:
        if svc is not None and svc.poll() is None:
            svc.kill()
        cleanup(app)
    res = json.loads(so.strip().splitlines()[-1])
    assert res["tiles_running"] == 3 and res["threads"] == 5 and res["frags"] == len(frags)
    want = [f for k in range(3) for f in reference_runs[(3, k)][1]]
    assert res["published"] == len(want)
    assert _normalized(parse_out(out)) == _normalized(want)


def _expect_tile_stops(stream, tmp_path, svc_args, needle, bound_s):
    path, _ = stream
    app = uuid.uuid4().hex[:10]
    svc = start_standin(app, 1, *svc_args)
    try:
        t0 = time.time()
        p = run_harness("verify_hip", path, str(tmp_path / "hip.bin"), app=app, timeout=60)
        so, se = p.communicate(timeout=90)
        dt = time.time() - t0
    finally:
        if svc.poll() is None:
            svc.kill()
        cleanup(app)
    assert p.returncode != 0 and p.returncode != 3, (p.returncode, so, se[-2000:])   # 3: the harness's own timeout
    assert needle in se, se[-2000:]
    assert dt < bound_s, dt
    return se


def test_tile_stops_when_service_dies(stream, tmp_path):
    """The service is killed mid-stream (SIGKILL after 400 verdicts): its
    heartbeat stops, and the sandboxed tile ends with FD_LOG_ERR within its
    1 s staleness bound (plus the harness's start-up) instead of waiting on
    the link forever -- the reference's reaction to a fatal tile condition,
    which takes the validator down."""
    _expect_tile_stops(stream, tmp_path, ("--die-after", "400"), "heartbeat stale", 15.0)


def test_tile_stops_when_service_fails(stream, tmp_path):
    """The service's failure policy: on a GPU failure it stops publishing and
    marks its links failed (here after 400 verdicts); the tile sees the
    status at its next housekeeping and ends."""
    _expect_tile_stops(stream, tmp_path, ("--fail-after", "400"), "verify service failed (link status -1700)", 15.0)


@pytest.mark.parametrize("bad", ["order", "size", "trailer", "verdict"])
def test_tile_refuses_protocol_violations(stream, tmp_path, bad):
    """A service that answers out of order, with a SUCCESS verdict that
    carries no trailer, with a trailer that belongs to a payload of another
    size, or with a verdict that does not exist: the tile marks its txn
    link failed (so the service stops too) and ends; nothing malformed is
    published."""
    path, frags = stream
    app = uuid.uuid4().hex[:10]
    txl = tile.ShLink(f"/fd_vhip_{app}_0_txn", 1024, create=True)
    vdl = tile.ShLink(f"/fd_vhip_{app}_0_vd", 1024, create=True)
    try:
        p = run_harness("verify_hip", path, str(tmp_path / "hip.bin"), app=app, timeout=60)
        t0 = time.time()
        n, beat = 0, 0

        def answer(body, sig):
            """publish a verdict frag, waiting for credit while the tile
            lives (it returns credits in groups, or when it finds the
            verdict link empty); False once it has exited"""
            while not vdl.publish(body, sig):
                if p.poll() is not None:
                    return False
                vdl.heartbeat(beat)
            return True
        while p.poll() is None and time.time() - t0 < 60:
            beat += 1
            vdl.heartbeat(beat)
            f = txl.consume()
            if f is None:
                continue
            payload, sig, ctl = f
            if n < 20:   # a few good filtered answers first
                ok = answer(bytes([0xFF]), sig)
            elif bad == "order":
                ok = answer(bytes([0xFF]), sig + (1 << 32))
            elif bad == "size":
                ok = answer(b"\0", sig)   # SUCCESS without the trailer
            elif bad == "trailer":   # fd_txn_t-sized, but its payload_sz is not this payload's
                ok = answer(b"\0" + bytes(64) + (len(payload) + 1).to_bytes(2, "little"), sig)
            else:
                ok = answer(bytes([0x05]), sig)
            if not ok:
                break
            n += 1
        so, se = p.communicate(timeout=30)
        status = txl.status()
    finally:
        if p.poll() is None:
            p.kill()
        txl.close()
        vdl.close()
    assert p.returncode not in (0, 3), (p.returncode, se[-2000:])
    assert "broke the frag protocol" in se, se[-2000:]
    assert status == tile.SHLINK_FAIL_PROTOCOL
    assert parse_out(str(tmp_path / "hip.bin")) == [] if os.path.exists(str(tmp_path / "hip.bin")) else True
