"""The accelerated verify tile under the reference's fd_mux_tile with the
real GPU verify service behind it (firedancer_amd/_lib/fd_verify_hip_service):
its published frags against the reference's fd_tile_verify on the same
stream, one tile and three tiles on one service process (the device's base
tables held once for all of them), and the service's failure policy.  The
CPU version with a stand-in service is test_mux_tile.py."""
import json
import os
import subprocess
import time
import uuid

import pytest

from firedancer_amd import tile
from test_mux_tile import HARNESS, MTU, assert_same_frags, cleanup, parse_out, run_harness
from txn_util import tile_workload

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SERVICE = os.path.join(REPO, "firedancer_amd", "_lib", "fd_verify_hip_service")

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not (os.path.exists(HARNESS) and os.path.exists(SERVICE)),
                                 reason="oracle/_ref/mux or the service binary not built")]


def start_service(app, tiles, *extra):
    env = dict(os.environ)
    env.setdefault("GPU_MAX_HW_QUEUES", "16")   # K tiles x 3 slots of one stream each
    svc = subprocess.Popen([SERVICE, "--prefix", f"/fd_vhip_{app}_", "--tiles", str(tiles), *extra],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    line = svc.stdout.readline()
    assert line.startswith("ready"), (line, svc.stderr.read() if svc.poll() is not None else "")
    return svc


def finish_service(svc):
    so, se = svc.communicate(timeout=60)
    return svc.returncode, json.loads(so.strip().splitlines()[-1]), se


@pytest.fixture(scope="module")
def stream(oracle, tmp_path_factory):
    frags = [p for p in tile_workload(oracle, 12, 2600) if len(p) <= MTU]
    path = str(tmp_path_factory.mktemp("gmux") / "payloads.bin")
    tile.write_payload_file(path, frags)
    return path, frags


@pytest.fixture(scope="module")
def reference_runs(stream, tmp_path_factory):
    path, _ = stream
    d = tmp_path_factory.mktemp("gmuxref")
    runs = {}
    for rr in ((1, 0), (3, 0), (3, 1), (3, 2)):
        out = str(d / f"ref_{rr[0]}_{rr[1]}.bin")
        p = run_harness("verify", path, out, rr=rr)
        so, se = p.communicate(timeout=120)
        assert p.returncode == 0, se[-2000:]
        runs[rr] = parse_out(out)
    return runs


@pytest.mark.parametrize("mode", [[], ["--gpu-parse"], ["--zero-copy"], ["--zero-copy", "--depth", "64"]],
                         ids=["host-parse", "gpu-parse", "zero-copy", "zero-copy-small-ring"])
def test_gpu_service_tile_matches_reference_tile(stream, reference_runs, tmp_path, mode):
    """The sandboxed tile under fd_mux_tile, the GPU service verifying in
    batches of 256 signatures with 3 in flight: the reference tile's frags,
    byte for byte and in order -- with the host parsing, the GPU parsing
    copies, and the GPU parsing payloads read in place from the txn link
    (the ring's wrap included: 2600 frags through a 1024-line link, and
    through a 64-line link whose ~84 KB dcache wraps every few batches, so
    batches take their payloads as two spans)."""
    path, frags = stream
    app = uuid.uuid4().hex[:10]
    svc = start_service(app, 1, "--batch", "256", "--depth", "1024", *mode)
    try:
        out = str(tmp_path / "hip.bin")
        p = run_harness("verify_hip", path, out, app=app, timeout=100)
        so, se = p.communicate(timeout=120)
        assert p.returncode == 0, se[-2000:]
        rc, res, se2 = finish_service(svc)
        assert rc == 0, se2[-2000:]
    finally:
        if svc.poll() is None:
            svc.kill()
        cleanup(app)
    assert res["txns"] == [len(frags)]
    assert_same_frags(reference_runs[(1, 0)], parse_out(out))


@pytest.fixture(scope="module")
def stream_30k(oracle, tmp_path_factory):
    """30,000 frags of the same mix, and the reference tile's output on them"""
    frags = [p for p in tile_workload(oracle, 30303, 30000) if len(p) <= MTU]
    d = tmp_path_factory.mktemp("gmux30k")
    path = str(d / "payloads.bin")
    tile.write_payload_file(path, frags)
    out = str(d / "ref.bin")
    p = run_harness("verify", path, out, rr=(1, 0))
    so, se = p.communicate(timeout=240)
    assert p.returncode == 0, se[-2000:]
    return path, frags, parse_out(out)


@pytest.mark.parametrize("mode", [[], ["--zero-copy"]], ids=["host-parse", "zero-copy"])
def test_gpu_service_tile_matches_reference_tile_at_scale(stream_30k, tmp_path, mode):
    """30,000 frags (≈90,000 signatures) through the sandboxed tile under
    fd_mux_tile and the GPU service (256-signature batches, the r16 form):
    the reference tile's frags byte for byte and in order."""
    path, frags, want = stream_30k
    app = uuid.uuid4().hex[:10]
    svc = start_service(app, 1, "--batch", "256", "--depth", "1024", *mode)
    try:
        out = str(tmp_path / "hip.bin")
        p = run_harness("verify_hip", path, out, app=app, timeout=200)
        so, se = p.communicate(timeout=240)
        assert p.returncode == 0, se[-2000:]
        rc, res, se2 = finish_service(svc)
        assert rc == 0, se2[-2000:]
    finally:
        if svc.poll() is None:
            svc.kill()
        cleanup(app)
    assert res["txns"] == [len(frags)]
    assert_same_frags(want, parse_out(out))


@pytest.mark.parametrize("mode", [["--zero-copy"], ["--zero-copy", "--links-per-thread", "3"],
                                  ["--links-per-thread", "2"], ["--zero-copy", "--cpus", "AFFINITY3"]],
                         ids=["zero-copy", "zero-copy-one-thread", "host-parse-two-per-thread", "zero-copy-pinned"])
def test_gpu_service_three_tiles_one_process(stream, reference_runs, tmp_path, mode):
    """Three verify tiles (seq % 3) on one service process (a thread per
    tile, or several tiles per thread): each publishes what the reference
    tile at its position does; the device's base tables (2 x 2 GiB) exist
    once in that process, and each further tile costs its own pipe only
    (batch-sized lane tables: well under 1 GiB)."""
    path, _ = stream
    app = uuid.uuid4().hex[:10]
    cpus = ",".join(str(c) for c in sorted(os.sched_getaffinity(0))[-3:])   # a service thread per tile, each on its CPU
    svc = start_service(app, 3, "--batch", "512", *[cpus if m == "AFFINITY3" else m for m in mode])
    try:
        procs = [(k, run_harness("verify_hip", path, str(tmp_path / f"hip{k}.bin"), app=app, rr=(3, k), timeout=100))
                 for k in range(3)]
        for k, p in procs:
            so, se = p.communicate(timeout=120)
            assert p.returncode == 0, (k, se[-2000:])
        rc, res, se2 = finish_service(svc)
        assert rc == 0, se2[-2000:]
    finally:
        if svc.poll() is None:
            svc.kill()
        cleanup(app)
    for k in range(3):
        assert_same_frags(reference_runs[(3, k)], parse_out(str(tmp_path / f"hip{k}.bin")))
    assert res["shared_device_bytes"] == 2 * (1 << 24) * 128
    assert all(0 < b < (1 << 30) for b in res["tile_device_bytes"]), res


def _vram_used():
    """Bytes of device 0's memory in use (rocm-smi), or None."""
    try:
        r = subprocess.run(["rocm-smi", "--showmeminfo", "vram", "--json"], capture_output=True, text=True, timeout=30)
        d = json.loads(r.stdout)
        card = d[sorted(d)[0]]
        return int(card["VRAM Total Used Memory (B)"])
    except Exception:
        return None


@pytest.mark.parametrize("per_thread", ["1", "2"], ids=["thread-per-tile", "one-thread"])
def test_gpu_service_tile_failure_ends_its_link_only(stream, per_thread):
    """Failure domains: tile 0 marks its txn link failed (as a tile does
    when the service broke the frag protocol); the service ends that link
    pair only and keeps serving tile 1, whose transactions still get their
    verdicts -- also when one service thread serves both; at the end it
    exits 3 with end codes [PROTOCOL, 0].  (A device failure still ends
    every link: test_gpu_service_fault.py.)"""
    _, frags = stream
    app = uuid.uuid4().hex[:10]
    svc = start_service(app, 2, "--batch", "256", "--links-per-thread", per_thread)
    links = []
    try:
        txl0, vdl0 = tile.ShLink(f"/fd_vhip_{app}_0_txn"), tile.ShLink(f"/fd_vhip_{app}_0_vd")
        txl1, vdl1 = tile.ShLink(f"/fd_vhip_{app}_1_txn"), tile.ShLink(f"/fd_vhip_{app}_1_vd")
        links = [txl0, vdl0, txl1, vdl1]
        t0 = time.time()
        while vdl0.heartbeat_query() == 0 and time.time() - t0 < 60:   # the service's first tick
            time.sleep(0.01)
        txl0.fail(tile.SHLINK_FAIL_PROTOCOL)
        t0 = time.time()
        while vdl0.status() == 0 and time.time() - t0 < 30:
            txl1.heartbeat(int(time.time() * 1e3))
            time.sleep(0.01)
        assert vdl0.status() == tile.SHLINK_FAIL_PROTOCOL
        assert vdl1.status() == 0                        # the other tile's link is untouched
        # tile 1 carries on: 200 transactions, then its end of stream
        sent, verdicts, beat = 0, [], 0
        t0 = time.time()
        while time.time() - t0 < 60:
            beat += 1
            txl1.heartbeat(beat)
            if sent < 200 and txl1.publish(frags[sent], sent << 32):
                sent += 1
            elif sent == 200 and txl1.publish(b"", 0, tile.SHLINK_CTL_EOS):
                sent += 1
            f = vdl1.consume()
            if f is not None:
                if f[2] & tile.SHLINK_CTL_EOS:
                    break
                verdicts.append((f[1] >> 32, f[0][0]))
        rc, res, se = finish_service(svc)
    finally:
        for link in links:
            link.close(unlink=False)
        if svc.poll() is None:
            svc.kill()
        cleanup(app)
    assert [k for k, _ in verdicts] == list(range(200))
    assert rc == 3, se[-2000:]
    assert res["end_codes"] == [tile.SHLINK_FAIL_PROTOCOL, 0]
    assert res["txns"][1] == 200


def test_gpu_service_exits_and_frees_the_device_when_its_tile_dies(stream, tmp_path):
    """The tile process is killed mid-stream: its heartbeat stops, the
    service ends the link pair after --tile-stale-ms, and with no tile left
    it exits (status 3) and removes its links; the device memory it held
    (4 GiB of base tables plus the pipe) is free again."""
    path, _ = stream
    app = uuid.uuid4().hex[:10]
    before = _vram_used()
    svc = start_service(app, 1, "--batch", "256", "--tile-stale-ms", "500")
    p = None
    try:
        p = run_harness("verify_hip", path, str(tmp_path / "hip.bin"), app=app, timeout=100, extra=("--rate", "300"))
        time.sleep(1.5)   # ~2600 frags at 300/s: mid-stream
        during = _vram_used()
        assert p.poll() is None
        p.kill()
        t0 = time.time()
        rc, res, se = finish_service(svc)
        dt = time.time() - t0
        left = sorted(f for f in os.listdir("/dev/shm") if f.startswith(f"fd_vhip_{app}_"))
        after = _vram_used()
    finally:
        if p is not None and p.poll() is None:
            p.kill()
        if svc.poll() is None:
            svc.kill()
        cleanup(app)
    assert rc == 3, se[-2000:]
    assert res["end_codes"] == [tile.SHLINK_FAIL_TILE_GONE]
    assert left == []
    assert dt < 15, dt
    if before is not None and during is not None and after is not None:
        assert during - before > (4 << 30)          # the service held its tables
        assert after - before < (256 << 20), (before, during, after)
