"""The verify service's lifecycle inside a validator, on CPU
with the stand-in service (oracle/_ref/mux/ref_vservice: the GPU service's
link code and lifecycle, the reference's verdicts) and sandboxed tiles
under the reference's fd_mux_tile (oracle/_ref/mux/mux_harness):

  - a tile that dies ends its own link pair; the service serves the other
    tiles on and exits (status 3, links removed) once every tile is gone;
  - a service killed with SIGKILL leaves its links behind; the next service
    reclaims them and comes up, while a second service next to a live one
    is refused;
  - the service exits when the process that started it dies, and on
    SIGTERM, ending every link (the tiles see the status and stop).

The reference supervises tiles the same way: a tile process that exits
takes the topology down (src/disco/topo/fd_topo_run.c:50-100) and liveness
is a cnc heartbeat (src/tango/cnc/fd_cnc.h:63-65,129-130).  The GPU
service's version of these checks is test_gpu_mux_tile.py."""
import json
import os
import signal
import subprocess
import sys
import time
import uuid

import pytest

from firedancer_amd import tile
from test_mux_tile import HARNESS, STANDIN, assert_same_frags, cleanup, parse_out, run_harness, start_standin
from test_mux_tile import reference_runs, stream  # noqa: F401  (fixtures)

pytestmark = pytest.mark.skipif(not (os.path.exists(HARNESS) and os.path.exists(STANDIN)),
                                reason="oracle/_ref/mux not built (make -C oracle ref-mux)")

STALE_MS = 400


def links_of(app):
    return sorted(f for f in os.listdir("/dev/shm") if f.startswith(f"fd_vhip_{app}_"))


def wait_exit(proc, bound_s):
    t0 = time.time()
    try:
        proc.wait(timeout=bound_s)
    except subprocess.TimeoutExpired:
        proc.kill()
        raise AssertionError(f"service still running {bound_s} s later")
    return time.time() - t0


def last_json(text):
    return json.loads(text.strip().splitlines()[-1])


def test_service_exits_once_every_tile_is_gone(stream, tmp_path):
    """Two tiles mid-stream (rate-limited producers) are killed with
    SIGKILL: their heartbeats stop, the service ends both links
    (FD_ED25519_HIP_SHLINK_FAIL_TILE_GONE) within the bound, removes the
    links and exits with status 3."""
    path, _ = stream
    app = uuid.uuid4().hex[:10]
    svc = start_standin(app, 2, "--tile-stale-ms", str(STALE_MS))
    tiles = []
    try:
        tiles = [run_harness("verify_hip", path, str(tmp_path / f"t{k}.bin"), app=app, rr=(2, k),
                             extra=("--rate", "500")) for k in range(2)]
        time.sleep(1.0)
        assert all(p.poll() is None for p in tiles)      # mid-stream
        for p in tiles:
            p.send_signal(signal.SIGKILL)
        dt = wait_exit(svc, 15)
        so, se = svc.communicate(timeout=10)
    finally:
        for p in tiles:
            if p.poll() is None:
                p.kill()
        if svc.poll() is None:
            svc.kill()
        leftover = links_of(app)
        cleanup(app)
    assert svc.returncode == 3, se[-2000:]
    assert last_json(so)["end_codes"] == [tile.SHLINK_FAIL_TILE_GONE] * 2
    assert "heartbeat stale" in se
    assert leftover == []
    assert dt < 10, dt


def test_service_serves_on_when_one_tile_dies(stream, reference_runs, tmp_path):  # noqa: F811
    """Three tiles (seq % 3) on one service; tile 2 is killed mid-stream.
    Its links end, tiles 0 and 1 run to the end and publish exactly what
    the reference tile at their positions does; the service then exits 3
    with end codes [0, 0, TILE_GONE]."""
    path, _ = stream
    app = uuid.uuid4().hex[:10]
    svc = start_standin(app, 3, "--tile-stale-ms", str(STALE_MS))
    procs = []
    try:
        procs = [run_harness("verify_hip", path, str(tmp_path / f"hip{k}.bin"), app=app, rr=(3, k),
                             extra=(("--rate", "500") if k == 2 else ())) for k in range(3)]
        time.sleep(0.5)
        procs[2].send_signal(signal.SIGKILL)
        for k in (0, 1):
            so, se = procs[k].communicate(timeout=120)
            assert procs[k].returncode == 0, (k, se[-2000:])
        wait_exit(svc, 15)
        so, se = svc.communicate(timeout=10)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        if svc.poll() is None:
            svc.kill()
        cleanup(app)
    assert svc.returncode == 3, se[-2000:]
    assert last_json(so)["end_codes"] == [0, 0, tile.SHLINK_FAIL_TILE_GONE]
    for k in (0, 1):
        assert_same_frags(reference_runs[(3, k)][1], parse_out(str(tmp_path / f"hip{k}.bin")))


def test_service_restarts_over_a_killed_services_links(stream, reference_runs, tmp_path):  # noqa: F811
    """A second service next to a live one is refused (exit 1: a running
    process holds the links).  SIGKILL leaves the first one's links in
    /dev/shm; a new service with the same prefix reclaims them, comes up,
    and a tile runs its stream to the reference's frags."""
    path, _ = stream
    app = uuid.uuid4().hex[:10]
    first = start_standin(app, 1)
    try:
        dup = subprocess.run([STANDIN, "--prefix", f"/fd_vhip_{app}_", "--tiles", "1", "--log-path", ""],
                             capture_output=True, text=True, timeout=30)
        assert dup.returncode == 1 and "a running process holds them" in dup.stderr, dup.stderr[-1000:]
        first.send_signal(signal.SIGKILL)
        first.wait(timeout=30)
        assert len(links_of(app)) == 2              # left behind
        second = start_standin(app, 1)              # reclaims them
        try:
            out = str(tmp_path / "hip.bin")
            p = run_harness("verify_hip", path, out, app=app)
            so, se = p.communicate(timeout=180)
            assert p.returncode == 0, se[-2000:]
            assert second.wait(timeout=30) == 0, second.stderr.read()[-2000:]
        finally:
            if second.poll() is None:
                second.kill()
        assert links_of(app) == []
    finally:
        if first.poll() is None:
            first.kill()
        cleanup(app)
    assert_same_frags(reference_runs[(1, 0)][1], parse_out(out))


def test_service_exits_when_its_parent_dies():
    """The service is started by a launcher process that is then killed
    (SIGKILL: no chance to clean up): the service notices (parent-death
    signal / parent pid watch), ends its links and removes them."""
    app = uuid.uuid4().hex[:10]
    code = ("import subprocess, sys, time; p = subprocess.Popen([%r, '--prefix', %r, '--tiles', '2', '--log-path', ''], "
            "stdout=subprocess.PIPE, text=True); print(p.pid, p.stdout.readline().strip(), flush=True); time.sleep(120)"
            % (STANDIN, f"/fd_vhip_{app}_"))
    launcher = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True)
    try:
        pid, ready = launcher.stdout.readline().split()[:2]
        pid = int(pid)
        assert ready == "ready" and len(links_of(app)) == 4
        launcher.send_signal(signal.SIGKILL)
        launcher.wait(timeout=30)
        t0 = time.time()
        while time.time() - t0 < 15:
            try:
                state = open(f"/proc/{pid}/stat").read().split(")")[-1].split()[0]
            except OSError:
                state = "gone"
            if state in ("gone", "Z", "X") and not links_of(app):
                break
            time.sleep(0.05)
        assert state in ("gone", "Z", "X"), state
        assert links_of(app) == []
        assert time.time() - t0 < 10
    finally:
        if launcher.poll() is None:
            launcher.kill()
        cleanup(app)


def test_sigterm_ends_every_link_and_the_tile_stops(stream, tmp_path):
    """SIGTERM to the service while a tile streams: every link is marked
    STOPPED, the service exits 3 with its links removed, and the sandboxed
    tile sees the status and stops (its fatal-condition exit) instead of
    waiting on the link."""
    path, _ = stream
    app = uuid.uuid4().hex[:10]
    svc = start_standin(app, 1)
    try:
        p = run_harness("verify_hip", path, str(tmp_path / "hip.bin"), app=app, timeout=60, extra=("--rate", "500"))
        time.sleep(0.8)
        svc.send_signal(signal.SIGTERM)
        wait_exit(svc, 15)
        so, se = svc.communicate(timeout=10)
        pso, pse = p.communicate(timeout=60)
    finally:
        if svc.poll() is None:
            svc.kill()
        cleanup(app)
    assert svc.returncode == 3, se[-2000:]
    assert last_json(so)["end_codes"] == [tile.SHLINK_FAIL_STOPPED]
    assert p.returncode not in (0, 3), pse[-2000:]
    assert f"verify service failed (link status {tile.SHLINK_FAIL_STOPPED})" in pse, pse[-2000:]
