"""The GPU verify service's failure policy with a real HIP failure (VERDICT
r2, next #3): the fault-injection build fails the third batch's launch
after its copies are on the stream.  The service must stop publishing,
mark both links failed with the code, report it, and exit without a hang;
the sandboxed tile side (the strict-mode producer) must see the failed
status and exit with its defined status (4) instead of waiting on verdicts
that will never come.  The verdicts it received before the failure are the
ones it would have received anyway (all SUCCESS here).  The service runs
in a child process, since the library is chosen at import."""
import os
import subprocess
import sys
import time
import uuid

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

FAULT_LIB = os.path.join(REPO, "firedancer_amd", "_lib", "libfd_ed25519_hip_faultinj.so")


@pytest.mark.parametrize("per_thread", [1, 2], ids=["thread-per-tile", "one-thread"])
def test_service_marks_links_failed_on_launch_failure(tmp_path, per_thread):
    if not os.path.exists(FAULT_LIB):
        pytest.fail(f"{FAULT_LIB} not built (make -C firedancer_amd/csrc)")
    from firedancer_amd import ed25519, tile, workload
    eng = ed25519.Engine(0, max_chunk=1 << 14)
    pay, _ = workload.txn_payloads(eng, 2000, 4242, msg_sz=200)
    eng.close()
    path = str(tmp_path / "payloads.bin")
    tile.write_payload_file(path, pay)
    tag = uuid.uuid4().hex[:12]
    txl = tile.ShLink(f"/fdf_tx_{tag}", 1024, create=True)
    vdl = tile.ShLink(f"/fdf_vd_{tag}", 1024, create=True)
    # a second tile's link pair on the same service, idle: a device failure
    # ends it too (the device is not trusted for anyone), marked STOPPED
    tx2 = tile.ShLink(f"/fdf_tx2_{tag}", 1024, create=True)
    vd2 = tile.ShLink(f"/fdf_vd2_{tag}", 1024, create=True)
    code = ("import sys; sys.path.insert(0, %r); from firedancer_amd import ed25519, tile; "
            "assert ed25519.LIB_PATH.endswith('libfd_ed25519_hip_faultinj.so'); "
            "a, b = tile.ShLink(%r), tile.ShLink(%r); c, d = tile.ShLink(%r), tile.ShLink(%r); "
            "rc, st = tile.vservice_serve([a, c], [b, d], batch_sigs=256, slot_cnt=3, gpu_parse=False, links_per_thread=%d); "
            "print(rc, [s['end_code'] for s in st]); "
            "print(tile._lib.fd_ed25519_hip_last_error().decode(), file=sys.stderr); sys.exit(1 if rc else 0)"
            % (REPO, txl.name, vdl.name, tx2.name, vd2.name, per_thread))
    env = dict(os.environ, FD_ED25519_HIP_LIB=FAULT_LIB)
    t0 = time.time()
    svc = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env)
    prod = subprocess.Popen([tile.PRODUCER_BIN, txl.name, vdl.name, path], stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE)
    try:
        pout, perr = prod.communicate(timeout=120)
        sout, serr = svc.communicate(timeout=60)
        dt = time.time() - t0
        status = (txl.status(), vdl.status())
        status2 = (tx2.status(), vd2.status())
    finally:
        for p in (prod, svc):
            if p.poll() is None:
                p.kill()
        for link in (txl, vdl, tx2, vd2):
            link.close()
    if prod.returncode == 3:
        pytest.skip(f"seccomp strict mode unavailable: {perr.decode()}")
    # the service reports the injected failure (a HIP error code, never an abort)
    assert svc.returncode not in (0, -6), (svc.returncode, serr.decode()[-2000:])
    assert b"injected launch failure" in serr, serr.decode()[-2000:]
    # both links carry the failure code the service marked, the other
    # tile's links the stop it caused
    assert status[0] == status[1] and status[0] < 0, status
    assert status2 == (tile.SHLINK_FAIL_STOPPED, tile.SHLINK_FAIL_STOPPED), status2
    rc, ends = sout.decode().split(" ", 1)
    assert int(rc) == status[0] and ends.strip() == f"[{status[0]}, {tile.SHLINK_FAIL_STOPPED}]", sout
    # the sandboxed tile side saw it and stopped with its defined status
    assert prod.returncode == 4, (prod.returncode, perr.decode())
    assert b"marked a link failed" in perr, perr.decode()
    assert dt < 90, dt
    # it never got a verdict that was not SUCCESS (the stream is all valid);
    # it wrote nothing (it exits before its output on a failure)
    assert len(pout) == 0 or (np.frombuffer(pout[:2000], np.int8) == 0).all()


SERVICE_BIN = os.path.join(REPO, "firedancer_amd", "_lib", "fd_verify_hip_service")


def test_service_exits_on_a_gpu_hang_without_waiting_on_the_device(tmp_path):
    """a hung GPU must not hang the service.  The fault-injection
    build holds the third batch on the device for 4 s (a bounded stand-in
    for a hang: one sleeping wave that exits on its own) and the service's
    hang bound is 0.5 s: the service must mark every link failed
    (FD_ED25519_HIP_ERR_TIMEOUT on the tile's pair, STOPPED on the idle
    second tile's), print its JSON line with gpu_hang true and exit with
    status 2 well before the stalled batch would have finished -- freeing
    its engines, or the HIP runtime's teardown, would wait on the device."""
    if not os.path.exists(FAULT_LIB):
        pytest.fail(f"{FAULT_LIB} not built (make -C firedancer_amd/csrc)")
    from firedancer_amd import ed25519, tile, workload
    eng = ed25519.Engine(0, max_chunk=1 << 14)
    pay, _ = workload.txn_payloads(eng, 3000, 4343, msg_sz=200)
    eng.close()
    path = str(tmp_path / "payloads.bin")
    tile.write_payload_file(path, pay)
    libdir = tmp_path / "lib"
    libdir.mkdir()
    (libdir / "libfd_ed25519_hip.so").symlink_to(FAULT_LIB)   # the name the service's RUNPATH loads
    env = dict(os.environ, LD_LIBRARY_PATH=str(libdir), FD_ED25519_HIP_FAULT_STALL_MS="4000")
    prefix = f"/fdh_{uuid.uuid4().hex[:10]}_"
    svc = subprocess.Popen([SERVICE_BIN, "--prefix", prefix, "--tiles", "2", "--batch", "256", "--slots", "3",
                            "--gpu-hang-ms", "500", "--no-parent-watch"], stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, env=env, text=True)
    prod = None
    try:
        line = svc.stdout.readline()
        assert line.startswith("ready 2"), (line, svc.stderr.read()[-2000:] if svc.poll() is not None else "")
        txl, vdl = tile.ShLink(prefix + "0_txn"), tile.ShLink(prefix + "0_vd")
        tx2, vd2 = tile.ShLink(prefix + "1_txn"), tile.ShLink(prefix + "1_vd")
        t0 = time.time()
        prod = subprocess.Popen([tile.PRODUCER_BIN, txl.name, vdl.name, path], stdout=subprocess.PIPE,
                                stderr=subprocess.PIPE)
        sout, serr = svc.communicate(timeout=30)
        dt = time.time() - t0
        pout, perr = prod.communicate(timeout=30)
        status, status2 = (txl.status(), vdl.status()), (tx2.status(), vd2.status())
        left = [f for f in os.listdir("/dev/shm") if f.startswith(prefix[1:])]
        for link in (txl, vdl, tx2, vd2):
            link.close(unlink=False)
    finally:
        for p in (prod, svc):
            if p is not None and p.poll() is None:
                p.kill()
        for f in os.listdir("/dev/shm"):
            if f.startswith(prefix[1:]):
                os.unlink(os.path.join("/dev/shm", f))
    if prod.returncode == 3:
        pytest.skip(f"seccomp strict mode unavailable: {perr.decode()}")
    assert svc.returncode == 2, (svc.returncode, serr[-2000:])
    assert "did not complete within 0.5 s (GPU hang)" in serr and "exiting without device teardown" in serr, serr[-2000:]
    import json
    res = json.loads(sout.strip().splitlines()[-1])
    assert res["gpu_hang"] is True and res["end_codes"] == [-110, tile.SHLINK_FAIL_STOPPED], res
    assert status == (-110, -110) and status2 == (tile.SHLINK_FAIL_STOPPED, tile.SHLINK_FAIL_STOPPED), (status, status2)
    # out within the hang bound and a margin, not after the 4 s the device holds the batch
    assert dt < 3.5, dt
    assert prod.returncode == 4 and b"marked a link failed" in perr, (prod.returncode, perr.decode())
    # the links' names went with the service (the mappings joined above stay valid until closed)
    assert not left, left


def test_zero_copy_count_changed_after_staging_is_a_parse_failure(tmp_path):
    """in zero-copy mode the host reads a payload's signature
    count (byte 0) from the live room when it stages the frag, the device
    parses the bytes the batch DMAs later.  The fault-injection build makes
    every 5th frag's count read as 12 at staging (as if the tile had
    rewritten byte 0 between the two reads and back): the device must
    reject those transactions as parse failures -- it copies signatures
    only from what its own parse validated -- and every other verdict is
    the one the stream has anyway (SUCCESS)."""
    if not os.path.exists(FAULT_LIB):
        pytest.fail(f"{FAULT_LIB} not built (make -C firedancer_amd/csrc)")
    from firedancer_amd import ed25519, tile, workload
    n = 1500
    eng = ed25519.Engine(0, max_chunk=1 << 14)
    pay, _ = workload.txn_payloads(eng, n, 4444, msg_sz=200)
    eng.close()
    path = str(tmp_path / "payloads.bin")
    tile.write_payload_file(path, pay)
    libdir = tmp_path / "lib"
    libdir.mkdir()
    (libdir / "libfd_ed25519_hip.so").symlink_to(FAULT_LIB)
    env = dict(os.environ, LD_LIBRARY_PATH=str(libdir), FD_ED25519_HIP_FAULT_ZC_COUNT="12")
    prefix = f"/fdz_{uuid.uuid4().hex[:10]}_"
    svc = subprocess.Popen([SERVICE_BIN, "--prefix", prefix, "--tiles", "1", "--batch", "256", "--slots", "3",
                            "--zero-copy", "--no-parent-watch"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           env=env, text=True)
    prod = None
    try:
        line = svc.stdout.readline()
        assert line.startswith("ready 1"), (line, svc.stderr.read()[-2000:] if svc.poll() is not None else "")
        prod = subprocess.Popen([tile.PRODUCER_BIN, prefix + "0_txn", prefix + "0_vd", path], stdout=subprocess.PIPE,
                                stderr=subprocess.PIPE)
        pout, perr = prod.communicate(timeout=120)
        sout, serr = svc.communicate(timeout=60)
    finally:
        for p in (prod, svc):
            if p is not None and p.poll() is None:
                p.kill()
        for f in os.listdir("/dev/shm"):
            if f.startswith(prefix[1:]):
                os.unlink(os.path.join("/dev/shm", f))
    if prod.returncode == 3:
        pytest.skip(f"seccomp strict mode unavailable: {perr.decode()}")
    assert prod.returncode == 0 and svc.returncode == 0, (prod.returncode, perr.decode()[-1000:], svc.returncode,
                                                          serr[-2000:])
    v = np.frombuffer(pout[:n], np.int8)
    tampered = np.arange(n) % 5 == 2
    assert (v[tampered] == tile.TXN_PARSE_FAILED).all(), np.unique(v[tampered], return_counts=True)
    assert (v[~tampered] == 0).all(), np.unique(v[~tampered], return_counts=True)
