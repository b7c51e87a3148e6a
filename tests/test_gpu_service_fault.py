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
