"""A pool batch that fails after its copies from the caller's arrays are
enqueued: fd_ed25519_hip_pool_run must report the error
only once those copies have finished (pool_submit synchronizes the slot's
stream), drain the batches already in flight, leave the pool usable, and
let the caller unregister and free its arrays without a hang.  The
fault-injection build fails the second batch's launch; run in a child
process, since the library is chosen at import."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

FAULT_LIB = os.path.join(REPO, "firedancer_amd", "_lib", "libfd_ed25519_hip_faultinj.so")


def test_pool_launch_failure_after_copies():
    if not os.path.exists(FAULT_LIB):
        pytest.fail(f"{FAULT_LIB} not built (make -C firedancer_amd/csrc)")
    env = dict(os.environ, FD_ED25519_HIP_LIB=FAULT_LIB)
    r = subprocess.run([sys.executable, "-u", os.path.join(REPO, "tests", "faultinj_pool_child.py")], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    for mode in ("direct", "staged"):
        got = res[mode]
        assert got["error"] and "injected launch failure" in got["error"], (mode, got)
        assert got["first_batch_ok"], (mode, got)
        assert got["rerun_ok"], (mode, got)
