"""The drop-ins' GPU-failure policy (include/fd_ed25519_hip.h,
fd_ed25519_hip_dropin_set_on_lost).  The fault-injection build fails the
drop-in launches $FD_ED25519_HIP_FAULT_DROPIN names (a:b = launches a ..
a+b-1, retries counted) after their inputs are staged:

  - one failed launch: the engine is re-created and the launch retried;
    every caller still gets the reference's code (the oracle's), the
    status stays usable and counts one recovery;
  - a launch that fails again on its retry, policy REJECT: that call and
    every later one return FD_ED25519_ERR_SIG without device work (fail
    closed: the valid signature is not accepted), the status reports the
    loss; fd_ed25519_hip_dropin_reset brings the drop-ins back and the codes
    are the reference's again;
  - the same with the default policy ABORT: the process stops with a
    message naming the failure and the policy (SIGABRT), after the calls
    before it returned the reference's codes.

Each case runs in a child process (the library is chosen at import)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

FAULT_LIB = os.path.join(REPO, "firedancer_amd", "_lib", "libfd_ed25519_hip_faultinj.so")
CHILD = os.path.join(REPO, "tests", "faultinj_dropin_child.py")


def _run(policy, fault, calls, *extra):
    if not os.path.exists(FAULT_LIB):
        pytest.fail(f"{FAULT_LIB} not built (make -C firedancer_amd/csrc)")
    env = dict(os.environ, FD_ED25519_HIP_LIB=FAULT_LIB, FD_ED25519_HIP_FAULT_DROPIN=fault)
    p = subprocess.run([sys.executable, CHILD, policy, str(calls), *extra], capture_output=True, text=True,
                       timeout=120, env=env)
    return p.returncode, [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")], p.stderr


def test_one_failed_launch_is_retried_on_a_new_engine():
    rc, rows, err = _run("reject", "3:1", 6)
    assert rc == 0, err[-2000:]
    assert [r["got"] for r in rows] == [r["want"] for r in rows] == [0, -3] * 3
    assert all(r["lost"] == 0 for r in rows)
    assert [r["recoveries"] for r in rows] == [0, 0, 1, 1, 1, 1]
    assert "injected launch failure" in err and "re-creating engine" in err


def test_lost_device_fails_closed_and_reset_recovers():
    rc, rows, err = _run("reject", "3:2", 4, "reset")
    assert rc == 0, err[-2000:]
    before, reset, after = rows[:4], rows[4], rows[5:]
    assert [r["got"] for r in before[:2]] == [r["want"] for r in before[:2]] == [0, -3]
    # launch 3 and its retry failed: lost, every call rejected, the valid one included, no device work
    assert [r["got"] for r in before[2:]] == [-1, -1] and before[2]["want"] == 0
    assert all(r["lost"] < 0 for r in before[2:])
    assert before[3]["launches"] == before[2]["launches"]
    assert reset == {"reset": 0}
    assert [r["got"] for r in after] == [r["want"] for r in after] == [0, -3, 0, -3]
    assert all(r["lost"] == 0 for r in after)
    assert "injected launch failure" in err


def test_lost_device_aborts_by_default():
    rc, rows, err = _run("abort", "3:2", 4)
    assert rc == -6, (rc, err[-2000:])
    assert [r["got"] for r in rows] == [r["want"] for r in rows] == [0, -3]   # the calls before the loss
    assert "FATAL" in err and "policy: abort" in err and "injected launch failure" in err
