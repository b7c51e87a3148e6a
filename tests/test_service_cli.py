"""fd_verify_hip_service's command line (CPU): arguments the service cannot
serve are refused with exit status 1 before its first HIP call -- slot
counts outside the pipe's 1..8, more hardware queues than the box allows
(32), malformed CPU lists, a missing prefix or tile count."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SERVICE = os.path.join(REPO, "firedancer_amd", "_lib", "fd_verify_hip_service")

pytestmark = pytest.mark.skipif(not os.path.exists(SERVICE), reason="service not built (__graft_entry__.build())")


@pytest.mark.parametrize("argv, msg", [
    (["--tiles", "1"], "usage"),
    (["--prefix", "/fd_vhip_cli_"], "usage"),
    (["--prefix", "/fd_vhip_cli_", "--tiles", "1", "--slots", "0"], "usage"),
    (["--prefix", "/fd_vhip_cli_", "--tiles", "1", "--slots", "9"], "usage"),
    (["--prefix", "/fd_vhip_cli_", "--tiles", "1", "--hw-queues", "33"], "usage"),
    (["--prefix", "/fd_vhip_cli_", "--tiles", "1", "--cpus", "3-1"], "bad --cpus"),
    (["--prefix", "/fd_vhip_cli_", "--tiles", "1", "--cpus", "a"], "bad --cpus"),
    (["--prefix", "/fd_vhip_cli_", "--tiles", "1", "--codes", "fast"], "usage"),
    (["--prefix", "/fd_vhip_cli_", "--tiles", "1", "--no-such-flag"], "usage"),
])
def test_bad_arguments_exit_1(argv, msg):
    p = subprocess.run([SERVICE, *argv], capture_output=True, text=True, timeout=60)
    assert p.returncode == 1, (p.returncode, p.stderr[-300:])
    assert msg in p.stderr
    assert not p.stdout.startswith("ready")
