"""The drop-in proven with the reference's own C callers (VERDICT r1,
missing #6): src/ballet/ed25519/test_ed25519.c's wycheproof, cctv and
cctv_batch suites (:1013-1082) and the verify tile's test_verify.c
(fd_txn_verify: success, failure, dedup), compiled from the reference's
sources with fd_ed25519_verify / fd_ed25519_verify_batch_single_msg bound
to libfd_ed25519_hip.so (oracle/Makefile ref-dropin), run to 'pass' on the
GPU."""
import os
import subprocess

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

DROPIN = os.path.join(REPO, "oracle", "_ref", "dropin")


@pytest.mark.parametrize("prog,expect", [
    ("test_ed25519_dropin", ["fd_ed25519_verify_wycheproof: ok", "fd_ed25519_verify_cctv: ok",
                             "fd_ed25519_verify_cctv_batch: ok", "pass"]),
    ("test_verify_dropin", ["test_verify_success", "test_verify_invalid_sigs_success",
                            "test_verify_invalid_dedup_success", "pass"]),
])
def test_reference_tests_pass_on_the_gpu_dropin(prog, expect, tmp_path):
    path = os.path.join(DROPIN, prog)
    if not os.path.exists(path):
        pytest.fail(f"{path} not built (make -C oracle ref-dropin)")
    r = subprocess.run([path], capture_output=True, text=True, timeout=240, cwd=tmp_path,
                       env=dict(os.environ, TMPDIR=str(tmp_path)))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    for e in expect:
        assert e in out, (e, out[-3000:])
    assert "libfd_ed25519_hip" not in out   # no engine failure message
