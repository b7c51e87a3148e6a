"""The host C that crosses the trust boundary under ASan + UBSan (VERDICT r3
#5; the reference's config/extra/with-asan.mk and with-ubsan.mk): the
shared-memory link and its peer checks, the accelerated verify tile
(integration/fd_verify_hip.c), the frag assembly, the txn parse core and
the tcache, the vtile / service loop and the stand-in service.

The CPU suites that drive that code run again in a child pytest against
the sanitized builds, once with ASan and once with UBSan (make -C
firedancer_amd/csrc san: the product library's host objects and the
sandboxed producer; make -C oracle ref-mux-san: the mux harness with the
tile, and the stand-in service), with the gcc sanitizer runtime preloaded
into the interpreter:

  test_shlink.py            hostile headers / frags / geometry, protocol
                            word, reclaim, producer under seccomp strict mode
  test_txn.py               fd_txn_parse parity on fixtures and mutations,
                            published frags, tcache
  test_frag_assemble.py     the tile's frag assembly (its own driver,
                            compiled here with the sanitizers too)
  test_mux_tile.py          the tile under fd_mux_tile: parity with the
                            reference tile, liveness, protocol violations
  test_service_lifecycle.py tiles dying, restarts, parent death, SIGTERM
  test_hsrec.py, test_hsdec.py  the drop-in's host scalars and host
                            decompressions on every fixture's signatures and
                            the edge encodings

Every sanitizer report goes to a log file (ASAN_OPTIONS / UBSAN_OPTIONS
log_path), from the interpreter and from every child program, so a report
is seen even where a test expects a child to fail; the run passes only
with the suites green and no report at all.  The sanitizer runtimes need
system calls seccomp forbids, so the tiles and the producer run
unsandboxed here (FD_TEST_SANITIZE); their code and checks are the same."""
import glob
import os
import subprocess
import sys

import pytest

from conftest import REPO

SUITES = ["test_shlink.py", "test_txn.py", "test_frag_assemble.py", "test_mux_tile.py", "test_service_lifecycle.py", "test_hsrec.py",
          "test_hsdec.py"]
# gcc's combined ASan + UBSan runtime writes UBSan's reports to stderr only
# (log_path is ignored), so each sanitizer has a build and a run of its own
RUNTIME = {"address": ("libasan.so", "ASAN_OPTIONS", "detect_leaks=0:halt_on_error=1"),
           "undefined": ("libubsan.so", "UBSAN_OPTIONS", "print_stacktrace=1:halt_on_error=1")}


def _runtime(name):
    r = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True)
    p = r.stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.parametrize("kind", ["address", "undefined"])
def test_trust_boundary_code_under_sanitizer(tmp_path, kind):
    lib = os.path.join(REPO, "firedancer_amd", "_lib", f"san-{kind}", "libfd_ed25519_hip.so")
    producer = os.path.join(REPO, "firedancer_amd", "_lib", f"san-{kind}", "fd_shlink_producer")
    mux = os.path.join(REPO, "oracle", "_ref", f"mux-san-{kind}")
    missing = [p for p in (lib, producer, os.path.join(mux, "mux_harness"), os.path.join(mux, "ref_vservice"))
               if not os.path.exists(p)]
    if missing:
        pytest.skip(f"sanitizer builds missing: {missing} (make -C firedancer_amd/csrc san; make -C oracle ref-mux-san)")
    so, var, opts = RUNTIME[kind]
    rt = _runtime(so)
    assert rt, f"gcc's {so} not found"
    logs = tmp_path / "san"
    logs.mkdir()
    env = dict(os.environ, LD_PRELOAD=rt, FD_ED25519_HIP_LIB=lib, FD_SHLINK_PRODUCER=producer, FD_TEST_MUX_DIR=mux,
               FD_TEST_SANITIZE=kind)
    # every report to a file, from the interpreter and from every child
    # program (leaks: the interpreter's own allocations at exit are not this code's)
    env[var] = f"{opts}:log_path={logs}/{kind}"
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu",
                        *[os.path.join(REPO, "tests", s) for s in SUITES]],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=1500)
    reports = sorted(glob.glob(str(logs / "*")))
    text = "".join(open(p, errors="replace").read()[:4000] for p in reports[:3])
    assert not reports, f"{len(reports)} sanitizer report(s):\n{text}"
    assert r.returncode == 0, (r.stdout[-4000:], r.stderr[-2000:])
    assert " passed" in r.stdout and " failed" not in r.stdout, r.stdout[-2000:]
