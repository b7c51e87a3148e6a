"""CPU-side checks of the C-ABI boundary: the library loads, exports every
symbol include/*.h declares, and the non-GPU entry points behave."""
import ctypes
import os
import re

import pytest

from conftest import REPO

LIB = os.path.join(REPO, "firedancer_amd", "_lib", "libfd_ed25519_hip.so")


def declared_symbols():
    syms = set()
    for f in os.listdir(os.path.join(REPO, "include")):
        if not f.endswith(".h"):
            continue
        text = open(os.path.join(REPO, "include", f)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^\s*(fd_[a-z0-9_]+)\s*\(", text, flags=re.M):
            syms.add(m.group(1))
    return syms


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} not built")
    return ctypes.CDLL(LIB)


def test_header_declares_dropins():
    syms = declared_symbols()
    for s in ("fd_ed25519_verify", "fd_ed25519_verify_batch_single_msg", "fd_ed25519_strerror",
              "fd_ed25519_hip_engine_new", "fd_ed25519_hip_verify_dev", "fd_ed25519_hip_verify_host"):
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_strerror_matches_reference(lib):
    lib.fd_ed25519_strerror.restype = ctypes.c_char_p
    assert lib.fd_ed25519_strerror(0) == b"success"
    assert lib.fd_ed25519_strerror(-1) == b"bad signature"
    assert lib.fd_ed25519_strerror(-2) == b"bad public key"
    assert lib.fd_ed25519_strerror(-3) == b"bad message"
    assert lib.fd_ed25519_strerror(1) == b"unknown"


def test_batch_size_guard_needs_no_gpu(lib):
    """batch_sz 0 or > 16 -> ERR_SIG before any device work
    (src/ballet/ed25519/fd_ed25519_user.c:238-240)."""
    f = lib.fd_ed25519_verify_batch_single_msg
    f.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_ubyte]
    assert f(b"m", 1, b"\0" * 64 * 17, b"\0" * 32 * 17, None, 0) == -1
    assert f(b"m", 1, b"\0" * 64 * 17, b"\0" * 32 * 17, None, 17) == -1


def test_engine_status_strings(lib):
    lib.fd_ed25519_hip_strerror.restype = ctypes.c_char_p
    assert lib.fd_ed25519_hip_strerror(0) == b"ok"
    assert lib.fd_ed25519_hip_strerror(-22) == b"invalid argument"


def test_python_mirror_imports_without_gpu():
    from firedancer_amd import ed25519
    assert ed25519.strerror(-2) == "bad public key"
    assert ed25519.SUCCESS == 0 and ed25519.ERR_MSG == -3
