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
        # header-only helpers (static inline) are not library symbols
        for m in re.finditer(r"^static inline [^\n]*\n\s*(fd_[a-z0-9_]+)\s*\(", text, flags=re.M):
            syms.discard(m.group(1))
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


def test_host_sha512_matches_hashlib(lib):
    """The library's host SHA-512 (fd_ed25519_hip_sha512: the drop-ins hash
    messages of 4 GiB and more with it) against hashlib, at every padding
    boundary, large inputs and unaligned starts.  The drop-in verdicts on
    such messages are tests/test_gpu_dropin_large.py."""
    import hashlib
    import random
    f = lib.fd_ed25519_hip_sha512
    f.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_char_p]
    rng = random.Random(512)
    sizes = list(range(0, 300)) + [383, 384, 385, 1232, 1 << 16, (1 << 20) + 7]
    for sz in sizes:
        data = bytes(rng.getrandbits(8) for _ in range(sz + 3)) if sz < 4096 else rng.randbytes(sz + 3)
        for shift in (0, 3) if sz < 400 else (1,):
            out = ctypes.create_string_buffer(64)
            buf = ctypes.create_string_buffer(data, len(data))
            f(ctypes.addressof(buf) + shift, sz, out)
            assert out.raw == hashlib.sha512(data[shift:shift + sz]).digest(), (sz, shift)


def test_engine_status_strings(lib):
    lib.fd_ed25519_hip_strerror.restype = ctypes.c_char_p
    assert lib.fd_ed25519_hip_strerror(0) == b"ok"
    assert lib.fd_ed25519_hip_strerror(-22) == b"invalid argument"


def test_python_mirror_imports_without_gpu():
    from firedancer_amd import ed25519
    assert ed25519.strerror(-2) == "bad public key"
    assert ed25519.SUCCESS == 0 and ed25519.ERR_MSG == -3


REF_SRC = "/root/reference/src"


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference sources not present (GPU box)")
def test_headers_compile_with_the_reference_header(tmp_path):
    """The drop-in prototypes are the reference's own: a translation unit
    that includes src/ballet/ed25519/fd_ed25519.h and include/*.h together
    compiles warning-free (-Werror, array-parameter bounds included), and
    the drop-ins convert to pointers of the reference's exact types."""
    import subprocess
    src = tmp_path / "both.c"
    src.write_text("""
#include "ballet/ed25519/fd_ed25519.h"
#include "fd_ed25519_hip.h"
#include "fd_ed25519_hip_tile.h"
static int (*p1)( uchar const *, ulong, uchar const *, uchar const *, fd_sha512_t * ) = fd_ed25519_verify;
static int (*p2)( uchar const *, ulong const, uchar const *, uchar const *, fd_sha512_t **, uchar const ) =
  fd_ed25519_verify_batch_single_msg;
static char const * (*p3)( int ) = fd_ed25519_strerror;
int main( void ) { return (p1!=0) + (p2!=0) + (p3!=0) - 3; }
""")
    defs = ["-DFD_HAS_INT128=1", "-DFD_HAS_DOUBLE=1", "-DFD_HAS_ALLOCA=1", "-DFD_HAS_X86=1", "-DFD_IS_X86_64=1",
            "-DFD_HAS_SSE=1", "-DFD_HAS_AVX=1", "-DFD_HAS_THREADS=1", "-DFD_HAS_ATOMIC=1"]
    r = subprocess.run(["gcc", "-std=c17", "-march=haswell", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", *defs,
                        "-I" + REF_SRC, "-I" + os.path.join(REPO, "include"), str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_headers_compile_as_c_and_cxx(tmp_path):
    """include/*.h alone, as C11 and as C++17 (extern "C"), warning-free."""
    import subprocess
    src = tmp_path / "h.c"
    src.write_text('#include "fd_ed25519_hip.h"\n#include "fd_ed25519_hip_tile.h"\nint main(void){return 0;}\n')
    for cc, std in (("gcc", "-std=c11"), ("g++", "-std=c++17")):
        args = [cc, std, "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-I" + os.path.join(REPO, "include")]
        if cc == "g++":
            args += ["-x", "c++"]
        r = subprocess.run(args + [str(src)], capture_output=True, text=True)
        assert r.returncode == 0, (cc, r.stderr)


DROPIN = os.path.join(REPO, "oracle", "_ref", "dropin")


@pytest.mark.skipif(not os.path.isdir(DROPIN), reason="oracle/_ref/dropin not built (make -C oracle ref-dropin)")
@pytest.mark.parametrize("prog", ["test_ed25519_dropin", "test_verify_dropin"])
def test_reference_tests_bind_to_the_dropin(prog, tmp_path):
    """The reference's own verify tests, compiled from its sources, call
    into libfd_ed25519_hip: here, without a GPU, its first verify call
    fails loudly in the product library's engine creation -- never a
    silent CPU verify (the reference's definitions are local to their
    object).  tests/test_gpu_dropin.py runs them to 'pass' on the GPU."""
    import subprocess
    r = subprocess.run([os.path.join(DROPIN, prog)], capture_output=True, text=True, timeout=120, cwd=tmp_path,
                       env=dict(os.environ, TMPDIR=str(tmp_path), HIP_VISIBLE_DEVICES="-1"))
    assert r.returncode != 0
    assert "libfd_ed25519_hip: FATAL: cannot create the drop-in GPU engines" in r.stderr, r.stderr[-2000:]
    assert "(policy: abort)" in r.stderr, r.stderr[-2000:]
