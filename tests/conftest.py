import ctypes
import os

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


def _oracle():
    path = os.path.join(REPO, "oracle", "liboracle_ed25519.so")
    if not os.path.exists(path):
        pytest.skip("oracle not built (python -c 'import __graft_entry__ as g; g.build()')")
    lib = ctypes.CDLL(path)
    lib.oracle_ed25519_verify.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_char_p,
                                          ctypes.c_int]
    lib.oracle_ed25519_verify_batch_single_msg.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p,
                                                           ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int]
    lib.oracle_ed25519_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p,
                                        ctypes.c_char_p]
    lib.oracle_ed25519_public_from_private.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    lib.oracle_ed25519_strerror.restype = ctypes.c_char_p
    lib.oracle_sha512.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64]
    lib.oracle_scalar_reduce.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    lib.oracle_base_mul_encode.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    lib.oracle_verify_many.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    return lib


@pytest.fixture(scope="session")
def oracle():
    return _oracle()


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


@pytest.fixture(scope="session")
def vectors():
    return load_golden("vectors")


@pytest.fixture(scope="session")
def adversarial():
    return load_golden("adversarial")


@pytest.fixture(scope="session")
def batch():
    return load_golden("batch")


def case(d, i):
    off, sz = int(d["msg_off"][i]), int(d["msg_sz"][i])
    return bytes(d["msgs"][off:off + sz]), d["sigs"][i].tobytes(), d["pubs"][i].tobytes()


def oracle_many(oracle, d, codes=0, nthreads=8):
    n = len(d["msg_sz"])
    out = np.zeros(n, dtype=np.int8)
    msgs = np.ascontiguousarray(d["msgs"]) if len(d["msgs"]) else np.zeros(1, np.uint8)
    off = np.ascontiguousarray(d["msg_off"], dtype=np.uint64)
    sz = np.ascontiguousarray(d["msg_sz"], dtype=np.uint32)
    sigs = np.ascontiguousarray(d["sigs"])
    pubs = np.ascontiguousarray(d["pubs"])
    rc = oracle.oracle_verify_many(n, msgs.ctypes.data, off.ctypes.data, sz.ctypes.data, sigs.ctypes.data,
                                   pubs.ctypes.data, out.ctypes.data, codes, nthreads)
    assert rc == 0
    return out


@pytest.fixture(scope="session")
def halfsize():
    return load_golden("halfsize")


@pytest.fixture(scope="session")
def longd():
    return load_golden("longd")


@pytest.fixture(scope="session")
def mixed_order():
    return load_golden("mixed_order")
