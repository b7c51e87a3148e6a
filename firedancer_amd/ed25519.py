"""Python mirror of the reference's ed25519 verify interface, backed by the
MI355X library libfd_ed25519_hip (C-ABI, include/fd_ed25519_hip.h).

Mirrors src/ballet/ed25519/fd_ed25519.h:96-138 of tigarcia/firedancer:

    verify(msg, sig, public_key)                    -> fd_ed25519_verify
    verify_batch_single_msg(msg, signatures, pubs)  -> fd_ed25519_verify_batch_single_msg
    strerror(err)                                   -> fd_ed25519_strerror

with the same argument meaning and return codes (SUCCESS 0, ERR_SIG -1,
ERR_PUBKEY -2, ERR_MSG -3), plus the batch Engine the verify tile and
bench.py drive.  There is no CPU fallback: importing this module without the
built library raises.
"""
import ctypes
import os

import numpy as np

SUCCESS = 0
ERR_SIG = -1
ERR_PUBKEY = -2
ERR_MSG = -3

FLAG_CODES_PORTABLE = 1
FLAG_HALF_STRICT = 2     # half-size |d| < 2^131 only (full-length form for the rest): tests / A-B
FLAG_DSM_QUAD = 4        # dsm with a quad of lanes per signature at every chunk size
FLAG_DSM_WIDE = 8        # dsm with one lane per signature at every chunk size
FLAG_DSM_OCT = 16        # dsm with two quads of lanes per signature at every chunk size
FLAG_ONE_STREAM = 32     # no decode side stream / second lane: for engines whose batches overlap one another
FLAG_NO_OVERLAP = 64     # a large chunk's phases in sequence (no decode side stream): tests / A-B
FLAG_NO_PIPELINE = 128   # a multi-chunk call on one set of work arrays (no second lane): tests / A-B
FLAG_COMPACT_TABLES = 256  # radix-2^16 base tables (2 x 8 MiB, shared) instead of radix 2^24 (2 x 2 GiB)
FLAG_DSM_R16 = 512       # dsm16 (field arithmetic over 16 lanes, two waves per signature) at every chunk size

# phases of a verify launch (FD_ED25519_HIP_PHASE_CNT, include/fd_ed25519_hip.h)
PHASES = ("hash", "scalar", "decode", "dsm")

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FD_ED25519_HIP_LIB", os.path.join(_HERE, "_lib", "libfd_ed25519_hip.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(f"libfd_ed25519_hip not built: {LIB_PATH} missing "
                      "(run `python -c 'import __graft_entry__ as g; g.build()'`); there is no CPU fallback")

_lib = ctypes.CDLL(LIB_PATH, use_errno=True)   # errno: shlink create / join report why they failed

_u8p = ctypes.c_void_p
_lib.fd_ed25519_verify.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]
_lib.fd_ed25519_verify.restype = ctypes.c_int
_lib.fd_ed25519_verify_batch_single_msg.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p,
                                                    ctypes.c_void_p, ctypes.c_ubyte]
_lib.fd_ed25519_verify_batch_single_msg.restype = ctypes.c_int
_lib.fd_ed25519_strerror.argtypes = [ctypes.c_int]
_lib.fd_ed25519_strerror.restype = ctypes.c_char_p
_lib.fd_ed25519_hip_engine_new.argtypes = [ctypes.c_int, ctypes.c_ulong, ctypes.c_int]
_lib.fd_ed25519_hip_engine_new.restype = ctypes.c_void_p
_lib.fd_ed25519_hip_engine_delete.argtypes = [ctypes.c_void_p]
_lib.fd_ed25519_hip_engine_set_forms.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_ulong]
_lib.fd_ed25519_hip_engine_set_r16_max.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
_lib.fd_ed25519_hip_engine_stream.argtypes = [ctypes.c_void_p]
_lib.fd_ed25519_hip_engine_stream.restype = ctypes.c_void_p
_lib.fd_ed25519_hip_engine_sync.argtypes = [ctypes.c_void_p]
_lib.fd_ed25519_hip_verify_dev.argtypes = [ctypes.c_void_p, ctypes.c_ulong] + [_u8p] * 7
_lib.fd_ed25519_hip_txn_combine_dev.argtypes = [ctypes.c_void_p, ctypes.c_ulong] + [_u8p] * 5
_lib.fd_ed25519_hip_verify_host.argtypes = [ctypes.c_void_p, ctypes.c_ulong] + [_u8p] * 6
_lib.fd_ed25519_hip_verify_txns_host.argtypes = [ctypes.c_void_p, ctypes.c_ulong] + [_u8p] * 9
_lib.fd_ed25519_hip_sign_dev.argtypes = [ctypes.c_void_p, ctypes.c_ulong] + [_u8p] * 7
_lib.fd_ed25519_hip_gen_dev.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_ulong, ctypes.c_ulong, _u8p,
                                        ctypes.c_ulong] + [_u8p] * 5
_lib.fd_ed25519_hip_corrupt_dev.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_ulong, ctypes.c_ulong,
                                            ctypes.c_uint] + [_u8p] * 8
_lib.fd_ed25519_hip_engine_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
_lib.fd_ed25519_hip_engine_timing_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                                   ctypes.POINTER(ctypes.c_ulong)]
_lib.fd_ed25519_hip_engine_check_base_tables.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulong)]
_lib.fd_ed25519_hip_engine_base_entry.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_ulong,
                                                  ctypes.POINTER(ctypes.c_int)]
BASE_TABLE_BITS = 24     # FD_ED25519_HIP_BASE_TABLE_BITS
BASE_TABLE_SHIFT = 144   # FD_ED25519_HIP_BASE_TABLE_SHIFT
_lib.fd_ed25519_hip_dev_alloc.argtypes = [ctypes.c_void_p, ctypes.c_ulong]
_lib.fd_ed25519_hip_dev_alloc.restype = ctypes.c_void_p
_lib.fd_ed25519_hip_dev_free.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
_lib.fd_ed25519_hip_memcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulong,
                                       ctypes.c_int]
_lib.fd_ed25519_hip_device_clock_mhz.argtypes = [ctypes.c_void_p]
_lib.fd_ed25519_hip_diag_half_scalars.argtypes = [ctypes.c_void_p, _u8p, ctypes.c_ulong, _u8p]
_lib.fd_ed25519_hip_strerror.argtypes = [ctypes.c_int]
_lib.fd_ed25519_hip_strerror.restype = ctypes.c_char_p
_lib.fd_ed25519_hip_last_error.restype = ctypes.c_char_p


class _Info(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("cu_cnt", ctypes.c_int), ("dsm_blocks_per_cu", ctypes.c_int),
                ("dsm_grid", ctypes.c_uint), ("max_chunk", ctypes.c_ulong), ("device_bytes", ctypes.c_ulong),
                ("flags", ctypes.c_int), ("arch", ctypes.c_char * 64), ("pci_domain", ctypes.c_int),
                ("pci_bus", ctypes.c_int), ("pci_device", ctypes.c_int)]


_lib.fd_ed25519_hip_engine_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(_Info)]


class HipError(RuntimeError):
    pass


def _check(rc):
    if rc:
        raise HipError(f"{_lib.fd_ed25519_hip_strerror(rc).decode()} ({_lib.fd_ed25519_hip_last_error().decode()})")


def library():
    """The loaded ctypes library (for callers that need raw entry points)."""
    return _lib


def strerror(err):
    return _lib.fd_ed25519_strerror(int(err)).decode()


def verify(msg, sig, public_key):
    """fd_ed25519_verify drop-in (synchronous, default engine)."""
    assert len(sig) == 64 and len(public_key) == 32
    msg = bytes(msg)
    return _lib.fd_ed25519_verify(msg, len(msg), bytes(sig), bytes(public_key), None)


def verify_batch_single_msg(msg, signatures, pubkeys, batch_sz=None):
    """fd_ed25519_verify_batch_single_msg drop-in: signatures is 64*n bytes,
    pubkeys 32*n bytes."""
    signatures, pubkeys, msg = bytes(signatures), bytes(pubkeys), bytes(msg)
    n = len(signatures) // 64 if batch_sz is None else batch_sz
    return _lib.fd_ed25519_verify_batch_single_msg(msg, len(msg), signatures or b"\0" * 64, pubkeys or b"\0" * 32,
                                                   None, n & 0xFF)


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


class Engine:
    """A libfd_ed25519_hip engine bound to one GPU."""

    def __init__(self, device=0, max_chunk=0, codes="avx512", half="extended", dsm="auto", one_stream=False,
                 overlap=True, pipeline=True, forms=None, compact=False, r16_max=None):
        flags = FLAG_CODES_PORTABLE if codes == "portable" else 0
        flags |= FLAG_ONE_STREAM if one_stream else 0
        flags |= 0 if overlap else FLAG_NO_OVERLAP
        flags |= 0 if pipeline else FLAG_NO_PIPELINE
        flags |= FLAG_COMPACT_TABLES if compact else 0
        flags |= FLAG_HALF_STRICT if half == "strict" else 0
        flags |= {"auto": 0, "quad": FLAG_DSM_QUAD, "wide": FLAG_DSM_WIDE, "oct": FLAG_DSM_OCT, "r16": FLAG_DSM_R16}[dsm]
        self._h = _lib.fd_ed25519_hip_engine_new(int(device), int(max_chunk), flags)
        if not self._h:
            raise HipError(f"engine_new failed: {_lib.fd_ed25519_hip_last_error().decode()}")
        self.codes = codes
        if forms is not None:   # (quad_max, oct_max): fd_ed25519_hip_engine_set_forms
            _check(_lib.fd_ed25519_hip_engine_set_forms(self._h, int(forms[0]), int(forms[1])))
        if r16_max is not None:   # dsm16 up to this chunk size: fd_ed25519_hip_engine_set_r16_max
            _check(_lib.fd_ed25519_hip_engine_set_r16_max(self._h, int(r16_max)))

    def close(self):
        if self._h:
            _lib.fd_ed25519_hip_engine_delete(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        i = _Info()
        _check(_lib.fd_ed25519_hip_engine_info(self._h, ctypes.byref(i)))
        return {f: (getattr(i, f).decode() if f == "arch" else getattr(i, f)) for f, _ in _Info._fields_}

    @property
    def stream(self):
        return _lib.fd_ed25519_hip_engine_stream(self._h)

    def sync(self):
        _check(_lib.fd_ed25519_hip_engine_sync(self._h))

    def verify_host(self, msgs, msg_off, msg_sz, sigs, pubs):
        """SoA host batch -> int8 codes (synchronous)."""
        n = len(msg_sz)
        out = np.zeros(n, dtype=np.int8)
        if n == 0:
            return out
        msgs = _c(msgs, np.uint8) if len(msgs) else np.zeros(1, np.uint8)
        off, sz = _c(msg_off, np.uint64), _c(msg_sz, np.uint32)
        sigs, pubs = _c(sigs, np.uint8).reshape(-1), _c(pubs, np.uint8).reshape(-1)
        assert len(sigs) >= 64 * n and len(pubs) >= 32 * n
        _check(_lib.fd_ed25519_hip_verify_host(self._h, n, _ptr(msgs), _ptr(off), _ptr(sz), _ptr(sigs), _ptr(pubs),
                                               _ptr(out)))
        return out

    def verify_txns_host(self, msgs, txn_msg_off, txn_msg_sz, txn_first, txn_cnt, sigs, pubs, want_sig_codes=False):
        """batch_single_msg semantics per transaction -> (txn codes, sig codes|None)."""
        ntxn = len(txn_cnt)
        out = np.zeros(ntxn, dtype=np.int8)
        nsig = len(sigs) if np.ndim(sigs) == 2 else len(sigs) // 64
        osig = np.zeros(max(nsig, 1), dtype=np.int8) if want_sig_codes else None
        if ntxn == 0:
            return out, osig
        msgs = _c(msgs, np.uint8) if len(msgs) else np.zeros(1, np.uint8)
        sigs = _c(sigs, np.uint8).reshape(-1) if nsig else np.zeros(64, np.uint8)
        pubs = _c(pubs, np.uint8).reshape(-1) if nsig else np.zeros(32, np.uint8)
        _check(_lib.fd_ed25519_hip_verify_txns_host(
            self._h, ntxn, _ptr(msgs), _ptr(_c(txn_msg_off, np.uint64)), _ptr(_c(txn_msg_sz, np.uint32)),
            _ptr(_c(txn_first, np.uint32)), _ptr(_c(txn_cnt, np.uint32)), _ptr(sigs), _ptr(pubs), _ptr(out),
            _ptr(osig)))
        return out, osig

    def verify_dev(self, n, d_msgs, d_off, d_sz, d_sigs, d_pubs, d_out, stream=None):
        """Device-resident batch: arguments are device addresses (ints); async."""
        _check(_lib.fd_ed25519_hip_verify_dev(self._h, int(n), d_msgs, d_off, d_sz, d_sigs, d_pubs, d_out, stream))

    def txn_combine_dev(self, ntxn, d_sig_codes, d_first, d_cnt, d_out, stream=None):
        _check(_lib.fd_ed25519_hip_txn_combine_dev(self._h, int(ntxn), d_sig_codes, d_first, d_cnt, d_out, stream))


    # ---- batched signing / synthetic workloads -------------------------
    def sign_dev(self, n, d_msgs, d_off, d_sz, d_privs, d_sigs, d_pubs, stream=None):
        _check(_lib.fd_ed25519_hip_sign_dev(self._h, int(n), d_msgs, d_off, d_sz, d_privs, d_sigs, d_pubs, stream))

    def gen_dev(self, n, seed, index_base, d_msgs, msg_bytes, d_off, d_sz, d_sigs, d_pubs, stream=None):
        _check(_lib.fd_ed25519_hip_gen_dev(self._h, int(n), int(seed), int(index_base), d_msgs, int(msg_bytes), d_off,
                                           d_sz, d_sigs, d_pubs, stream))

    def corrupt_dev(self, n, seed, index_base, ppm, d_msgs, d_off, d_sz, d_sigs, d_pubs, d_expect=None, d_cls=None,
                    stream=None):
        _check(_lib.fd_ed25519_hip_corrupt_dev(self._h, int(n), int(seed), int(index_base), int(ppm), d_msgs, d_off,
                                               d_sz, d_sigs, d_pubs, d_expect, d_cls, stream))

    # ---- measurement ------------------------------------------------------
    def timing(self, enable=True):
        _check(_lib.fd_ed25519_hip_engine_timing(self._h, 1 if enable else 0))

    def timing_read(self):
        ms = (ctypes.c_double * len(PHASES))()
        cnt = ctypes.c_ulong(0)
        _check(_lib.fd_ed25519_hip_engine_timing_read(self._h, ms, ctypes.byref(cnt)))
        return {name: ms[i] for i, name in enumerate(PHASES)}, cnt.value

    def check_base_tables(self):
        """per base table ([e]B, [e][2^144]B, and the full-length form's
        [0..2^15]B), the count of entries e with entry e+1 != entry e +
        entry 1 ((0, 0, 0) for correct tables)"""
        bad = (ctypes.c_ulong * 3)()
        _check(_lib.fd_ed25519_hip_engine_check_base_tables(self._h, bad))
        return bad[0], bad[1], bad[2]

    def base_entry(self, which, index):
        """entry `index` of wide base table `which` (0: [e]B, 1: [e][2^144]B):
        int32 [30] = (y+x, y-x, 2dxy) in radix-2^25.5 limbs"""
        out = (ctypes.c_int * 30)()
        _check(_lib.fd_ed25519_hip_engine_base_entry(self._h, which, index, out))
        return np.array(out[:], dtype=np.int64)

    def diag_half_scalars(self, k_words):
        """Diagnostic: the device's half-size scalar search for k given as
        uint32 [n][8]; returns uint32 [n][12] (ok, d<0, c[5], |d|[5])."""
        k = np.ascontiguousarray(k_words, dtype=np.uint32).reshape(-1, 8)
        out = np.zeros((len(k), 12), dtype=np.uint32)
        if len(k):
            _check(_lib.fd_ed25519_hip_diag_half_scalars(self._h, k.ctypes.data_as(_u8p), len(k),
                                                         out.ctypes.data_as(_u8p)))
        return out

    def clock_mhz(self):
        return _lib.fd_ed25519_hip_device_clock_mhz(self._h)

    # ---- device memory ----------------------------------------------------
    def alloc(self, nbytes):
        return DeviceBuffer(self, nbytes)


class DeviceBuffer:
    """Device memory owned by an engine's HIP runtime."""

    def __init__(self, engine, nbytes):
        self.engine, self.nbytes = engine, int(nbytes)
        self.ptr = _lib.fd_ed25519_hip_dev_alloc(engine._h, max(self.nbytes, 1))
        if not self.ptr:
            raise HipError(f"dev_alloc({nbytes}) failed: {_lib.fd_ed25519_hip_last_error().decode()}")

    def upload(self, arr):
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        _check(_lib.fd_ed25519_hip_memcpy(self.engine._h, self.ptr, arr.ctypes.data, arr.nbytes, 0))
        return self

    def download(self, dtype, count, offset_bytes=0):
        out = np.empty(count, dtype=dtype)
        assert offset_bytes + out.nbytes <= self.nbytes
        _check(_lib.fd_ed25519_hip_memcpy(self.engine._h, out.ctypes.data, self.ptr + offset_bytes, out.nbytes, 1))
        return out

    def download_into(self, out, offset_bytes=0):
        """D2H straight into a caller's contiguous array (e.g. a slice of a
        page-locked host window), no intermediate copy."""
        assert out.flags["C_CONTIGUOUS"] and offset_bytes + out.nbytes <= self.nbytes
        if out.nbytes:
            _check(_lib.fd_ed25519_hip_memcpy(self.engine._h, out.ctypes.data, self.ptr + offset_bytes, out.nbytes, 1))
        return out

    def free(self):
        if self.ptr:
            _lib.fd_ed25519_hip_dev_free(self.engine._h, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceWorkload:
    """A signature batch resident in HBM (SoA), generated on the device."""

    def __init__(self, engine, n, lo, hi, ppm, seed, index_base=0):
        from . import workload
        self.n = n
        sizes = workload.msg_sizes(seed, index_base, n, lo, hi)
        off = workload.msg_offsets(sizes)
        self.msg_bytes = int(sizes.astype(np.uint64).sum())
        self.sizes = sizes
        self.msgs = engine.alloc(self.msg_bytes + 16)
        self.off = engine.alloc(8 * n).upload(off)
        self.sz = engine.alloc(4 * n).upload(sizes)
        self.sigs = engine.alloc(64 * n)
        self.pubs = engine.alloc(32 * n)
        self.out = engine.alloc(n)
        self.expect = engine.alloc(n)
        self.cls = engine.alloc(n)
        engine.gen_dev(n, seed, index_base, self.msgs.ptr, self.msg_bytes, self.off.ptr, self.sz.ptr, self.sigs.ptr,
                       self.pubs.ptr)
        engine.corrupt_dev(n, seed, index_base, ppm, self.msgs.ptr, self.off.ptr, self.sz.ptr, self.sigs.ptr,
                           self.pubs.ptr, self.expect.ptr, self.cls.ptr)
        engine.sync()
        self.engine = engine

    def verify(self, stream=None):
        self.engine.verify_dev(self.n, self.msgs.ptr, self.off.ptr, self.sz.ptr, self.sigs.ptr, self.pubs.ptr,
                               self.out.ptr, stream)

    def free(self):
        for b in (self.msgs, self.off, self.sz, self.sigs, self.pubs, self.out, self.expect, self.cls):
            b.free()


_lib.fd_ed25519_hip_device_count.restype = ctypes.c_int


_lib.fd_ed25519_hip_dropin_stats.argtypes = [ctypes.POINTER(ctypes.c_ulong), ctypes.POINTER(ctypes.c_ulong)]
_lib.fd_ed25519_hip_dropin_device_bytes.restype = ctypes.c_ulong
_lib.fd_ed25519_hip_shared_device_bytes.argtypes = [ctypes.c_int]
_lib.fd_ed25519_hip_shared_device_bytes.restype = ctypes.c_ulong


def dropin_stats():
    """(launches, calls): the drop-ins' combined launches and the calls they carried."""
    a, b = ctypes.c_ulong(), ctypes.c_ulong()
    _lib.fd_ed25519_hip_dropin_stats(ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


DROPIN_ON_LOST_ABORT, DROPIN_ON_LOST_REJECT = 0, 1
_lib.fd_ed25519_hip_dropin_set_on_lost.argtypes = [ctypes.c_int]
_lib.fd_ed25519_hip_dropin_status.argtypes = [ctypes.POINTER(ctypes.c_ulong)]


def dropin_set_on_lost(policy):
    """The drop-ins' lost-device policy (fd_ed25519_hip_dropin_set_on_lost):
    DROPIN_ON_LOST_ABORT (default) or DROPIN_ON_LOST_REJECT; returns the previous."""
    return _lib.fd_ed25519_hip_dropin_set_on_lost(int(policy))


def dropin_status():
    """(lost, recoveries): 0 or the code that lost the device, and the launches
    that succeeded on a re-created engine (fd_ed25519_hip_dropin_status)."""
    r = ctypes.c_ulong()
    lost = _lib.fd_ed25519_hip_dropin_status(ctypes.byref(r))
    return lost, r.value


def dropin_reset():
    """Re-creates the drop-in engines (fd_ed25519_hip_dropin_reset): 0 or an error code."""
    return _lib.fd_ed25519_hip_dropin_reset()


def dropin_device_bytes():
    """Device memory the drop-ins hold: their engines plus the process's shared base tables."""
    return _lib.fd_ed25519_hip_dropin_device_bytes()


def shared_device_bytes(device=0):
    return _lib.fd_ed25519_hip_shared_device_bytes(int(device))


def device_count():
    """Visible HIP devices, from the library's own runtime."""
    return _lib.fd_ed25519_hip_device_count()
