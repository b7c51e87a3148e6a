"""Python mirror of the verify-tile side of libfd_ed25519_hip
(include/fd_ed25519_hip_tile.h): the transaction parser, the tcache, the
batched verify-tile core, the latency mode and the multi-GPU pool.

Names follow the reference: txn_parse ~ fd_txn_parse
(src/ballet/txn/fd_txn_parse.c), TCache ~ fd_tcache
(src/tango/tcache/fd_tcache.h), VerifyTile.frag / .poll ~ the verify tile's
after_frag + fd_txn_verify (src/app/fdctl/run/tiles/fd_verify.{c,h}), with
the verdicts TXN_VERIFY_SUCCESS / FAILED / DEDUP (fd_verify.h:9-11).
"""
import ctypes

import numpy as np

from .ed25519 import HipError, _c, _check, _lib, _ptr

TXN_VERIFY_SUCCESS = 0
TXN_VERIFY_FAILED = -1
TXN_VERIFY_DEDUP = -2
TXN_PARSE_FAILED = -3

TXN_MTU = 1232
TXN_MAX_SZ = 852                          # FD_TXN_MAX_SZ: the largest fd_txn_t
TPU_DCACHE_MTU = TXN_MTU + TXN_MAX_SZ + 2   # a published frag: payload, pad, fd_txn_t, payload_sz
SHLINK_MTU = 1 + TPU_DCACHE_MTU            # a verdict frag: verdict byte + published frag
VTILE_GPU_PARSE = 2   # FD_ED25519_HIP_VTILE_GPU_PARSE: fd_txn_parse on the device


class Txn(ctypes.Structure):
    _fields_ = [("transaction_version", ctypes.c_ubyte), ("signature_cnt", ctypes.c_ubyte),
                ("signature_off", ctypes.c_ushort), ("message_off", ctypes.c_ushort),
                ("readonly_signed_cnt", ctypes.c_ubyte), ("readonly_unsigned_cnt", ctypes.c_ubyte),
                ("acct_addr_cnt", ctypes.c_ushort), ("acct_addr_off", ctypes.c_ushort),
                ("recent_blockhash_off", ctypes.c_ushort), ("instr_cnt", ctypes.c_ushort),
                ("addr_table_lookup_cnt", ctypes.c_ubyte), ("addr_table_adtl_writable_cnt", ctypes.c_ubyte),
                ("addr_table_adtl_cnt", ctypes.c_ubyte)]

    FIELDS = [f for f, _ in _fields_]

    def as_tuple(self):
        return tuple(getattr(self, f) for f in self.FIELDS)


class LatencyResult(ctypes.Structure):
    _fields_ = [("offered_txn_per_s", ctypes.c_double), ("achieved_txn_per_s", ctypes.c_double),
                ("achieved_sig_per_s", ctypes.c_double), ("seconds", ctypes.c_double),
                ("txn_cnt", ctypes.c_ulong), ("sig_cnt", ctypes.c_ulong), ("batches", ctypes.c_ulong),
                ("ring_overruns", ctypes.c_ulong)]


_v = ctypes.c_void_p
_lib.fd_ed25519_hip_txn_parse.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.POINTER(Txn)]
_lib.fd_ed25519_hip_txn_parse.restype = ctypes.c_int
_lib.fd_ed25519_hip_txn_parse_full.argtypes = [ctypes.c_char_p, ctypes.c_ulong, _v]
_lib.fd_ed25519_hip_txn_parse_full.restype = ctypes.c_ulong
_lib.fd_ed25519_hip_txn_frag.argtypes = [ctypes.c_char_p, ctypes.c_ulong, _v]
_lib.fd_ed25519_hip_txn_frag.restype = ctypes.c_ulong
_lib.fd_ed25519_hip_tcache_new.argtypes = [ctypes.c_ulong, ctypes.c_ulong]
_lib.fd_ed25519_hip_tcache_new.restype = _v
_lib.fd_ed25519_hip_tcache_delete.argtypes = [_v]
_lib.fd_ed25519_hip_tcache_query.argtypes = [_v, ctypes.c_ulong]
_lib.fd_ed25519_hip_tcache_insert.argtypes = [_v, ctypes.c_ulong]
_lib.fd_ed25519_hip_vtile_new.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_ulong, ctypes.c_ulong, ctypes.c_ulong,
                                          ctypes.c_int]
_lib.fd_ed25519_hip_vtile_new.restype = _v
_lib.fd_ed25519_hip_vtile_delete.argtypes = [_v]
_lib.fd_ed25519_hip_vtile_frag.argtypes = [_v, ctypes.c_char_p, ctypes.c_ulong, ctypes.c_ulong]
_lib.fd_ed25519_hip_vtile_flush.argtypes = [_v, ctypes.c_int]
_lib.fd_ed25519_hip_vtile_poll.argtypes = [_v, ctypes.c_int, ctypes.c_ulong, _v, _v, _v]
_lib.fd_ed25519_hip_vtile_poll.restype = ctypes.c_ulong
_lib.fd_ed25519_hip_vtile_poll_frags.argtypes = [_v, ctypes.c_int, ctypes.c_ulong, _v, _v, _v, _v, _v, _v,
                                                 ctypes.c_ulong]
_lib.fd_ed25519_hip_vtile_poll_frags.restype = ctypes.c_ulong
_lib.fd_ed25519_hip_vtile_pending.argtypes = [_v]
_lib.fd_ed25519_hip_vtile_pending.restype = ctypes.c_ulong
_lib.fd_ed25519_hip_latency_run.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_ulong, _v, _v, _v, ctypes.c_ulong,
                                            ctypes.c_double, ctypes.c_ulong, ctypes.c_int, _v, _v,
                                            ctypes.POINTER(LatencyResult)]
_lib.fd_ed25519_hip_latency_run_tiles.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_uint, ctypes.c_ulong, _v, _v, _v,
                                                  ctypes.c_ulong, ctypes.c_double, ctypes.c_ulong, ctypes.c_int, _v,
                                                  _v, ctypes.POINTER(LatencyResult)]
_lib.fd_ed25519_hip_pool_verify.argtypes = [_v, ctypes.c_uint, ctypes.c_uint, ctypes.c_ulong, ctypes.c_ulong, _v, _v,
                                            _v, _v, _v, _v, ctypes.POINTER(ctypes.c_double)]


class Slot(ctypes.Structure):
    """fd_ed25519_hip_slot_t: one batch of a pipe (pinned host arrays)."""
    _fields_ = [("msgs", ctypes.POINTER(ctypes.c_ubyte)), ("msg_off", ctypes.POINTER(ctypes.c_ulong)),
                ("msg_sz", ctypes.POINTER(ctypes.c_uint)), ("sigs", ctypes.POINTER(ctypes.c_ubyte)),
                ("pubs", ctypes.POINTER(ctypes.c_ubyte)), ("txn_first", ctypes.POINTER(ctypes.c_uint)),
                ("txn_sig_cnt", ctypes.POINTER(ctypes.c_uint)), ("sig_out", ctypes.POINTER(ctypes.c_byte)),
                ("txn_out", ctypes.POINTER(ctypes.c_byte)), ("txn_trailer", ctypes.POINTER(ctypes.c_ubyte)),
                ("sig_cap", ctypes.c_ulong), ("msg_cap", ctypes.c_ulong), ("txn_cap", ctypes.c_ulong),
                ("sig_cnt", ctypes.c_ulong), ("msg_bytes", ctypes.c_ulong), ("txn_cnt", ctypes.c_ulong),
                ("seq", ctypes.c_ulong), ("t_submit", ctypes.c_double), ("t_done", ctypes.c_double),
                ("user", ctypes.c_ulong)]


_lib.fd_ed25519_hip_pipe_new.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_ulong, ctypes.c_ulong, ctypes.c_ulong,
                                         ctypes.c_int]
_lib.fd_ed25519_hip_pipe_new.restype = _v
_lib.fd_ed25519_hip_pipe_delete.argtypes = [_v]
_lib.fd_ed25519_hip_pipe_acquire.argtypes = [_v]
_lib.fd_ed25519_hip_pipe_acquire.restype = ctypes.POINTER(Slot)
_lib.fd_ed25519_hip_pipe_submit.argtypes = [_v, ctypes.POINTER(Slot), ctypes.c_ulong, ctypes.c_ulong, ctypes.c_ulong]
_lib.fd_ed25519_hip_pipe_submit_txns.argtypes = [_v, ctypes.POINTER(Slot), ctypes.c_ulong, ctypes.c_ulong]
_lib.fd_ed25519_hip_pipe_poll.argtypes = [_v, ctypes.c_int]
_lib.fd_ed25519_hip_pipe_poll.restype = ctypes.POINTER(Slot)
_lib.fd_ed25519_hip_pipe_release.argtypes = [_v, ctypes.POINTER(Slot)]


class Pipe:
    """fd_ed25519_hip_pipe_*: slot_cnt batches in flight on one device, the
    caller staging each batch in place in its slot's pinned arrays."""

    def __init__(self, device=0, slot_cnt=2, sig_cap=4096, msg_cap=None, txn_cap=None, flags=0):
        msg_cap = sig_cap * TXN_MTU if msg_cap is None else msg_cap
        txn_cap = sig_cap if txn_cap is None else txn_cap
        self._p = _lib.fd_ed25519_hip_pipe_new(device, slot_cnt, sig_cap, msg_cap, txn_cap, flags)
        if not self._p:
            raise HipError("pipe_new failed")

    def acquire(self):
        s = _lib.fd_ed25519_hip_pipe_acquire(self._p)
        return s if s else None

    @staticmethod
    def arrays(slot):
        """numpy views of a slot's staging and output arrays"""
        c = slot.contents
        return {"msgs": np.ctypeslib.as_array(c.msgs, (c.msg_cap,)),
                "msg_off": np.ctypeslib.as_array(c.msg_off, (max(c.sig_cap, c.txn_cap),)),
                "msg_sz": np.ctypeslib.as_array(c.msg_sz, (max(c.sig_cap, c.txn_cap),)),
                "sigs": np.ctypeslib.as_array(c.sigs, (c.sig_cap * 64,)),
                "pubs": np.ctypeslib.as_array(c.pubs, (c.sig_cap * 32,)),
                "txn_first": np.ctypeslib.as_array(c.txn_first, (max(c.txn_cap, 1),)),
                "txn_sig_cnt": np.ctypeslib.as_array(c.txn_sig_cnt, (max(c.txn_cap, 1),)),
                "sig_out": np.ctypeslib.as_array(c.sig_out, (c.sig_cap,)),
                "txn_out": np.ctypeslib.as_array(c.txn_out, (max(c.txn_cap, 1),))}

    def submit(self, slot, sig_cnt, msg_bytes, txn_cnt=0):
        """the library's status code (0, or FD_ED25519_HIP_ERR_* with nothing enqueued)"""
        return _lib.fd_ed25519_hip_pipe_submit(self._p, slot, sig_cnt, msg_bytes, txn_cnt)

    def submit_txns(self, slot, txn_cnt, payload_bytes):
        return _lib.fd_ed25519_hip_pipe_submit_txns(self._p, slot, txn_cnt, payload_bytes)

    def poll(self, wait=True):
        s = _lib.fd_ed25519_hip_pipe_poll(self._p, 1 if wait else 0)
        return s if s else None

    def release(self, slot):
        _lib.fd_ed25519_hip_pipe_release(self._p, slot)

    def close(self):
        if self._p:
            _lib.fd_ed25519_hip_pipe_delete(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PoolStats(ctypes.Structure):
    _fields_ = [("direct_batches", ctypes.c_ulong), ("staged_batches", ctypes.c_ulong), ("h2d_bytes", ctypes.c_ulong)]


_lib.fd_ed25519_hip_pool_new.argtypes = [_v, ctypes.c_uint, ctypes.c_uint, ctypes.c_ulong, ctypes.c_ulong]
_lib.fd_ed25519_hip_pool_new.restype = _v
_lib.fd_ed25519_hip_pool_run.argtypes = [_v, ctypes.c_ulong, _v, _v, _v, _v, _v, _v, ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(PoolStats)]
_lib.fd_ed25519_hip_pool_delete.argtypes = [_v]
_lib.fd_ed25519_hip_host_register.argtypes = [_v, ctypes.c_ulong]
_lib.fd_ed25519_hip_host_unregister.argtypes = [_v]
_lib.fd_ed25519_hip_h2d_gbps.argtypes = [ctypes.c_int, ctypes.c_ulong, ctypes.c_uint]
_lib.fd_ed25519_hip_h2d_gbps.restype = ctypes.c_double


def txn_parse(payload):
    """fd_txn_parse: the parsed fields as a dict, or None if rejected."""
    t = Txn()
    payload = bytes(payload)
    if not _lib.fd_ed25519_hip_txn_parse(payload, len(payload), ctypes.byref(t)):
        return None
    return {f: getattr(t, f) for f in Txn.FIELDS}


def txn_parse_full(payload):
    """fd_txn_parse: the fd_txn_t bytes (its footprint), or None."""
    payload = bytes(payload)
    buf = ctypes.create_string_buffer(TXN_MAX_SZ)
    r = _lib.fd_ed25519_hip_txn_parse_full(payload, len(payload), buf)
    return buf.raw[:r] if r else None


def txn_frag(payload):
    """after_frag's output frag (payload, pad, fd_txn_t, payload_sz), or
    None when the parse filter drops the payload."""
    payload = bytes(payload)
    buf = ctypes.create_string_buffer(TPU_DCACHE_MTU)
    r = _lib.fd_ed25519_hip_txn_frag(payload, len(payload), buf)
    return buf.raw[:r] if r else None


class TCache:
    def __init__(self, depth=16, map_cnt=64):
        self._h = _lib.fd_ed25519_hip_tcache_new(depth, map_cnt)
        if not self._h:
            raise ValueError("bad tcache geometry (map_cnt must be a power of two >= depth+2)")

    def query(self, tag):
        return bool(_lib.fd_ed25519_hip_tcache_query(self._h, int(tag)))

    def insert(self, tag):
        """1 if tag was a duplicate (nothing inserted)."""
        return bool(_lib.fd_ed25519_hip_tcache_insert(self._h, int(tag)))

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.fd_ed25519_hip_tcache_delete(self._h)
            self._h = None


class VerifyTile:
    """The verify tile's batched core on one GPU."""

    def __init__(self, device=0, slot_cnt=3, batch_sigs=4096, tcache_depth=16, tcache_map_cnt=64, codes="avx512",
                 gpu_parse=False):
        flags = (1 if codes == "portable" else 0) | (VTILE_GPU_PARSE if gpu_parse else 0)
        self._h = _lib.fd_ed25519_hip_vtile_new(int(device), int(slot_cnt), int(batch_sigs), int(tcache_depth),
                                                int(tcache_map_cnt), flags)
        if not self._h:
            raise HipError(f"vtile_new failed: {_lib.fd_ed25519_hip_last_error().decode()}")

    def frag(self, payload, cookie):
        payload = bytes(payload)
        return _lib.fd_ed25519_hip_vtile_frag(self._h, payload, len(payload), int(cookie))

    def flush(self):
        return _lib.fd_ed25519_hip_vtile_flush(self._h, 1)

    def poll(self, wait=False, max_n=1 << 16):
        ck = np.zeros(max_n, np.uint64)
        vd = np.zeros(max_n, np.int8)
        tg = np.zeros(max_n, np.uint64)
        n = _lib.fd_ed25519_hip_vtile_poll(self._h, 1 if wait else 0, max_n, _ptr(ck), _ptr(vd), _ptr(tg))
        return ck[:n], vd[:n], tg[:n]

    def poll_frags(self, wait=False, max_n=4096):
        """As poll, plus the frag published for each SUCCESS (bytes) or None."""
        ck = np.zeros(max_n, np.uint64)
        vd = np.zeros(max_n, np.int8)
        tg = np.zeros(max_n, np.uint64)
        fo = np.zeros(max_n, np.uint64)
        fs = np.zeros(max_n, np.uint64)
        cap = max_n * ((TPU_DCACHE_MTU + 63) & ~63)
        fb = np.zeros(cap, np.uint8)
        n = _lib.fd_ed25519_hip_vtile_poll_frags(self._h, 1 if wait else 0, max_n, _ptr(ck), _ptr(vd), _ptr(tg),
                                                 _ptr(fo), _ptr(fs), _ptr(fb), cap)
        frags = [fb[int(fo[k]):int(fo[k]) + int(fs[k])].tobytes() if fs[k] else None for k in range(n)]
        return ck[:n], vd[:n], tg[:n], frags

    def pending(self):
        return _lib.fd_ed25519_hip_vtile_pending(self._h)

    def run(self, payloads, frags=False):
        """Every payload through the tile in order -> (verdicts, tags[,
        published frags]) by index."""
        n = len(payloads)
        verdict = np.full(n, 99, np.int8)
        tags = np.zeros(n, np.uint64)
        out = [None] * n

        def take(r):
            ck, vd, tg = r[:3]
            verdict[ck] = vd
            tags[ck] = tg
            if frags:
                for c, f in zip(ck, r[3]):
                    out[int(c)] = f

        poll = self.poll_frags if frags else self.poll
        for i, p in enumerate(payloads):
            self.frag(p, i)
            take(poll(False))
        self.flush()
        while self.pending():
            take(poll(True))
        return (verdict, tags, out) if frags else (verdict, tags)

    def close(self):
        if self._h:
            _lib.fd_ed25519_hip_vtile_delete(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pack_payloads(payloads):
    sz = np.array([len(p) for p in payloads], np.uint32)
    off = np.zeros(len(payloads), np.uint64)
    if len(payloads) > 1:
        np.cumsum(sz[:-1], dtype=np.uint64, out=off[1:])
    buf = np.frombuffer(b"".join(bytes(p) for p in payloads) or b"\0", np.uint8).copy()
    return buf, off, sz


_lib.fd_ed25519_hip_latency_set_cpus.argtypes = [ctypes.c_int, ctypes.c_int]
_lib.fd_ed25519_hip_pipe_set_host_scalars.argtypes = [ctypes.c_ulong]


def pipe_set_host_scalars(max_sigs):
    """fd_ed25519_hip_pipe_set_host_scalars: pipe batches of at most
    max_sigs signatures take the host-scalar path (0: none; default 4)"""
    _lib.fd_ed25519_hip_pipe_set_host_scalars(int(max_sigs))


_lib.fd_ed25519_hip_pipe_set_host_decode.argtypes = [ctypes.c_ulong]
_lib.fd_ed25519_hip_pipe_set_host_decode.restype = None


def pipe_set_host_decode(max_sigs):
    """fd_ed25519_hip_pipe_set_host_decode: host-scalar batches of at most
    max_sigs signatures also decompress A and R on the submitting thread
    (0: never; the library's default is 4)."""
    _lib.fd_ed25519_hip_pipe_set_host_decode(int(max_sigs))


_lib.fd_ed25519_hip_pipe_set_split_waves.argtypes = [ctypes.c_int]
_lib.fd_ed25519_hip_pipe_set_split_waves.restype = None


def pipe_set_split_waves(waves):
    """fd_ed25519_hip_pipe_set_split_waves: host-decoded pipe batches over
    4 or 8 waves (dsm16s) or dsm16's 2 (the default)."""
    _lib.fd_ed25519_hip_pipe_set_split_waves(int(waves))


def latency_set_cpus(producer_cpu=-1, tile_cpu=-1):
    """fd_ed25519_hip_latency_set_cpus: pin latency_run's producer and tile
    threads (one tile) to these CPUs for each run; -1 leaves one unpinned."""
    _check(_lib.fd_ed25519_hip_latency_set_cpus(int(producer_cpu), int(tile_cpu)))


def physical_cores(cpus):
    """one logical CPU per physical core among cpus (the lowest SMT
    sibling), in order"""
    out, seen = [], set()
    for c in sorted(cpus):
        try:
            sib = open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
        except OSError:
            sib = str(c)
        if sib not in seen:
            seen.add(sib)
            out.append(c)
    return out


def core_siblings(cpu):
    """every logical CPU of cpu's physical core (cpu itself without SMT)"""
    try:
        txt = open(f"/sys/devices/system/cpu/cpu{cpu}/topology/thread_siblings_list").read().strip()
    except OSError:
        return {cpu}
    out = set()
    for part in txt.split(","):
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out or {cpu}


def latency_run(payloads, offered_txn_per_s, device=0, slot_cnt=3, batch_sigs=256, ring_depth=4096, gpu_parse=False,
                tiles=1):
    """Latency mode (C5): a producer thread publishes the payloads into a
    tango-style ring at the offered rate; the verify tile consumes them.
    payloads: a list of byte strings, or a uint8 array [n][size] of
    equal-size payloads.  Returns (per-txn latency seconds, verdicts,
    result dict)."""
    if isinstance(payloads, np.ndarray) and payloads.ndim == 2:
        n, size = payloads.shape
        buf = np.ascontiguousarray(payloads).reshape(-1)
        off = np.arange(n, dtype=np.uint64) * np.uint64(size)
        sz = np.full(n, size, np.uint32)
    else:
        buf, off, sz = pack_payloads(payloads)
        n = len(payloads)
    lat = np.zeros(n, np.float64)
    verdict = np.zeros(n, np.int8)
    res = LatencyResult()
    if tiles > 1:   # several verify tiles, transaction i to tile i % tiles
        _check(_lib.fd_ed25519_hip_latency_run_tiles(int(device), int(tiles), int(slot_cnt), int(batch_sigs), _ptr(buf),
                                                     _ptr(off), _ptr(sz), n, float(offered_txn_per_s), int(ring_depth),
                                                     VTILE_GPU_PARSE if gpu_parse else 0, _ptr(lat), _ptr(verdict),
                                                     ctypes.byref(res)))
    else:
        _check(_lib.fd_ed25519_hip_latency_run(int(device), int(slot_cnt), int(batch_sigs), _ptr(buf), _ptr(off),
                                               _ptr(sz), n, float(offered_txn_per_s), int(ring_depth),
                                               VTILE_GPU_PARSE if gpu_parse else 0, _ptr(lat), _ptr(verdict),
                                               ctypes.byref(res)))
    return lat, verdict, {f: getattr(res, f) for f, _ in LatencyResult._fields_}


class Pool:
    """fd_ed25519_hip_pool: one feeder thread per entry of `devices`,
    slot_cnt batches of batch_sigs signatures in flight on each, msg_cap
    message bytes per batch; set up once, run many times."""

    def __init__(self, devices, batch_sigs=65536, slot_cnt=3, msg_cap=None):
        devs = np.ascontiguousarray(devices, np.int32)
        cap = int(msg_cap if msg_cap is not None else batch_sigs * TXN_MTU)
        self._h = _lib.fd_ed25519_hip_pool_new(_ptr(devs), len(devs), int(slot_cnt), int(batch_sigs), cap)
        if not self._h:
            raise HipError(f"pool_new failed: {_lib.fd_ed25519_hip_last_error().decode()}")

    def run(self, msgs, msg_off, msg_sz, sigs, pubs, out=None):
        """-> (codes, seconds, transfer stats).  Arrays registered with
        HostRegistration are DMA'd in place; others are staged."""
        n = len(msg_sz)
        if out is None:
            out = np.zeros(max(n, 1), np.int8)
        msgs = msgs if len(msgs) else np.zeros(1, np.uint8)
        arrs = [_c(msgs, np.uint8), _c(msg_off, np.uint64), _c(msg_sz, np.uint32), _c(sigs, np.uint8).reshape(-1),
                _c(pubs, np.uint8).reshape(-1)]
        sec = ctypes.c_double(0.0)
        st = PoolStats()
        _check(_lib.fd_ed25519_hip_pool_run(self._h, n, *[_ptr(a) for a in arrs], _ptr(out), ctypes.byref(sec),
                                            ctypes.byref(st)))
        return out[:n], sec.value, {f: getattr(st, f) for f, _ in PoolStats._fields_}

    def close(self):
        if self._h:
            _lib.fd_ed25519_hip_pool_delete(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def max_span(msg_off, msg_sz, batch_sigs):
    """The message capacity a pool needs for these batches: the largest
    span (or packed size) of a batch."""
    off = np.asarray(msg_off, np.uint64)
    end = off + np.asarray(msg_sz, np.uint64)
    cap = 1
    for i0 in range(0, len(off), batch_sigs):
        lo, hi = int(off[i0:i0 + batch_sigs].min()), int(end[i0:i0 + batch_sigs].max())
        byt = int(np.asarray(msg_sz[i0:i0 + batch_sigs], np.uint64).sum())
        cap = max(cap, hi - lo if hi - lo <= 2 * byt + 65536 else byt)
    return cap


def pool_verify(devices, msgs, msg_off, msg_sz, sigs, pubs, batch_sigs=65536, slot_cnt=3, out=None, stats=False):
    """Signatures dealt round-robin in batches over `devices` (one host
    feeder thread per entry) -> (codes, seconds[, stats]); a pool set up for
    this one call."""
    pool = Pool(devices, batch_sigs, slot_cnt, max_span(msg_off, msg_sz, batch_sigs) if len(msg_sz) else 1)
    try:
        codes, sec, st = pool.run(msgs, msg_off, msg_sz, sigs, pubs, out)
    finally:
        pool.close()
    return (codes, sec, st) if stats else (codes, sec)


class HostRegistration:
    """Page-locks numpy arrays for direct DMA (fd_ed25519_hip_host_register)
    for the life of the context."""

    def __init__(self, *arrays):
        self.arrays = [a for a in arrays if a is not None and a.nbytes]
        self.done = []

    def __enter__(self):
        for a in self.arrays:
            assert a.flags["C_CONTIGUOUS"]
            _check(_lib.fd_ed25519_hip_host_register(a.ctypes.data, a.nbytes))
            self.done.append(a)
        return self

    def __exit__(self, *exc):
        for a in self.done:
            _lib.fd_ed25519_hip_host_unregister(a.ctypes.data)
        self.done = []
        return False


def device_cpus(info):
    """The host CPUs on the NUMA node of an engine's device (from its PCI
    address, /sys/bus/pci/devices/<bdf>/local_cpulist), within this
    process's affinity; empty if unknown."""
    bdf = f"{info['pci_domain']:04x}:{info['pci_bus']:02x}:{info['pci_device']:02x}.0"
    try:
        text = open(f"/sys/bus/pci/devices/{bdf}/local_cpulist").read().strip()
    except OSError:
        return set()
    cpus = set()
    for part in text.split(","):
        if "-" in part:
            lo, hi = part.split("-")
            cpus.update(range(int(lo), int(hi) + 1))
        elif part:
            cpus.add(int(part))
    import os
    return cpus & os.sched_getaffinity(0)


class NearDevice:
    """Runs the enclosed block on the CPUs of the device's NUMA node, so
    that host buffers first touched there (numpy allocations) sit next to
    the GPU's PCIe link: DMA from the far socket crosses the inter-socket
    fabric."""

    def __init__(self, info):
        import os
        self.cpus = device_cpus(info)
        self.saved = os.sched_getaffinity(0)

    def __enter__(self):
        import os
        if self.cpus:
            os.sched_setaffinity(0, self.cpus)
        return self

    def __exit__(self, *exc):
        import os
        os.sched_setaffinity(0, self.saved)
        return False


_lib.fd_ed25519_hip_host_alloc.argtypes = [ctypes.c_ulong]
_lib.fd_ed25519_hip_host_alloc.restype = _v
_lib.fd_ed25519_hip_host_free.argtypes = [_v]


class _HostMem:
    def __init__(self, nbytes):
        self.ptr = _lib.fd_ed25519_hip_host_alloc(max(int(nbytes), 1))
        if not self.ptr:
            raise HipError(f"host_alloc({nbytes}) failed: {_lib.fd_ed25519_hip_last_error().decode()}")

    def __del__(self):
        if getattr(self, "ptr", None):
            _lib.fd_ed25519_hip_host_free(self.ptr)
            self.ptr = None


def host_array(shape, dtype, kind="thp"):
    """A host array for a host-fed stream: "numpy" (default allocation),
    "thp" (anonymous mmap with MADV_HUGEPAGE: 2 MB pages when the kernel
    grants them, fewer DMA translations), or "hostmalloc" (page-locked by
    the HIP driver, fd_ed25519_hip_host_alloc; needs no registration)."""
    dtype = np.dtype(dtype)
    nbytes = int(np.prod(shape)) * dtype.itemsize
    if kind == "numpy":
        return np.zeros(shape, dtype)
    if kind == "hostmalloc":
        mem = _HostMem(nbytes)
        buf = (ctypes.c_uint8 * max(nbytes, 1)).from_address(mem.ptr)
        buf._mem = mem   # the array's base keeps the allocation alive
        return np.frombuffer(buf, np.uint8, count=nbytes).view(dtype).reshape(shape)
    import mmap
    m = mmap.mmap(-1, max(nbytes, 1), flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    if hasattr(mmap, "MADV_HUGEPAGE"):
        try:
            m.madvise(mmap.MADV_HUGEPAGE)
        except OSError:
            pass
    return np.frombuffer(m, np.uint8, count=nbytes).view(dtype).reshape(shape)


def h2d_gbps(device=0, nbytes=256 << 20, reps=8):
    """Host -> device copy bandwidth from pinned memory, GB/s."""
    return _lib.fd_ed25519_hip_h2d_gbps(int(device), int(nbytes), int(reps))


# ---- shlink + verify service (the GPU process behind a sandboxed tile) ----

SHLINK_CTL_EOS = 1
PRODUCER_BIN = (__import__("os").environ.get("FD_SHLINK_PRODUCER") or   # the sanitizer run's build
                __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)),
                                           "_lib", "fd_shlink_producer"))


class VServiceStats(ctypes.Structure):
    _fields_ = [("txn_cnt", ctypes.c_ulong), ("batches", ctypes.c_ulong), ("seconds", ctypes.c_double),
                ("device_bytes", ctypes.c_ulong), ("shared_device_bytes", ctypes.c_ulong), ("end_code", ctypes.c_int),
                ("leaked_on_hang", ctypes.c_uint)]


_lib.fd_ed25519_hip_shlink_create.argtypes = [ctypes.c_char_p, ctypes.c_ulong]
_lib.fd_ed25519_hip_shlink_create.restype = _v
_lib.fd_ed25519_hip_shlink_join.argtypes = [ctypes.c_char_p]
_lib.fd_ed25519_hip_shlink_join.restype = _v
_lib.fd_ed25519_hip_shlink_leave.argtypes = [_v, ctypes.c_int]
_lib.fd_ed25519_hip_shlink_depth.argtypes = [_v]
_lib.fd_ed25519_hip_shlink_depth.restype = ctypes.c_ulong
_lib.fd_ed25519_hip_shlink_publish.argtypes = [_v, ctypes.c_char_p, ctypes.c_ulong, ctypes.c_ulong, ctypes.c_uint]
_lib.fd_ed25519_hip_shlink_publish.restype = ctypes.c_int
_lib.fd_ed25519_hip_shlink_consume.argtypes = [_v, _v, ctypes.POINTER(ctypes.c_ulong), ctypes.POINTER(ctypes.c_ulong),
                                               ctypes.POINTER(ctypes.c_uint)]
_lib.fd_ed25519_hip_shlink_consume.restype = ctypes.c_int
_lib.fd_ed25519_hip_vservice_run.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_ulong, ctypes.c_int, _v, _v,
                                             ctypes.POINTER(VServiceStats)]
# the library and these ctypes mirrors must describe the same ABI
_lib.fd_ed25519_hip_abi_check.argtypes = [ctypes.c_uint, ctypes.c_ulong, ctypes.c_ulong, ctypes.c_ulong]
ABI_VERSION = 10   # FD_ED25519_HIP_ABI_VERSION
if _lib.fd_ed25519_hip_abi_check(ABI_VERSION, ctypes.sizeof(Slot), ctypes.sizeof(__import__(
        "firedancer_amd.ed25519", fromlist=["_Info"])._Info), ctypes.sizeof(VServiceStats)) != 0:
    raise ImportError("libfd_ed25519_hip ABI mismatch: " + _lib.fd_ed25519_hip_last_error().decode())
_lib.fd_ed25519_hip_shlink_heartbeat.argtypes = [_v, ctypes.c_ulong]
_lib.fd_ed25519_hip_shlink_heartbeat_query.argtypes = [_v]
_lib.fd_ed25519_hip_shlink_heartbeat_query.restype = ctypes.c_ulong
_lib.fd_ed25519_hip_shlink_fail.argtypes = [_v, ctypes.c_int]
_lib.fd_ed25519_hip_shlink_status.argtypes = [_v]
_lib.fd_ed25519_hip_shlink_status.restype = ctypes.c_int
SHLINK_FAIL_PROTOCOL = -100
SHLINK_FAIL_STOPPED = -101
SHLINK_FAIL_TILE_GONE = -102
SHLINK_PROTO = 6          # FD_ED25519_HIP_SHLINK_PROTO


class ShLinkWatch(ctypes.Structure):
    """fd_ed25519_hip_shlink_watch_t: a consumer's view of its producer's
    heartbeat; check() -> 1 never ticked, 0 alive, -1 stale."""
    _fields_ = [("last", ctypes.c_ulong), ("t_ns", ctypes.c_long), ("seen", ctypes.c_int)]

    def check(self, link, now_ns, stale_ns):
        return _lib.fd_ed25519_hip_shlink_watch(ctypes.byref(self), link._h, int(now_ns), int(stale_ns))


_lib.fd_ed25519_hip_shlink_watch.argtypes = [ctypes.POINTER(ShLinkWatch), _v, ctypes.c_long, ctypes.c_long]
_lib.fd_ed25519_hip_shlink_watch.restype = ctypes.c_int


class ShLink:
    """fd_ed25519_hip_shlink: a tango-style mcache/dcache in POSIX shared
    memory, one producer and one consumer process (one handle per side)."""

    def __init__(self, name, depth=0, create=False):
        self.name = name
        h = (_lib.fd_ed25519_hip_shlink_create(name.encode(), int(depth)) if create
             else _lib.fd_ed25519_hip_shlink_join(name.encode()))
        if not h:
            import errno as _errno
            e = ctypes.get_errno()
            raise HipError(-1, f"shlink {'create' if create else 'join'} {name} failed "
                               f"({_errno.errorcode.get(e, e)})")
        self._h, self._owner = h, create
        self._buf = ctypes.create_string_buffer(SHLINK_MTU)

    @property
    def depth(self):
        return _lib.fd_ed25519_hip_shlink_depth(self._h)

    def publish(self, payload, sig, ctl=0):
        """True if published, False if no credit (retry)."""
        r = _lib.fd_ed25519_hip_shlink_publish(self._h, bytes(payload), len(payload), int(sig), int(ctl))
        if r < 0:
            _check(r)
        return r == 0

    def consume(self):
        """(payload, sig, ctl), or None if nothing is published yet."""
        sz, sig, ctl = ctypes.c_ulong(), ctypes.c_ulong(), ctypes.c_uint()
        r = _lib.fd_ed25519_hip_shlink_consume(self._h, self._buf, ctypes.byref(sz), ctypes.byref(sig),
                                               ctypes.byref(ctl))
        if r == 1:
            return None
        if r:
            raise HipError(r, "shlink overrun")
        return self._buf.raw[:sz.value], sig.value, ctl.value

    def heartbeat(self, value):
        """The producer's liveness tick (fd_ed25519_hip_shlink_heartbeat)."""
        _lib.fd_ed25519_hip_shlink_heartbeat(self._h, int(value))

    def heartbeat_query(self):
        return _lib.fd_ed25519_hip_shlink_heartbeat_query(self._h)

    def fail(self, code):
        _lib.fd_ed25519_hip_shlink_fail(self._h, int(code))

    def status(self):
        return _lib.fd_ed25519_hip_shlink_status(self._h)

    def close(self, unlink=None):
        if self._h:
            _lib.fd_ed25519_hip_shlink_leave(self._h, int(self._owner if unlink is None else unlink))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def vservice_run(in_link, out_link, device=0, slot_cnt=3, batch_sigs=4096, gpu_parse=True, codes="avx512"):
    """The GPU side of a sandboxed verify tile: serves in_link -> out_link
    until the EOS frag (fd_ed25519_hip_vservice_run).  Returns its stats."""
    from .ed25519 import FLAG_CODES_PORTABLE
    flags = (VTILE_GPU_PARSE if gpu_parse else 0) | (FLAG_CODES_PORTABLE if codes == "portable" else 0)
    st = VServiceStats()
    _check(_lib.fd_ed25519_hip_vservice_run(int(device), int(slot_cnt), int(batch_sigs), flags, in_link._h,
                                            out_link._h, ctypes.byref(st)))
    return {f: getattr(st, f) for f, _ in VServiceStats._fields_}


class VServiceOpts(ctypes.Structure):
    _fields_ = [("stop", ctypes.c_void_p), ("tile_stale_ns", ctypes.c_long), ("gpu_hang_ns", ctypes.c_long),
                ("ready", ctypes.c_void_p), ("ready_ctx", ctypes.c_void_p), ("links_per_thread", ctypes.c_uint),
                ("link_cpus", ctypes.POINTER(ctypes.c_int)), ("link_cpu_cnt", ctypes.c_uint)]


_lib.fd_ed25519_hip_vservice_serve.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_ulong, ctypes.c_int,
                                               ctypes.POINTER(_v), ctypes.POINTER(_v), ctypes.c_uint,
                                               ctypes.POINTER(VServiceStats), ctypes.POINTER(VServiceOpts)]


def vservice_serve(in_links, out_links, device=0, slot_cnt=3, batch_sigs=4096, gpu_parse=True, codes="avx512",
                   tile_stale_s=0.0, gpu_hang_s=0.0, links_per_thread=1, cpus=None):
    """Several link pairs on one device (fd_ed25519_hip_vservice_serve),
    links_per_thread pairs per service thread, thread t on cpus[t % len]
    (None: the process's affinity):
    -> (status, [stats per pair]); status 0 when every pair ended with EOS,
    else the device failure's code or the first link-local end."""
    from .ed25519 import FLAG_CODES_PORTABLE
    flags = (VTILE_GPU_PARSE if gpu_parse else 0) | (FLAG_CODES_PORTABLE if codes == "portable" else 0)
    k = len(in_links)
    ins = (_v * k)(*[l._h for l in in_links])
    outs = (_v * k)(*[l._h for l in out_links])
    st = (VServiceStats * k)()
    cpu_arr = (ctypes.c_int * len(cpus))(*cpus) if cpus else None
    opts = VServiceOpts(None, int(tile_stale_s * 1e9), int(gpu_hang_s * 1e9), None, None, int(links_per_thread),
                        cpu_arr, len(cpus) if cpus else 0)
    rc = _lib.fd_ed25519_hip_vservice_serve(int(device), int(slot_cnt), int(batch_sigs), flags, ins, outs, k, st,
                                            ctypes.byref(opts))
    return rc, [{f: getattr(x, f) for f, _ in VServiceStats._fields_} for x in st]


def parse_producer_frags(blob):
    """The producer tool's frag records (u32 size, bytes) -> list of bytes."""
    out, i = [], 0
    while i < len(blob):
        k = int.from_bytes(blob[i:i + 4], "little")
        out.append(bytes(blob[i + 4:i + 4 + k]))
        i += 4 + k
    return out


def write_payload_file(path, payloads):
    """The producer tool's input: u64 n, n x u32 sizes, the payloads."""
    with open(path, "wb") as f:
        f.write(np.uint64(len(payloads)).tobytes())
        f.write(np.array([len(p) for p in payloads], np.uint32).tobytes())
        for p in payloads:
            f.write(bytes(p))
