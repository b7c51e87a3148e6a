"""Parity at BASELINE.json's full sizes, checked signature by signature
against the reference itself (fd_ed25519_verify of the AVX-512 backend,
compiled from its sources into oracle/_ref, on the box's host cores):

  C2  the whole 1,048,576-signature workload bench.py measures
      (64-1232 B messages, 2% invalid in seven classes)
  C4  a 12,582,912-signature stream of the same distribution (>= 10M, the
      north star's parity target), verified on the GPU in 1M chunks; its
      verdict-stream SHA-256 is recorded in gpurun_out/ (and, per round,
      in profiles/) next to the 64M stream's."""
import ctypes
import hashlib
import json
import os
import time

import numpy as np
import pytest

from conftest import REPO
from txn_util import cpu_has_avx512ifma

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ref():
    flavour = "avx512" if cpu_has_avx512ifma() else "portable"
    path = os.path.join(REPO, "oracle", "_ref", f"libfdref_{flavour}.so")
    if not os.path.exists(path):
        pytest.fail(f"{path} not built")
    lib = ctypes.CDLL(path)
    lib.fdref_verify_many.restype = ctypes.c_long
    lib.fdref_verify_many.argtypes = [ctypes.c_ulong] + [ctypes.c_void_p] * 6 + [ctypes.c_int, ctypes.c_ulong]
    lib.flavour = flavour
    return lib


def _ref_codes(ref, wl, n, threads):
    sizes = wl.sizes[:n].astype(np.uint64)
    off = np.zeros(n, np.uint64)
    np.cumsum(sizes[:-1], out=off[1:])
    msgs = wl.msgs.download(np.uint8, max(int(sizes.sum()), 1))
    sigs = wl.sigs.download(np.uint8, 64 * n)
    pubs = wl.pubs.download(np.uint8, 32 * n)
    sz = wl.sizes[:n].astype(np.uint32)
    out = np.zeros(n, np.int8)
    ns = ref.fdref_verify_many(n, msgs.ctypes.data, off.ctypes.data, sz.ctypes.data, sigs.ctypes.data,
                               pubs.ctypes.data, out.ctypes.data, threads, 1)
    assert ns > 0
    return out, ns * 1e-9


def test_c2_full_size(ref):
    from firedancer_amd import ed25519, workload
    cfg = workload.CONFIGS["C2"]
    threads, _ = workload.host_cores()
    eng = ed25519.Engine(0, max_chunk=1 << 20)
    wl = ed25519.DeviceWorkload(eng, cfg["n"], cfg["lo"], cfg["hi"], cfg["ppm"], seed=0x5EED)
    try:
        wl.verify()
        eng.sync()
        got = wl.out.download(np.int8, wl.n)
        labels = wl.expect.download(np.int8, wl.n)
        want, _ = _ref_codes(ref, wl, wl.n, threads)
    finally:
        wl.free()
        eng.close()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(int(i), int(got[i]), int(want[i])) for i in bad[:8]]
    assert np.array_equal(want, labels)
    assert 0.015 < (want != 0).mean() < 0.025


@pytest.fixture(scope="module")
def c2_small_chunks(ref):
    """the C2 workload and the reference's codes for it, once for the
    small-chunk forms below"""
    from firedancer_amd import ed25519, workload
    cfg = workload.CONFIGS["C2"]
    threads, _ = workload.host_cores()
    eng = ed25519.Engine(0, max_chunk=1 << 20)
    wl = ed25519.DeviceWorkload(eng, cfg["n"], cfg["lo"], cfg["hi"], cfg["ppm"], seed=0x5EED)
    want, _ = _ref_codes(ref, wl, wl.n, threads)
    yield wl, want
    wl.free()
    eng.close()


@pytest.mark.parametrize("chunk,opts", [(256, {}), (4096, {}), (16384, {}), (1 << 20, {"compact": True}),
                                        (1 << 20, {"half": "strict"}), (256, {"half": "strict"})],
                         ids=["r16", "oct", "quad", "wide-compact", "wide-strict", "r16-strict"])
def test_c2_full_size_small_chunks(c2_small_chunks, chunk, opts):
    """The whole C2 workload through an engine of small chunks -- the
    latency forms a tile slot or a drop-in launch takes: 256 signatures a
    chunk (prep16 + dsm16), 4096 (dsm8), 16384 (dsm4) -- and through the
    throughput form with the compact base tables (the drop-ins') or with
    FLAG_HALF_STRICT (every k without a 131-bit pair, ~0.16%, in the
    full-length form: the one-lane dsm kernel's items, or prep16's lanes at
    256 a chunk), code by code against the reference."""
    from firedancer_amd import ed25519
    wl, want = c2_small_chunks
    eng = ed25519.Engine(0, max_chunk=chunk, **opts)
    out = eng.alloc(wl.n)
    try:
        eng.verify_dev(wl.n, wl.msgs.ptr, wl.off.ptr, wl.sz.ptr, wl.sigs.ptr, wl.pubs.ptr, out.ptr)
        eng.sync()
        got = out.download(np.int8, wl.n)
    finally:
        out.free()
        eng.close()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(int(i), int(got[i]), int(want[i])) for i in bad[:8]]


def test_dropin_on_c2_sample(c2_small_chunks):
    """fd_ed25519_verify, one synchronous call per signature (the drop-in's
    latency path: a one-signature launch reading the pinned block in place),
    over the first 20,000 signatures of the C2 workload -- its invalid
    classes included -- against the reference's codes."""
    from firedancer_amd import ed25519
    wl, want = c2_small_chunks
    n = 20000
    sizes = wl.sizes[:n].astype(np.uint64)
    off = np.zeros(n, np.uint64)
    np.cumsum(sizes[:-1], out=off[1:])
    msgs = wl.msgs.download(np.uint8, int(sizes.sum()))
    sigs = wl.sigs.download(np.uint8, 64 * n).reshape(n, 64)
    pubs = wl.pubs.download(np.uint8, 32 * n).reshape(n, 32)
    got = np.array([ed25519.verify(msgs[int(off[i]):int(off[i] + sizes[i])].tobytes(), sigs[i].tobytes(),
                                   pubs[i].tobytes()) for i in range(n)], np.int8)
    assert (want[:n] != 0).sum() > 100   # the sample holds every invalid class several times over
    bad = np.nonzero(got != want[:n])[0]
    assert len(bad) == 0, [(int(i), int(got[i]), int(want[i])) for i in bad[:8]]


def test_c2_full_size_portable_codes(c2_small_chunks):
    """The C2 workload with FD_ED25519_HIP_FLAG_CODES_PORTABLE (the
    reference's portable backend's error codes: a public key that does not
    decode is ERR_PUBKEY there, ERR_SIG in the AVX-512 backend), code by
    code against the reference's portable build; the verdicts (zero or
    not) equal the AVX-512 reference's."""
    from firedancer_amd import ed25519, workload
    wl, want_avx = c2_small_chunks
    path = os.path.join(REPO, "oracle", "_ref", "libfdref_portable.so")
    if not os.path.exists(path):
        pytest.fail(f"{path} not built")
    lib = ctypes.CDLL(path)
    lib.fdref_verify_many.restype = ctypes.c_long
    lib.fdref_verify_many.argtypes = [ctypes.c_ulong] + [ctypes.c_void_p] * 6 + [ctypes.c_int, ctypes.c_ulong]
    threads, _ = workload.host_cores()
    want, _ = _ref_codes(lib, wl, wl.n, threads)
    eng = ed25519.Engine(0, max_chunk=1 << 20, codes="portable")
    out = eng.alloc(wl.n)
    try:
        eng.verify_dev(wl.n, wl.msgs.ptr, wl.off.ptr, wl.sz.ptr, wl.sigs.ptr, wl.pubs.ptr, out.ptr)
        eng.sync()
        got = out.download(np.int8, wl.n)
    finally:
        out.free()
        eng.close()
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(int(i), int(got[i]), int(want[i])) for i in bad[:8]]
    assert np.array_equal(want != 0, want_avx != 0)
    assert (want != want_avx).any()   # the workload holds the classes whose codes differ


def test_c4_stream_12m(ref):
    """>= 10M signatures (12M: 12 chunks of 1M, seed 0xC4C4, the 64M
    stream's first 12M) code by code against the reference."""
    from firedancer_amd import ed25519, workload
    cfg = workload.CONFIGS["C2"]
    threads, _ = workload.host_cores()
    total, chunk, seed = 12 << 20, 1 << 20, 0xC4C4
    eng = ed25519.Engine(0, max_chunk=chunk)
    dig = hashlib.sha256()
    mism = label_mism = 0
    t_gpu = t_ref = 0.0
    codes = {c: 0 for c in (0, -1, -2, -3)}
    t_start = time.time()
    try:
        for base in range(0, total, chunk):
            wl = ed25519.DeviceWorkload(eng, chunk, cfg["lo"], cfg["hi"], cfg["ppm"], seed=seed, index_base=base)
            t0 = time.perf_counter()
            wl.verify()
            eng.sync()
            t_gpu += time.perf_counter() - t0
            got = wl.out.download(np.int8, chunk)
            label_mism += int((got != wl.expect.download(np.int8, chunk)).sum())
            want, dt = _ref_codes(ref, wl, chunk, threads)
            t_ref += dt
            mism += int((got != want).sum())
            for c in codes:
                codes[c] += int((got == c).sum())
            dig.update(got.tobytes())
            wl.free()
            print(f"c4 stream: {base + chunk} verified, mismatches {mism} ({time.time() - t_start:.0f} s)", flush=True)
    finally:
        eng.close()
    rec = {"stream": f"C2 distribution, {total} signatures in chunks of {chunk}, seed {seed:#x} "
                     f"(the first {total} of the 64M stream of profiles/r1_parity_stream_64M_v12.json)",
           "signatures": total, "reference": f"fd_ed25519_verify ({ref.flavour} backend, compiled from the reference "
                                             f"sources), {threads} threads",
           "reference_mismatches": mism, "label_mismatches": label_mism, "code_counts": {str(k): v for k, v in codes.items()},
           "gpu_seconds": t_gpu, "gpu_verifies_per_s": total / t_gpu, "reference_seconds": t_ref,
           "reference_verifies_per_s": total / t_ref, "verdict_stream_sha256": dig.hexdigest(),
           "bit_exact": mism == 0 and label_mism == 0}
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    json.dump(rec, open(os.path.join(REPO, "gpurun_out", "c4_stream_12m.json"), "w"), indent=1)
    assert mism == 0 and label_mism == 0, rec
