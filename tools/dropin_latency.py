#!/usr/bin/env python3
"""Per-call latency of the synchronous drop-ins (fd_ed25519_verify,
fd_ed25519_verify_batch_single_msg on the library's default engine) next
to the reference's CPU verify of the same inputs (oracle/_ref, one call,
one core): the numbers behind INTEGRATION.md's advice on which callers
keep the CPU path.

    python tools/dropin_latency.py [--calls 2000] [--out gpurun_out/dropin_latency.json]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def pct(a):
    a = np.asarray(a) * 1e6
    return {"p50_us": float(np.percentile(a, 50)), "p99_us": float(np.percentile(a, 99)), "mean_us": float(a.mean())}


def thread_scaling(ed25519, msgs, sigs, pubs, calls):
    """fd_ed25519_verify from 1, 2, 4, 8 threads at once (the drop-in's flat
    combining: concurrent callers share launches); calls per second over
    all threads and the per-call p50 / p99."""
    import threading
    out = {}
    for nth in (1, 2, 4, 8):
        per = max(50, calls // nth)
        lat = [[] for _ in range(nth)]

        def run(k):
            for j in range(per):
                i = (k * 31 + j) % 64
                t = time.perf_counter()
                assert ed25519.verify(msgs[200 * i:200 * i + 200].tobytes(), sigs[i].tobytes(), pubs[i].tobytes()) == 0
                lat[k].append(time.perf_counter() - t)
        th = [threading.Thread(target=run, args=(k,)) for k in range(nth)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        out[str(nth)] = dict(pct(np.concatenate([np.asarray(x) for x in lat])), calls_per_s=nth * per / dt)
    return out


def large_messages(ed25519, lib, ref, sizes, reps):
    """fd_ed25519_verify on one message of each size (device SHA-512: below
    the 4 GiB host-hash limit), signed on the GPU (fd_ed25519_hip_sign_dev),
    next to the reference's CPU verify of the same bytes."""
    eng = ed25519.Engine(0, max_chunk=1 << 12)
    rng = np.random.default_rng(17)
    out = {}
    for sz in [int(x) for x in str(sizes).split(",") if x and x != "none"]:
        m = rng.integers(0, 256, sz, dtype=np.uint8)
        bufs = [eng.alloc(max(sz, 1)).upload(m), eng.alloc(8).upload(np.zeros(1, np.uint64)),
                eng.alloc(4).upload(np.array([sz], np.uint32)),
                eng.alloc(32).upload(rng.integers(0, 256, 32, dtype=np.uint8)), eng.alloc(64), eng.alloc(32)]
        eng.sign_dev(1, *[b.ptr for b in bufs])
        eng.sync()
        sig, pub = bufs[4].download(np.uint8, 64).tobytes(), bufs[5].download(np.uint8, 32).tobytes()
        for b in bufs:
            b.free()
        mb = m.tobytes()
        t_gpu, t_cpu = [], []
        for _ in range(reps + 2):
            t = time.perf_counter()
            rc = lib.fd_ed25519_verify(mb, sz, sig, pub, None)
            t_gpu.append(time.perf_counter() - t)
            assert rc == 0, (sz, rc)
            t = time.perf_counter()
            rc = ref.fdref_verify(mb, sz, sig, pub)
            t_cpu.append(time.perf_counter() - t)
            assert rc == 0, (sz, rc)
        out[str(sz)] = {"gpu_dropin": pct(t_gpu[2:]), "reference_cpu_one_core": pct(t_cpu[2:]),
                        "path": "host scalars (message hashed on the calling thread, not staged)"}
    eng.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "dropin_latency.json"))
    ap.add_argument("--host-scalars", type=int, default=None,
                    help="fd_ed25519_hip_dropin_set_host_scalars (A/B; default: the library's)")
    ap.add_argument("--host-decode", type=int, default=None,
                    help="fd_ed25519_hip_dropin_set_host_decode (A/B; default: the library's)")
    ap.add_argument("--split", type=int, default=None, help="fd_ed25519_hip_dropin_set_split_waves (A/B: 2, 4, 8)")
    ap.add_argument("--threads", action="store_true", help="also the 1/2/4/8-thread scaling")
    ap.add_argument("--large", default="16384,65376,65377,1048576,8388608",
                    help="message sizes (bytes) for the device-hashed large-message latencies")
    args = ap.parse_args()
    from firedancer_amd import ed25519, workload
    eng = ed25519.Engine(0, max_chunk=1 << 12)
    wl = ed25519.DeviceWorkload(eng, 64, 200, 200, 0, seed=3)
    msgs = wl.msgs.download(np.uint8, wl.msg_bytes)
    sigs = wl.sigs.download(np.uint8, 64 * 64).reshape(64, 64)
    pubs = wl.pubs.download(np.uint8, 32 * 64).reshape(64, 32)
    wl.free()
    eng.close()
    lib = ed25519.library()
    res = {}
    if args.host_scalars is not None:
        lib.fd_ed25519_hip_dropin_set_host_scalars.argtypes = [ctypes.c_ulong]
        lib.fd_ed25519_hip_dropin_set_host_scalars(args.host_scalars)
        res["host_scalars_max_sigs"] = args.host_scalars
    if args.split is not None:
        lib.fd_ed25519_hip_dropin_set_split_waves.argtypes = [ctypes.c_int]
        lib.fd_ed25519_hip_dropin_set_split_waves(args.split)
        res["split_waves"] = args.split
    if args.host_decode is not None:
        lib.fd_ed25519_hip_dropin_set_host_decode.argtypes = [ctypes.c_ulong]
        lib.fd_ed25519_hip_dropin_set_host_decode(args.host_decode)
        res["host_decode_max_sigs"] = args.host_decode
    for _ in range(20):   # warm-up: the default engine, code objects
        ed25519.verify(msgs[:200].tobytes(), sigs[0].tobytes(), pubs[0].tobytes())
    t_one = []
    for i in range(args.calls):
        k = i % 64
        m, s, p = msgs[200 * k:200 * k + 200].tobytes(), sigs[k].tobytes(), pubs[k].tobytes()
        t = time.perf_counter()
        rc = lib.fd_ed25519_verify(m, 200, s, p, None)
        t_one.append(time.perf_counter() - t)
        assert rc == 0
    res["fd_ed25519_verify_gpu_dropin"] = pct(t_one)
    if args.threads:
        res["thread_scaling"] = thread_scaling(ed25519, msgs, sigs, pubs, args.calls)
    # fd_ed25519_verify_batch_single_msg on the golden batch's valid
    # transactions of 1, 2 and 4 signatures (one message, several signers)
    bd = np.load(os.path.join(REPO, "tests", "golden", "batch.npz"))
    res["batch_single_msg_gpu_dropin"] = {}
    for want in (1, 2, 4):
        txns = [t for t in range(len(bd["txn_cnt"])) if int(bd["txn_cnt"][t]) == want and int(bd["codes_avx512"][t]) == 0]
        if not txns:
            continue
        calls = []
        for t in txns[:16]:
            o, z, f = int(bd["txn_msg_off"][t]), int(bd["txn_msg_sz"][t]), int(bd["txn_first"][t])
            calls.append((bytes(bd["msgs"][o:o + z]), bd["sigs"][f:f + want].tobytes(), bd["pubs"][f:f + want].tobytes()))
        lat = []
        for i in range(max(200, args.calls // 4)):
            m, s, p = calls[i % len(calls)]
            t0 = time.perf_counter()
            assert ed25519.verify_batch_single_msg(m, s, p, want) == 0
            lat.append(time.perf_counter() - t0)
        res["batch_single_msg_gpu_dropin"][f"{want}_signatures"] = pct(lat[10:])
    # a 4-signer transaction over one message (sign the first message with 4 keys on the device)
    ref = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libfdref_portable.so"))
    ref.fdref_verify.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p]
    flavour = "portable"
    try:
        flags = next(l for l in open("/proc/cpuinfo") if l.startswith("flags")).split()
        if "avx512ifma" in flags and "avx512vbmi" in flags:
            ref = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libfdref_avx512.so"))
            ref.fdref_verify.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p]
            flavour = "avx512"
    except StopIteration:
        pass
    t_ref = []
    for i in range(args.calls):
        k = i % 64
        m, s, p = msgs[200 * k:200 * k + 200].tobytes(), sigs[k].tobytes(), pubs[k].tobytes()
        t = time.perf_counter()
        rc = ref.fdref_verify(m, 200, s, p)
        t_ref.append(time.perf_counter() - t)
        assert rc == 0
    res[f"fd_ed25519_verify_reference_cpu_{flavour}_one_core"] = pct(t_ref)
    res["msg_sz"] = 200
    res["large_messages"] = large_messages(ed25519, lib, ref, args.large, max(4, args.calls // 100))
    res["note"] = ("synchronous per-call latency through ctypes (~1 us of the GPU figure is the call itself); a call "
                   "of at most 4 single-signature requests (every case here) takes host scalars: the calling thread "
                   "hashes R||A||M and finds the half-size scalars; at most 2 (the one-caller case here) also "
                   "decompresses A and R on that thread and launches dsm16 alone, which reads the scalars, points, "
                   "signature and key from the pinned block in place (3-4: prep16's decode blocks run meanwhile); no "
                   "copy launches, and the host polls the block for the codes; the message is never staged for the "
                   "device")
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
