#!/usr/bin/env python3
"""Bit-exact parity of the MI355X engine with the reference over a long
stream (north star: >= 10M mixed valid/invalid signatures; C4: a 64M
stream), run on the GPU box.

The stream is the C2 distribution (64-1232 B messages, 2% invalid in seven
classes), generated chunk by chunk on the GPU (distinct keys per global
index).  Every chunk is verified on the GPU and its codes are checked
against the class labels; the first --ref-chunks chunks are also verified
by the reference's own fd_ed25519_verify (AVX-512 backend compiled from its
sources into oracle/_ref, one pthread per host core) and compared code by
code.  A SHA-256 digest of the GPU verdict stream is reported.

    python tools/parity_stream.py --total 67108864 --ref-total 16777216 --out gpurun_out/parity.json
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total", type=int, default=64 << 20)
    ap.add_argument("--ref-total", type=int, default=16 << 20)
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--seed", type=int, default=0xC4C4)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "parity_stream.json"))
    args = ap.parse_args()

    from firedancer_amd import ed25519, workload
    cfg = workload.CONFIGS["C2"]
    eng = ed25519.Engine(0, max_chunk=args.chunk)
    flavour = "avx512"
    ref = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", f"libfdref_{flavour}.so"))
    ref.fdref_verify_many.restype = ctypes.c_long
    ref.fdref_verify_many.argtypes = [ctypes.c_ulong] + [ctypes.c_void_p] * 6 + [ctypes.c_int, ctypes.c_ulong]

    dig = hashlib.sha256()
    t_gpu = t_ref = 0.0
    n_done = n_ref = label_mism = ref_mism = 0
    classes = np.zeros(8, np.int64)
    codes_hist = {c: 0 for c in (0, -1, -2, -3)}
    first_bad = []
    base = 0
    t_start = time.time()
    while base < args.total:
        n = min(args.chunk, args.total - base)
        wl = ed25519.DeviceWorkload(eng, n, cfg["lo"], cfg["hi"], cfg["ppm"], seed=args.seed, index_base=base)
        t0 = time.perf_counter()
        wl.verify()
        eng.sync()
        t_gpu += time.perf_counter() - t0
        out = wl.out.download(np.int8, n)
        expect = wl.expect.download(np.int8, n)
        cls = wl.cls.download(np.uint8, n)
        classes += np.bincount(cls, minlength=8)[:8]
        for c in codes_hist:
            codes_hist[c] += int((out == c).sum())
        bad = np.nonzero(out != expect)[0]
        label_mism += len(bad)
        first_bad += [(base + int(i), int(out[i]), int(expect[i]), "label") for i in bad[:4]]
        dig.update(out.tobytes())
        if n_ref < args.ref_total:
            m = min(n, args.ref_total - n_ref)
            sizes = wl.sizes[:m].astype(np.uint64)
            off = np.zeros(m, np.uint64)
            np.cumsum(sizes[:-1], out=off[1:])
            msgs = wl.msgs.download(np.uint8, max(int(sizes.sum()), 1))
            sigs = wl.sigs.download(np.uint8, 64 * m)
            pubs = wl.pubs.download(np.uint8, 32 * m)
            sz = wl.sizes[:m].astype(np.uint32)
            ro = np.zeros(m, np.int8)
            ns = ref.fdref_verify_many(m, msgs.ctypes.data, off.ctypes.data, sz.ctypes.data, sigs.ctypes.data,
                                       pubs.ctypes.data, ro.ctypes.data, args.threads, 1)
            t_ref += ns * 1e-9
            rb = np.nonzero(ro != out[:m])[0]
            ref_mism += len(rb)
            first_bad += [(base + int(i), int(out[i]), int(ro[i]), "reference") for i in rb[:4]]
            n_ref += m
        wl.free()
        n_done += n
        base += n
        print(f"{n_done}/{args.total} verified, {n_ref} checked by the reference, mismatches label={label_mism} "
              f"ref={ref_mism}  ({time.time() - t_start:.0f} s)", file=sys.stderr, flush=True)
    eng.close()
    res = {
        "stream": f"C2 distribution, {args.total} signatures in chunks of {args.chunk}, seed {args.seed:#x}",
        "signatures": n_done, "gpu_seconds": t_gpu, "gpu_verifies_per_s": n_done / t_gpu,
        "label_mismatches": label_mism,
        "reference_checked": n_ref, "reference_mismatches": ref_mism,
        "reference": f"fd_ed25519_verify, {flavour} backend compiled from the reference sources, {args.threads} threads",
        "reference_seconds": t_ref, "reference_verifies_per_s": n_ref / t_ref if t_ref else None,
        "class_counts": dict(zip(workload.CLASS_NAMES, classes.tolist())),
        "code_counts": {str(k): v for k, v in codes_hist.items()},
        "verdict_stream_sha256": dig.hexdigest(),
        "first_mismatches": first_bad[:16],
        "bit_exact": label_mism == 0 and ref_mism == 0,
    }
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)
    print(json.dumps(res))
    return 0 if res["bit_exact"] else 1


if __name__ == "__main__":
    sys.exit(main())
