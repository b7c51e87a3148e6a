#!/usr/bin/env python3
"""A/B of the verify-tile host path between two builds of the library:
the same GPU-signed transactions through fd_ed25519_hip_latency_run
(unpaced) of each .so, interleaved reps.

    python tools/tile_ab.py LIB_A LIB_B [--txns 1000000] [--batch 4096] [--slots 3] [--reps 2]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class Res(ctypes.Structure):
    _fields_ = [("offered", ctypes.c_double), ("txn_per_s", ctypes.c_double), ("sig_per_s", ctypes.c_double),
                ("seconds", ctypes.c_double), ("txn_cnt", ctypes.c_ulong), ("sig_cnt", ctypes.c_ulong),
                ("batches", ctypes.c_ulong), ("overruns", ctypes.c_ulong)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs=2)
    ap.add_argument("--txns", type=int, default=1000000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--slots", type=int, default=3)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    from firedancer_amd import ed25519, workload
    eng = ed25519.Engine(0, max_chunk=1 << 16)
    pay, size = workload.txn_payloads(eng, args.txns, 99, msg_sz=200)
    eng.close()
    n = len(pay)
    buf = np.ascontiguousarray(pay).reshape(-1)
    off = np.arange(n, dtype=np.uint64) * np.uint64(size)
    sz = np.full(n, size, np.uint32)
    libs = [ctypes.CDLL(os.path.abspath(p)) for p in args.libs]
    for rep in range(args.reps):
        for name, lib in zip(args.libs, libs):
            for gpu_parse in (0, 2):
                lat = np.zeros(n, np.float64)
                v = np.zeros(n, np.int8)
                r = Res()
                rc = lib.fd_ed25519_hip_latency_run(ctypes.c_int(0), ctypes.c_uint(args.slots), ctypes.c_ulong(args.batch),
                                                    ctypes.c_void_p(buf.ctypes.data), ctypes.c_void_p(off.ctypes.data),
                                                    ctypes.c_void_p(sz.ctypes.data), ctypes.c_ulong(n),
                                                    ctypes.c_double(0.0), ctypes.c_ulong(1 << 14), ctypes.c_int(gpu_parse),
                                                    ctypes.c_void_p(lat.ctypes.data), ctypes.c_void_p(v.ctypes.data),
                                                    ctypes.byref(r))
                print(json.dumps({"lib": name, "rep": rep, "gpu_parse": bool(gpu_parse), "rc": rc,
                                  "txn_per_s": r.txn_per_s, "p50_ms": float(np.percentile(lat, 50) * 1e3),
                                  "ok": bool((v == 0).all())}), flush=True)


if __name__ == "__main__":
    main()
