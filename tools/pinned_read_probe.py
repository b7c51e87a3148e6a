#!/usr/bin/env python3
"""CPU read/write bandwidth of page-locked host memory from hipHostMalloc
(fd_ed25519_hip_host_alloc, the pipe's staging and the drop-ins' blocks)
against ordinary pageable memory: whether the host side of a batch
(staging writes, resolve reads) pays for the pinned mapping.

    python tools/pinned_read_probe.py [--mb 8] [--reps 50]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import ed25519  # noqa: E402

lib = ed25519._lib
lib.fd_ed25519_hip_host_alloc.argtypes = [ctypes.c_ulong]
lib.fd_ed25519_hip_host_alloc.restype = ctypes.c_void_p
lib.fd_ed25519_hip_host_free.argtypes = [ctypes.c_void_p]


def bw(a, b, reps):
    """GB/s of b[:] = a (read a, write b) and of a.sum() (read only)"""
    np.copyto(b, a)
    t = time.perf_counter()
    for _ in range(reps):
        np.copyto(b, a)
    copy = reps * a.nbytes / (time.perf_counter() - t) / 1e9
    a64 = a.view(np.uint64)
    a64.sum()
    t = time.perf_counter()
    for _ in range(reps):
        a64.sum()
    read = reps * a.nbytes / (time.perf_counter() - t) / 1e9
    return copy, read


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=8)
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    n = args.mb << 20
    ed25519.Engine(0, max_chunk=4096).close()   # the HIP runtime up
    p = lib.fd_ed25519_hip_host_alloc(n)
    q = lib.fd_ed25519_hip_host_alloc(n)
    pa = np.ctypeslib.as_array((ctypes.c_ubyte * n).from_address(p))
    pb = np.ctypeslib.as_array((ctypes.c_ubyte * n).from_address(q))
    pa[:] = 7
    pb[:] = 1
    ua, ub = np.full(n, 7, np.uint8), np.ones(n, np.uint8)
    res = {"mb": args.mb}
    res["pageable_copy_GBps"], res["pageable_read_GBps"] = bw(ua, ub, args.reps)
    res["pinned_copy_GBps"], res["pinned_read_GBps"] = bw(pa, pb, args.reps)
    res["pinned_to_pageable_copy_GBps"], _ = bw(pa, ub, args.reps)
    res["pageable_to_pinned_copy_GBps"], _ = bw(ua, pb, args.reps)
    lib.fd_ed25519_hip_host_free(p)
    lib.fd_ed25519_hip_host_free(q)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
