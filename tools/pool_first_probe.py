#!/usr/bin/env python3
"""Diagnostic: host-fed stream rate of the first pool a process creates vs
the next ones (A/B for HIP stream -> hardware queue placement).

    python tools/pool_first_probe.py SLOTS [--side 0|1] [--pools 2]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import ed25519, tile, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("slots", type=int)
    ap.add_argument("--side", type=int, default=1, help="verify once on the main engine first (creates its side stream)")
    ap.add_argument("--pools", type=int, default=2)
    ap.add_argument("--batch", type=int, default=131072)
    args = ap.parse_args()
    cfg = workload.CONFIGS["C2"]
    eng = ed25519.Engine(0, max_chunk=1 << 20)
    wl = ed25519.DeviceWorkload(eng, cfg["n"], cfg["lo"], cfg["hi"], cfg["ppm"], seed=0x5EED)
    if args.side:
        wl.verify()
        eng.sync()
    n, mb, k = wl.n, wl.msg_bytes, 4
    msgs1 = wl.msgs.download(np.uint8, mb)
    off1 = wl.off.download(np.uint64, n)
    msgs = np.concatenate([msgs1] * k + [np.zeros(16, np.uint8)])
    off = np.concatenate([off1 + np.uint64(c * mb) for c in range(k)])
    sz = np.tile(wl.sizes.astype(np.uint32), k)
    sigs = np.tile(wl.sigs.download(np.uint8, 64 * n), k)
    pubs = np.tile(wl.pubs.download(np.uint8, 32 * n), k)
    out = np.zeros(k * n, np.int8)
    cap = tile.max_span(off, sz, args.batch)
    with tile.HostRegistration(msgs, off, sz, sigs, pubs, out):
        for p in range(args.pools):
            pool = tile.Pool([0], args.batch, args.slots, cap)
            pool.run(msgs, off, sz, sigs, pubs, out)
            t = time.perf_counter()
            for _ in range(3):
                pool.run(msgs, off, sz, sigs, pubs, out)
            dt = time.perf_counter() - t
            pool.close()
            print(json.dumps({"slots": args.slots, "side": args.side, "pool": p, "verifies_per_s": 3 * k * n / dt}),
                  flush=True)


if __name__ == "__main__":
    main()
