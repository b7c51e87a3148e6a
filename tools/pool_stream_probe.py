#!/usr/bin/env python3
"""Diagnostic: host-fed pool rate against what the process created before
the pool (stream placement on the device's hardware queues).

    python tools/pool_stream_probe.py gen PATH             # C2 host arrays -> PATH (.npz)
    python tools/pool_stream_probe.py run PATH [--engines K] [--verify 0|1] [--one-stream 0|1]
                                                [--slots S] [--after-engines K2]

`run` loads the arrays (no engine needed), creates K engines (optionally
verifying once on the first, which creates its decode side stream), then a
pool of S slots, streams the set 4 times x 3 and prints the rate; then K2
more engines and the same pool run again.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from firedancer_amd import ed25519, tile, workload  # noqa: E402


def gen(path):
    cfg = workload.CONFIGS["C2"]
    eng = ed25519.Engine(0, max_chunk=1 << 20)
    wl = ed25519.DeviceWorkload(eng, cfg["n"], cfg["lo"], cfg["hi"], cfg["ppm"], seed=0x5EED)
    n, mb = wl.n, wl.msg_bytes
    np.savez(path, msgs=wl.msgs.download(np.uint8, mb), off=wl.off.download(np.uint64, n),
             sz=wl.sizes.astype(np.uint32), sigs=wl.sigs.download(np.uint8, 64 * n),
             pubs=wl.pubs.download(np.uint8, 32 * n), expect=wl.expect.download(np.int8, n))
    wl.free()
    eng.close()


def run(args):
    d = np.load(args.path)
    k = 4
    mb = len(d["msgs"])
    n = len(d["sz"])
    msgs = np.concatenate([d["msgs"]] * k + [np.zeros(16, np.uint8)])
    off = np.concatenate([d["off"] + np.uint64(c * mb) for c in range(k)])
    sz = np.tile(d["sz"], k)
    sigs, pubs = np.tile(d["sigs"], k), np.tile(d["pubs"], k)
    out = np.zeros(k * n, np.int8)
    expect = np.tile(d["expect"], k)
    engines = []

    def make(cnt):
        for _ in range(cnt):
            engines.append(ed25519.Engine(0, max_chunk=1 << 20, one_stream=bool(args.one_stream)))
        if cnt and args.verify:
            m = 65536   # a large chunk: the throughput form, side stream included
            engines[0].verify_host(d["msgs"], d["off"][:m], d["sz"][:m], d["sigs"][:64 * m], d["pubs"][:32 * m])

    make(args.engines)
    cap = tile.max_span(off, sz, args.batch)
    res = []
    with tile.HostRegistration(msgs, off, sz, sigs, pubs, out):
        pool = tile.Pool([0], args.batch, args.slots, cap)
        for phase in range(2):
            pool.run(msgs, off, sz, sigs, pubs, out)
            t = time.perf_counter()
            for _ in range(3):
                pool.run(msgs, off, sz, sigs, pubs, out)
            dt = time.perf_counter() - t
            res.append({"phase": phase, "engines_before": len(engines), "verifies_per_s": 3 * k * n / dt,
                        "ok": bool(np.array_equal(out, expect))})
            if phase == 0:
                make(args.after_engines)
        pool.close()
    print(json.dumps({"slots": args.slots, "one_stream": args.one_stream, "verify": args.verify, "runs": res}),
          flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["gen", "run"])
    ap.add_argument("path")
    ap.add_argument("--engines", type=int, default=0)
    ap.add_argument("--after-engines", type=int, default=0)
    ap.add_argument("--verify", type=int, default=1)
    ap.add_argument("--one-stream", type=int, default=0)
    ap.add_argument("--slots", type=int, default=3)
    ap.add_argument("--batch", type=int, default=131072)
    args = ap.parse_args()
    if args.mode == "gen":
        gen(args.path)
    else:
        run(args)


if __name__ == "__main__":
    main()
