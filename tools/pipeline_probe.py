#!/usr/bin/env python3
"""Multi-chunk calls with and without the engine's two-lane pipeline: one
verify_dev call of --chunks x max_chunk signatures (C2 distribution),
timed with host wall clock around call + sync, alternating the two engines
rep by rep so box drift hits both alike; the codes of the two agree.

    python tools/pipeline_probe.py [--chunk 1048576] [--chunks 4] [--reps 8]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from firedancer_amd import ed25519  # noqa: E402


def engine(pipeline, chunk):
    return ed25519.Engine(0, max_chunk=chunk, pipeline=pipeline)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--reps", type=int, default=8)
    args = ap.parse_args()
    n = args.chunk * args.chunks
    engs = {"one_lane": engine(False, args.chunk), "two_lanes": engine(True, args.chunk)}
    wls = {k: ed25519.DeviceWorkload(e, n, 64, 1232, 20000, seed=0xC4C4) for k, e in engs.items()}
    ts = {k: [] for k in engs}
    for k, e in engs.items():      # warm: lane 1's scratch is made on the first call
        wls[k].verify()
        e.sync()
    for _ in range(args.reps):
        for k, e in engs.items():
            t0 = time.perf_counter()
            wls[k].verify()
            e.sync()
            ts[k].append(time.perf_counter() - t0)
    outs = {k: wls[k].out.download(np.int8, n) for k in engs}
    agree = bool(np.array_equal(outs["one_lane"], outs["two_lanes"]))
    labels = wls["one_lane"].expect.download(np.int8, n)
    rec = {"signatures_per_call": n, "chunk": args.chunk, "reps": args.reps, "codes_agree": agree,
           "codes_match_labels": bool(np.array_equal(outs["two_lanes"], labels))}
    for k, v in ts.items():
        med = float(np.median(v))
        rec[k] = {"median_ms": 1e3 * med, "min_ms": 1e3 * min(v), "verifies_per_s": n / med}
    rec["gain"] = rec["two_lanes"]["verifies_per_s"] / rec["one_lane"]["verifies_per_s"]
    print(json.dumps(rec), flush=True)
    for w in wls.values():
        w.free()
    for e in engs.values():
        e.close()
    if not agree:
        sys.exit(1)


if __name__ == "__main__":
    main()
