#!/usr/bin/env python3
"""Per-phase time per signature at several chunk sizes (one chunk per
launch): t(n) = a n + tail separates the per-signature cost from the
launch's fixed and tail costs (the last waves of a persistent kernel
finishing unevenly).

    python tools/dsm_tail_probe.py [--sizes 262144,524288,1048576,2097152] [--reps 5]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from firedancer_amd import ed25519  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="262144,524288,1048576,2097152")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    sizes = [int(x) for x in args.sizes.split(",")]
    eng = ed25519.Engine(0, max_chunk=max(sizes))
    for n in sizes:
        wl = ed25519.DeviceWorkload(eng, n, 64, 1232, 20000, seed=11)
        wl.verify()
        eng.sync()
        eng.timing(True)
        for _ in range(args.reps):
            wl.verify()
        eng.sync()
        ph, cnt = eng.timing_read()
        eng.timing(False)
        per = {k: v / cnt for k, v in ph.items()}
        print(json.dumps({"n": n, "ms": per, "ns_per_sig": {k: 1e6 * v / n for k, v in per.items()}}), flush=True)
        wl.free()


if __name__ == "__main__":
    main()
